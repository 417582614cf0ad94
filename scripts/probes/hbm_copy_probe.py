"""Probe: achievable HBM rates (measured: read 5.25, copy 5.42, add 5.86, fill
6.73 TB/s) for the conv epilogues' traffic mixes on this
device -- read-only (sum), copy (1 read : 1 write), residual add
(2 reads : 1 write) -- with torch's own elementwise kernels on 201 MB tensors
(the res2 activation size at batch 64)."""
import torch

n = 64 * 96 * 32 * 256
a = torch.randn(n, device='cuda')
b = torch.randn(n, device='cuda')
c = torch.empty(n, device='cuda')
s = torch.empty((), device='cuda')


def t(fn, nbytes, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return ms * 1e3, nbytes / (ms * 1e-3) / 1e12


for name, fn, nb in (('read (sum)', lambda: torch.sum(a, dim=(0,), out=s), 4 * n),
                     ('copy', lambda: c.copy_(a), 8 * n),
                     ('add (2R 1W)', lambda: torch.add(a, b, out=c), 12 * n),
                     ('fill (W)', lambda: c.fill_(1.0), 4 * n)):
    us, tbs = t(fn, nb)
    print('%-12s %7.1f us  %.2f TB/s' % (name, us, tbs), flush=True)
