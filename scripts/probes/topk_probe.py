import sys, os, torch
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from pps_amd import ops
def t(d, k):
    for _ in range(2): ops.topk(d, k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5): ops.topk(d, k)
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / 5
for (R, C) in [(19889, 19889), (2228, 17661), (10000, 125000)]:
    d = torch.rand(R, C, device='cuda')
    dp = ops.dist_buffer(R, C, 'cuda')  # rows padded to 16 bytes: the dwordx4 path
    dp.copy_(d)
    for name, x in (('dense', d), ('padded', dp)):
        if name == 'padded' and C % 4 == 0:
            continue  # same layout as dense
        for k in (21, 100):
            ms = t(x, k)
            print('%dx%d %s k=%d %.3f ms  %.0f GB/s' % (R, C, name, k, ms, R * C * 4 / ms / 1e6),
                  flush=True)
    del d, dp
