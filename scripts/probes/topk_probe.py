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
    for k in (21, 100):
        ms = t(d, k)
        print('%dx%d k=%d %.3f ms  %.0f GB/s' % (R, C, k, ms, R * C * 4 / ms / 1e6), flush=True)
