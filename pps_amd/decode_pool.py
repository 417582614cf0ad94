"""Multi-process JPEG decoding for the feature-extraction loop.

The reference decodes with cv2.imread inside its test loop
(detectron/core/test_engine.py:282-315 -> utils/blob.py:97-117).  Here the
decode is PIL (libjpeg-turbo, the same library and default IDCT /
upsampling as cv2's), and PIL's JPEG plugin parses markers in Python under
the GIL: ~0.25-0.5 ms of GIL-held time per 128x64 image, so decode threads
do not scale and cap the loop near 6.6k images/s while the GPU runs 14k+.
Decoding therefore runs in worker PROCESSES.

The workers come from a `forkserver` started by `start()`.  Call it before
the process initialises the GPU (the CLI entry points and bench.py do, first
thing): the fork server is then started from a process that has not touched
the GPU, and every worker is forked from it.  `pool()` returns None when no
pool was started, and the loop falls back to threads.
"""
import multiprocessing as mp

import numpy as np

_POOL = None
_WORKERS = 0


def decode_bgr(path):
    """cv2.imread(path, IMREAD_COLOR) equivalent: uint8 HxWx3, BGR order."""
    from PIL import Image
    with Image.open(path) as im:
        rgb = np.asarray(im.convert('RGB'), dtype=np.uint8)
    return np.ascontiguousarray(rgb[..., ::-1])


def decode_many(paths):
    return [decode_bgr(p) for p in paths]


def _ready(_):
    return 0


def start(workers):
    """Start `workers` decode processes (no-op if a pool is running or
    workers < 1).  Returns the pool or None."""
    global _POOL, _WORKERS
    if _POOL is not None or workers < 1:
        return _POOL
    ctx = mp.get_context('forkserver')
    ctx.set_forkserver_preload(['numpy', 'PIL.Image', 'PIL.JpegImagePlugin'])
    _POOL = ctx.Pool(workers)
    _POOL.map(_ready, range(workers))   # every worker up before the GPU work starts
    _WORKERS = workers
    return _POOL


def pool():
    return _POOL


def workers():
    return _WORKERS


def stop():
    global _POOL, _WORKERS
    if _POOL is not None:
        _POOL.terminate()
        _POOL.join()
    _POOL, _WORKERS = None, 0


def default_workers(share=1):
    """Decode processes for this process: the CPUs it may use, capped by a
    cgroup CPU quota, divided by `share` (ranks on the node), minus one for
    the main loop."""
    import os
    n = len(os.sched_getaffinity(0))
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, p = f.read().split()
        if q != 'max':
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return max(1, n // max(1, share) - 1)
