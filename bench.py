"""Benchmark: PPS re-ID inference + retrieval on MI355X (BASELINE.json metric
"gallery images/sec + distmat GB/s; mAP/Rank-1 parity on Market-1501",
workload configs[1]: Market-1501 ResNet-50 PPS, 1xMI355X, batch 64,
3368q x 15913g L2 distmat).

  python bench.py [--gpus N] [--steps K] [--warmup W]

A step = one batch of 64 synthetic Market-sized images (uint8 BGR 128x64,
resident in HBM) through the whole feature path: preprocess (mean-subtract +
bicubic to 384x128) -> ResNet-50/stride-1 res5 -> part power set -> 31 heads
-> L2 normalise.  value = images/s over all ranks (weak scaling: 64 per rank
per step).  The retrieval stage (distance matrix + count-based mAP/CMC at
Market sizes; gallery-sharded across ranks with an all-gather of queries) is
timed after the step loop and reported as distmat_GBps etc.

Multi-GPU: launched by torch.distributed.run, one process per GPU, RCCL.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md chip table (dense f32 MFMA)
PEAK_BF16_MFMA_TFLOPS = 16 * PEAK_FP32_MFMA_TFLOPS   # bf16 MFMA = 16x the f32 rate (~2.5 PF)
# bf16x3 path: every f32 product costs 6 bf16 MFMA terms -> its own MFMA roof
PEAK_X3_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6
# f16x2 distance path (csrc/gemm_h2.hip): 3 f16 MFMA terms per f32-level
# product (f16 MFMA: the bf16 rate) -> its roof in f32-equivalent TFLOP/s
PEAK_H2_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 3
TRAFFIC_FILE = os.path.join(ROOT, 'profiles', 'r06', 'pmc_traffic.json')
PEAK_HBM_GBPS = 8000.0          # MI355X HBM3E spec
Q_MARKET, G_MARKET, D_FEAT = 3368, 15913, 3968


def ops_dist_math():
    from pps_amd import ops
    return ops.dist_math()


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=None,
                   help='ranks (one per GPU); > 1 without WORLD_SIZE in the environment '
                        'launches them (torch.distributed.run, before any GPU call)')
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=3)
    p.add_argument('--batch', type=int, default=64)
    p.add_argument('--no-graph', action='store_true', help='eager launches (no hipGraph)')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-duke', action='store_true',
                   help='skip the Duke configuration leg (configs[2], rank 0 at N = 1)')
    p.add_argument('--no-e2e', action='store_true',
                   help='skip the end-to-end JPEG-files stage (e2e block of the line)')
    p.add_argument('--e2e-images', type=int, default=Q_MARKET + G_MARKET)
    p.add_argument('--dist-reps', type=int, default=5)
    p.add_argument('--no-autotune', action='store_true')
    p.add_argument('--dry-run', action='store_true',
                   help='no GPU work: exercise the launch / rendezvous / reporting path only')
    p.add_argument('--sharded-legs', action='store_true',
                   help='also run the config_cuhk03 / config_1m legs at N = 1 (they run by '
                        'default at N > 1)')
    p.add_argument('--no-sharded-legs', action='store_true')
    p.add_argument('--tiles-file', default=None,
                   help='JSON {layer: tile}: reuse (if present) or save the autotune result, '
                        'so profiling passes run the same kernels as the timed run')
    return p.parse_args()


def launch_ranks(n):
    """`--gpus n` (n > 1) without a launcher: start n ranks of this script
    with torch.distributed.run as a CHILD process (this process has touched
    no GPU and is not replaced), wait, and return its exit code.  Rank 0
    prints the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(n), '--master-addr', '127.0.0.1', '--master-port', str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get(
        'HSA_ENABLE_IPC_MODE_LEGACY', '0'))
    return subprocess.call(cmd, env=env)


def market_cfg():
    from pps_amd import config
    cfg = config.cfg
    cfg.MODEL.NUM_CLASSES = 752
    cfg.MODEL.USE_BN = True
    cfg.RESNETS.RES5_STRIDE = 1
    cfg.REID.SCALE = (128, 384)
    cfg.REID.BPM_STRIP_NUM = 5
    cfg.REID.BPM_DIM = 128
    cfg.REID.NORMALIZE_FEATURE = True
    cfg.REID.MAX_AVE_FEATURE = True
    cfg.REID.RERANK = False
    return cfg


def synth_features(n, ids, gen, noise=4.0, n_ids=750, dim=D_FEAT, device='cuda'):
    """SURVEY §8(d) recipe on the device: centroid[id] + noise*N(0,1), L2 norm."""
    cent = torch.randn((n_ids + 1, dim), generator=gen, device=device)
    x = cent[ids] + noise * torch.randn((n, dim), generator=gen, device=device)
    return (x / x.norm(dim=1, keepdim=True)).contiguous()


def retrieval_inputs(nq, ng, n_distractors, n_ids, dim=D_FEAT, device='cuda'):
    """Seeded ids / cams and the [nq + ng, dim] features (queries first) of a
    retrieval workload: the same global data on every rank."""
    rng = np.random.RandomState(0)
    qid = rng.randint(1, n_ids + 1, nq)
    gid = np.concatenate([rng.randint(1, n_ids + 1, ng - n_distractors),
                          np.zeros(n_distractors, int)])
    qcam = rng.randint(1, 7, nq)
    gcam = rng.randint(1, 7, ng)
    gen = torch.Generator(device=device)
    gen.manual_seed(0)
    allf = synth_features(nq + ng, torch.from_numpy(np.concatenate([qid, gid])).to(device), gen,
                          n_ids=n_ids, dim=dim, device=device)
    return qid, gid, qcam, gcam, allf


def retrieval_stage(rank, world, reps, tune=True, nq=Q_MARKET, ng=G_MARKET,
                    n_distractors=2793, n_ids=750, backend=None, device='cuda', dim=D_FEAT):
    """Distance matrix + mAP/CMC (default: Market sizes; the config_cuhk03
    leg and scripts/bench_retrieval_sharded.py pass other splits).  Gallery
    sharded over ranks, queries all-gathered.  Returns timings
    (ms) and scores.  backend / device: the product HipBackend on the GPU, or
    (tests/test_distributed_cpu.py) the oracle's CpuBackend on CPU with gloo,
    which runs the same collective code with host timers and no rooflines."""
    from pps_amd import distributed as pdist
    Q_MARKET, G_MARKET = nq, ng   # local names: the sizes of this run
    qid, gid, qcam, gcam, allf = retrieval_inputs(nq, ng, n_distractors, n_ids, dim, device)
    qsl = pdist.shard_range(Q_MARKET, rank, world)
    gsl = pdist.shard_range(G_MARKET, rank, world)
    q_local = allf[qsl[0]:qsl[1]].contiguous()
    g_local = allf[Q_MARKET + gsl[0]:Q_MARKET + gsl[1]].contiguous()
    del allf
    ev = pdist.ShardedEvaluator(qid, qcam, gid, gcam, rank, world, backend=backend)
    gpu = device == 'cuda'
    tune = tune and gpu
    if tune:
        # distance-GEMM tile choice on this shard's shape (outside the timed runs)
        from pps_amd import ops
        gen = torch.Generator(device='cuda')
        gen.manual_seed(1)
        qa = torch.empty((Q_MARKET, dim), device='cuda').normal_(generator=gen)
        # gallery index and query planes prepared once: the tiles compete on the
        # GEMM alone (what roofline_distmat times)
        h2 = ops.dist_math() == 'h2' and dim % 32 == 0
        if h2:   # f16x2 split of both operands; the h2 tiles compete
            gidx = ops.GalleryIndex(g_local, math='h2')
            q2, qrs, qsq = ops.split_h2_tiled(qa)
            qt = None
            cands = [(t, False) for t in range(1, ops.h2_num_tiles())]
        else:
            gidx = ops.GalleryIndex(g_local, tiled=dim % 32 == 0, math='x3')
            qt, qsq = ops.split_sqnorm_tiled(qa) if dim % 32 == 0 else (None, None)
            # (the 3x3-patch ids 56+ run tile 38 on a distance matrix)
            cands = [(t, False) for t in range(1, ops.TILE_C16_FIRST)]
            if ops.dist_math() == 'x3' and dim % 32 == 0:  # queries as planes too
                cands += [(t, True) for t in range(ops.TILE_P_FIRST, ops.TILE_C16_FIRST)]
        dout = ops.dist_buffer(Q_MARKET, g_local.shape[0], 'cuda')

        def launch_dist(t, qp):
            if h2:
                ops.distmat_h2(q2, qrs, qsq, gidx, dout, tile=t)
            elif qp:
                ops.distmat_planes(None, qsq, gidx, dout, tile=t, q_tiled=qt, Q=Q_MARKET,
                                   D=dim)
            else:
                ops.compute_dist(qa, gidx, out=dout, tile=t)

        def time_dist(t, qp, n):
            launch_dist(t, qp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                launch_dist(t, qp)
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / n

        # one launch each to screen, then the 4 best re-timed in three
        # interleaved rounds of 5 launches, min per tile (single launches left
        # the pick to +-3 % noise between close tiles; interleaving keeps a
        # drifting clock from favouring whichever ran first)
        screen = {c: time_dist(c[0], c[1], 1) for c in cands}
        fin = sorted(screen, key=screen.get)[:4]
        final = {c: 1e30 for c in fin}
        for _ in range(3):
            for c in fin:
                final[c] = min(final[c], time_dist(c[0], c[1], 5))
        best = min(final, key=final.get)
        pdist.HipBackend.distmat_tile = best[0]
        pdist.HipBackend.distmat_qplanes = best[1]
        del qa, gidx, qt, dout
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    # warm-up
    res = ev.run(q_local, g_local)
    sync()
    t_gather, t_dist, t_rank, t_total = [], [], [], []
    for _ in range(reps):
        pdist.barrier(world)
        sync()
        t0 = time.perf_counter()
        res = ev.run(q_local, g_local, timed=True, keep_dist=True)
        sync()
        if gpu:
            t_gather.append(res['t_gather_ms'])
            t_dist.append(res['t_distmat_ms'])
            t_rank.append(res['t_rank_ms'])
            t_total.append(res['t_total_ms'])
        else:   # host timers: the whole run only
            t_total.append((time.perf_counter() - t0) * 1e3)
    rank_roof = rank_roofline(ev, res['dist']) if gpu else None
    argsort_roof = argsort_roofline(res['dist']) if gpu else None
    dist_roof = distmat_roofline(q_local, g_local, world) if gpu else None
    del res['dist']
    med = lambda v: float(np.median(v)) if v else None   # noqa: E731
    be = ev.backend
    out = dict(rank_roofline=rank_roof, dist_roofline=dist_roof, argsort_roofline=argsort_roof,
               distmat_tile=getattr(be, 'distmat_tile', None),
               distmat_qplanes=getattr(be, 'distmat_qplanes', None),
               gather_ms=med(t_gather), distmat_ms=med(t_dist), rank_eval_ms=med(t_rank),
               retrieval_ms=med(t_total), mAP=res['mAP'], cmc=[float(c) for c in res['cmc']],
               cmc1=float(res['cmc'][0]), cmc5=float(res['cmc'][4]),
               cmc10=float(res['cmc'][9]), G_local=gsl[1] - gsl[0])
    return out


def distmat_roofline(q_local, g_local, world, reps=10):
    """The distance GEMM launch alone (gemm_h2_kernel, or gemm_x3p_kernel
    EPI_DIST, on the bench's tile), the way a gallery index is used: gallery
    split + norms prepared once (GalleryIndex), queries split once; `reps`
    launches between HIP events on the kernel's stream.  Algorithmic work
    2 Q G_r D FLOP, priced against the MFMA roof of the arithmetic the kernel
    runs (h2: 3 f16 terms per product; x3: 6 bf16 terms)."""
    from pps_amd import ops
    from pps_amd import distributed as pdist
    be = pdist.HipBackend
    dm = ops.dist_math()
    if dm == 'f32':
        return None
    q_all = pdist.all_gather_rows(q_local, [q_local.shape[0]] * world) if world > 1 else q_local
    Q, D = q_all.shape
    h2 = dm == 'h2' and D % 32 == 0
    idx = ops.GalleryIndex(g_local, math='h2' if h2 else 'x3')
    out = ops.dist_buffer(Q, g_local.shape[0], q_all.device)
    qp = bool(be.distmat_qplanes)
    if h2:
        q2, qrs, qsq = ops.split_h2_tiled(q_all)
        launch = lambda: ops.distmat_h2(q2, qrs, qsq, idx, out, tile=be.distmat_tile)
    elif qp:
        q3, qsq = ops.split_sqnorm(q_all)
        q3t = ops.tile_planes(q3) if D % 32 == 0 else None
        launch = lambda: ops.distmat_planes(q3, qsq, idx, out, tile=be.distmat_tile, q_tiled=q3t)
    else:
        launch = lambda: ops.compute_dist(q_all, idx, out=out, tile=be.distmat_tile)
    for _ in range(2):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    G = g_local.shape[0]
    flops = 2.0 * Q * G * D
    # the operand planes read once + the matrix written once
    byt = (Q + G) * D * (4 if h2 else 6) + Q * G * 4
    tf = flops / (us * 1e-6) / 1e12
    peak = PEAK_H2_TFLOPS if h2 else PEAK_X3_TFLOPS
    return dict(achieved=round(tf, 2), peak=round(peak, 1), frac=round(tf / peak, 4),
                frac_of_x3_roof=round(tf / PEAK_X3_TFLOPS, 4),
                math='h2' if h2 else 'x3',
                avg_launch_us=round(us, 2), flops_per_launch=flops,
                operand_and_output_bytes_per_launch=byt, queries_as_planes=bool(qp or h2),
                timing='%d launches between HIP events, gallery index and query split '
                       'prepared once' % reps)


def rank_roofline(ev, dist, reps=20):
    """The rank stage's dominant kernel, rank_count_stream (one pure stream
    over the [Q, G_r] distance block), timed with HIP events on the stream it
    runs on: algorithmic bytes = Q * G_r * 4 (every distance read once; the
    sorted positive lists and counts are kilobytes) per launch."""
    from pps_amd import ops
    from pps_amd import distributed as pdist
    state = ev._state or pdist.HipBackend.prepare(ev)
    pd_, pi_, pc_, junk = ops.collect_matches(dist, state, ev.g_offset, ev.pmax)
    sp = ops.rank_prepare(pd_[None], pi_[None], pc_[None])
    hist, before = ops.rank_count_stream(dist, ev.g_offset, sp, junk)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.rank_count_stream(dist, ev.g_offset, sp, junk, hist, before)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    Q, G = dist.shape
    byt = Q * G * 4
    return dict(bound='hbm', achieved=round(byt / (us * 1e-6) / 1e9, 1), peak=PEAK_HBM_GBPS,
                unit='GB/s', frac=round(byt / (us * 1e-6) / 1e9 / PEAK_HBM_GBPS, 4),
                traffic=_pmc_traffic('rank', ops.default_math(), None),
                kernel='rank_count_stream_kernel (one 16-byte stream per row chunk, '
                       'binary search + LDS histogram against the sorted positives)',
                avg_launch_us=round(us, 2), algorithmic_bytes_per_launch=byt,
                rows=Q, cols=G, row_stride=dist.stride(0))


def argsort_roofline(dist, reps=10):
    """The full stable rank list of the same distance block (the reference's
    np.argsort(distmat, axis=1), reid_dataset_evaluator.py:319,420) by
    pps_argsort_rows, timed with HIP events on its stream: algorithmic bytes
    = Q * G * 4 read + Q * G * 4 indices written per launch.  Reported beside
    the evaluator's path (which needs only the ranks of the positives)."""
    from pps_amd import ops
    Q, G = dist.shape
    if G > ops._lib.lib().pps_argsort_rows_cap():
        return None
    idx = ops.argsort_rows(dist)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.argsort_rows(dist)
    e1.record()
    e1.synchronize()
    del idx
    us = e0.elapsed_time(e1) * 1e3 / reps
    byt = 2 * Q * G * 4
    return dict(bound='hbm', achieved=round(byt / (us * 1e-6) / 1e9, 1), peak=PEAK_HBM_GBPS,
                unit='GB/s', frac=round(byt / (us * 1e-6) / 1e9 / PEAK_HBM_GBPS, 4),
                kernel='argsort_rows_kernel (row in LDS: bucket histogram / scatter, in-bucket '
                       'ranks, sorted row streamed out)',
                avg_launch_us=round(us, 2), algorithmic_bytes_per_launch=byt, rows=Q, cols=G)


# BASELINE configs[3] / configs[4]: CUHK03-detected (new
# protocol) and the synthetic 1M-gallery x 10k-query, 2048-d shard stress
CUHK03 = dict(nq=1400, ng=5332, n_distractors=0, n_ids=700)
SHARD_1M = dict(nq=10000, ng=1000000, dim=2048, k=100)


class _Stamps(object):
    """Stage boundaries: HIP events on the GPU (read after one sync), host
    clocks on the CPU rehearsal."""

    def __init__(self, gpu):
        self.gpu, self.t = gpu, []

    def mark(self):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.t.append(e)
        else:
            self.t.append(time.perf_counter())

    def ms(self):
        if self.gpu:
            self.t[-1].synchronize()
            return [a.elapsed_time(b) for a, b in zip(self.t, self.t[1:])]
        return [(b - a) * 1e3 for a, b in zip(self.t, self.t[1:])]


def config_cuhk03(rank, world, reps=5, backend=None, device='cuda', sizes=None):
    """BASELINE configs[3]: CUHK03-detected retrieval, 1400 queries x 5332
    gallery, the gallery sharded over the ranks, queries
    all-gathered over RCCL, each rank's distance block + per-shard match
    lists (all-gathered) + additive counts (all-reduced), mAP / CMC -- the
    product path of pps_amd/distributed.py (replaces the reference's
    subprocess fan-out + one-host evaluation, utils/subprocess.py:39-103,
    core/test_engine.py:184-229).  Stage times are medians over `reps`, the
    max over ranks."""
    from pps_amd import distributed as pdist
    sz = dict(CUHK03, **(sizes or {}))
    dim = sz.pop('dim', D_FEAT)
    ret = retrieval_stage(rank, world, reps, tune=True, backend=backend, device=device, dim=dim,
                          **sz)
    mx = lambda v: None if v is None else round(pdist.max_over_ranks(v, world), 4)  # noqa: E731
    nq, ng = sz['nq'], sz['ng']
    total_ms = mx(ret['retrieval_ms'])
    out = dict(workload='CUHK03-detected retrieval, %dq x %dg, D=%d, L2, gallery-sharded over %d '
                        'rank(s), queries all-gathered, counts all-reduced' % (nq, ng, dim, world),
               n_ranks=world, G_local_rank0=ret['G_local'],
               query_allgather_ms=mx(ret['gather_ms']), distmat_ms=mx(ret['distmat_ms']),
               rank_eval_ms=mx(ret['rank_eval_ms']), retrieval_ms=total_ms,
               queries_per_s=round(nq / (total_ms * 1e-3), 1) if total_ms else None,
               distmat_GBps=(round(((nq + ng) * dim * 4 + nq * ng * 4) /
                                   (mx(ret['distmat_ms']) * 1e-3) / 1e9, 2)
                             if ret['distmat_ms'] else None),
               mAP_synthetic=round(ret['mAP'], 9), cmc=ret['cmc'],
               cmc1_synthetic=ret['cmc1'], cmc5_synthetic=ret['cmc5'],
               roofline_distmat_rank0=ret['dist_roofline'],
               roofline_rank_rank0=ret['rank_roofline'],
               timing='median of %d runs per rank (HIP events: all-gather / GEMM / lists + '
                      'counts + all-reduce + AP), max over ranks' % reps,
               data='synthetic (SURVEY §8(d) recipe: 700 centroids + noise 4.0, L2 norm)')
    return out


def synth_rows(a, b, dim, seed, device='cuda', chunk=8192):
    """Rows [a, b) of a seeded, L2-normalised Gaussian [*, dim] matrix whose
    rows do not depend on how it is sharded: chunk c of `chunk` rows is drawn
    from seed * 1000003 + c."""
    out = torch.empty((max(b - a, 0), dim), dtype=torch.float32, device=device)
    gen = torch.Generator(device=device)
    for c in range(a // chunk, (b + chunk - 1) // chunk):
        lo, hi = max(a, c * chunk), min(b, (c + 1) * chunk)
        if lo >= hi:
            continue
        gen.manual_seed(seed * 1000003 + c)
        blk = torch.randn((chunk, dim), generator=gen, device=device)
        out[lo - a:hi - a] = blk[lo - c * chunk:hi - c * chunk]
    out /= out.norm(dim=1, keepdim=True)
    return out


def config_1m(rank, world, reps=3, backend=None, device='cuda', sizes=None, keep=False):
    """BASELINE configs[4]: the synthetic 1M-gallery x 10k-query, 2048-d
    sharded distance matrix (the HBM-roofline stress):
    rank r owns gallery rows shard_range(1M, r, world) (a [10k, 1M/world]
    block), the query shards are all-gathered, each rank takes the stable
    top-100 of its block (pps_topk), the lists are all-gathered and merged
    by (distance, global index) (pps_topk_merge) into the global top-100 of
    every query -- the reference's np.argsort(distmat, axis=1)[:, :100]
    (reid_dataset_evaluator.py:319,420) over the unsharded matrix.  Features:
    synth_rows (seeded normalised Gaussian, sharding-independent).  keep:
    also return the merged (vals, idx) (the CPU rehearsal checks them)."""
    from pps_amd import distributed as pdist
    be = backend or pdist.HipBackend
    sz = dict(SHARD_1M, **(sizes or {}))
    nq, ng, dim, k = sz['nq'], sz['ng'], sz['dim'], sz['k']
    gpu = device == 'cuda'
    qa, qb = pdist.shard_range(nq, rank, world)
    ga, gb = pdist.shard_range(ng, rank, world)
    q_sizes = [b - a for a, b in (pdist.shard_range(nq, r, world) for r in range(world))]
    offsets = [pdist.shard_range(ng, r, world)[0] for r in range(world)]
    q_local = synth_rows(qa, qb, dim, 1, device)
    g_local = synth_rows(ga, gb, dim, 2, device)
    G = gb - ga
    kin = min(k, G)
    st = _Stamps(gpu)
    if gpu:
        from pps_amd import ops
        # the gallery prepared once per shard, in sub-blocks whose f16x2 planes
        # stay under the 2 GiB a buffer resource addresses (1M / 2 ranks =
        # 500k rows of 2048-d: 4 GB of planes), each scored into its columns
        sub = max(4, min(G, ((2 ** 31 - 2 ** 20) // (dim * 4)) // 4 * 4))
        st.mark()
        index = [(a, ops.GalleryIndex(g_local[a:a + sub])) for a in range(0, G, sub)]
        st.mark()
        index_ms = st.ms()[0]
        dist = ops.dist_buffer(nq, G, device)

        def gemm(q_all):
            for a, ix in index:
                ops.compute_dist(q_all, ix, out=dist[:, a:a + ix.shape[0]], tile=be.distmat_tile)
            return dist
    else:
        index, index_ms, dist = g_local, None, None

    def once():
        s = _Stamps(gpu)
        s.mark()
        q_all = pdist.all_gather_rows(q_local, q_sizes)
        s.mark()
        if gpu:
            d = gemm(q_all)
        else:
            d = be.distmat(q_all, index, 'euclidean')
        s.mark()
        vals, idx = be.topk(d, kin)
        if kin < k:   # a shard shorter than k: pad its list with (+inf, -1)
            pv = torch.full((nq, k), float('inf'), dtype=torch.float32, device=vals.device)
            pi = torch.full((nq, k), -1, dtype=torch.int32, device=vals.device)
            pv[:, :kin], pi[:, :kin] = vals, idx
            vals, idx = pv, pi
        s.mark()
        av = pdist.all_gather_rows(vals.contiguous()[None], [1] * world)
        ai = pdist.all_gather_rows(idx.contiguous()[None], [1] * world)
        mv, mi = be.topk_merge(av.contiguous(), ai.contiguous(), offsets, k)
        s.mark()
        return s.ms(), (mv, mi)

    once()   # warm-up
    times = []
    for _ in range(reps):
        pdist.barrier(world)
        if gpu:
            torch.cuda.synchronize()
        t, merged = once()
        times.append(t)
    med = [float(np.median([t[i] for t in times])) for i in range(4)]
    mx = [pdist.max_over_ranks(v, world) for v in med]
    total = pdist.max_over_ranks(float(np.median([sum(t) for t in times])), world)
    out = dict(workload='synthetic %dq x %dg, D=%d, L2, gallery-sharded over %d rank(s) (%d rows '
                        'each), per-rank stable top-%d + all-gather + merge'
                        % (nq, ng, dim, world, G, k),
               n_ranks=world, G_local_rank0=G,
               gallery_index_ms_rank0=round(index_ms, 3) if index_ms is not None else None,
               query_allgather_ms=round(mx[0], 3), distmat_ms=round(mx[1], 3),
               topk_ms=round(mx[2], 3), list_allgather_merge_ms=round(mx[3], 3),
               total_ms=round(total, 3), queries_per_s=round(nq / (total * 1e-3), 1),
               distmat_GBps=round(((nq + ng) * dim * 4 + nq * ng * 4) / (mx[1] * 1e-3) / 1e9, 2),
               timing='median of %d runs per rank, stage boundaries by %s, max over ranks'
                      % (reps, 'HIP events' if gpu else 'host clock'),
               data='synthetic (seeded normalised Gaussian rows, synth_rows)')
    if gpu:
        from pps_amd import ops
        # the two kernels of the leg on their own, rank 0's shard: the
        # distance GEMM (f16x2 roof) and the stable top-k stream (HBM)
        n = 3
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        q_all = pdist.all_gather_rows(q_local, q_sizes)
        e0.record()
        for _ in range(n):
            gemm(q_all)
        e1.record()
        for _ in range(n):
            be.topk(dist, kin)
        e2.record()
        e2.synchronize()
        gemm_us = e0.elapsed_time(e1) * 1e3 / n
        topk_us = e1.elapsed_time(e2) * 1e3 / n
        flops = 2.0 * nq * G * dim
        h2 = index[0][1].math == 'h2'
        peak = PEAK_H2_TFLOPS if h2 else PEAK_X3_TFLOPS
        tb = nq * G * 4 + nq * kin * 8
        out['roofline_distmat_rank0'] = dict(
            bound='mfma', achieved=round(flops / gemm_us / 1e6, 2), peak=round(peak, 1),
            unit='TFLOP/s', frac=round(flops / gemm_us / 1e6 / peak, 4),
            math='h2' if h2 else 'x3', avg_launch_us=round(gemm_us, 1),
            note='compute_dist on the prepared GalleryIndex sub-blocks (%d; query split + '
                 'GEMM per sub-block)' % len(index))
        out['roofline_topk_rank0'] = dict(
            bound='hbm', achieved=round(tb / topk_us / 1e3, 1),
            peak=PEAK_HBM_GBPS, unit='GB/s',
            frac=round(tb / topk_us / 1e3 / PEAK_HBM_GBPS, 4), avg_launch_us=round(topk_us, 1),
            algorithmic_bytes_per_launch=tb,
            kernel='topk_wave_kernel (stable top-%d, one stream over the block)' % kin)
    if keep:
        out['merged'] = merged
    return out


def _pmc_traffic(key, math, batch):
    """HBM bytes per launch measured by rocprofv3 PMC passes of this bench
    (scripts/pmc_traffic.py -> profiles/r06/pmc_traffic.json): FETCH_SIZE x 2
    (gfx950 reports half of wide streaming reads) + WRITE_SIZE, per launch.
    None unless the file was measured for the same math and batch."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    e = t.get(key)
    # conv entries carry the model's base arithmetic as model_math (their
    # `math` names the f16x2 / bf16x3 launch mix)
    if not e or (e.get('model_math', e.get('math', math)) != math) or \
            (batch is not None and e.get('batch', batch) != batch):
        return None
    return e.get('bytes_per_launch')


def _pmc_mfma(math, batch):
    """Conv stack's MFMA-busy fraction from the committed PMC pass
    (SQ_VALU_MFMA_BUSY_CYCLES over the launches' trace durations, at 2.4 GHz
    and at the DPM clock the bench sampled; scripts/pmc_traffic.py), same
    model arithmetic and batch."""
    try:
        with open(TRAFFIC_FILE) as f:
            e = json.load(f).get('conv_mfma')
    except (OSError, ValueError):
        return None
    if not e or e.get('model_math', e.get('math')) != math or e.get('batch') != batch:
        return None
    return {k: e[k] for k in ('mfma_busy_frac_at_2p4GHz', 'mfma_busy_frac_at_dpm_clock',
                              'dpm_clock_MHz', 'math') if k in e}


def conv_roofline(nm, x, reps=20):
    """Conv-stack roofline from the timed execution, through the whole-network
    C entry point: pps_forward captured in a hipGraph and replayed `reps`
    times between two HIP events on the kernels' stream gives the forward's
    time as the timed step runs it; eager passes of pps_forward_layers, one
    layer each with an event between layers (median of five), split it by
    launch.  The events add ~1-10 us per launch to the eager split, so the
    split is rescaled to the graph-replay total (ROCm does not allow event
    nodes inside a captured graph, which would time launches in the replay
    directly)."""
    from pps_amd import ops
    N = int(x.shape[0])
    layers = nm.layers(N)
    out = torch.empty((N, nm.feat_dim), dtype=torch.float32, device='cuda')
    nm.forward(x, out=out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        nm.forward(x, out=out)
    for _ in range(3):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    e1.synchronize()
    fwd_ms = e0.elapsed_time(e1) / reps
    # launch units: a PPS_TILE_SEAM layer and the next branch2a it computes
    # are one launch (timed as forward_layers(i, i + 2))
    units, i = [], 0
    while i < len(layers):
        n = 2 if (layers[i]['tile'] & ops.TILE_SEAM) and i + 1 < len(layers) else 1
        units.append((i, n))
        i += n
    splits = []
    for _ in range(5):   # per-launch medians of five eager passes
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(units) + 1)]
        evs[0].record()
        for u, (i, n) in enumerate(units):
            nm.forward_layers(x, i, i + n, out=out, keep_amax=True)
            evs[u + 1].record()
        torch.cuda.synchronize()
        splits.append([evs[u].elapsed_time(evs[u + 1]) for u in range(len(units))])
    eager = [float(v) for v in np.median(np.array(splits), axis=0)]
    scale = fwd_ms / sum(eager)
    per = {}
    for (i, n), t in zip(units, eager):
        L = layers[i]
        if n == 1:
            per[L['name']] = dict(op=L['op'], flops=L['flops'], ms=t * scale, ms_eager=t,
                                  bytes=L['bytes'], tile=L['tile'], planes_out=L['planes_out'],
                                  gemm=L['gemm'])
        else:   # the seam: both layers' FLOPs; the trunk is not re-read by branch2a
            X = layers[i + 1]
            trunk = 4.0 * float(np.prod(L['out_shape']))
            per[L['name'] + '+' + X['name']] = dict(
                op='seam', flops=L['flops'] + X['flops'], ms=t * scale, ms_eager=t,
                bytes=L['bytes'] + X['bytes'] - trunk, tile=L['tile'], planes_out=False,
                gemm=True)
    conv = [v for v in per.values() if v['gemm']]
    conv_ms = sum(v['ms'] for v in conv)
    conv_flops = sum(v['flops'] for v in conv)
    conv_bytes = sum(v['bytes'] for v in conv)
    n_launch = len(conv)
    achieved = conv_flops / (conv_ms * 1e-3) / 1e12
    # f16x2 launches (PPS_TILE_H2) run 3 f16 MFMA terms per product, the rest
    # 6 bf16 terms: the roof of a mixed table is the flop-weighted harmonic
    # blend of the two (the time the whole stack takes at both peaks)
    h2_flops = sum(v['flops'] for v in conv if v['tile'] & ops.TILE_H2)
    if nm.math == 'x3' and h2_flops:
        peak = conv_flops / (h2_flops / PEAK_H2_TFLOPS + (conv_flops - h2_flops) / PEAK_X3_TFLOPS)
        kernel = ('implicit-GEMM conv, %d f16x2 launches (PPS_TILE_H2: 3 f16 MFMA terms per '
                  'product, per-tensor power-of-two activation scale) + %d bf16x3 launches '
                  '(6 bf16 terms): gemm_x3p_kernel<*>, gemm_x3c_kernel<*>, gemm_ws_kernel<*>, the '
                  'fused stem; per-layer autotune; peak = flop-weighted blend of %.1f and %.1f '
                  'TF/s' % (sum(1 for v in conv if v['tile'] & ops.TILE_H2),
                            sum(1 for v in conv if not v['tile'] & ops.TILE_H2),
                            PEAK_H2_TFLOPS, PEAK_X3_TFLOPS))
    elif nm.math == 'x3':
        peak, kernel = PEAK_X3_TFLOPS, ('implicit-GEMM conv: gemm_x3p_kernel<*> (LDS-DMA pipelined), gemm_x3c_kernel<*> (3x3 '
                                        'from LDS input patches), gemm_ws_kernel<*> (weight-stationary 1x1), per-layer autotune; '
                                        '+ the fused stem (stem_ring_x3_kernel); f32 products as 6 '
                                        'bf16 MFMA terms (%d launches/forward, run by pps_forward)' % n_launch)
    else:
        peak, kernel = PEAK_FP32_MFMA_TFLOPS, ('gemm_f32_kernel<*> implicit-GEMM conv '
                                               '(%d launches/forward, run by pps_forward)' % n_launch)
    return dict(bound='mfma', achieved=round(achieved, 2), peak=round(peak, 1),
                unit='TFLOP/s', frac=round(achieved / peak, 4),
                traffic=_pmc_traffic('conv', nm.math, N), kernel=kernel,
                pmc_mfma=_pmc_mfma(nm.math, N),
                launches=n_launch, flops_per_forward=conv_flops,
                algorithmic_bytes_per_launch=round(conv_bytes / n_launch),
                avg_launch_us=round(conv_ms * 1e3 / n_launch, 2),
                forward_graph_ms=round(fwd_ms, 3),
                forward_eager_event_ms=round(sum(eager), 3),
                timing='pps_forward hipGraph replayed %d x between HIP events; per-launch split '
                       'from eager pps_forward_layers passes with events between layers (median '
                       'of 5), rescaled to the replay total' % reps,
                frac_of_f32_mfma_peak=round(achieved / PEAK_FP32_MFMA_TFLOPS, 4),
                frac_of_x3_roof=round(achieved / PEAK_X3_TFLOPS, 4),
                h2_flop_share=round(h2_flops / conv_flops, 4)), per


def usable_cores():
    """(threads to use, sched_getaffinity count, cgroup CPU quota or None):
    the CPUs this process may run on, capped by a cgroup v2 quota if one is
    set (a GPU box's share of a larger host)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, period = f.read().split()[:2]
        if q != 'max':
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    return use, aff, quota


class ClockSampler(object):
    """Shader clock of this rank's GPU during the timed loop (VERDICT r03:
    tell box-to-box spread from a regression).  Reads the driver's current
    sclk level (sysfs pp_dpm_sclk, the '*' line) from a host thread every
    `period` s while the GPU replays the step; the host thread only waits on
    the GPU meanwhile.  pp_dpm_sclk is the DPM level the SMU reports, up to
    ~10 % above the in-kernel clock of MFMA-dense kernels
    (MI355X_MICROARCH.md, DVFS give-back): a box-spread indicator, not the
    effective clock (the PMC pass's GRBM_GUI_ACTIVE is that)."""

    def __init__(self, device=0, period=0.02):
        import threading
        self.path = self._find(device)
        self.period = period
        self.samples = []
        self._stop = threading.Event()
        self._thread = None

    @staticmethod
    def _find(device):
        import glob
        try:
            pr = torch.cuda.get_device_properties(device)
            bdf = '%04x:%02x:%02x.0' % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
        except Exception:
            return None
        cands = ['/sys/bus/pci/devices/%s/pp_dpm_sclk' % bdf]
        for p in glob.glob('/sys/class/drm/card*/device/pp_dpm_sclk'):
            if os.path.basename(os.path.realpath(os.path.dirname(p))) == bdf:
                cands.append(p)
        for p in cands:
            if os.path.exists(p):
                return p
        return None

    def read(self):
        if not self.path:
            return None
        try:
            with open(self.path) as f:
                for line in f:
                    if line.rstrip().endswith('*'):
                        return float(line.split(':', 1)[1].strip().rstrip('*').strip()
                                     .lower().replace('mhz', ''))
        except (OSError, ValueError, IndexError):
            return None
        return None

    def _run(self):
        while not self._stop.is_set():
            v = self.read()
            if v is not None:
                self.samples.append(v)
            self._stop.wait(self.period)

    def __enter__(self):
        import threading
        self.before = self.read()
        if self.path:
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._thread is not None:
            self._thread.join()
        self.after = self.read()

    def summary(self):
        s = np.array(self.samples, np.float64)
        if not self.path:
            return dict(source=None, note='pp_dpm_sclk not readable on this host')
        return dict(source=self.path, unit='MHz', before=self.before, after=self.after,
                    samples=int(s.size),
                    median=float(np.median(s)) if s.size else None,
                    min=float(s.min()) if s.size else None,
                    max=float(s.max()) if s.size else None,
                    note='DPM level during the timed loop (host thread, %g s period); '
                         'the in-kernel clock of MFMA-dense kernels reads up to ~10 %% '
                         'lower' % self.period)


def table_digest(nm):
    """The tuning table behind `value`: a digest of (layer, tile, planes,
    split-K) and the layer count per rounding group (tests/_tiles.py: the
    32x32x16 group below tile 38, the 16x16x32 group 38-55 incl. the
    weight-stationary 54, the patch-staged 3x3 group 56-59; the stem and the
    head reduction are fixed kernels)."""
    import hashlib
    from pps_amd import ops
    layers = nm.layers()
    planes = set(nm.planes())
    rows, groups = [], {}
    for L in layers:
        if L['op'] not in ('conv', 'conv_dual', 'heads', 'conv_pps', 'stem_pool'):
            continue
        t = L['tile']
        rows.append('%s:%d:%d:%d' % (L['name'], t, int(L['name'] in planes), L['splitk']))
        base = t & 0xff
        g = ('auto' if base == 0 else 'x32' if base < ops.TILE_P16_FIRST else
             'x16' if base < ops.TILE_C16_FIRST else 'patch')
        if t & ops.TILE_H2:   # f16x2 arithmetic: its own rounding groups
            g = 'h2_' + ('x16' if base < ops.TILE_C16_FIRST else 'patch')
        if L['op'] == 'stem_pool':
            g = 'stem_h2' if t & ops.TILE_H2 else 'stem'
            if t & ops.TILE_H2:
                rows[-1] += ':h2'   # (the stem's tile alone, 0 / 0x800, would collide with nothing)
        groups[g] = groups.get(g, 0) + 1
    return dict(sha1=hashlib.sha1('\n'.join(rows).encode()).hexdigest()[:16],
                layers_per_rounding_group=groups, plane_edges=len(planes),
                splitk_layers=sum(1 for L in layers if L['splitk'] > 1),
                seam_pairs=sum(1 for L in layers if L['tile'] & ops.TILE_SEAM),
                h2_layers=sum(1 for L in layers if L['tile'] & ops.TILE_H2),
                h2_plane_inputs=sum(1 for L in layers if L['tile'] & ops.TILE_H2P),
                h2_plane_edges=sum(1 for L in layers if L['tile'] & ops.TILE_H2E))


def e2e_stage(nm, rank, world, n_images, batch, threads):
    """End-to-end images/s from image FILES (north_star "end-to-end
    images/sec"; the reference's loop is detectron/core/test_engine.py:
    282-315): Market-sized 128x64 JPEGs written to local disk, then the
    product loop pps_amd.test_engine.extract_features -- PIL decode in the
    decode processes main() started before touching the GPU (threads if
    none), one pinned H2D copy per batch, the preprocessing kernel and
    pps_forward on the GPU -- followed (one rank) by the
    distance matrix + mAP/CMC of the first 3368 images as queries against
    the rest.  Images are split over ranks; the rate is all images / the
    slowest rank's time."""
    import shutil
    import tempfile
    import concurrent.futures as cf
    from PIL import Image
    from pps_amd import distributed as pdist
    from pps_amd import test_engine
    a, b = pdist.shard_range(n_images, rank, world)
    n = b - a
    d = tempfile.mkdtemp(prefix='pps_e2e_', dir='/tmp')
    try:
        rng = np.random.RandomState(100 + rank)
        base = rng.randint(0, 256, (64, 32, 16, 3)).astype(np.float32)

        def write(i):   # smooth colour blobs + noise: JPEG-typical content
            im = np.kron(base[i % 64], np.ones((4, 4, 1), np.float32))
            im = im + np.random.RandomState(i).randint(-24, 24, im.shape)
            p = os.path.join(d, '%08d.jpg' % i)
            Image.fromarray(np.clip(im, 0, 255).astype(np.uint8)).save(p, quality=95)
            return p
        with cf.ThreadPoolExecutor(threads) as pool:
            paths = list(pool.map(write, range(n)))
        jpeg_bytes = sum(os.path.getsize(p) for p in paths)
        feats = torch.empty((n, nm.feat_dim), dtype=torch.float32, device='cuda')
        # warm: the decode pool, pinned allocations, the batch shapes
        test_engine.extract_features(nm, lambda i: test_engine._decode_bgr(paths[i]),
                                     min(n, 2 * batch), batch=batch, out=feats, workers=threads,
                                     paths=paths)
        pdist.barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        test_engine.extract_features(nm, lambda i: test_engine._decode_bgr(paths[i]), n,
                                     batch=batch, out=feats, workers=threads, paths=paths)
        torch.cuda.synchronize()
        t_ext = time.perf_counter() - t0
        t_max = pdist.max_over_ranks(t_ext, world)
        from pps_amd import decode_pool
        procs = decode_pool.workers()
        out = dict(images=n_images, decode='%d processes' % procs if procs else
                   '%d threads' % threads, jpeg_MB=round(jpeg_bytes / 1e6, 2),
                   extract_s=round(t_max, 4), images_per_s=round(n_images / t_max, 2),
                   note='JPEG files on local disk (page-cached after writing) -> PIL decode '
                        'in worker processes -> pinned H2D -> pps_preprocess_bgr_ragged -> '
                        'pps_forward (test_engine.extract_features); rate = all images / '
                        'slowest rank')
        if world == 1 and n > Q_MARKET:
            from pps_amd.distributed import ShardedEvaluator
            rs = np.random.RandomState(0)
            ids = rs.randint(1, 751, n)
            cams = rs.randint(1, 7, n)
            t1 = time.perf_counter()
            ev = ShardedEvaluator(ids[:Q_MARKET], cams[:Q_MARKET], ids[Q_MARKET:],
                                  cams[Q_MARKET:], 0, 1)
            ev.run(feats[:Q_MARKET], feats[Q_MARKET:])
            t_ret = time.perf_counter() - t1
            out.update(retrieval_s=round(t_ret, 4), total_s=round(t_ext + t_ret, 4),
                       total_images_per_s=round(n / (t_ext + t_ret), 2))
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def _cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or 'unknown'


def cpu_baseline(blobs, n_img=8, n_q=400, runs=3):
    """SURVEY §8(d) "How the CPU path is timed": the build's CPU restatement
    of the reference path (oracle/: the recorded reference graph in torch CPU
    fp32, the NumPy evaluator) per stage, median of `runs` after one warm-up,
    on this host's cores.  Workload = BASELINE configs[1] sizes: the forward
    on n_img images 384x128; the Market-size distance matrix (3368 x 15913,
    D=3968, SURVEY §8(d) feature recipe) in full; argsort / mAP / CMC on the
    first n_q query rows of that matrix against the whole gallery, scaled by
    3368 / n_q (per-query work is independent of the other queries)."""
    from oracle import evaluator as ev
    from oracle.forward import GraphForward
    threads, aff, quota = usable_cores()
    torch.set_num_threads(threads)

    def med(fn):
        fn()
        ts = []
        for _ in range(runs):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    fw = GraphForward(blobs)
    rng = np.random.RandomState(0)
    x = (rng.randn(n_img, 3, 384, 128) * 50).astype(np.float32)
    fwd_s = med(lambda: fw(x))
    # Market-size features, SURVEY §8(d) recipe (750 centroids + 4.0 noise, L2 norm)
    Q, G = Q_MARKET, G_MARKET
    qid = rng.randint(1, 751, Q)
    gid = np.concatenate([rng.randint(1, 751, G - 2793), np.zeros(2793, int)])
    qcam, gcam = rng.randint(1, 7, Q), rng.randint(1, 7, G)
    cent = rng.randn(751, D_FEAT).astype(np.float32)
    f = cent[np.concatenate([qid, gid])]
    f += (4.0 * rng.randn(*f.shape)).astype(np.float32)
    f /= np.linalg.norm(f, axis=1, keepdims=True)
    qf, gf = f[:Q], f[Q:]
    box = {}
    dist_s = med(lambda: box.__setitem__('d', ev.compute_dist(qf, gf)))
    d = box['d'][:n_q]
    scale = Q / float(n_q)
    argsort_s = med(lambda: np.argsort(d, axis=1)) * scale
    map_s = med(lambda: ev.mean_ap(d, qid[:n_q], gid, qcam[:n_q], gcam)) * scale
    cmc_s = med(lambda: ev.cmc(d, qid[:n_q], gid, qcam[:n_q], gcam, topk=10,
                               first_match_break=True)) * scale
    byt = (Q + G) * D_FEAT * 4 + Q * G * 4
    return dict(value=round(n_img / fwd_s, 3), unit='images/s', cores=threads, kind='port',
                sample='forward: %d images 384x128 through oracle/forward.py (the recorded '
                       'reference graph, torch CPU fp32); retrieval: Market 3368 x 15913 x '
                       '3968 distance in full, argsort / mAP / CMC on %d query rows scaled x%.2f; '
                       'median of %d after 1 warm-up' % (n_img, n_q, scale, runs),
                cpu_model=_cpu_model(), cpu_count=os.cpu_count(), affinity_cpus=aff,
                cgroup_cpu_quota=quota,
                stages=dict(forward_img_s=round(n_img / fwd_s, 3),
                            distmat_s=round(dist_s, 3), distmat_GBps=round(byt / dist_s / 1e9, 3),
                            argsort_s=round(argsort_s, 3), mAP_s=round(map_s, 3),
                            cmc_s=round(cmc_s, 3),
                            retrieval_total_s=round(dist_s + argsort_s + map_s + cmc_s, 3)))


def dry_run(args, rank, world):
    """--dry-run: the rendezvous, barrier, timing and reporting path of a
    multi-rank run with no GPU work (gloo), so `--gpus N` is testable on CPU."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group('gloo')
    pdist_barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)
    pdist_barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    pdist_barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        print(json.dumps({'metric': 'gallery images/sec + distmat GB/s; mAP/Rank-1 parity on '
                          'Market-1501', 'value': None, 'unit': 'images/s', 'n_gpus': world,
                          'steps': args.steps, 'warmup': args.warmup, 'dry_run': True,
                          'ms_per_step': el * 1e3 / max(args.steps, 1)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def build_bench_model(batch, rank=0, table=None, autotune=True, flags=0):
    """The measured configuration: seeded weights of the PPS architecture,
    the whole-network C handle, the rank's seeded uint8 Market-sized images,
    their preprocessed NHWC4 batch, and the tuning table -- `table` (a saved
    tiles file) or pps_model_autotune on this device at this batch.
    tests/test_gpu_bench_table.py builds the same thing, so the table the
    parity tests check is the one the timed loop runs."""
    from pps_amd import model, native, ops
    cfg = market_cfg()
    plan = model.build_plan()
    blobs = model.synthetic_weights(plan, seed=0)
    # the product form: one handle behind the whole-network C ABI
    # (pps_model_create / pps_forward_bgr)
    nm = native.NativeModel(blobs)
    H, W = cfg.REID.SCALE[1], cfg.REID.SCALE[0]
    g = torch.Generator(device='cuda')
    g.manual_seed(1234 + rank)
    imgs = torch.randint(0, 256, (batch, 128, 64, 3), generator=g, device='cuda',
                         dtype=torch.int64).to(torch.uint8)
    xbuf = torch.empty((batch, H, W, 4), dtype=torch.float32, device='cuda')
    ops.preprocess_bgr(imgs, cfg.PIXEL_MEANS.ravel(), (H, W), xbuf)
    if table is not None:
        nm.apply_table(table)
    elif autotune:
        nm.autotune(xbuf, flags)
    return nm, blobs, imgs, xbuf


def main():
    args = parse()
    env_world = os.environ.get('WORLD_SIZE')
    if args.gpus is not None and args.gpus > 1 and env_world is None:
        # one process per GPU: this process only launches them (no GPU call yet)
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or 1)
    if args.gpus is not None and args.gpus != world:
        raise SystemExit('bench.py: --gpus %d but WORLD_SIZE=%d' % (args.gpus, world))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.dry_run:
        return dry_run(args, rank, world)
    # PPS_DIST_BACKEND=gloo: rehearse the N>1 path with several ranks sharing
    # the devices there are (one-GPU box); the product path is nccl (= RCCL)
    backend = os.environ.get('PPS_DIST_BACKEND', 'nccl')
    if backend == 'gloo':
        local = local % torch.cuda.device_count()
    if not args.no_e2e:
        # JPEG decode processes for the e2e stage, forked from a server started
        # before this process touches the GPU; the host's CPUs split over the
        # node's ranks
        from pps_amd import decode_pool
        lw = int(os.environ.get('LOCAL_WORLD_SIZE', world))
        decode_pool.start(decode_pool.default_workers(share=max(1, lw)))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    from pps_amd import native
    from pps_amd import distributed as pdist
    B = args.batch
    saved = None
    if args.tiles_file and os.path.exists(args.tiles_file):
        with open(args.tiles_file) as f:
            saved = json.load(f)
        pdist.HipBackend.distmat_tile = int(saved.get('__distmat__', 0))
        pdist.HipBackend.distmat_qplanes = bool(saved.get('__distmat_qplanes__', False))
        # a table tuned for another distance arithmetic: its tile id means nothing here
        if saved.get('__distmat_math__', 'x3') != ops_dist_math():
            pdist.HipBackend.distmat_tile, pdist.HipBackend.distmat_qplanes = 0, False
    # per-layer tile / plane choice on this device, outside the timed region
    # (PPS_AUTOTUNE_SPLITK=1: also try conv split-K)
    nm, blobs, imgs, xbuf = build_bench_model(
        B, rank, table=saved, autotune=not args.no_autotune,
        flags=(native.AUTOTUNE_SPLITK if os.environ.get('PPS_AUTOTUNE_SPLITK') == '1' else 0) |
        (native.AUTOTUNE_NO_H2 if os.environ.get('PPS_AUTOTUNE_NO_H2') == '1' else 0) |
        (native.AUTOTUNE_NO_H2E if os.environ.get('PPS_AUTOTUNE_NO_H2E') == '1' else 0) |
        (native.AUTOTUNE_NO_GROUPS if os.environ.get('PPS_AUTOTUNE_NO_GROUPS') == '1' else 0))
    cfg = market_cfg()
    H, W = cfg.REID.SCALE[1], cfg.REID.SCALE[0]
    feat = torch.empty((B, nm.feat_dim), dtype=torch.float32, device='cuda')
    from pps_amd import ops
    nm.reserve(B)

    def step():   # uint8 images -> preprocess -> forward, one C call
        nm.forward_bgr(imgs, out=feat)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    graph = None
    if not args.no_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()
    run = graph.replay if graph is not None else step

    pdist.barrier(world)
    torch.cuda.synchronize()
    with ClockSampler(local) as clk:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        pdist.barrier(world)
        elapsed = time.perf_counter() - t0
    elapsed = pdist.max_over_ranks(elapsed, world)
    ms_per_step = elapsed * 1e3 / args.steps
    value = world * B * args.steps / elapsed

    # PCIe-inclusive rate: the test loop hands the library host
    # images, so also time the step with each batch's uint8 images copied
    # from pinned host memory first (same stream, ordered before the replay).
    # Reported beside `value`, never as it.
    host = torch.empty(imgs.shape, dtype=torch.uint8, pin_memory=True)
    host.copy_(imgs.cpu())
    for _ in range(2):
        imgs.copy_(host, non_blocking=True)
        run()
    pdist.barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        imgs.copy_(host, non_blocking=True)
        run()
    torch.cuda.synchronize()
    pdist.barrier(world)
    el_h2d = pdist.max_over_ranks(time.perf_counter() - t0, world)
    pcie = dict(value=round(world * B * args.steps / el_h2d, 2), unit='images/s',
                ms_per_step=round(el_h2d * 1e3 / args.steps, 3),
                h2d_bytes_per_step=int(host.numel()),
                note='uint8 BGR batch copied from pinned host memory before every step')
    del graph

    roof, per_layer = conv_roofline(nm, xbuf)
    tiles_saved = bool(args.tiles_file and os.path.exists(args.tiles_file))
    ret = retrieval_stage(rank, world, args.dist_reps,
                          tune=not (args.no_autotune or tiles_saved))
    if args.tiles_file and not tiles_saved and rank == 0:
        with open(args.tiles_file, 'w') as f:
            json.dump(dict(nm.tiles(), __distmat__=ret['distmat_tile'],
                           __distmat_qplanes__=ret['distmat_qplanes'],
                           __distmat_math__=ops_dist_math(),
                           __planes__=nm.planes(), __splitk__=nm.splitks()), f, indent=0)
    e2e = None
    if not args.no_e2e:
        e2e = e2e_stage(nm, rank, world, args.e2e_images, B, min(16, usable_cores()[0]))
    dist_bytes = (Q_MARKET + ret['G_local']) * D_FEAT * 4 + Q_MARKET * ret['G_local'] * 4
    dist_flops = 2.0 * Q_MARKET * ret['G_local'] * D_FEAT
    dist_tflops = dist_flops / (ret['distmat_ms'] * 1e-3) / 1e12
    dist_math = ops.dist_math()
    dist_peak = {'h2': PEAK_H2_TFLOPS, 'x3': PEAK_X3_TFLOPS}.get(dist_math, PEAK_FP32_MFMA_TFLOPS)
    droof = ret['dist_roofline'] or {}
    # whole-job distmat GB/s: all ranks' shards / the slowest rank's time
    dist_ms_max = pdist.max_over_ranks(ret['distmat_ms'], world)
    total_bytes = (Q_MARKET + G_MARKET) * D_FEAT * 4 + Q_MARKET * G_MARKET * 4
    out = {
        'metric': 'gallery images/sec + distmat GB/s; mAP/Rank-1 parity on Market-1501',
        'value': round(value, 2), 'unit': 'images/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 3),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        # f32 operands and outputs; the products run as exact-split f16 / bf16
        # MFMA terms with f32 accumulation
        'dtype': ('f32 (f16x2 3-term / bf16x3 6-term MFMA emulation, f32 accumulate)'
                  if nm.math == 'x3' else 'f32 (f32 MFMA)'),
        'math': dict(conv_launches=dict(
                         f16x2=sum(1 for v in per_layer.values()
                                   if v['gemm'] and v['tile'] & ops.TILE_H2),
                         bf16x3=sum(1 for v in per_layer.values()
                                    if v['gemm'] and not v['tile'] & ops.TILE_H2)),
                     distance=ops.dist_math(), accumulate='f32',
                     note='f16x2: each f32 operand as two f16 terms on a power-of-two scale, '
                          'three f16 MFMA products; bf16x3: three bf16 terms, six products'),
        'data': 'synthetic (uint8 images, seeded weights of the PPS R-50 architecture)',
        'config': {'workload': 'Market-1501 ResNet-50 PPS (stride-1 res5, 31 part subsets), '
                               'batch %d/GPU, 384x128, 3368q x 15913g L2 distmat' % B,
                   'global_batch': B * world, 'input_hw': [H, W], 'feat_dim': nm.feat_dim,
                   'parallelism': 'dp%d' % world, 'hipgraph': not args.no_graph,
                   'entry_point': 'pps_forward_bgr (whole-network C ABI)',
                   'act_plane_edges': len(nm.planes()), 'splitk_layers': len(nm.splitks()),
                   'tuning_table': table_digest(nm)},
        'gpu_clock': clk.summary(),
        'distmat_GBps': round(total_bytes / (dist_ms_max * 1e-3) / 1e9, 2),
        'distmat_ms': round(dist_ms_max, 3),
        'distmat_TFLOPs_per_gpu': round(dist_tflops, 2),
        'pcie_inclusive': pcie,
        'e2e_from_jpeg': e2e,
        'rank_eval_ms': round(ret['rank_eval_ms'], 3),
        'retrieval_ms': round(ret['retrieval_ms'], 3),
        'mAP_synthetic': round(ret['mAP'], 6), 'cmc1_synthetic': round(ret['cmc1'], 6),
        'roofline': roof,
        'roofline_rank': ret['rank_roofline'],
        'roofline_argsort': ret['argsort_roofline'],
        'roofline_distmat': dict(
            bound='mfma',
            achieved=droof.get('achieved', round(dist_tflops, 2)),
            peak=droof.get('peak', round(dist_peak, 1)),
            unit='TFLOP/s',
            frac=droof.get('frac', round(dist_tflops / dist_peak, 4)),
            frac_of_x3_roof=droof.get('frac_of_x3_roof'),
            math=dist_math,
            peak_note=('f32-equivalent TFLOP/s: dense f16 MFMA rate / 3 terms per product '
                       '(h2); / 6 bf16 terms (x3); exact f32 MFMA rate (f32)'),
            avg_launch_us=droof.get('avg_launch_us'),
            with_index_prep=dict(ms=round(ret['distmat_ms'], 3), TFLOPs=round(dist_tflops, 2),
                                 note='gallery shard split + norms + query gather + GEMM, '
                                      'as retrieval_ms runs it'),
            hbm_GBps=round(dist_bytes / (ret['distmat_ms'] * 1e-3) / 1e9, 2),
            traffic=_pmc_traffic('distmat', dist_math, Q_MARKET),
            algorithmic_bytes_per_launch=dist_bytes,
            timing=droof.get('timing'),
            kernel=('gemm_h2_kernel (f16x2, pps_distmat_h2_tiled), tile %d' % ret['distmat_tile']
                    if dist_math == 'h2' else
                    '%s EPI_DIST, tile %d' % (
                        'gemm_x3p_kernel' if dist_math == 'x3' else 'gemm_f32_kernel',
                        ret['distmat_tile']) + (
                        ', queries and gallery as chunk-tiled bf16x3 planes '
                        '(pps_distmat_x3p_tiled)' if ret['distmat_qplanes'] else ''))),
    }
    if (world > 1 or args.sharded_legs) and not args.no_sharded_legs:
        # BASELINE configs[3] and configs[4] on the ranks this run has (the
        # driver's N = 2 / 4 / 8 runs): gallery-sharded, RCCL collectives
        torch.cuda.empty_cache()
        out['config_cuhk03'] = config_cuhk03(rank, world)
        torch.cuda.empty_cache()
        out['config_1m'] = config_1m(rank, world)
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_duke:
        # BASELINE configs[2] (Duke sizes, cosine + k-reciprocal re-ranking),
        # timed after the headline workload: distance / re-ranking / rank
        # stages and their rooflines (scripts/bench_duke_rerank.py)
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), 'scripts'))
        from bench_duke_rerank import run_duke
        torch.cuda.empty_cache()
        out['config_duke'] = run_duke(reps=3)
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(blobs)
    if rank == 0:
        if os.environ.get('PPS_BENCH_LAYERS'):
            with open(os.environ['PPS_BENCH_LAYERS'], 'w') as f:
                json.dump({k: v for k, v in per_layer.items()}, f, indent=0)
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
