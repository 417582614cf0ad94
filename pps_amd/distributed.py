"""Multi-GPU retrieval: gallery-sharded distance + rank evaluation.

SURVEY §8(e).  The reference tests on several GPUs by spawning one process per
GPU over contiguous image ranges and exchanging pickle files
(detectron/utils/subprocess.py:39-103, np.array_split :53); its parent then
vstacks all features and evaluates on one host.  Here each rank keeps its
gallery shard resident in HBM:

  1. all-gather the query embeddings (RCCL over xGMI; Market 53.5 MB total),
  2. distance block [Q, G_r] on the local shard (HIP FP32 MFMA),
  3. each rank lists its shard's true matches per query; all-gather the
     lists ([R, Q, Pmax] distances + global gallery indices, kilobytes),
  4. each rank bins its shard against the merged, sorted positives
     (additive counts), all-reduce(SUM) of the counts,
  5. AP / first-match rank per query from the summed counts.

Only the all-gathers and one all-reduce cross ranks: there is no ring
all-reduce of big tensors anywhere on this path.

The per-stage kernels come from a backend object so the collective logic can
be exercised with world_size > 1 on CPU (gloo) in tests; the product backend
is HipBackend (libpps_hip.so).
"""
import numpy as np
import torch

from . import ops


def shard_range(n, rank, world):
    """Contiguous, balanced split (np.array_split semantics, subprocess.py:53)."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def barrier(world):
    if world > 1:
        torch.distributed.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    dev = 'cuda' if torch.distributed.get_backend() == 'nccl' else 'cpu'
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def all_gather_rows(x, sizes):
    """Gather [n_r, ...] blocks of unequal n_r (known on every rank)."""
    world = len(sizes)
    if world == 1:
        return x
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[:x.shape[0]] = x
    bufs = [torch.empty_like(pad) for _ in range(world)]
    torch.distributed.all_gather(bufs, pad)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], 0).contiguous()


class HipBackend(object):
    """libpps_hip.so kernels (the product path)."""
    device = 'cuda'
    distmat_tile = 0   # GEMM tile for the distance matrix (0 = heuristic; bench tunes it)
    distmat_qplanes = False  # queries pre-split into bf16x3 planes (ops.compute_dist)

    @classmethod
    def distmat(cls, q, g, metric):
        return ops.compute_dist(q, g, metric=metric, tile=cls.distmat_tile,
                                q_planes=cls.distmat_qplanes)

    @staticmethod
    def collect(dist, qid, qcam, gid, gcam, g_offset, pmax):
        return ops.collect_positives(dist, qid, qcam, gid, gcam, g_offset, pmax)

    @staticmethod
    def counts(dist, qid, qcam, gid, gcam, g_offset, pos_d, pos_idx, pos_cnt):
        return ops.rank_counts(dist, qid, qcam, gid, gcam, g_offset, pos_d, pos_idx,
                               pos_cnt)

    @staticmethod
    def finalize(sorted_d, pos_total, hist, before):
        return ops.ap_finalize(sorted_d, pos_total, hist, before)


class ShardedEvaluator(object):
    """Market protocol (separate_camera_set=False, single_gallery_shot=False,
    first_match_break=True, topk=10; reid_dataset_evaluator.py:35-37,92)."""

    def __init__(self, qid, qcam, gid, gcam, rank, world, backend=None, metric='euclidean',
                 topk=10):
        self.backend = backend or HipBackend
        self.rank, self.world = rank, world
        self.metric, self.topk = metric, topk
        qid, qcam = np.asarray(qid), np.asarray(qcam)
        gid, gcam = np.asarray(gid), np.asarray(gcam)
        self.Q, self.G = len(qid), len(gid)
        self.q_sizes = [b - a for a, b in (shard_range(self.Q, r, world) for r in range(world))]
        self.g_ranges = [shard_range(self.G, r, world) for r in range(world)]
        g0, g1 = self.g_ranges[rank]
        self.g_offset = g0
        # Pmax: max true matches per query inside any one shard (host metadata)
        self.pmax = max(1, max(ops.max_positives(qid, qcam, gid[a:b], gcam[a:b])
                               for a, b in self.g_ranges))
        dev = self.backend.device
        i32 = torch.int32
        self.qid = torch.from_numpy(qid.astype(np.int32)).to(dev)
        self.qcam = torch.from_numpy(qcam.astype(np.int32)).to(dev)
        self.gid = torch.from_numpy(gid[g0:g1].astype(np.int32)).to(dev)
        self.gcam = torch.from_numpy(gcam[g0:g1].astype(np.int32)).to(dev)
        assert self.qid.dtype == i32

    def run(self, q_local, g_local, timed=False):
        be = self.backend
        use_ev = timed and be.device == 'cuda'
        if use_ev:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            evs[0].record()
        q_all = all_gather_rows(q_local, self.q_sizes)
        if use_ev:
            evs[1].record()
        dist = be.distmat(q_all, g_local, self.metric)
        if use_ev:
            evs[2].record()
        pos_d, pos_idx, pos_cnt = be.collect(dist, self.qid, self.qcam, self.gid, self.gcam,
                                             self.g_offset, self.pmax)
        if self.world > 1:
            pos_d = all_gather_rows(pos_d[None], [1] * self.world)
            pos_idx = all_gather_rows(pos_idx[None], [1] * self.world)
            pos_cnt = all_gather_rows(pos_cnt[None], [1] * self.world)
        else:
            pos_d, pos_idx, pos_cnt = pos_d[None], pos_idx[None], pos_cnt[None]
        sorted_d, _, pos_total, hist, before = be.counts(
            dist, self.qid, self.qcam, self.gid, self.gcam, self.g_offset, pos_d, pos_idx,
            pos_cnt)
        if self.world > 1:
            torch.distributed.all_reduce(hist)
            torch.distributed.all_reduce(before)
        ap, valid, first = be.finalize(sorted_d, pos_total, hist, before)
        if use_ev:
            evs[3].record()
        ap = ap.cpu().numpy()
        valid = valid.cpu().numpy().astype(bool)
        first = first.cpu().numpy()
        if np.any(pos_cnt.cpu().numpy() > self.pmax):
            raise RuntimeError('positive list overflow: Pmax=%d too small' % self.pmax)
        nvalid = int(valid.sum())
        mAP = float(ap.sum()) / nvalid if nvalid else float('nan')
        hits = np.zeros(self.topk)
        fr = first[valid]
        np.add.at(hits, fr[fr < self.topk], 1)
        cmc = np.cumsum(hits) / max(nvalid, 1)
        res = dict(mAP=mAP, cmc=cmc, ap=ap, valid=valid, first_rank=first)
        if use_ev:
            res['t_distmat_ms'] = evs[1].elapsed_time(evs[2])
            res['t_rank_ms'] = evs[2].elapsed_time(evs[3])
            res['t_total_ms'] = evs[0].elapsed_time(evs[3])
        return res
