"""Multi-GPU retrieval: gallery-sharded distance, rank list and evaluation.

SURVEY §8(e).  The reference tests on several GPUs by spawning one process per
GPU over contiguous image ranges and exchanging pickle files
(detectron/utils/subprocess.py:39-103, np.array_split :53); its parent then
vstacks all features and evaluates on one host
(detectron/core/test_engine.py:184-229, reid_dataset_evaluator.py:29-209).
Here each rank keeps its gallery shard resident in HBM:

  1. all-gather the query embeddings (RCCL over xGMI; Market 53.5 MB total),
  2. distance block [Q, G_r] on the local shard (HIP MFMA GEMM),
  3. each rank lists its shard's true matches per query from a per-identity
     index of its shard (capacity = the most same-id entries of any query in
     any shard, exact from the ids every rank holds); all-gather of the
     positive lists ([R, Q, Pmax], kilobytes),
  4. each rank streams its block once, binning every entry against the
     merged, sorted positives and taking its own junk entries back out
     (additive counts), all-reduce(SUM) of the counts,
  5. AP / first-match rank per query from the summed counts.

Rank list (the reference's np.argsort(distmat, axis=1), :319,:420): each
rank takes the stable top-k of its block, the lists are all-gathered
(Q·k·8 B per shard) and merged on the device by (distance, global index)
(pps_topk_merge): equal to the top-k of the unsharded matrix.

Multi-query (:131-159): the mq image features are all-gathered in global
order and pooled per (id, cam) on every rank (bit-identical to the one-GPU
pooling), then scored like single queries.  Re-ranking (:161-207) needs the
whole (Q+G)^2 neighbour structure: it is gathered to rank 0 (replica work
would only repeat it), whose scores are broadcast.

Only all-gathers, two SUM all-reduces of small count arrays and one
broadcast of scalars cross ranks: no ring all-reduce of big tensors.

The per-stage kernels come from a backend object so the collective logic can
be exercised with world_size > 1 on CPU (gloo) in tests; the product backend
is HipBackend (libpps_hip.so).
"""
from collections import OrderedDict

import numpy as np
import torch

from . import ops


def shard_range(n, rank, world):
    """Contiguous, balanced split (np.array_split semantics, subprocess.py:53)."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def max_same_id(qid, gid):
    """The most gallery entries sharing any query's id (>= 1): an exact bound
    on a query's positive and junk lists in that gallery (shard)."""
    qid, gid = np.asarray(qid), np.asarray(gid)
    if len(qid) == 0 or len(gid) == 0:
        return 1
    ids, cnt = np.unique(gid, return_counts=True)
    pos = np.searchsorted(ids, qid)
    pos = np.minimum(pos, len(ids) - 1)
    per_q = np.where(ids[pos] == qid, cnt[pos], 0)
    return max(1, int(per_q.max()))


def _active(world):
    """Collectives run whenever a process group exists, also at world size 1
    (a one-rank RCCL communicator), and are skipped only without one."""
    return world > 1 or (torch.distributed.is_available() and torch.distributed.is_initialized())


def barrier(world):
    if _active(world):
        torch.distributed.barrier()


def _coll_device(x):
    """Collectives run on the tensors' device for nccl (RCCL), host for gloo."""
    return x.device if torch.distributed.get_backend() == 'nccl' else torch.device('cpu')


def max_over_ranks(x, world):
    if not _active(world):
        return x
    dev = 'cuda' if torch.distributed.get_backend() == 'nccl' else 'cpu'
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def all_gather_rows(x, sizes):
    """Gather [n_r, ...] blocks of unequal n_r (known on every rank)."""
    world = len(sizes)
    if not _active(world):
        return x
    mx = max(max(sizes), 1)
    dev = _coll_device(x)
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=dev)
    pad[:x.shape[0]] = x
    bufs = [torch.empty_like(pad) for _ in range(world)]
    torch.distributed.all_gather(bufs, pad)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], 0).to(x.device).contiguous()


def _padded(x, mx, dim):
    """x padded with zeros to mx along dim (0 = rows, 1 = columns), on the
    collective's device."""
    dev = _coll_device(x)
    shape = list(x.shape)
    shape[dim] = mx
    pad = torch.zeros(shape, dtype=x.dtype, device=dev)
    pad.narrow(dim, 0, x.shape[dim]).copy_(x)
    return pad


def gather_blocks(x, sizes, dim=0, dst=0):
    """Gather blocks of unequal extent sizes[r] along `dim` (0: rows [n_r, ...],
    1: columns [m, n_r]) to rank `dst` only, concatenated in rank order;
    None on the other ranks.  For tensors only one rank consumes (the
    features.npy dump, the re-ranking inputs): 1/world of an all-gather's
    traffic."""
    world = len(sizes)
    if not _active(world):
        return x
    pad = _padded(x, max(max(sizes), 1), dim)
    me = torch.distributed.get_rank()
    bufs = [torch.empty_like(pad) for _ in range(world)] if me == dst else None
    torch.distributed.gather(pad, bufs, dst=dst)
    if me != dst:
        return None
    return torch.cat([b.narrow(dim, 0, s) for b, s in zip(bufs, sizes)],
                     dim).to(x.device).contiguous()


def broadcast_object(obj, world, src=0):
    if not _active(world):
        return obj
    box = [obj]
    torch.distributed.broadcast_object_list(box, src=src)
    return box[0]


class HipBackend(object):
    """libpps_hip.so kernels (the product path)."""
    device = 'cuda'
    distmat_math = None   # distance arithmetic (None = ops.dist_math(): 'h2' by default)
    distmat_tile = 0   # GEMM tile of that arithmetic (0 = default; bench tunes it)
    distmat_qplanes = False  # x3: queries pre-split into bf16x3 planes (ops.compute_dist)

    @classmethod
    def distmat(cls, q, g, metric):
        return ops.compute_dist(q, g, metric=metric, tile=cls.distmat_tile,
                                q_planes=cls.distmat_qplanes, pad_rows=True,
                                math=cls.distmat_math)

    @staticmethod
    def prepare(ev):
        """Per-identity index of this rank's gallery shard (host ids, once)."""
        return ops.MatchIndex(ev.qid_np, ev.qcam_np, ev.gid_np, ev.gcam_np)

    @staticmethod
    def collect(dist, ev, state, pmax):
        """This shard's positive lists [Q, pmax] (+ its junk lists, kept local)."""
        pos_d, pos_idx, pos_cnt, junk = ops.collect_matches(dist, state, ev.g_offset, pmax)
        return pos_d, pos_idx, pos_cnt, junk

    @staticmethod
    def counts(dist, ev, state, pos_d, pos_idx, pos_cnt, local):
        """Merged + sorted positives of all shards, this shard's additive counts."""
        sp = ops.rank_prepare(pos_d, pos_idx, pos_cnt)
        hist, before = ops.rank_count_stream(dist, ev.g_offset, sp, local)
        return sp.sorted_d, sp.sorted_idx, sp.pos_total, hist, before

    @staticmethod
    def finalize(sorted_d, pos_total, hist, before):
        return ops.ap_finalize(sorted_d, pos_total, hist, before)

    @staticmethod
    def topk(dist, k):
        return ops.topk(dist, k)

    @staticmethod
    def topk_merge(vals, idx, offsets, k):
        return ops.topk_merge(vals, idx, offsets, k)

    @staticmethod
    def group_mean(x, groups):
        return ops.group_mean(x, groups)

    @staticmethod
    def self_dist(x, metric):
        return ops.compute_dist(x, x, metric=metric, pad_rows=True)

    @staticmethod
    def re_ranking(q_g, q_q, g_g):
        # strided blocks go in as they are (a copy would drop the symmetric mark)
        return ops.re_ranking(q_g, q_q, g_g)

    @staticmethod
    def rank_eval(dist, qid, gid, qcam, gcam):
        from .reid_dataset_evaluator import rank_eval
        return rank_eval(dist, qid, gid, qcam, gcam)


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
        # list capacity: the most same-id entries any query has in any shard
        # -- exact, from the ids every rank holds (no collective, no overflow)
        self.pmax = max(max_same_id(qid, gid[a:b]) for a, b in self.g_ranges)
        self.qid_np, self.qcam_np = qid, qcam
        self.gid_np, self.gcam_np = gid[g0:g1], gcam[g0:g1]
        self._state = None
        dev = self.backend.device
        i32 = torch.int32
        self.qid = torch.from_numpy(qid.astype(np.int32)).to(dev)
        self.qcam = torch.from_numpy(qcam.astype(np.int32)).to(dev)
        self.gid = torch.from_numpy(gid[g0:g1].astype(np.int32)).to(dev)
        self.gcam = torch.from_numpy(gcam[g0:g1].astype(np.int32)).to(dev)
        assert self.qid.dtype == i32

    def _all_reduce(self, t, op=None):
        """In-place all-reduce of a backend tensor (host-staged for gloo)."""
        if not _active(self.world):
            return t
        op = op if op is not None else torch.distributed.ReduceOp.SUM
        dev = _coll_device(t)
        s = t if t.device == dev else t.to(dev)
        torch.distributed.all_reduce(s, op=op)
        if s is not t:
            t.copy_(s)
        return t

    def _gather_lists(self, *ts):
        if not _active(self.world):
            return [t[None] for t in ts]
        return [all_gather_rows(t[None], [1] * self.world) for t in ts]

    def run(self, q_local, g_local, timed=False, dist=None, keep_dist=False):
        be = self.backend
        use_ev = timed and be.device == 'cuda'
        if use_ev:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            evs[0].record()
        if dist is None:
            q_all = all_gather_rows(q_local, self.q_sizes)
            if use_ev:
                evs[1].record()
            dist = be.distmat(q_all, g_local, self.metric)
        elif use_ev:
            evs[1].record()
        if use_ev:
            evs[2].record()
        if self._state is None:
            self._state = be.prepare(self)
        pos_d, pos_idx, pos_cnt, local = be.collect(dist, self, self._state, self.pmax)
        pos_d, pos_idx, pos_cnt = self._gather_lists(pos_d, pos_idx, pos_cnt)
        sorted_d, _, pos_total, hist, before = be.counts(
            dist, self, self._state, pos_d, pos_idx, pos_cnt, local)
        self._all_reduce(hist)
        self._all_reduce(before)
        ap, valid, first = be.finalize(sorted_d, pos_total, hist, before)
        if use_ev:
            evs[3].record()
        ap = ap.cpu().numpy()
        valid = valid.cpu().numpy().astype(bool)
        first = first.cpu().numpy()
        nvalid = int(valid.sum())
        mAP = float(ap.sum()) / nvalid if nvalid else float('nan')
        hits = np.zeros(self.topk)
        fr = first[valid]
        np.add.at(hits, fr[fr < self.topk], 1)
        cmc = np.cumsum(hits) / max(nvalid, 1)
        res = dict(mAP=mAP, cmc=cmc, ap=ap, valid=valid, first_rank=first)
        if keep_dist:
            res['dist'] = dist
        if use_ev:
            res['t_gather_ms'] = evs[0].elapsed_time(evs[1])   # the query all-gather
            res['t_distmat_ms'] = evs[1].elapsed_time(evs[2])
            res['t_rank_ms'] = evs[2].elapsed_time(evs[3])
            res['t_total_ms'] = evs[0].elapsed_time(evs[3])
        return res

    def rank_list(self, q_local=None, g_local=None, k=100, dist=None):
        """Global stable top-k rank list [Q, k] (distances, global gallery
        indices) on every rank: local top-k, all-gather, k-way merge."""
        be = self.backend
        if dist is None:
            q_all = all_gather_rows(q_local, self.q_sizes)
            dist = be.distmat(q_all, g_local, self.metric)
        kin = min(k, dist.shape[1])
        if kin > 0:
            vals, idx = be.topk(dist, kin)
        else:
            vals = torch.zeros((self.Q, 1), dtype=torch.float32, device=dist.device)
            idx = torch.full((self.Q, 1), -1, dtype=torch.int32, device=dist.device)
        if kin < k and kin > 0:   # short shard: pad its list to k entries
            pv = torch.full((self.Q, k), float('inf'), dtype=torch.float32, device=dist.device)
            pi = torch.full((self.Q, k), -1, dtype=torch.int32, device=dist.device)
            pv[:, :kin] = vals
            pi[:, :kin] = idx
            vals, idx = pv, pi
        elif kin == 0:
            vals = torch.full((self.Q, k), float('inf'), dtype=torch.float32,
                              device=dist.device)
            idx = torch.full((self.Q, k), -1, dtype=torch.int32, device=dist.device)
        vals, idx = self._gather_lists(vals.contiguous(), idx.contiguous())
        offsets = [a for a, _ in self.g_ranges]
        return be.topk_merge(vals.contiguous(), idx.contiguous(), offsets, k)


def _score(ap, valid, first, topk=10):
    ap, valid, first = (np.asarray(t.cpu().numpy() if isinstance(t, torch.Tensor) else t)
                        for t in (ap, valid, first))
    valid = valid.astype(bool)
    nvalid = int(valid.sum())
    mAP = float(ap.sum()) / nvalid if nvalid else float('nan')
    hits = np.zeros(topk)
    fr = first[valid]
    np.add.at(hits, fr[(fr >= 0) & (fr < topk)], 1)
    return mAP, np.cumsum(hits) / max(nvalid, 1)


def mq_groups(mq_ids, mq_cams):
    """Per-(id, cam) member lists in first-appearance order
    (reid_dataset_evaluator.py:136-140) -> (keys [n, 2], groups)."""
    groups = OrderedDict()
    for k, key in enumerate(zip(np.asarray(mq_ids).tolist(), np.asarray(mq_cams).tolist())):
        groups.setdefault(key, []).append(k)
    keys = np.array(list(groups.keys()), dtype=np.int64).reshape(-1, 2)
    return keys, list(groups.values())


def evaluate_sharded(q_local, g_local, mq_local, ids, cams, marks, rank, world,
                     backend=None, metric='euclidean', rerank=False, verbose=False):
    """The reference's evaluate() (reid_dataset_evaluator.py:29-209) over
    features sharded across ranks: q_local / g_local / mq_local are this
    rank's contiguous shards (shard_range) of the query (mark 0), gallery
    (mark 1) and multi-query (mark 2) features in dataset order; ids / cams /
    marks cover the whole dataset.  Returns (mAP, cmc, mq_mAP, mq_cmc) on
    every rank, equal to the one-process evaluate."""
    be = backend or HipBackend
    ids, cams, marks = np.asarray(ids), np.asarray(cams), np.asarray(marks)
    q, g, mq = marks == 0, marks == 1, marks == 2
    ev = ShardedEvaluator(ids[q], cams[q], ids[g], cams[g], rank, world, backend=be,
                          metric=metric)
    q_all = all_gather_rows(q_local, ev.q_sizes)
    q_g = be.distmat(q_all, g_local, metric)
    res = ev.run(None, g_local, dist=q_g)
    mAP, cmc = res['mAP'], res['cmc']
    mq_mAP = mq_cmc = None
    if mq.any():
        n_mq = int(mq.sum())
        mq_sizes = [b - a for a, b in (shard_range(n_mq, r, world) for r in range(world))]
        mq_all = all_gather_rows(mq_local, mq_sizes)
        keys, groups = mq_groups(ids[mq], cams[mq])
        pooled = be.group_mean(mq_all, groups)
        ev_mq = ShardedEvaluator(keys[:, 0], keys[:, 1], ids[g], cams[g], rank, world,
                                 backend=be, metric=metric)
        mq_g = be.distmat(pooled, g_local, metric)
        r = ev_mq.run(None, g_local, dist=mq_g)
        mq_mAP, mq_cmc = r['mAP'], r['cmc']
    if rerank:
        # the whole (Q+G)^2 neighbour structure on rank 0: the gallery
        # features (for g x g) and the shards' q x g blocks already computed
        # above, gathered there only (not recomputed, not sent to every rank)
        g_sizes = [b - a for a, b in ev.g_ranges]
        g_all = gather_blocks(g_local, g_sizes)
        qg_full = gather_blocks(q_g.contiguous(), g_sizes, dim=1)
        mqg_full = gather_blocks(mq_g.contiguous(), g_sizes, dim=1) if mq.any() else None
        scores = None
        if rank == 0:
            g_g = be.self_dist(g_all, metric)
            rr = be.re_ranking(qg_full, be.self_dist(q_all, metric), g_g)
            s_sq = _score(*be.rank_eval(rr, ids[q], ids[g], cams[q], cams[g]))
            s_mq = None
            if mq.any():
                rr_mq = be.re_ranking(mqg_full, be.self_dist(pooled, metric), g_g)
                s_mq = _score(*be.rank_eval(rr_mq, keys[:, 0], ids[g], keys[:, 1], cams[g]))
            scores = (s_sq, s_mq)
        s_sq, s_mq = broadcast_object(scores, world)
        mAP, cmc = s_sq
        if s_mq is not None:
            mq_mAP, mq_cmc = s_mq
    return mAP, cmc, mq_mAP, mq_cmc
