"""ORACLE (test infrastructure only) -- NumPy restatement of the count-based
rank evaluation kernels in pps_amd/csrc/rank.hip, used as a CPU backend so the
gallery-sharded collective logic (pps_amd/distributed.py) can be tested with
torch.distributed gloo, world_size > 1, without a GPU.  Same semantics as the
HIP kernels: positives = same id & different cam; junk = same id & same cam;
stable (distance, global gallery index) order; counts additive over shards.
"""
import numpy as np
import torch

from oracle import evaluator as ev


def merge_topk(vals, idx, offsets, k):
    """Stable (distance, global index) top-k of R per-shard lists [R, Q, k_in]
    with local indices (idx < 0 = pad): the semantics of pps_topk_merge."""
    R, Q, kin = vals.shape
    out_v = np.full((Q, k), np.inf, np.float32)
    out_i = np.full((Q, k), -1, np.int32)
    gidx = idx.astype(np.int64) + np.asarray(offsets, np.int64)[:, None, None]
    for q in range(Q):
        ok = idx[:, q, :] >= 0
        v, g = vals[:, q, :][ok], gidx[:, q, :][ok]
        o = np.lexsort((g, v))[:k]
        out_v[q, :len(o)] = v[o]
        out_i[q, :len(o)] = g[o]
    return out_v, out_i


class CpuBackend(object):
    device = 'cpu'

    @staticmethod
    def distmat(q, g, metric):
        return torch.from_numpy(ev.compute_dist(q.numpy(), g.numpy(), metric))

    @staticmethod
    def prepare(ev):
        return None

    @staticmethod
    def collect(dist, ev, state, pmax):
        pos = CpuBackend.collect_positives(dist, ev.qid, ev.qcam, ev.gid, ev.gcam, ev.g_offset,
                                           pmax)
        return pos + (None,)

    @staticmethod
    def counts(dist, ev, state, pos_d, pos_idx, pos_cnt, local):
        return CpuBackend.rank_counts(dist, ev.qid, ev.qcam, ev.gid, ev.gcam, ev.g_offset,
                                      pos_d, pos_idx, pos_cnt)

    @staticmethod
    def collect_positives(dist, qid, qcam, gid, gcam, g_offset, pmax):
        d, qi, qc, gi, gc = (t.numpy() for t in (dist, qid, qcam, gid, gcam))
        Q = d.shape[0]
        pos_d = np.zeros((Q, pmax), np.float32)
        pos_idx = np.zeros((Q, pmax), np.int32)
        cnt = np.zeros(Q, np.int32)
        for q in range(Q):
            hit = np.nonzero((gi == qi[q]) & (gc != qc[q]))[0]
            cnt[q] = len(hit)
            k = min(len(hit), pmax)
            pos_d[q, :k] = d[q, hit[:k]]
            pos_idx[q, :k] = hit[:k] + g_offset
        return torch.from_numpy(pos_d), torch.from_numpy(pos_idx), torch.from_numpy(cnt)

    @staticmethod
    def rank_counts(dist, qid, qcam, gid, gcam, g_offset, pos_d, pos_idx, pos_cnt):
        d, qi, qc, gi, gc = (t.numpy() for t in (dist, qid, qcam, gid, gcam))
        pd, px, pc = pos_d.numpy(), pos_idx.numpy(), pos_cnt.numpy()
        R, Q, pmax = pd.shape
        ptot = R * pmax
        sd = np.full((Q, ptot), np.inf, np.float32)
        si = np.full((Q, ptot), -1, np.int32)
        total = np.zeros(Q, np.int32)
        hist = np.zeros((Q, ptot), np.int32)
        before = np.zeros(Q, np.int32)
        G = d.shape[1]
        gidx = np.arange(G) + g_offset
        for q in range(Q):
            vals = [(pd[r, q, p], px[r, q, p]) for r in range(R)
                    for p in range(min(pc[r, q], pmax))]
            vals.sort()
            P = len(vals)
            total[q] = P
            if P == 0:
                continue
            sd[q, :P] = [v[0] for v in vals]
            si[q, :P] = [v[1] for v in vals]
            valid = ~((gi == qi[q]) & (gc == qc[q]))
            dv = d[q, valid]
            lb = np.searchsorted(sd[q, :P], dv, side='left')
            np.add.at(hist[q], lb[lb < P], 1)
            df, idf = sd[q, 0], si[q, 0]
            before[q] = np.sum((dv < df) | ((dv == df) & (gidx[valid] < idf)))
        return (torch.from_numpy(sd), torch.from_numpy(si), torch.from_numpy(total),
                torch.from_numpy(hist), torch.from_numpy(before))

    @staticmethod
    def topk(dist, k):
        d = dist.numpy()
        order = np.argsort(d, axis=1, kind='stable')[:, :k]
        return (torch.from_numpy(np.take_along_axis(d, order, axis=1).astype(np.float32)),
                torch.from_numpy(order.astype(np.int32)))

    @staticmethod
    def topk_merge(vals, idx, offsets, k):
        return tuple(torch.from_numpy(a) for a in
                     merge_topk(vals.numpy(), idx.numpy(), offsets, k))

    @staticmethod
    def group_mean(x, groups):
        xn = x.numpy()
        return torch.from_numpy(np.stack([xn[g].mean(axis=0) for g in groups])
                                .astype(np.float32))

    @staticmethod
    def self_dist(x, metric):
        return CpuBackend.distmat(x, x, metric)

    @staticmethod
    def re_ranking(q_g, q_q, g_g):
        return torch.from_numpy(ev.re_ranking(q_g.numpy(), q_q.numpy(), g_g.numpy()))

    @staticmethod
    def rank_eval(dist, qid, gid, qcam, gcam):
        d = dist.numpy() if isinstance(dist, torch.Tensor) else np.asarray(dist)
        ap, valid = ev.mean_ap(d, qid, gid, qcam, gcam, average=False)
        first = ev.first_match_rank(d, qid, gid, qcam, gcam)
        return ap, valid.astype(np.int32), first

    @staticmethod
    def finalize(sorted_d, pos_total, hist, before):
        sd, tot, h, b = (t.numpy() for t in (sorted_d, pos_total, hist, before))
        Q = sd.shape[0]
        ap = np.zeros(Q)
        valid = (tot > 0).astype(np.int32)
        first = np.where(tot > 0, b, -1).astype(np.int32)
        for q in range(Q):
            P = tot[q]
            if P == 0:
                continue
            le = np.cumsum(h[q, :P])
            pos_le = np.searchsorted(sd[q, :P], sd[q, :P], side='right')
            ap[q] = np.sum(pos_le / le) / P
        return torch.from_numpy(ap), torch.from_numpy(valid), torch.from_numpy(first)
