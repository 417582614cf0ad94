"""ORACLE (test infrastructure only) -- NumPy restatement of the reference's
retrieval evaluator, detectron/datasets/reid_dataset_evaluator.py.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline.  The product path
(pps_amd) never imports it.

Parity pinning: every function here is checked against golden vectors that
tests/golden/make_golden.py produced by importing the reference evaluator
unchanged (NumPy 2.2.6, scikit-learn 1.7.2).  AP follows scikit-learn >= 0.19
`average_precision_score` (step-wise, tie-grouped thresholds), which is what
the reference computes with any sklearn other than 0.18.1 (:390-407).
"""
from collections import OrderedDict

import numpy as np


def compute_dist(array1, array2, type='euclidean'):
    """reid_dataset_evaluator.py:244-272 (euclidean branch, float32 NumPy):
    d^2 = -2 a.b^T + |a|^2 + |b|^2, negatives clamped to 0, sqrt.
    'cosine' here is the true cosine DISTANCE 1 - cos (the reference branch
    :259-263 is broken: `normalize` undefined, and it returns similarity)."""
    assert type in ('cosine', 'euclidean', 'sqeuclidean')
    a = np.asarray(array1, np.float32)
    b = np.asarray(array2, np.float32)
    if type == 'cosine':
        an = a / np.maximum(np.linalg.norm(a, axis=1, keepdims=True), 1e-12)
        bn = b / np.maximum(np.linalg.norm(b, axis=1, keepdims=True), 1e-12)
        return (1.0 - an @ bn.T).astype(np.float32)
    sq1 = np.sum(np.square(a), axis=1)[:, None]
    sq2 = np.sum(np.square(b), axis=1)[None, :]
    d2 = -2 * (a @ b.T) + sq1 + sq2
    d2[d2 < 0] = 0
    return d2 if type == 'sqeuclidean' else np.sqrt(d2)


def pairwise_distance(X):
    """detectron/ops/pairwise_distance_op.cu:9-21 -- difference form, squared."""
    X = np.asarray(X, np.float64)
    diff = X[:, None, :] - X[None, :, :]
    return np.sum(diff * diff, axis=2).astype(np.float32)


def average_precision(y_true, y_score):
    """sklearn>=0.19 average_precision_score restated: thresholds are the
    distinct scores in decreasing order; AP = sum_t (R_t - R_{t-1}) * P_t."""
    y_true = np.asarray(y_true, bool)
    y_score = np.asarray(y_score)
    order = np.argsort(-y_score, kind='mergesort')
    s = y_score[order]
    t = y_true[order]
    last = np.r_[np.nonzero(np.diff(s))[0], len(s) - 1]  # end of each tie group
    tps = np.cumsum(t)[last].astype(np.float64)
    fps = (last + 1) - tps
    precision = tps / (tps + fps)
    recall = tps / tps[-1]
    prev = np.r_[0.0, recall[:-1]]
    return float(np.sum((recall - prev) * precision))


def _valid_mask(gallery_ids, gallery_cams, qid, qcam, order):
    return (gallery_ids[order] != qid) | (gallery_cams[order] != qcam)


def mean_ap(distmat, query_ids, gallery_ids, query_cams, gallery_cams, average=True):
    """reid_dataset_evaluator.py:366-439 (argsort made stable)."""
    distmat = np.asarray(distmat)
    m = distmat.shape[0]
    order = np.argsort(distmat, axis=1, kind='stable')
    aps = np.zeros(m)
    is_valid = np.zeros(m)
    for i in range(m):
        valid = _valid_mask(gallery_ids, gallery_cams, query_ids[i], query_cams[i], order[i])
        y_true = gallery_ids[order[i]][valid] == query_ids[i]
        if not np.any(y_true):
            continue
        y_score = -distmat[i][order[i]][valid]
        is_valid[i] = 1
        aps[i] = average_precision(y_true, y_score)
    if average:
        return float(np.sum(aps)) / np.sum(is_valid)
    return aps, is_valid


def cmc(distmat, query_ids, gallery_ids, query_cams, gallery_cams, topk=100,
        separate_camera_set=False, single_gallery_shot=False, first_match_break=False,
        average=True, rng=None):
    """reid_dataset_evaluator.py:283-363 (argsort made stable)."""
    distmat = np.asarray(distmat)
    m = distmat.shape[0]
    order = np.argsort(distmat, axis=1, kind='stable')
    ret = np.zeros([m, topk])
    is_valid = np.zeros(m)
    nvalid = 0
    rng = rng or np.random
    for i in range(m):
        valid = _valid_mask(gallery_ids, gallery_cams, query_ids[i], query_cams[i], order[i])
        if separate_camera_set:
            valid &= gallery_cams[order[i]] != query_cams[i]
        matches = gallery_ids[order[i]] == query_ids[i]
        if not np.any(matches[valid]):
            continue
        is_valid[i] = 1
        repeat = 100 if single_gallery_shot else 1
        if single_gallery_shot:
            inds = np.nonzero(valid)[0]
            by_id = OrderedDict()
            for j, x in zip(inds, gallery_ids[order[i]][valid]):
                by_id.setdefault(x, []).append(j)
        for _ in range(repeat):
            if single_gallery_shot:
                pick = np.zeros(len(valid), bool)
                for idx_list in by_id.values():
                    pick[rng.choice(idx_list)] = True
                hits = np.nonzero(matches[valid & pick])[0]
            else:
                hits = np.nonzero(matches[valid])[0]
            delta = 1.0 / (len(hits) * repeat)
            for j, k in enumerate(hits):
                if k - j >= topk:
                    break
                if first_match_break:
                    ret[i, k - j] += 1
                    break
                ret[i, k - j] += delta
        nvalid += 1
    if nvalid == 0:
        raise RuntimeError('No valid query')
    ret = ret.cumsum(axis=1)
    if average:
        return np.sum(ret, axis=0) / nvalid
    return ret, is_valid


def first_match_rank(distmat, query_ids, gallery_ids, query_cams, gallery_cams):
    """Per query, the CMC index `k - j` at which reid_dataset_evaluator.py
    :340-355 (first_match_break=True) books its hit: the number of valid
    entries ranked before the first true match in the stable argsort order;
    -1 for queries without a valid match (:336-338).  Not capped at topk."""
    distmat = np.asarray(distmat)
    order = np.argsort(distmat, axis=1, kind='stable')
    out = np.full(distmat.shape[0], -1, np.int64)
    for i in range(distmat.shape[0]):
        valid = _valid_mask(gallery_ids, gallery_cams, query_ids[i], query_cams[i], order[i])
        hits = np.nonzero(gallery_ids[order[i]][valid] == query_ids[i])[0]
        if len(hits):
            out[i] = hits[0]
    return out


def re_ranking(q_g_dist, q_q_dist, g_g_dist, k1=20, k2=6, lambda_value=0.3):
    """k-reciprocal re-ranking, reid_dataset_evaluator.py:442-519 (Zhong et
    al., CVPR'17), restated with the same float32 intermediates."""
    nq = q_g_dist.shape[0]
    full = np.block([[q_q_dist, q_g_dist], [q_g_dist.T, g_g_dist]])
    full = np.power(full, 2).astype(np.float32)
    full = np.transpose(1. * full / np.max(full, axis=0))          # :452-454
    n = full.shape[0]
    ranks = np.argsort(full).astype(np.int32)                        # :456
    half = int(np.around(k1 / 2.))

    def reciprocal(i, k):
        fwd = ranks[i, :k + 1]
        bwd = ranks[fwd, :k + 1]
        return fwd[np.where(bwd == i)[0]]

    V = np.zeros_like(full).astype(np.float32)
    for i in range(n):
        core = reciprocal(i, k1)
        expanded = core
        for cand in core:
            cand_set = reciprocal(cand, half)
            if len(np.intersect1d(cand_set, core)) > 2. / 3 * len(cand_set):
                expanded = np.append(expanded, cand_set)
        expanded = np.unique(expanded)
        w = np.exp(-full[i, expanded])
        V[i, expanded] = 1. * w / np.sum(w)                          # :486-488
    orig_q = full[:nq, ]
    if k2 != 1:                                                      # :490-494
        Vqe = np.zeros_like(V, dtype=np.float32)
        for i in range(n):
            Vqe[i, :] = np.mean(V[ranks[i, :k2], :], axis=0)
        V = Vqe
    inv = [np.where(V[:, j] != 0)[0] for j in range(n)]              # :497-499
    jac = np.zeros_like(orig_q, dtype=np.float32)
    for i in range(nq):                                               # :503-511
        tmin = np.zeros(shape=[1, n], dtype=np.float32)
        nz = np.where(V[i, :] != 0)[0]
        for j in nz:
            tmin[0, inv[j]] = tmin[0, inv[j]] + np.minimum(V[i, j], V[inv[j], j])
        jac[i] = 1 - tmin / (2. - tmin)
    final = jac * (1 - lambda_value) + orig_q * lambda_value
    return final[:nq, nq:]


def _row_topk_stable(a, k):
    """Per row, the k smallest entries in (value, index) order: the first k
    columns of a stable argsort, from argpartition + a (value, index) sort
    of the k + ties candidates (whole-row argsort is O(N^2 log N) at
    N ~ 16k)."""
    n = a.shape[1]
    kk = min(n, k)
    part = np.argpartition(a, kk - 1, axis=1)[:, :kk]
    out = np.empty((a.shape[0], kk), np.int64)
    for i in range(a.shape[0]):
        kth = a[i, part[i]].max()
        cand = np.nonzero(a[i] <= kth)[0]          # every entry tied with the k-th too
        order = np.lexsort((cand, a[i, cand]))      # value, then index
        out[i] = cand[order[:kk]]
    return out


def re_ranking_sparse(q_g_dist, q_q_dist, g_g_dist, k1=20, k2=6, lambda_value=0.3):
    """re_ranking above for N = Q + G in the tens of thousands, with the same
    float32 values in the same operation order (sparse V / V_qe rows, the
    inverted index as row lists) -- test infrastructure for the long-row GPU
    check (tests/test_gpu_configs.py).  Ranks are the stable (value, index)
    order, which equals np.argsort's wherever the first k1 + 1 values of a
    row are distinct.  Pinned: equal to re_ranking on the golden fixture and
    on random cases (tests/test_oracle_golden.py)."""
    nq = q_g_dist.shape[0]
    full = np.block([[q_q_dist, q_g_dist], [q_g_dist.T, g_g_dist]])
    full = np.power(full, 2).astype(np.float32)
    full = np.ascontiguousarray(np.transpose(1. * full / np.max(full, axis=0)))
    n = full.shape[0]
    half = int(np.around(k1 / 2.))
    ranks = _row_topk_stable(full, max(k1 + 1, k2)).astype(np.int32)

    def reciprocal(i, k):
        fwd = ranks[i, :k + 1]
        bwd = ranks[fwd, :k + 1]
        return fwd[np.where(bwd == i)[0]]

    V = [None] * n    # row i: (sorted columns, float32 weights)
    for i in range(n):
        core = reciprocal(i, k1)
        expanded = core
        for cand in core:
            cand_set = reciprocal(cand, half)
            if len(np.intersect1d(cand_set, core)) > 2. / 3 * len(cand_set):
                expanded = np.append(expanded, cand_set)
        expanded = np.unique(expanded)
        w = np.exp(-full[i, expanded])
        V[i] = (expanded, (1. * w / np.sum(w)).astype(np.float32))
    if k2 != 1:
        # np.mean(V[rows, :], axis=0): float32 sum down the k2 rows in row
        # order (zeros of the other rows included), then / k2
        Vqe = [None] * n
        for i in range(n):
            rows = [V[r] for r in ranks[i, :k2]]
            cols = np.unique(np.concatenate([c for c, _ in rows]))
            acc = np.zeros(len(cols), np.float32)
            for c, v in rows:
                dense = np.zeros(len(cols), np.float32)
                dense[np.searchsorted(cols, c)] = v
                acc = acc + dense
            Vqe[i] = (cols, (acc / np.float32(k2)).astype(np.float32))
        V = Vqe
    inv = {}
    for r in range(n):                     # V[:, j] != 0, rows ascending
        c, v = V[r]
        for j in c[v != 0]:
            inv.setdefault(int(j), []).append(r)
    vget = [dict(zip(c.tolist(), v.tolist())) for c, v in V]
    jac = np.zeros((nq, n), np.float32)
    for i in range(nq):
        tmin = np.zeros(n, np.float32)
        c, v = V[i]
        for j, vij in zip(c, v):
            if vij == 0:
                continue
            rows = np.asarray(inv[int(j)])
            other = np.asarray([vget[r][int(j)] for r in rows], np.float32)
            tmin[rows] = tmin[rows] + np.minimum(np.float32(vij), other)
        jac[i] = 1 - tmin / (2. - tmin)
    final = jac * (1 - lambda_value) + full[:nq] * lambda_value
    return final[:nq, nq:]


def parse_im_name(im_name, parse_type='id'):
    """reid_dataset_evaluator.py:224-231."""
    assert parse_type in ('id', 'cam')
    return int(im_name[:8]) if parse_type == 'id' else int(im_name[9:13])


def evaluate_arrays(feat, ids, cams, marks, rerank=False, verbose=False):
    """reid_dataset_evaluator.py:29-209 orchestration on arrays: q/g/mq split
    by mark, euclidean distances, mAP + CMC(top-10, first-match-break),
    multi-query mean pooling per (id, cam) in first-appearance order."""
    feat = np.asarray(feat, np.float32)
    q, g, mq = marks == 0, marks == 1, marks == 2

    def score(d, qi, gi, qc, gc):
        return (mean_ap(d, qi, gi, qc, gc),
                cmc(d, qi, gi, qc, gc, first_match_break=True, topk=10))

    qg = compute_dist(feat[q], feat[g])
    mAP, cmc_s = score(qg, ids[q], ids[g], cams[q], cams[g])
    mq_mAP = mq_cmc = None
    if mq.any():
        groups = OrderedDict()
        for k, (i, c) in enumerate(zip(ids[mq], cams[mq])):
            groups.setdefault((i, c), []).append(k)
        mf = np.stack([feat[mq][v].mean(axis=0) for v in groups.values()])
        keys = np.array(list(groups.keys()))
        mq_g = compute_dist(mf, feat[g])
        mq_mAP, mq_cmc = score(mq_g, keys[:, 0], ids[g], keys[:, 1], cams[g])
    if rerank:                                                        # :161-207
        qq = compute_dist(feat[q], feat[q])
        gg = compute_dist(feat[g], feat[g])
        rr = re_ranking(qg, qq, gg)
        mAP, cmc_s = score(rr, ids[q], ids[g], cams[q], cams[g])
        if mq.any():                                                  # :185-206
            mqmq = compute_dist(mf, mf)
            rr_mq = re_ranking(mq_g, mqmq, gg)
            mq_mAP, mq_cmc = score(rr_mq, keys[:, 0], ids[g], keys[:, 1], cams[g])
    return mAP, cmc_s, mq_mAP, mq_cmc
