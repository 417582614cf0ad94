"""Near-tie-aware exact ranking parity (north_star: "bit-exact on rank
indices ... mAP/Rank-1 equal to the CPU reference").

Two float32 computations of the same distance matrix differ by at most
e = max|d_gpu - d_ref| per entry, so two entries a, b can swap order between
them only if |d_ref[a] - d_ref[b]| <= 2e.  These helpers therefore demand:

* rank indices: position j of the GPU's stable top-k equals position j of the
  oracle's stable argsort, except where the two entries there are a near-tie
  (their oracle distances differ by <= 2e); and in every position the GPU's
  entry has the oracle distance of the j-th order statistic within 2e;
* AP per query: equal (<= 1e-12, float64 summation order) for every query
  none of whose true matches has another valid entry within 2e; first-match
  rank equal for every query whose first true match has no valid neighbour
  within 2e; mAP and CMC equal (<= 1e-12) when no query is affected.

Each check returns the counts so that tests can print how many near-tie
positions / queries there actually were.
"""
import numpy as np

from oracle import evaluator as ev


def tie_eps(d_gpu, d_ref):
    """2 x the largest per-entry difference, plus one float32 ulp at the
    largest distance (so an exact-equality pair never counts as a flip)."""
    d_gpu = np.asarray(d_gpu, np.float32)
    d_ref = np.asarray(d_ref, np.float32)
    err = float(np.abs(d_gpu.astype(np.float64) - d_ref).max()) if d_ref.size else 0.0
    ulp = float(np.spacing(np.float32(max(1.0, float(np.abs(d_ref).max()) if d_ref.size
                                          else 1.0))))
    return 2.0 * err + ulp


def check_topk(idx_gpu, d_ref, k, eps, order_ref=None):
    """idx_gpu [Q, k] global gallery indices from the GPU; d_ref [Q, G] oracle
    distances.  Returns the number of positions where the index differs (all
    of them near-ties, else AssertionError)."""
    idx_gpu = np.asarray(idx_gpu).astype(np.int64)
    Q, G = d_ref.shape
    assert idx_gpu.shape == (Q, min(k, G)), idx_gpu.shape
    assert idx_gpu.min() >= 0 and idx_gpu.max() < G
    srt = np.sort(idx_gpu, axis=1)
    assert not np.any(srt[:, 1:] == srt[:, :-1]), 'duplicate index in a GPU top-k row'
    if order_ref is None:
        order_ref = np.argsort(d_ref, axis=1, kind='stable')[:, :k]
    d_at_gpu = np.take_along_axis(d_ref, idx_gpu, axis=1).astype(np.float64)
    d_at_ref = np.take_along_axis(d_ref, order_ref, axis=1).astype(np.float64)
    gap = np.abs(d_at_gpu - d_at_ref)
    bad = gap > eps
    assert not bad.any(), ('top-k rank index differs beyond the near-tie bound at %d '
                           'positions (max oracle gap %.3g > eps %.3g), first at %s'
                           % (int(bad.sum()), float(gap.max()), eps,
                              tuple(np.argwhere(bad)[0])))
    return int((idx_gpu != order_ref).sum())


def affected_queries(d_ref, qid, gid, qcam, gcam, eps):
    """(ap_affected, first_affected) boolean [Q] masks: a query is
    AP-affected when one of its true matches has another valid gallery entry
    within eps of its oracle distance, first-match-affected when its first
    true match (stable order) does."""
    d_ref = np.asarray(d_ref)
    qid, gid = np.asarray(qid), np.asarray(gid)
    qcam, gcam = np.asarray(qcam), np.asarray(gcam)
    Q, G = d_ref.shape
    ap_aff = np.zeros(Q, bool)
    first_aff = np.zeros(Q, bool)
    for i in range(Q):
        junk = (gid == qid[i]) & (gcam == qcam[i])
        pos = (gid == qid[i]) & ~junk
        if not pos.any():
            continue
        row = d_ref[i].astype(np.float64)
        s = np.sort(row[~junk])
        dp = row[pos]
        n_near = np.searchsorted(s, dp + eps, 'right') - np.searchsorted(s, dp - eps, 'left')
        ap_aff[i] = bool((n_near > 1).any())
        pidx = np.nonzero(pos)[0]
        first = pidx[np.lexsort((pidx, row[pidx]))[0]]
        dp0 = row[first]
        first_aff[i] = (np.searchsorted(s, dp0 + eps, 'right')
                        - np.searchsorted(s, dp0 - eps, 'left')) > 1
    return ap_aff, first_aff


def check_rank_metrics(ap, valid, first, d_ref, qid, gid, qcam, gcam, eps, topk=10):
    """GPU per-query (ap, valid, first_rank) vs the oracle on d_ref.  Returns a
    dict of counts; raises AssertionError on any difference the near-tie bound
    does not explain."""
    ap = np.asarray(ap, np.float64)
    valid = np.asarray(valid).astype(bool)
    first = np.asarray(first).astype(np.int64)
    ap_o, valid_o = ev.mean_ap(d_ref, qid, gid, qcam, gcam, average=False)
    valid_o = valid_o.astype(bool)
    first_o = ev.first_match_rank(d_ref, qid, gid, qcam, gcam)
    np.testing.assert_array_equal(valid, valid_o)
    ap_aff, first_aff = affected_queries(d_ref, qid, gid, qcam, gcam, eps)
    ok = valid & ~ap_aff
    np.testing.assert_allclose(ap[ok], ap_o[ok], rtol=0, atol=1e-12)
    okf = valid & ~first_aff
    np.testing.assert_array_equal(first[okf], first_o[okf])
    nvalid = int(valid.sum())
    mAP = float(ap[valid].sum()) / nvalid
    mAP_o = float(ap_o[valid].sum()) / nvalid

    def cmc_of(fr):
        hits = np.zeros(topk)
        f = fr[valid]
        np.add.at(hits, f[(f >= 0) & (f < topk)], 1)
        return np.cumsum(hits) / nvalid

    cmc, cmc_o = cmc_of(first), cmc_of(first_o)
    n_ap, n_first = int((valid & ap_aff).sum()), int((valid & first_aff).sum())
    if n_ap == 0:
        assert abs(mAP - mAP_o) <= 1e-12, (mAP, mAP_o)
    else:
        # each affected query's AP is in [0, 1]
        assert abs(mAP - mAP_o) <= float(n_ap) / nvalid, (mAP, mAP_o, n_ap)
    if n_first == 0:
        np.testing.assert_allclose(cmc, cmc_o, rtol=0, atol=1e-12)
    else:
        assert np.abs(cmc - cmc_o).max() <= float(n_first) / nvalid + 1e-12
    return dict(eps=eps, nvalid=nvalid, ap_affected=n_ap, first_affected=n_first,
                ap_differs=int((np.abs(ap - ap_o) > 1e-12)[valid].sum()),
                first_differs=int((first != first_o)[valid].sum()),
                mAP=mAP, mAP_ref=mAP_o, cmc1=float(cmc[0]), cmc1_ref=float(cmc_o[0]))
