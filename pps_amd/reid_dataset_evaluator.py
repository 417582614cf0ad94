"""Re-ID retrieval evaluation on the GPU -- same API as the reference's
detectron/datasets/reid_dataset_evaluator.py, computed by libpps_hip.so.

  compute_dist(array1, array2, type)      :244-272  -> HIP FP32-MFMA distmat
  mean_ap(distmat, ids/cams..., average)  :366-439  -> count-based AP kernels
  cmc(distmat, ..., topk, first_match_break) :283-363
  evaluate(json_dataset, all_feats, output_dir) :29-209
  get_info / parse_im_name                :212-231

Inputs may be NumPy arrays (copied to the current device) or CUDA tensors.
Outputs of compute_dist are CUDA tensors when the inputs were, NumPy
otherwise.  The ranking is a stable (distance, gallery index) order; the
reference's np.argsort is unstable, so the two agree except for exact ties,
where CMC can differ by construction and mAP cannot (AP groups ties).
"""
import contextlib
import os
import time
from collections import OrderedDict

import numpy as np
import torch

from . import ops
from .config import cfg


def _to_dev(x, dtype=torch.float32):
    if isinstance(x, torch.Tensor):
        t = x if x.is_cuda else x.cuda()
        return t.to(dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(x)).to(dtype).cuda()


@contextlib.contextmanager
def measure_time(enter_msg, verbose=True):
    """reid_dataset_evaluator.py:234-241 (same printed format)."""
    st = time.time()
    if verbose:
        print(enter_msg)
    yield
    if verbose:
        torch.cuda.synchronize()
        print('Done, {:.2f}s'.format(time.time() - st))


def compute_dist(array1, array2, type='euclidean'):
    """[m1,n] x [m2,n] -> [m1,m2]; 'euclidean' | 'sqeuclidean' | 'cosine'
    (cosine = 1 - cos, a distance; see include/pps_abi.h)."""
    assert type in ['cosine', 'euclidean', 'sqeuclidean']
    as_numpy = not isinstance(array1, torch.Tensor)
    d = ops.compute_dist(_to_dev(array1), _to_dev(array2), metric=type)
    return d.cpu().numpy() if as_numpy else d


def _host_ids(x):
    return x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


def rank_eval(distmat, query_ids, gallery_ids, query_cams, gallery_cams, index=None):
    """Per-query (ap float64, valid int32, first_rank int32) on the device:
    true matches listed from a per-identity gallery index (ops.MatchIndex,
    built from the ids unless given), then one streaming count pass over the
    distance rows (pps_collect_matches / pps_rank_prepare /
    pps_rank_count_stream / pps_ap_finalize).  No capacity limit on a
    query's true matches (pps_rank_prepare sorts lists beyond its LDS merge
    in global memory)."""
    d = distmat if isinstance(distmat, torch.Tensor) and distmat.is_cuda and \
        distmat.dtype == torch.float32 and distmat.dim() == 2 and \
        (distmat.shape[0] < 2 or distmat.stride(1) == 1) else _to_dev(distmat)
    if index is None:
        index = ops.MatchIndex(_host_ids(query_ids), _host_ids(query_cams),
                               _host_ids(gallery_ids), _host_ids(gallery_cams), d.device)
    pos_d, pos_idx, pos_cnt, junk = ops.collect_matches(d, index)
    sp = ops.rank_prepare(pos_d[None], pos_idx[None], pos_cnt[None])
    hist, before = ops.rank_count_stream(d, 0, sp, junk)
    return ops.ap_finalize(sp.sorted_d, sp.pos_total, hist, before)


def _np(x):
    return x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


def scores_from_ranks(ap, valid, first_rank, topk=10):
    """mAP and CMC[topk] from per-query results (host, O(Q))."""
    ap, valid, first_rank = _np(ap), _np(valid).astype(bool), _np(first_rank)
    nvalid = int(valid.sum())
    mAP = float(np.sum(ap)) / nvalid if nvalid else float('nan')
    if nvalid == 0:
        return mAP, None
    hits = np.zeros(topk)
    fr = first_rank[valid]
    np.add.at(hits, fr[fr < topk], 1)
    return mAP, np.cumsum(hits) / nvalid


def mean_ap(distmat, query_ids=None, gallery_ids=None, query_cams=None,
            gallery_cams=None, average=True):
    ap, valid, _ = rank_eval(distmat, query_ids, gallery_ids, query_cams, gallery_cams)
    ap, valid = _np(ap), _np(valid).astype(np.float64)
    if average:
        return float(np.sum(ap)) / np.sum(valid)
    return ap, valid


def cmc(distmat, query_ids=None, gallery_ids=None, query_cams=None, gallery_cams=None,
        topk=100, separate_camera_set=False, single_gallery_shot=False,
        first_match_break=False, average=True, rng=None):
    """reid_dataset_evaluator.py:283-363 with the same defaults and outputs:
    the fractional CMC (first_match_break=False), the first-match CMC, and
    separate_camera_set, from per-positive counts on the device
    (pps_cmc_counts / pps_cmc_finalize; the Market protocol evaluate() uses
    takes the mAP pass's first-match ranks instead).  The ranking is the
    stable (distance, index) order.  single_gallery_shot (:334-346) draws one
    valid gallery entry per identity 100 times per valid query with `rng`
    (default: the global np.random, as the reference's np.random.choice):
    the same draws in the same order, so a seeded call equals the
    reference's; the grouping and ranking run on the device (_cmc_sgs)."""
    if single_gallery_shot:
        ret, valid = _cmc_sgs(distmat, query_ids, gallery_ids, query_cams, gallery_cams, topk,
                              separate_camera_set, first_match_break, rng)
        if not valid.any():
            raise RuntimeError('No valid query')
        if average:
            return np.sum(ret, axis=0) / valid.sum()
        return ret, valid.astype(np.float64)
    d = distmat if isinstance(distmat, torch.Tensor) and distmat.is_cuda and \
        distmat.dtype == torch.float32 and distmat.dim() == 2 and \
        (distmat.shape[0] < 2 or distmat.stride(1) == 1) else _to_dev(distmat)
    if first_match_break and not separate_camera_set:
        _, valid, first = rank_eval(d, query_ids, gallery_ids, query_cams, gallery_cams)
        valid, first = _np(valid).astype(bool), _np(first)
        ret = np.zeros((len(valid), topk))
        rows = np.nonzero(valid & (first < topk))[0]
        ret[rows, first[rows]] = 1
        ret = ret.cumsum(axis=1)
    else:
        index = ops.MatchIndex(_host_ids(query_ids), _host_ids(query_cams),
                               _host_ids(gallery_ids), _host_ids(gallery_cams), d.device)
        pos_d, pos_idx, pos_cnt, junk = ops.collect_matches(d, index)
        sp = ops.rank_prepare(pos_d[None], pos_idx[None], pos_cnt[None])
        hist = ops.cmc_counts(d, 0, sp, junk, index, separate_camera_set)
        ret, valid = ops.cmc_finalize(sp.pos_total, hist, topk, first_match_break)
        ret, valid = _np(ret), _np(valid).astype(bool)
    if not valid.any():
        raise RuntimeError('No valid query')
    if average:
        return np.sum(ret, axis=0) / valid.sum()
    return ret, valid.astype(np.float64)


SGS_MAX_IDS = 16384   # pps_sgs_keys / pps_sgs_groups (include/pps_abi.h)


def _cmc_sgs(distmat, query_ids, gallery_ids, query_cams, gallery_cams, topk,
             separate_camera_set, first_match_break, rng, repeat=100):
    """CMC single_gallery_shot (reid_dataset_evaluator.py:321-363 with
    :334-346): stable rank list (pps_argsort_rows), per-query identity groups
    in `ids_dict` order (pps_sgs_keys / pps_sgs_groups), the reference's
    draws (`_unique_sample` :275-280: one np.random.choice per identity and
    repeat, reproduced call for call by one randint per query), and the
    query identity's rank among the draws (pps_sgs_ranks).  rng: a legacy
    np.random.RandomState or the np.random module (the reference's stream);
    a np.random.Generator draws with .integers -- valid draws, but not the
    reference's sequence."""
    rng = np.random if rng is None else rng
    if isinstance(rng, np.random.Generator):
        randint = rng.integers
    elif hasattr(rng, 'randint'):
        randint = rng.randint
    else:
        raise TypeError('rng must be a np.random.RandomState, the np.random module or a '
                        'np.random.Generator, got %r' % type(rng).__name__)
    d = _to_dev(distmat)
    Q, G = d.shape
    gid = np.asarray(gallery_ids).astype(np.int64)
    qid = np.asarray(query_ids).astype(np.int64)
    uniq = np.unique(gid)
    U = len(uniq)
    if U > SGS_MAX_IDS:
        raise ValueError('single_gallery_shot: %d distinct gallery identities, the device '
                         'grouping holds at most %d' % (U, SGS_MAX_IDS))
    gdense = np.searchsorted(uniq, gid)
    qpos = np.minimum(np.searchsorted(uniq, qid), U - 1)
    qdense = np.where(uniq[qpos] == qid, qpos, -1)
    dev = d.device
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.int32)).to(dev)
    order = ops.argsort_rows(d)
    perm, gstart, glen, nids, qt = ops.sgs_groups(order, i32(gdense), i32(gallery_cams),
                                                  i32(qdense), i32(query_cams), U,
                                                  separate_camera_set)
    del order
    glen_h, nids_h, qt_h = _np(glen), _np(nids), _np(qt)
    valid = qt_h >= 0
    rows = np.nonzero(valid)[0]
    ret = np.zeros((Q, topk))
    delta = 1. if first_match_break else 1. / (1 * repeat)   # one hit per repeat (:347-356)
    if len(rows):
        ldd = int(nids_h[rows].max())
        chunk = max(1, (64 << 20) // (repeat * ldd * 4))
        for c0 in range(0, len(rows), chunk):
            rs = rows[c0:c0 + chunk]
            draws = np.zeros((len(rs), repeat, ldd), dtype=np.int32)
            for i, q in enumerate(rs):   # query order, as the reference draws
                n = int(nids_h[q])
                draws[i, :, :n] = randint(0, np.tile(glen_h[q, :n], repeat)).reshape(repeat, n)
            k = _np(ops.sgs_ranks(perm, gstart, glen, nids, qt, i32(rs), i32(draws)))
            qq = np.repeat(rs, repeat)
            kk = k.reshape(-1)
            keep = kk < topk
            np.add.at(ret, (qq[keep], kk[keep]), delta)
    return ret.cumsum(axis=1), valid


def parse_im_name(im_name, parse_type='id'):
    """reid_dataset_evaluator.py:224-231."""
    assert parse_type in ('id', 'cam')
    return int(im_name[:8]) if parse_type == 'id' else int(im_name[9:13])


def get_info(entry):
    """reid_dataset_evaluator.py:212-221."""
    im_name = os.path.basename(entry['image'])
    return (parse_im_name(im_name, 'id'), parse_im_name(im_name, 'cam'), im_name,
            entry['mark'], entry['image'])


def print_scores(mAP, cmc_scores):
    """:95-98 -- the line tools/loss_vs_map.py:80 parses."""
    print('[mAP: {:5.2%}], [cmc1: {:5.2%}], [cmc5: {:5.2%}], [cmc10: {:5.2%}]'
          .format(mAP, *cmc_scores[[0, 4, 9]]))


def evaluate(json_dataset, all_feats, output_dir, verbose=True):
    """reid_dataset_evaluator.py:29-209.  Returns (mAP, cmc, mq_mAP, mq_cmc)."""
    roidb = json_dataset.get_roidb(gt=True)
    info = [get_info(e) for e in roidb]
    ids = np.array([i[0] for i in info])
    cams = np.array([i[1] for i in info])
    marks = np.array([i[3] for i in info])
    return evaluate_arrays(all_feats, ids, cams, marks, verbose=verbose)


def evaluate_arrays(all_feats, ids, cams, marks, verbose=True, metric=None):
    metric = metric or cfg.REID.get('DISTANCE', 'euclidean')
    feat = _to_dev(all_feats)
    ids, cams, marks = np.asarray(ids), np.asarray(cams), np.asarray(marks)
    q_inds, g_inds, mq_inds = marks == 0, marks == 1, marks == 2
    qi = torch.from_numpy(np.nonzero(q_inds)[0]).cuda()
    gi = torch.from_numpy(np.nonzero(g_inds)[0]).cuda()
    if verbose:
        print('-' * 40)
        print('Starting eval')

    def compute_score(dist, q_ids, g_ids, q_cams, g_cams):
        ap, valid, first = rank_eval(dist, q_ids, g_ids, q_cams, g_cams)
        return scores_from_ranks(ap, valid, first, topk=10)

    tiled = ops.dist_math() in ('h2', 'x3') and feat.shape[1] % 32 == 0
    # re-ranking on the h2 / x3 paths: ONE mirrored self-distance of [queries;
    # gallery] gives q_g, q_q and g_g as blocks of one exactly symmetric
    # matrix (re-ranking then reads q_g^T in place, PPS_RERANK_WHOLE)
    whole = bool(cfg.REID.RERANK) and tiled
    if whole:
        x = feat.index_select(0, torch.cat([qi, gi])).contiguous()
        qf, gf = x[:len(qi)], x[len(qi):]
    else:
        qf = feat.index_select(0, qi).contiguous()
        gf = feat.index_select(0, gi).contiguous()
    with measure_time('Computing distance...', verbose):
        if verbose:
            print('Array size: ', tuple(qf.shape), tuple(gf.shape))
        # the gallery split once (h2: f16x2 planes; x3: chunk-tiled bf16x3
        # planes): q_g and the multi-query mq_g read it
        gsrc = ops.GalleryIndex(gf, tiled=True) if tiled else gf
        if whole:
            _, q_g, q_q, g_g = ops.self_distance_blocks(x, len(qi), metric=metric)
        else:
            q_g = ops.compute_dist(qf, gsrc, metric=metric, pad_rows=True, q_planes=tiled)
    with measure_time('Computing scores...', verbose):
        mAP, cmc_scores = compute_score(q_g, ids[q_inds], ids[g_inds], cams[q_inds],
                                        cams[g_inds])
    if verbose:
        print('{:<30}'.format('Single Query:'), end='')
        print_scores(mAP, cmc_scores)

    mq_mAP, mq_cmc = None, None
    if mq_inds.any():
        groups = OrderedDict()
        for k, key in enumerate(zip(ids[mq_inds], cams[mq_inds])):
            groups.setdefault(key, []).append(k)
        mq_rows = np.nonzero(mq_inds)[0]
        pooled = ops.group_mean(feat, [mq_rows[v] for v in groups.values()])
        keys = np.array(list(groups.keys()))
        with measure_time('Multi Query, Computing distance...', verbose):
            mq_g = ops.compute_dist(pooled, gsrc, metric=metric, pad_rows=True,
                                    q_planes=tiled)
        with measure_time('Multi Query, Computing scores...', verbose):
            mq_mAP, mq_cmc = compute_score(mq_g, keys[:, 0], ids[g_inds], keys[:, 1],
                                           cams[g_inds])
        if verbose:
            print('{:<30}'.format('Multi Query:'), end='')
            print_scores(mq_mAP, mq_cmc)

    if cfg.REID.RERANK:
        # :161-207 -- re-ranked scores overwrite the plain ones
        with measure_time('Re-ranking distance...', verbose):
            # 16-byte rows: re-ranking reads the blocks in place (no N x N copy)
            if whole:
                rr = ops.re_ranking(q_g, q_q, g_g, symmetric=True, whole=True)
            else:
                q_q = ops.compute_dist(qf, qf, metric=metric, pad_rows=True)
                g_g = ops.compute_dist(gf, gsrc, metric=metric, pad_rows=True)
                rr = ops.re_ranking(q_g, q_q, g_g)
        with measure_time('Computing scores for re-ranked distance...', verbose):
            mAP, cmc_scores = compute_score(rr, ids[q_inds], ids[g_inds], cams[q_inds],
                                            cams[g_inds])
        if verbose:
            print('{:<30}'.format('Re-ranked Single Query:'), end='')
            print_scores(mAP, cmc_scores)
        if mq_inds.any():
            with measure_time('Multi Query, Re-ranking distance...', verbose):
                mq_mq = ops.compute_dist(pooled, pooled, metric=metric, pad_rows=True)
                # g_g a block of the whole matrix: exactly symmetric, untagged
                sym = True if whole and getattr(mq_mq, '_pps_symmetric', False) else None
                rr_mq = ops.re_ranking(mq_g, mq_mq, g_g, symmetric=sym)
            with measure_time('Multi Query, Computing scores for re-ranked distance...',
                              verbose):
                mq_mAP, mq_cmc = compute_score(rr_mq, keys[:, 0], ids[g_inds], keys[:, 1],
                                               cams[g_inds])
            if verbose:
                print('{:<30}'.format('Re-ranked Multi Query:'), end='')
                print_scores(mq_mAP, mq_cmc)
    return mAP, cmc_scores, mq_mAP, mq_cmc


def re_ranking(q_g_dist, q_q_dist, g_g_dist, k1=20, k2=6, lambda_value=0.3):
    """:442-519 on the GPU; NumPy in -> NumPy out, CUDA tensors in -> tensor out."""
    as_numpy = not isinstance(q_g_dist, torch.Tensor)
    out = ops.re_ranking(_to_dev(q_g_dist), _to_dev(q_q_dist), _to_dev(g_g_dist), k1, k2,
                         lambda_value)
    return out.cpu().numpy() if as_numpy else out
