"""Market-1501-scale retrieval parity (BASELINE configs[1] sizes: Q=3368,
G=15913, D=3968) on synthetic features of the SURVEY §8(d) distribution.

* distances: GPU (x3 and exact-f32 kernels) vs the oracle's NumPy
  restatement of compute_dist, within 1e-4 (north_star);
* ranking: the oracle's stable-argsort mean_ap / cmc on the GPU's own
  distances vs the GPU count-based kernels -- AP per query within 1e-12 and
  CMC exact (identical inputs, so the rank of every positive must agree);
* end to end: mAP / CMC@1 of the GPU path vs the all-CPU oracle path; these
  can differ only through near-tied distances whose fp32 rounding differs
  (|Δd| < 1e-5), which moves a positive by a rank: mAP within 1e-4, CMC@k
  within 2 queries.
"""
import numpy as np
import pytest
import torch

from oracle import evaluator as ev

pytestmark = pytest.mark.gpu

Q, G, D = 3368, 15913, 3968


@pytest.fixture(scope='module')
def market():
    rng = np.random.RandomState(0)
    qid = rng.randint(1, 751, Q)
    gid = np.concatenate([rng.randint(1, 751, G - 2793), np.zeros(2793, int)])
    qcam = rng.randint(1, 7, Q)
    gcam = rng.randint(1, 7, G)
    cent = rng.randn(751, D).astype(np.float32)
    f = cent[np.concatenate([qid, gid])] + 4.0 * rng.randn(Q + G, D).astype(np.float32)
    f /= np.linalg.norm(f, axis=1, keepdims=True)
    f = f.astype(np.float32)
    ref = ev.compute_dist(f[:Q], f[Q:])
    return dict(qf=f[:Q], gf=f[Q:], qid=qid, gid=gid, qcam=qcam, gcam=gcam, ref=ref)


@pytest.mark.parametrize('math', ['x3', 'f32'])
def test_market_scale_parity(market, math):
    from pps_amd import ops
    from pps_amd import reid_dataset_evaluator as gev
    m = market
    d = ops.compute_dist(torch.from_numpy(m['qf']).cuda(), torch.from_numpy(m['gf']).cuda(),
                         math=math)
    dn = d.cpu().numpy()
    err = np.abs(dn - m['ref']).max()
    assert err < 1e-4, err
    # ranking on identical distances: exact
    ap, valid, first = gev.rank_eval(d, m['qid'], m['gid'], m['qcam'], m['gcam'])
    ap, valid, first = ap.cpu().numpy(), valid.cpu().numpy().astype(bool), first.cpu().numpy()
    ap_o, valid_o = ev.mean_ap(dn, m['qid'], m['gid'], m['qcam'], m['gcam'], average=False)
    np.testing.assert_array_equal(valid, valid_o.astype(bool))
    np.testing.assert_allclose(ap[valid], ap_o[valid_o.astype(bool)], rtol=0, atol=1e-12)
    cmc_o = ev.cmc(dn, m['qid'], m['gid'], m['qcam'], m['gcam'], topk=10,
                   first_match_break=True)
    mAP, cmc = gev.scores_from_ranks(ap, valid, first, topk=10)
    np.testing.assert_allclose(cmc, cmc_o, rtol=0, atol=1e-12)
    # end to end against the all-CPU path
    mAP_ref = ev.mean_ap(m['ref'], m['qid'], m['gid'], m['qcam'], m['gcam'])
    cmc_ref = ev.cmc(m['ref'], m['qid'], m['gid'], m['qcam'], m['gcam'], topk=10,
                     first_match_break=True)
    assert abs(mAP - mAP_ref) < 1e-4, (mAP, mAP_ref)
    assert np.abs(cmc - cmc_ref).max() <= 2.0 / valid.sum(), (cmc, cmc_ref)
    assert 0.5 < mAP < 0.9   # non-trivial regime (~0.69)
