"""Pin the oracle: its NumPy restatement of the reference evaluator must
reproduce the golden vectors produced by the reference itself
(tests/golden/make_golden.py, reference imported unchanged)."""
import os

import numpy as np
import pytest

from oracle import evaluator as ev
from tests.conftest import GOLDEN


@pytest.mark.parametrize('case', ['market_small', 'full_dim'])
def test_compute_dist_matches_reference(golden, case):
    g = golden(case)
    d = ev.compute_dist(g['qf'], g['gf'], 'euclidean')
    np.testing.assert_allclose(d, g['dist'], rtol=0, atol=2e-6)


@pytest.mark.parametrize('case', ['market_small', 'full_dim'])
def test_mean_ap_matches_reference(golden, case):
    g = golden(case)
    aps, valid = ev.mean_ap(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'],
                            average=False)
    np.testing.assert_array_equal(valid, g['valid_ap'])
    np.testing.assert_allclose(aps, g['aps'], rtol=0, atol=1e-12)
    m = ev.mean_ap(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'])
    assert abs(m - float(g['mAP'])) < 1e-12


@pytest.mark.parametrize('case', ['market_small', 'full_dim'])
def test_cmc_matches_reference(golden, case):
    g = golden(case)
    ret, valid = ev.cmc(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'], topk=10,
                        first_match_break=True, average=False)
    np.testing.assert_array_equal(valid, g['valid_cmc'])
    np.testing.assert_allclose(ret, g['cmc_all'], atol=0)
    avg = ev.cmc(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'], topk=10,
                 first_match_break=True)
    np.testing.assert_allclose(avg, g['cmc'], atol=1e-15)


def test_ap_tie_grouping_matches_reference(golden):
    g = golden('ties')
    aps, valid = ev.mean_ap(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'],
                            average=False)
    np.testing.assert_allclose(aps, g['aps'], atol=1e-12)
    # the fixture really has ties
    assert any(len(np.unique(r)) < len(r) for r in g['dist'])


def test_rerank_matches_reference(golden):
    g = golden('rerank')
    rr = ev.re_ranking(g['q_g'], g['q_q'], g['g_g'], k1=20, k2=6, lambda_value=0.3)
    np.testing.assert_allclose(rr, g['rerank'], rtol=0, atol=1e-6)
    m = ev.mean_ap(rr, g['qid'], g['gid'], g['qcam'], g['gcam'])
    assert abs(m - float(g['mAP'])) < 1e-9


def test_evaluate_orchestration_matches_reference(golden):
    g = golden('evaluate')
    names = [str(n) for n in g['names']]
    ids = np.array([ev.parse_im_name(n, 'id') for n in names])
    cams = np.array([ev.parse_im_name(n, 'cam') for n in names])
    np.testing.assert_array_equal(ids, g['ids'])
    np.testing.assert_array_equal(cams, g['cams'])
    mAP, cmc, mq_mAP, mq_cmc = ev.evaluate_arrays(g['feat'], ids, cams, g['marks'])
    assert abs(mAP - float(g['mAP'])) < 1e-9
    np.testing.assert_allclose(cmc, g['cmc'], atol=1e-12)
    assert mq_mAP is None


def test_log_line_format():
    # the exact line the reference prints and tools/loss_vs_map.py:80 parses
    with open(os.path.join(GOLDEN, 'evaluate_log.txt')) as f:
        ref = [l for l in f.read().splitlines() if l.startswith('Single Query:')][0]
    import re
    assert re.search(r'Single Query:[ ]+\[mAP: [0-9]+([.][0-9]+)?%\]', ref)


def test_pairwise_distance_oracle_matches_norm_form():
    rng = np.random.RandomState(0)
    X = rng.randn(17, 12).astype(np.float32)
    Z = ev.pairwise_distance(X)
    assert np.all(np.diag(Z) == 0)
    np.testing.assert_allclose(Z, ev.compute_dist(X, X, 'sqeuclidean'), atol=1e-4)


def test_oracle_cmc_all_modes_vs_reference(golden):
    """The reference `cmc` beyond the Market protocol (cmc_modes.npz, made by
    the reference evaluator itself): its defaults (topk=100, fractional
    first_match_break=False) and separate_camera_set=True."""
    g = golden('cmc_modes')
    for tag in ('market_small', 'dense'):
        d, qid, gid = g[tag + '_dist'], g[tag + '_qid'], g[tag + '_gid']
        qcam, gcam = g[tag + '_qcam'], g[tag + '_gcam']
        for sep in (0, 1):
            for fmb in (0, 1):
                key = '%s_sep%d_fmb%d' % (tag, sep, fmb)
                got = ev.cmc(d, qid, gid, qcam, gcam, separate_camera_set=bool(sep),
                             first_match_break=bool(fmb))
                np.testing.assert_allclose(got, g[key], rtol=0, atol=1e-12, err_msg=key)
                ret, valid = ev.cmc(d, qid, gid, qcam, gcam, separate_camera_set=bool(sep),
                                    first_match_break=bool(fmb), average=False)
                np.testing.assert_allclose(ret, g[key + '_all'], rtol=0, atol=1e-12)
                np.testing.assert_array_equal(valid, g[key + '_valid'])
        np.testing.assert_allclose(ev.cmc(d, qid, gid, qcam, gcam), g[tag + '_default'],
                                   rtol=0, atol=1e-12)
        np.testing.assert_allclose(ev.cmc(d, qid, gid, qcam, gcam, topk=5,
                                          separate_camera_set=True),
                                   g[tag + '_sep1_fmb0_top5'], rtol=0, atol=1e-12)


def test_oracle_cmc_single_gallery_shot_vs_reference_golden(golden):
    """The oracle cmc(single_gallery_shot=True) draws what the reference draws
    (cmc_sgs.npz, the reference run after np.random.seed(s)): identical
    per-query rows, averages and RNG state left behind."""
    g = golden('cmc_sgs')
    d, qid, gid, qcam, gcam = g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam']
    for seed, sep, fmb, topk in ((0, 0, 0, 100), (1, 1, 0, 100), (2, 0, 1, 20), (3, 1, 1, 10)):
        key = 'seed%d_sep%d_fmb%d_top%d' % (seed, sep, fmb, topk)
        kw = dict(topk=topk, separate_camera_set=bool(sep), single_gallery_shot=True,
                  first_match_break=bool(fmb))
        np.random.seed(seed)
        ret, valid = ev.cmc(d, qid, gid, qcam, gcam, average=False, **kw)
        np.testing.assert_array_equal(ret, g[key + '_all'], err_msg=key)
        np.testing.assert_array_equal(valid, g[key + '_valid'])
        assert np.random.randint(1 << 30) == g[key + '_next_draw']
        np.testing.assert_array_equal(
            ev.cmc(d, qid, gid, qcam, gcam, rng=np.random.RandomState(seed), **kw), g[key])


def test_sgs_draws_are_the_reference_choice_stream():
    """The product path draws one randint(0, tile(lens, repeat)) per query;
    NumPy's legacy RandomState gives exactly the values (and state) of the
    reference's per-identity np.random.choice calls, one-entry lists
    consuming nothing."""
    rs = np.random.RandomState(0)
    lens = rs.randint(1, 40, size=500)
    lens[::7] = 1
    a, b = np.random.RandomState(5), np.random.RandomState(5)
    seq = [a.choice(list(range(n))) for _ in range(3) for n in lens]
    np.testing.assert_array_equal(seq, b.randint(0, np.tile(lens.astype(np.int32), 3)))
    assert a.randint(1 << 30) == b.randint(1 << 30)


@pytest.mark.parametrize('k2', [6, 1])
def test_rerank_sparse_restatement_equals_oracle(golden, k2):
    """oracle.re_ranking_sparse (the long-row GPU test's checker) computes the
    same float32 values as oracle.re_ranking, which the golden pins."""
    g = golden('rerank')
    a = ev.re_ranking(g['q_g'], g['q_q'], g['g_g'], k1=20, k2=k2, lambda_value=0.3)
    b = ev.re_ranking_sparse(g['q_g'], g['q_q'], g['g_g'], k1=20, k2=k2, lambda_value=0.3)
    np.testing.assert_array_equal(a, b)
    rng = np.random.RandomState(5)
    Q, G, D = 60, 340, 32
    cent = rng.randn(40, D).astype(np.float32)
    ids = rng.randint(0, 40, Q + G)
    f = cent[ids] + 1.5 * rng.randn(Q + G, D).astype(np.float32)
    qg = ev.compute_dist(f[:Q], f[Q:])
    qq = ev.compute_dist(f[:Q], f[:Q])
    gg = ev.compute_dist(f[Q:], f[Q:])
    a = ev.re_ranking(qg, qq, gg, k1=20, k2=k2, lambda_value=0.3)
    b = ev.re_ranking_sparse(qg, qq, gg, k1=20, k2=k2, lambda_value=0.3)
    np.testing.assert_array_equal(a, b)
