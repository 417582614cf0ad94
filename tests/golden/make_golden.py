"""Generate golden vectors for the retrieval path from the REFERENCE evaluator.

Run in the build container only (it needs /root/reference, which does not exist
on the GPU box):

    python tests/golden/make_golden.py

It loads `/root/reference/detectron/datasets/reid_dataset_evaluator.py`
unchanged via importlib, with small stubs for modules it imports but that are
not on the hot path (cv2, pycocotools, detectron.core.config.cfg,
detectron.utils.{io,boxes}). It then calls the reference's own
`compute_dist` (:244-272), `mean_ap` (:366-439), `cmc` (:283-363),
`re_ranking` (:442-519) and `evaluate` (:29-209) on seeded synthetic inputs
and writes the inputs + outputs as small .npz fixtures next to this script.

Versions used to make the committed fixtures: Python 3.10, NumPy 2.2.6,
scikit-learn 1.7.2 (step-wise AP), SciPy 1.15.3.

Only data is written; no reference source is copied.
"""
import contextlib
import importlib.util
import io
import json
import os
import sys
import types

import numpy as np

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _Attr(dict):
    def __getattr__(self, k):
        return self[k]


def load_reference_evaluator(rerank=False):
    """Import the reference evaluator file with stubs for off-path deps."""
    _stub('cv2')
    _stub('pycocotools')
    _stub('pycocotools.cocoeval', COCOeval=object)
    _stub('detectron')
    _stub('detectron.core')
    cfg = _Attr(REID=_Attr(RERANK=rerank, VIS=False))
    _stub('detectron.core.config', cfg=cfg, get_output_dir=lambda *a, **k: '/tmp')
    _stub('detectron.utils')
    _stub('detectron.utils.io', save_object=lambda *a, **k: None)
    _stub('detectron.utils.boxes')
    path = os.path.join(REF, 'detectron/datasets/reid_dataset_evaluator.py')
    spec = importlib.util.spec_from_file_location('ref_reid_eval', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod, cfg


def synth_features(n_ids, per_id, D, noise, seed, n_distract=0):
    """SURVEY §8(d) feature recipe: centroid[id] + noise*N(0,1), L2-normalised."""
    rng = np.random.RandomState(seed)
    cent = rng.randn(n_ids + 1, D).astype(np.float32)
    ids = np.repeat(np.arange(1, n_ids + 1), per_id)
    ids = np.concatenate([ids, np.zeros(n_distract, dtype=ids.dtype)])
    x = cent[ids] + noise * rng.randn(len(ids), D).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    cams = rng.randint(1, 7, size=len(ids))
    return x.astype(np.float32), ids.astype(np.int64), cams.astype(np.int64)


def split_qg(x, ids, cams, q_frac, seed):
    rng = np.random.RandomState(seed + 1)
    is_q = rng.rand(len(ids)) < q_frac
    is_q[ids == 0] = False  # distractors are gallery-only, as in Market
    return (x[is_q], ids[is_q], cams[is_q]), (x[~is_q], ids[~is_q], cams[~is_q])


def quiet(fn, *a, **k):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = fn(*a, **k)
    return out, buf.getvalue()


def case_retrieval(ev, name, n_ids, per_id, D, noise, seed, n_distract, q_frac):
    x, ids, cams = synth_features(n_ids, per_id, D, noise, seed, n_distract)
    (qf, qid, qcam), (gf, gid, gcam) = split_qg(x, ids, cams, q_frac, seed)
    dist, _ = quiet(ev.compute_dist, qf, gf, type='euclidean')
    aps, valid_ap = ev.mean_ap(dist, qid, gid, qcam, gcam, average=False)
    mAP, _ = quiet(ev.mean_ap, dist, qid, gid, qcam, gcam)
    cmc_all, valid_cmc = ev.cmc(dist, qid, gid, qcam, gcam,
                                separate_camera_set=False,
                                single_gallery_shot=False,
                                first_match_break=True, topk=10, average=False)
    cmc_avg = ev.cmc(dist, qid, gid, qcam, gcam, separate_camera_set=False,
                     single_gallery_shot=False, first_match_break=True,
                     topk=10)
    order = np.argsort(dist, axis=1, kind='stable').astype(np.int32)
    np.savez_compressed(
        os.path.join(HERE, name + '.npz'),
        qf=qf, gf=gf, qid=qid, gid=gid, qcam=qcam, gcam=gcam,
        dist=dist.astype(np.float32), order_stable=order,
        aps=aps, valid_ap=valid_ap, mAP=np.float64(mAP),
        cmc_all=cmc_all, valid_cmc=valid_cmc, cmc=cmc_avg)
    return dict(name=name, Q=len(qid), G=len(gid), D=D, mAP=float(mAP),
                cmc1=float(cmc_avg[0]))


def case_ties(ev):
    """Exact duplicate gallery rows -> tied distances (AP is tie-invariant)."""
    x, ids, cams = synth_features(20, 6, 64, 1.0, 7, 10)
    (qf, qid, qcam), (gf, gid, gcam) = split_qg(x, ids, cams, 0.2, 7)
    gf = np.concatenate([gf, gf[:40]])
    gid = np.concatenate([gid, gid[:40]])
    gcam = np.concatenate([gcam, (gcam[:40] % 6) + 1])
    dist, _ = quiet(ev.compute_dist, qf, gf, type='euclidean')
    aps, valid_ap = ev.mean_ap(dist, qid, gid, qcam, gcam, average=False)
    mAP, _ = quiet(ev.mean_ap, dist, qid, gid, qcam, gcam)
    np.savez_compressed(os.path.join(HERE, 'ties.npz'), qf=qf, gf=gf, qid=qid,
                        gid=gid, qcam=qcam, gcam=gcam, dist=dist, aps=aps,
                        valid_ap=valid_ap, mAP=np.float64(mAP))
    return dict(name='ties', Q=len(qid), G=len(gid), mAP=float(mAP))


def case_rerank(ev):
    x, ids, cams = synth_features(25, 6, 64, 1.5, 11, 20)
    (qf, qid, qcam), (gf, gid, gcam) = split_qg(x, ids, cams, 0.2, 11)
    q_g, _ = quiet(ev.compute_dist, qf, gf, type='euclidean')
    q_q, _ = quiet(ev.compute_dist, qf, qf, type='euclidean')
    g_g, _ = quiet(ev.compute_dist, gf, gf, type='euclidean')
    rr = ev.re_ranking(q_g, q_q, g_g, k1=20, k2=6, lambda_value=0.3)
    mAP, _ = quiet(ev.mean_ap, rr, qid, gid, qcam, gcam)
    cmc_avg = ev.cmc(rr, qid, gid, qcam, gcam, first_match_break=True, topk=10)
    np.savez_compressed(os.path.join(HERE, 'rerank.npz'), qf=qf, gf=gf,
                        qid=qid, gid=gid, qcam=qcam, gcam=gcam, q_g=q_g,
                        q_q=q_q, g_g=g_g, rerank=rr.astype(np.float32),
                        mAP=np.float64(mAP), cmc=cmc_avg)
    return dict(name='rerank', Q=len(qid), G=len(gid), mAP=float(mAP))


def case_cmc_modes(ev):
    """The reference `cmc` beyond the Market protocol: its own defaults
    (topk=100, first_match_break=False: fractional CMC, delta = 1/#matches,
    :283-292,349-356) and separate_camera_set=True (:329-331), with and
    without first_match_break, averaged and per query."""
    out = {}
    for tag, args in (('market_small', dict(n_ids=60, per_id=8, D=128, noise=1.6, seed=0,
                                            n_distract=80, q_frac=0.2)),
                      ('dense', dict(n_ids=15, per_id=12, D=32, noise=2.5, seed=4,
                                     n_distract=30, q_frac=0.2))):
        x, ids, cams = synth_features(args['n_ids'], args['per_id'], args['D'], args['noise'],
                                      args['seed'], args['n_distract'])
        (qf, qid, qcam), (gf, gid, gcam) = split_qg(x, ids, cams, args['q_frac'], args['seed'])
        dist, _ = quiet(ev.compute_dist, qf, gf, type='euclidean')
        out[tag + '_qid'], out[tag + '_gid'] = qid, gid
        out[tag + '_qcam'], out[tag + '_gcam'] = qcam, gcam
        out[tag + '_dist'] = dist.astype(np.float32)
        for sep in (False, True):
            for fmb in (False, True):
                key = '%s_sep%d_fmb%d' % (tag, sep, fmb)
                out[key] = ev.cmc(dist, qid, gid, qcam, gcam, separate_camera_set=sep,
                                  first_match_break=fmb)
                out[key + '_all'], out[key + '_valid'] = ev.cmc(
                    dist, qid, gid, qcam, gcam, separate_camera_set=sep,
                    first_match_break=fmb, average=False)
        out[tag + '_default'] = ev.cmc(dist, qid, gid, qcam, gcam)   # the signature defaults
        out[tag + '_sep1_fmb0_top5'] = ev.cmc(dist, qid, gid, qcam, gcam, topk=5,
                                              separate_camera_set=True)
    np.savez_compressed(os.path.join(HERE, 'cmc_modes.npz'), **out)
    return dict(name='cmc_modes', keys=len(out))


def case_sgs(ev):
    """The reference `cmc(single_gallery_shot=True)` (:334-346): 100 repeats
    per valid query, one gallery entry drawn per identity with the global
    np.random (`_unique_sample`, :275-280), seeded here before each call.
    The distances are given as float32 values with no tie inside a row, so
    the reference's quicksort argsort is the stable order."""
    out = {}
    for fseed in range(31, 64):   # the first feature seed without a tie in any row
        x, ids, cams = synth_features(40, 6, 64, 1.8, fseed, 40)
        (qf, qid, qcam), (gf, gid, gcam) = split_qg(x, ids, cams, 0.15, fseed)
        dist, _ = quiet(ev.compute_dist, qf, gf, type='euclidean')
        dist = dist.astype(np.float32)
        s = np.sort(dist, axis=1)
        if not np.any(s[:, 1:] == s[:, :-1]):
            break
    else:
        raise AssertionError('tied distances in every candidate')
    out.update(qid=qid, gid=gid, qcam=qcam, gcam=gcam, dist=dist)
    for seed, sep, fmb, topk in ((0, False, False, 100), (1, True, False, 100),
                                 (2, False, True, 20), (3, True, True, 10)):
        key = 'seed%d_sep%d_fmb%d_top%d' % (seed, sep, fmb, topk)
        np.random.seed(seed)
        out[key + '_all'], out[key + '_valid'] = ev.cmc(
            dist.astype(np.float64), qid, gid, qcam, gcam, topk=topk, separate_camera_set=sep,
            single_gallery_shot=True, first_match_break=fmb, average=False)
        np.random.seed(seed)
        out[key] = ev.cmc(dist.astype(np.float64), qid, gid, qcam, gcam, topk=topk,
                          separate_camera_set=sep, single_gallery_shot=True,
                          first_match_break=fmb)
        out[key + '_next_draw'] = np.random.randint(1 << 30)   # the RNG state left behind
    np.savez_compressed(os.path.join(HERE, 'cmc_sgs.npz'), **out)
    return dict(name='cmc_sgs', Q=len(qid), G=len(gid), keys=len(out))


class _FakeJsonDataset(object):
    def __init__(self, entries):
        self.entries = entries
        self.name = 'synthetic'

    def get_roidb(self, gt=True):
        return self.entries


def case_evaluate(ev):
    """Drive the reference `evaluate()` (single-query path) end to end and
    keep its printed log lines (the `Single Query: [mAP: ..]` format that
    tools/loss_vs_map.py:80 parses)."""
    x, ids, cams = synth_features(30, 5, 96, 1.2, 23, 15)
    rng = np.random.RandomState(5)
    marks = (rng.rand(len(ids)) < 0.25).astype(np.int64) ^ 1  # 0=q,1=g
    marks[ids == 0] = 1
    names = ['%08d_%04d_%05d.jpg' % (i, c, k)
             for k, (i, c) in enumerate(zip(ids, cams))]
    entries = [dict(image='/data/' + n, mark=int(m))
               for n, m in zip(names, marks)]
    (mAP, cmc_s, mq_mAP, mq_cmc), log = quiet(
        ev.evaluate, _FakeJsonDataset(entries), x, '/tmp')
    lines = [l for l in log.splitlines()
             if l.startswith('Single Query:') or 'Array size' in l]
    np.savez_compressed(os.path.join(HERE, 'evaluate.npz'), feat=x, ids=ids,
                        cams=cams, marks=marks, names=np.array(names),
                        mAP=np.float64(mAP), cmc=cmc_s)
    with open(os.path.join(HERE, 'evaluate_log.txt'), 'w') as f:
        f.write('\n'.join(lines) + '\n')
    return dict(name='evaluate', N=len(ids), mAP=float(mAP))


def main():
    ev, _ = load_reference_evaluator(rerank=False)
    if '--only' in sys.argv:   # one case, the other fixtures untouched
        name = sys.argv[sys.argv.index('--only') + 1]
        print(globals()['case_' + name](ev))
        return
    meta = []
    meta.append(case_retrieval(ev, 'market_small', n_ids=60, per_id=8, D=128,
                               noise=1.6, seed=0, n_distract=80, q_frac=0.2))
    meta.append(case_retrieval(ev, 'full_dim', n_ids=12, per_id=5, D=3968,
                               noise=4.0, seed=3, n_distract=8, q_frac=0.25))
    meta.append(case_ties(ev))
    meta.append(case_rerank(ev))
    meta.append(case_evaluate(ev))
    meta.append(case_cmc_modes(ev))
    meta.append(case_sgs(ev))
    import sklearn
    meta = dict(cases=meta, numpy=np.__version__, sklearn=sklearn.__version__,
                python=sys.version.split()[0],
                source='reference reid_dataset_evaluator.py imported unchanged')
    with open(os.path.join(HERE, 'golden_meta.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == '__main__':
    main()
