"""End to end on the GPU: JPEG files + COCO json -> test_engine.run_inference
(decode, H2D, preprocess kernel, PPS forward, distance, count-based mAP/CMC)
vs the CPU oracle pipeline on the same decoded pixels."""
import os

import numpy as np
import pytest
import torch
from _parity import check_rank_metrics, tie_eps

pytestmark = pytest.mark.gpu


def _make_dataset(tmp, n_ids=8, per_id=4, seed=0):
    from PIL import Image
    from pps_amd import json_dataset as jd
    rng = np.random.RandomState(seed)
    names, marks = [], []
    base = rng.randint(0, 256, (n_ids, 128, 64, 3))
    k = 0
    for i in range(1, n_ids + 1):
        for j in range(per_id):
            cam = 1 + (j % 3)
            im = np.clip(base[i - 1] + rng.randint(-40, 40, (128, 64, 3)), 0, 255)
            h, w = (128, 64) if (k % 5) else (110, 50)     # a few ragged sizes
            im = np.ascontiguousarray(im[:h, :w].astype(np.uint8))
            fn = '%08d_%04d_%08d.jpg' % (i, cam, k)
            Image.fromarray(im).save(os.path.join(tmp, fn), quality=92)
            names.append(fn)
            marks.append(0 if j == 0 else 1)
            k += 1
    jd.write_coco_json(os.path.join(tmp, 'test.json'), names, marks)
    return names, np.array(marks)


def test_run_inference_end_to_end(tmp_path):
    from oracle import evaluator as ev
    from oracle import preprocess as pre
    from oracle.forward import GraphForward
    from pps_amd import config, model, test_engine, weights
    tmp = str(tmp_path)
    names, marks = _make_dataset(tmp)
    cfg = config.cfg
    config.merge_cfg_from_file(os.path.join(os.path.dirname(__file__), '..', 'configs',
                                            'market1501', 'pps_crm_triplet_R-50_1x.yaml'))
    cfg.TEST.DATASETS = (os.path.join(tmp, 'test.json'),)
    cfg.OUTPUT_DIR = tmp
    cfg.TEST.IMS_PER_BATCH = 16
    plan = model.build_plan()
    blobs = model.synthetic_weights(plan, seed=1)
    weights.save_npz(os.path.join(tmp, 'w.npz'), blobs)
    res = test_engine.run_inference(os.path.join(tmp, 'w.npz'))
    # features.pkl = {'all_feats', 'cfg'} (test_engine.py:356-368); written
    # by this test's own run, so unpickling it is safe
    import pickle
    with open(os.path.join(test_engine.get_output_dir(cfg.TEST.DATASETS[0]),
                           'features.pkl'), 'rb') as f:
        saved = pickle.load(f)
    assert set(saved) == {'all_feats', 'cfg'} and 'REID' in saved['cfg']
    feats = saved['all_feats']
    # oracle pipeline on identical decoded pixels
    ims = [test_engine._decode_bgr(os.path.join(tmp, n)) for n in names]
    x = pre.im_list_to_blob([pre.prep_im_for_blob(im) for im in ims])
    ref = GraphForward(blobs)(x).numpy()
    np.testing.assert_allclose(feats, ref, rtol=0, atol=1e-4)
    ids = np.array([int(n[:8]) for n in names])
    cams = np.array([int(n[9:13]) for n in names])
    q, g = marks == 0, marks == 1
    r = list(res.values())[0]['ReID']
    # the reported scores are the GPU ranking of the GPU features' distances
    from pps_amd import ops
    from pps_amd import reid_dataset_evaluator as gev
    ft = torch.from_numpy(feats).cuda()
    d_gpu = ops.compute_dist(ft[torch.from_numpy(np.nonzero(q)[0]).cuda()].contiguous(),
                             ft[torch.from_numpy(np.nonzero(g)[0]).cuda()].contiguous())
    ap, valid, first = gev.rank_eval(d_gpu, ids[q], ids[g], cams[q], cams[g])
    mAP_gpu, cmc_gpu = gev.scores_from_ranks(ap, valid, first)
    assert r['mAP'] == mAP_gpu and r['CMC1'] == cmc_gpu[0]
    # vs the all-CPU oracle pipeline (oracle features -> oracle distances ->
    # oracle mean_ap / cmc): exact outside near-ties, which are counted
    d_ref = ev.compute_dist(ref[q], ref[g])
    eps = tie_eps(d_gpu.cpu().numpy(), d_ref)
    out = check_rank_metrics(ap.cpu().numpy(), valid.cpu().numpy(), first.cpu().numpy(),
                             d_ref, ids[q], ids[g], cams[q], cams[g], eps)
    print('end to end vs oracle pipeline: %s' % out)
    mAP_ref, cmc_ref, _, _ = ev.evaluate_arrays(ref, ids, cams, marks)
    assert abs(out['mAP_ref'] - mAP_ref) <= 1e-12
    if out['ap_affected'] == 0:
        assert abs(r['mAP'] - mAP_ref) <= 1e-12
    if out['first_affected'] == 0:
        assert abs(r['CMC1'] - cmc_ref[0]) <= 1e-12
