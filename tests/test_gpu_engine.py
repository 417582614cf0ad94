"""End to end on the GPU: JPEG files + COCO json -> test_engine.run_inference
(decode, H2D, preprocess kernel, PPS forward, distance, count-based mAP/CMC)
vs the CPU oracle pipeline on the same decoded pixels."""
import os

import numpy as np
import pytest
import torch

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
    feats = np.load(os.path.join(test_engine.get_output_dir(cfg.TEST.DATASETS[0]),
                                 'features.npy'))
    # oracle pipeline on identical decoded pixels
    ims = [test_engine._decode_bgr(os.path.join(tmp, n)) for n in names]
    x = pre.im_list_to_blob([pre.prep_im_for_blob(im) for im in ims])
    ref = GraphForward(blobs)(x).numpy()
    np.testing.assert_allclose(feats, ref, rtol=0, atol=1e-4)
    ids = np.array([int(n[:8]) for n in names])
    cams = np.array([int(n[9:13]) for n in names])
    # ranking parity on the same features (the oracle ranks with NumPy fp32
    # distances; a rank can only flip where two distances are within ~1e-6)
    mAP, cmc, _, _ = ev.evaluate_arrays(feats, ids, cams, marks)
    r = list(res.values())[0]['ReID']
    q, g = marks == 0, marks == 1
    d = ev.compute_dist(feats[q], feats[g])
    gaps = np.diff(np.sort(d, axis=1), axis=1)
    tol = 1e-9 if gaps.min() > 1e-5 else 0.05
    assert abs(r['mAP'] - mAP) < tol
    assert abs(r['CMC1'] - cmc[0]) < max(tol, 1e-9)
    # and the end-to-end features agree with the oracle pipeline's
    mAP_ref, _, _, _ = ev.evaluate_arrays(ref, ids, cams, marks)
    assert abs(mAP_ref - mAP) < 0.02
