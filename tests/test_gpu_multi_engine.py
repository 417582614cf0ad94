"""The multi-GPU test API on the HIP kernels: tools/test_net.py
--multi-gpu-testing's path (test_engine.multi_gpu_test_net_on_dataset ->
distributed.evaluate_sharded) run by 2 ranks that share this box's one GPU
over gloo (the product uses RCCL, one rank per GPU), on a JPEG dataset with
query, gallery and multi-query images and REID.RERANK on.  Must reproduce
the one-process run_inference: features in dataset order within f32
rounding of the per-shard batches, and the same single-query, multi-query
and re-ranked scores (test_engine.py:184-229, reid_dataset_evaluator.py:29-209)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_dataset(tmp, n_ids=8, per_id=6, seed=3):
    """Identities share most of their appearance (a common image + a small
    per-identity part + heavy noise), so the ranking is far from perfect."""
    from PIL import Image
    from pps_amd import json_dataset as jd
    rng = np.random.RandomState(seed)
    names, marks = [], []
    common = rng.randint(0, 256, (128, 64, 3)).astype(np.float64)
    base = 0.8 * common + 0.2 * rng.randint(0, 256, (n_ids, 128, 64, 3))
    k = 0
    for i in range(1, n_ids + 1):
        for j in range(per_id):
            cam = 1 + (j % 3)
            im = np.clip(base[i - 1] + rng.randint(-90, 90, (128, 64, 3)), 0, 255)
            im = np.ascontiguousarray(im.astype(np.uint8))
            fn = '%08d_%04d_%08d.jpg' % (i, cam, k)
            Image.fromarray(im).save(os.path.join(tmp, fn), quality=92)
            names.append(fn)
            marks.append(0 if j == 0 else (2 if j == 1 else 1))
            k += 1
    jd.write_coco_json(os.path.join(tmp, 'test.json'), names, marks)
    return names


def _setup_cfg(tmp, out_dir):
    from pps_amd import config
    cfg = config.cfg
    config.merge_cfg_from_file(os.path.join(ROOT, 'configs', 'market1501',
                                            'pps_crm_triplet_R-50_1x.yaml'))
    cfg.TEST.DATASETS = (os.path.join(tmp, 'test.json'),)
    cfg.OUTPUT_DIR = out_dir
    cfg.TEST.IMS_PER_BATCH = 8
    cfg.REID.RERANK = True
    return cfg


def _worker(rank, world, port, tmp, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK='0')
    torch.cuda.set_device(0)
    torch.distributed.init_process_group('gloo', rank=rank, world_size=world)
    from pps_amd import test_engine
    cfg = _setup_cfg(tmp, os.path.join(tmp, 'multi'))
    name = cfg.TEST.DATASETS[0]
    res = test_engine.multi_gpu_test_net_on_dataset(os.path.join(tmp, 'w.npz'), name,
                                                    test_engine.get_output_dir(name))
    out[rank] = dict(list(res.values())[0]['ReID'])
    torch.distributed.destroy_process_group()


def test_multi_gpu_test_net_matches_single_process(tmp_path):
    from pps_amd import config, model, test_engine, weights
    tmp = str(tmp_path)
    _make_dataset(tmp)
    cfg = _setup_cfg(tmp, os.path.join(tmp, 'single'))
    blobs = model.synthetic_weights(model.build_plan(), seed=2)
    weights.save_npz(os.path.join(tmp, 'w.npz'), blobs)
    single = list(test_engine.run_inference(os.path.join(tmp, 'w.npz')).values())[0]['ReID']
    import pickle
    with open(os.path.join(test_engine.get_output_dir(cfg.TEST.DATASETS[0]),
                           'features.pkl'), 'rb') as f:   # written by this run
        feats1 = pickle.load(f)['all_feats']
    config.reset_cfg()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), tmp, out), nprocs=2, join=True)
    feats2 = np.load(os.path.join(tmp, 'multi', 'test', 'test', 'features.npy'))
    np.testing.assert_allclose(feats2, feats1, rtol=0, atol=2e-6)
    print('single-process scores: %s' % dict(single))
    assert single['mAP'] < 0.999 or single['mq_mAP'] < 0.999   # a non-trivial ranking
    for r in range(2):
        m = out[r]
        assert m['mq_mAP'] != -1 and single['mq_mAP'] != -1
        for key in ('mAP', 'CMC1', 'CMC5', 'CMC10', 'mq_mAP', 'mq_CMC1', 'mq_CMC5',
                    'mq_CMC10'):
            assert abs(m[key] - single[key]) < 1e-6, (key, m[key], single[key])
