"""Dataset json ingestion and weights files (CPU)."""
import os

import numpy as np
import pytest


def test_json_roundtrip_sorted_and_marks(tmp_path):
    from pps_amd import json_dataset as jd
    names = ['%08d_%04d_%08d.jpg' % (i, c, k) for k, (i, c) in
             enumerate([(3, 1), (1, 2), (2, 2), (1, 5)])]
    marks = [1, 0, 1, 2]
    p = tmp_path / 'test.json'
    jd.write_coco_json(str(p), names, marks)
    ds = jd.JsonDataset('x', image_directory=str(tmp_path), annotation_file=str(p))
    roidb = ds.get_roidb(gt=True)
    assert [os.path.basename(e['image']) for e in roidb] == names
    assert [e['mark'] for e in roidb] == marks
    from pps_amd.reid_dataset_evaluator import get_info
    pid, cam, name, mark, path = get_info(roidb[3])
    assert (pid, cam, mark) == (1, 5, 2)


def test_catalog_names_cover_reference_sets():
    from pps_amd import json_dataset as jd
    for n in ('market1501_test', 'duke_test', 'cuhk03_test', 'cuhk03_detected_test'):
        im, ann = jd.dataset_paths(n)
        assert ann.endswith('.json')
    with pytest.raises(KeyError):
        jd.dataset_paths('nope')


def test_weights_npz_roundtrip_and_pickle_refusal(tmp_path):
    from pps_amd import weights
    blobs = {'gpu_0/conv1_w': np.ones((64, 3, 7, 7)), 'conv1_w_momentum': np.zeros(3),
             'res_conv1_bn_riv': np.ones(64)}
    p = tmp_path / 'w.npz'
    weights.save_npz(str(p), blobs)
    got = weights.load_weights(str(p))
    assert set(got) == {'conv1_w', 'res_conv1_bn_riv'}
    assert got['conv1_w'].dtype == np.float32
    pk = tmp_path / 'w.pkl'
    pk.write_bytes(b'not really a pickle')
    with pytest.raises(RuntimeError, match='Refusing to unpickle'):
        weights.load_weights(str(pk))


def test_check_complete_reports_missing():
    from pps_amd import config, model, weights
    config.cfg.REID.BPM_STRIP_NUM = 5
    config.cfg.REID.BPM_DIM = 128
    plan = model.build_plan()
    blobs = model.synthetic_weights(plan, 0)
    weights.check_complete(blobs, plan)
    blobs.pop('res4_2_branch2b_w')
    with pytest.raises(RuntimeError, match='1 missing'):
        weights.check_complete(blobs, plan)
