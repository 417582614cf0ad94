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


def test_detectron_py2_pickle_weights():
    """A Detectron weights file as the reference's Python 2 tools write it
    (protocol 2, byte-string keys and array bytes, 'gpu_0/' scopes,
    '_momentum' optimizer blobs, BN `_s/_b/_rm/_riv`; fixture from
    tests/golden/make_weights_pickle.py, written by this repo): loaded with
    latin1 decoding (utils/io.py:72-83), unscoped (net.py:73-76), momentum
    dropped, every blob float32 (net.py:116-118 astype(np.float32))."""
    import sys
    from pps_amd import weights
    here = os.path.join(os.path.dirname(__file__), 'golden')
    sys.path.insert(0, here)
    import make_weights_pickle as mk
    path = os.path.join(here, 'weights_py2.pkl')
    with open(path, 'rb') as f:
        assert f.read() == mk.build()     # the committed file is the script's output
    with pytest.raises(RuntimeError, match='Refusing to unpickle'):
        weights.load_weights(path)
    got = weights.load_weights(path, trusted=True)
    exp = mk.expected()
    assert set(got) == {'conv1_w', 'res_conv1_bn_s', 'res_conv1_bn_b', 'res_conv1_bn_rm',
                        'res_conv1_bn_riv', 'pps01_conv_w', 'pps01_conv_b'}
    for k, v in exp.items():
        if k.endswith('_momentum'):
            continue
        name = k.split('/')[-1]
        assert got[name].dtype == np.float32
        np.testing.assert_array_equal(got[name], v.astype(np.float32))


def test_test_reid_sh_reference_convention(tmp_path):
    """scripts/test_reid.sh ARGS... <snapshot_dir> (reference
    scripts/test_reid.sh:7-55): OUTPUT_DIR names the experiment, the log goes
    to ${EXP_DIR}/../_logs, snapshots model_epoch{1,11,...,171}, NUM_GPUS > 1
    launches one process per GPU, a .pkl needs PPS_TRUSTED_WEIGHTS=1."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    snap = tmp_path / 'snap'
    snap.mkdir()
    (snap / 'model_epoch1.npz').write_bytes(b'')
    (snap / 'model_epoch11.pkl').write_bytes(b'')
    exp = tmp_path / 'exp' / 'run1'
    env = dict(os.environ, PPS_DRY_RUN='1')
    args = ['bash', os.path.join(root, 'scripts', 'test_reid.sh'), '--cfg', 'c.yaml',
            'OUTPUT_DIR', str(exp), 'NUM_GPUS', '2', str(snap)]
    r = subprocess.run(args, env=env, capture_output=True, text=True)
    assert r.returncode == 1 and 'PPS_TRUSTED_WEIGHTS' in r.stderr + r.stdout
    env['PPS_TRUSTED_WEIGHTS'] = '1'
    r = subprocess.run(args, env=env, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if 'test_net.py' in l]
    assert len(lines) == 18                       # ITER = 1, 11, ..., 171
    assert '--nproc-per-node 2' in lines[0] and 'model_epoch1.npz' in lines[0]
    assert '--trusted-weights' in lines[1] and 'model_epoch11.pkl' in lines[1]
    assert 'OUTPUT_DIR %s' % exp in lines[2] and 'model_epoch21.pkl' in lines[2]
    assert '--trusted-weights' not in lines[2]
    logs = os.listdir(str(tmp_path / 'exp' / '_logs'))
    assert logs and all(l.startswith('run1 test_reid.sh') for l in logs)
