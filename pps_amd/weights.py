"""Weights files in the reference's Detectron format.

detectron/utils/net.py:53-135 `initialize_gpu_from_weights_file` and
:138-178 `save_model_to_weights_file`; detectron/utils/io.py:72-83: a pickle of
{'blobs': {unscoped_name: ndarray}, 'cfg': yaml-string}, py2 pickles read with
encoding='latin1'.  BN parameters follow tools/pickle_caffe_blobs_keep_bn.py
:141-159 (`_s`, `_b`, `_rm`, `_riv` with `_riv` = running variance).

Loading a pickle executes code from the file, so `load_weights` only unpickles
when the caller passes trusted=True (the user's own training snapshots, as
scripts/test_reid.sh:54 does with model_epoch*.pkl).  The safe container is
.npz (`save_npz` / `load_weights`), which never unpickles.
"""
import os

import numpy as np


def _unscope(name):
    # 'gpu_0/res2_0_branch2a_w' -> 'res2_0_branch2a_w' (net.py:91-94 scoping)
    return name.split('/')[-1]


def _clean(blobs):
    out = {}
    for k, v in blobs.items():
        k = _unscope(k)
        if k.endswith('_momentum'):
            continue  # optimizer state (net.py:153-156 saves it; unused at test)
        out[k] = np.asarray(v, dtype=np.float32)
    return out


def load_weights(path, trusted=False):
    """Return {blob name: float32 ndarray}."""
    ext = os.path.splitext(path)[1].lower()
    if ext == '.npz':
        with np.load(path, allow_pickle=False) as z:
            return _clean({k: z[k] for k in z.files})
    if ext in ('.pkl', '.pickle'):
        if not trusted:
            raise RuntimeError(
                'Refusing to unpickle %s: pickles execute code on load. Pass '
                'trusted=True (CLI: --trusted-weights) for your own snapshots, or '
                'convert with `tools/convert_weights.py` to .npz.' % path)
        import pickle
        with open(path, 'rb') as f:
            data = pickle.load(f, encoding='latin1')
        blobs = data['blobs'] if isinstance(data, dict) and 'blobs' in data else data
        return _clean(blobs)
    raise RuntimeError('Unknown weights format: %s' % path)


def save_npz(path, blobs):
    np.savez(path, **{k: np.asarray(v, np.float32) for k, v in blobs.items()})


def check_complete(blobs, plan):
    """Every parameter the plan needs must be present with the right shape."""
    missing, bad = [], []
    for name, shape in plan.params.items():
        if name not in blobs:
            if not name.endswith('_conv_b'):
                missing.append(name)
            continue
        if tuple(blobs[name].shape) != tuple(shape):
            bad.append((name, blobs[name].shape, shape))
    if missing or bad:
        raise RuntimeError('weights do not match the PPS plan: %d missing (e.g. %s), '
                           '%d with wrong shape (e.g. %s)' % (len(missing), missing[:3],
                                                              len(bad), bad[:3]))
