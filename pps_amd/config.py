"""Config: the subset of Detectron's global `cfg` that the PPS test path reads.

Mirrors detectron/core/config.py (AttrDict cfg, merge_cfg_from_file :1228,
merge_cfg_from_list :1240-1262, assert_and_infer_cfg :1165).  Only the keys the
re-ID inference + retrieval path consumes are defined; any other
key found in a reference YAML (training schedule, solver, loss switches) is
accepted and kept under its path but has no effect here.
"""
import ast
import copy

import numpy as np
import yaml


class AttrDict(dict):
    """Nested config node: keys readable and writable as attributes, and a
    recursive freeze (the behaviour of the reference's AttrDict,
    detectron/utils/collections.py:24-60, that detectron/core/config.py
    relies on: cfg.A.B access, cfg.immutable(True) after
    assert_and_infer_cfg so later writes raise AttributeError)."""

    def __init__(self, *args, **kwargs):
        dict.__init__(self, *args, **kwargs)
        object.__setattr__(self, '_frozen', False)

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError:
            raise AttributeError(key)

    def __setattr__(self, key, value):
        if object.__getattribute__(self, '_frozen'):
            raise AttributeError('config is frozen: cannot set %s = %r' % (key, value))
        self[key] = value

    def immutable(self, frozen):
        """Freeze (True) or thaw (False) this node and every node below it."""
        object.__setattr__(self, '_frozen', bool(frozen))
        for child in self.values():
            if isinstance(child, AttrDict):
                child.immutable(frozen)

    def is_immutable(self):
        return object.__getattribute__(self, '_frozen')


def _defaults():
    C = AttrDict()
    C.NUM_GPUS = 1
    C.OUTPUT_DIR = '.'
    C.RNG_SEED = 3
    # reference config.py:957 (BGR order)
    C.PIXEL_MEANS = np.array([[[102.9801, 115.9465, 122.7717]]])
    C.MODEL = AttrDict(TYPE='generalized_reid',
                       CONV_BODY='ResNet.add_ResNet50_conv5_body',
                       NUM_CLASSES=-1, USE_BN=False, USE_GN=False,
                       EXECUTION_TYPE='dag')
    C.RESNETS = AttrDict(NUM_GROUPS=1, WIDTH_PER_GROUP=64, STRIDE_1X1=True,
                         TRANS_FUNC='bottleneck_transformation',
                         STEM_FUNC='basic_bn_stem',
                         SHORTCUT_FUNC='basic_bn_shortcut',
                         RES5_DILATION=1, RES5_STRIDE=2)
    C.FPN = AttrDict(FPN_ON=False, DIM=256, COARSEST_STRIDE=32)
    C.FAST_RCNN = AttrDict(ROI_BOX_HEAD='')
    C.TEST = AttrDict(WEIGHTS='', DATASETS=(), SCALE=600, MAX_SIZE=1000,
                      PRECOMPUTED_PROPOSALS=False, IMS_PER_BATCH=64)
    C.TRAIN = AttrDict(WEIGHTS='', DATASETS=())
    # reference config.py:1016-1088 (REID block) -- inference-relevant keys
    C.REID = AttrDict(SCALE=(128, 384), VIS=False, RERANK=True, BPM_DIM=256,
                      BPM_STRIP_NUM=6, NORMALIZE_FEATURE=False,
                      MAX_AVE_FEATURE=False, FPN_SHARED=False, FPN_NUM=4,
                      CRM=False, DISTANCE='euclidean', AP_MODE='sklearn')
    return C


cfg = _defaults()


def reset_cfg():
    global cfg
    fresh = _defaults()
    cfg.immutable(False)
    cfg.clear()
    cfg.update(fresh)
    return cfg


def _coerce(old, new, key):
    if isinstance(new, str) and not isinstance(old, str):
        try:
            new = ast.literal_eval(new)
        except (ValueError, SyntaxError):
            pass
    if isinstance(old, tuple) and isinstance(new, list):
        new = tuple(new)
    if isinstance(old, np.ndarray):
        new = np.array(new, dtype=old.dtype).reshape(old.shape)
    if isinstance(old, float) and isinstance(new, int):
        new = float(new)
    return new


def _merge(a, b, stack=''):
    for k, v in a.items():
        full = stack + k
        if isinstance(v, dict):
            if k not in b or not isinstance(b[k], AttrDict):
                b[k] = AttrDict()
            _merge(v, b[k], full + '.')
        else:
            b[k] = _coerce(b.get(k), v, full) if k in b else v


def merge_cfg_from_file(filename):
    """reference config.py:1228 -- load a YAML and merge into `cfg`."""
    with open(filename, 'r') as f:
        y = yaml.safe_load(f)
    _merge(y or {}, cfg)


def merge_cfg_from_list(opts):
    """reference config.py:1240-1262 -- ['A.B', value, ...] overrides."""
    assert len(opts) % 2 == 0, 'Specify config overrides as KEY VALUE pairs'
    for full, v in zip(opts[0::2], opts[1::2]):
        d = cfg
        parts = full.split('.')
        for p in parts[:-1]:
            if p not in d:
                d[p] = AttrDict()
            d = d[p]
        d[parts[-1]] = _coerce(d.get(parts[-1]), v, full) if parts[-1] in d else v


def assert_and_infer_cfg(make_immutable=True):
    if make_immutable:
        cfg.immutable(True)
    return cfg


def snapshot():
    return copy.deepcopy(dict(cfg))
