"""Write tests/golden/weights_py2.pkl: a tiny Detectron weights file laid out
exactly as the reference's Python 2 tools write them
(detectron/utils/net.py:138-178 save_model_to_weights_file ->
utils/io.py:39-60 save_object, pickle protocol 2;
tools/pickle_caffe_blobs_keep_bn.py:141-159 BN names), so the loader's
py2/latin1 path (utils/io.py:72-83 load_object) is exercised without Python 2:

  {'blobs': {'gpu_0/conv1_w': f32 [4,3,7,7], 'conv1_w_momentum': ...,
             'res_conv1_bn_s' / '_b' / '_rm' / '_riv': f32 [4],
             'pps01_conv_w': f32 [2,6,1,1], 'pps01_conv_b': f64 [2]},
   'cfg': <yaml string>}

Python 2 pickles keys and raw array bytes as byte strings (BINSTRING /
SHORT_BINSTRING opcodes) and arrays through numpy.core.multiarray._reconstruct
+ BUILD; those opcodes are emitted here by hand.  The arrays are
deterministic (see `expected()`), so the test rebuilds them instead of
storing a second copy.
"""
import os
import struct

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'weights_py2.pkl')


def expected():
    rng = np.random.RandomState(7)
    return {
        'gpu_0/conv1_w': rng.randn(4, 3, 7, 7).astype(np.float32),
        'gpu_0/conv1_w_momentum': rng.randn(4, 3, 7, 7).astype(np.float32),
        'res_conv1_bn_s': rng.uniform(0.5, 1.5, 4).astype(np.float32),
        'res_conv1_bn_b': rng.randn(4).astype(np.float32),
        'res_conv1_bn_rm': rng.randn(4).astype(np.float32),
        'res_conv1_bn_riv': rng.uniform(0.5, 1.5, 4).astype(np.float32),
        'pps01_conv_w': rng.randn(2, 6, 1, 1).astype(np.float32),
        'pps01_conv_b': rng.randn(2).astype(np.float64),   # a float64 blob
    }


CFG_YAML = 'MODEL:\n  NUM_CLASSES: 752\nREID:\n  BPM_STRIP_NUM: 5\n'


class P2(object):
    """Minimal protocol-2 opcode writer with Python 2 string semantics."""

    def __init__(self):
        self.b = bytearray(b'\x80\x02')        # PROTO 2

    def str_(self, s):                         # py2 str -> (SHORT_)BINSTRING
        raw = s if isinstance(s, bytes) else s.encode('latin1')
        if len(raw) < 256:
            self.b += b'U' + bytes([len(raw)]) + raw
        else:
            self.b += b'T' + struct.pack('<i', len(raw)) + raw

    def int_(self, v):
        self.b += b'J' + struct.pack('<i', v)  # BININT

    def glob(self, mod, name):
        self.b += b'c' + mod.encode() + b'\n' + name.encode() + b'\n'

    def tuple_(self, items):
        self.b += b'('                         # MARK
        for it in items:
            it()
        self.b += b't'                         # TUPLE

    def dtype(self, dt):
        self.glob('numpy', 'dtype')
        self.tuple_([lambda: self.str_(dt.str[1:]), lambda: self.int_(0),
                     lambda: self.int_(1)])
        self.b += b'R'                         # REDUCE
        # state (3, '<', None, None, None, -1, -1, 0)
        self.tuple_([lambda: self.int_(3), lambda: self.str_('<'), lambda: self.none(),
                     lambda: self.none(), lambda: self.none(), lambda: self.int_(-1),
                     lambda: self.int_(-1), lambda: self.int_(0)])
        self.b += b'b'                         # BUILD

    def none(self):
        self.b += b'N'

    def array(self, a):
        a = np.ascontiguousarray(a)
        self.glob('numpy.core.multiarray', '_reconstruct')
        self.tuple_([lambda: self.glob('numpy', 'ndarray'),
                     lambda: self.tuple_([lambda: self.int_(0)]),
                     lambda: self.str_('b')])
        self.b += b'R'
        self.tuple_([lambda: self.int_(1),
                     lambda: self.tuple_([(lambda d=d: self.int_(d)) for d in a.shape]),
                     lambda: self.dtype(a.dtype),
                     lambda: self.b.extend(b'\x89'),   # NEWFALSE (not Fortran order)
                     lambda: self.str_(a.tobytes())])
        self.b += b'b'

    def dict_(self, items):
        self.b += b'}('                        # EMPTY_DICT, MARK
        for k, v in items:
            self.str_(k)
            v()
        self.b += b'u'                         # SETITEMS

    def stop(self):
        self.b += b'.'
        return bytes(self.b)


def build():
    p = P2()
    blobs = expected()
    p.dict_([('blobs', lambda: p.dict_([(k, (lambda v=v: p.array(v)))
                                         for k, v in blobs.items()])),
             ('cfg', lambda: p.str_(CFG_YAML))])
    return p.stop()


if __name__ == '__main__':
    with open(OUT, 'wb') as f:
        f.write(build())
    print('wrote', OUT)
