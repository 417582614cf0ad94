"""The whole-network C entry point (include/pps_abi.h "whole network":
pps_model_create / pps_forward / pps_model_destroy) from Python.

`NativeModel` is the product form of the feature extractor: one handle that
owns the weights, the activation buffers and the tuning table, and one C call
per forward -- what a non-Python caller (a Caffe2 `PPSForward` operator
replacing `workspace.RunNet` at detectron/core/test.py:163-165, see
INTEGRATION.md) links against.  `pps_amd.model.PPSModel` runs the same
launches orchestrated from Python op by op (autotune, per-layer inspection);
`apply_table(PPSModel)` copies its tile / plane / split-K choices, after
which both compute identical bits (tests/test_gpu_native.py).
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import call
from .config import cfg as _cfg

MATH = {'x3': 0, 'f32': 1}
AUTOTUNE_NO_PLANES, AUTOTUNE_SPLITK, AUTOTUNE_NO_SEAM, AUTOTUNE_NO_H2 = 1, 2, 4, 8
AUTOTUNE_NO_H2E, AUTOTUNE_NO_GROUPS = 16, 32
FWD_KEEP_AMAX = 1   # pps_abi.h PPS_FWD_KEEP_AMAX


class PpsBlob(ctypes.Structure):
    _fields_ = [('name', ctypes.c_char_p), ('data', ctypes.c_void_p), ('ndim', ctypes.c_int),
                ('shape', ctypes.c_int64 * 4)]


class PpsModelConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        'struct_size', 'height', 'width', 'strip_num', 'bpm_dim', 'num_groups',
        'width_per_group', 'stride_1x1', 'res5_stride', 'res5_dilation', 'fpn_on', 'fpn_dim',
        'max_ave', 'normalize', 'math', 'fused_stem', 'fused_pps', 'act_planes')] + \
        [('pixel_means', ctypes.c_float * 3)]


class PpsLayerInfo(ctypes.Structure):
    _fields_ = [('name', ctypes.c_char_p), ('op', ctypes.c_char_p), ('tile', ctypes.c_int),
                ('splitk', ctypes.c_int), ('planes_in', ctypes.c_int),
                ('planes_out', ctypes.c_int), ('gemm', ctypes.c_int),
                ('flops', ctypes.c_double), ('bytes', ctypes.c_double),
                ('out_shape', ctypes.c_int64 * 4), ('output', ctypes.c_char_p)]


def _env_flag(name):
    return os.environ.get(name, '1') != '0'


def config_from_cfg(c=None, math=None, fused_stem=None, fused_pps=None, act_planes=None):
    """PpsModelConfig from the Detectron-style cfg (pps_amd.config; the keys
    the reference's test net reads) and the same fusion defaults / env
    switches as PPSModel (PPS_MATH, PPS_FUSED_STEM, PPS_FUSED_PPS,
    PPS_ACT_PLANES)."""
    from . import ops
    c = c or _cfg
    k = PpsModelConfig()
    call('pps_model_config_default', ctypes.addressof(k))
    k.height, k.width = int(c.REID.SCALE[1]), int(c.REID.SCALE[0])
    k.strip_num, k.bpm_dim = int(c.REID.BPM_STRIP_NUM), int(c.REID.BPM_DIM)
    k.num_groups, k.width_per_group = int(c.RESNETS.NUM_GROUPS), int(c.RESNETS.WIDTH_PER_GROUP)
    k.stride_1x1 = int(bool(c.RESNETS.STRIDE_1X1))
    k.res5_stride, k.res5_dilation = int(c.RESNETS.RES5_STRIDE), int(c.RESNETS.RES5_DILATION)
    k.fpn_on, k.fpn_dim = int(bool(c.FPN.FPN_ON)), int(c.FPN.DIM)
    k.max_ave, k.normalize = int(bool(c.REID.MAX_AVE_FEATURE)), int(bool(c.REID.NORMALIZE_FEATURE))
    k.math = MATH[math or ops.default_math()]
    k.fused_stem = int(_env_flag('PPS_FUSED_STEM') if fused_stem is None else bool(fused_stem))
    k.fused_pps = int(_env_flag('PPS_FUSED_PPS') if fused_pps is None else bool(fused_pps))
    k.act_planes = int(_env_flag('PPS_ACT_PLANES') if act_planes is None else bool(act_planes))
    for i, v in enumerate(np.asarray(c.PIXEL_MEANS, np.float64).ravel()[:3]):
        k.pixel_means[i] = float(v)
    return k


class NativeModel(object):
    """Device-resident PPS extractor behind the whole-network C ABI.

    blobs: {name: ndarray} Detectron-format weights (pps_amd.weights /
    model.synthetic_weights).  forward(x_nhwc4) -> [N, feat_dim] on torch's
    current stream (capturable once the batch size is reserved)."""

    def __init__(self, blobs, config=None, **kw):
        self.config = config or config_from_cfg(**kw)
        arrays = []
        table = (PpsBlob * max(1, len(blobs)))()
        for i, (name, a) in enumerate(sorted(blobs.items())):
            a = np.ascontiguousarray(a, dtype=np.float32)
            arrays.append(a)
            table[i].name = name.encode()
            table[i].data = a.ctypes.data
            table[i].ndim = a.ndim
            for d, s in enumerate(a.shape[:4]):
                table[i].shape[d] = s
            if a.ndim > 4:
                raise ValueError('blob %s has %d dims' % (name, a.ndim))
        h = ctypes.c_void_p()
        call('pps_model_create', ctypes.addressof(table), len(blobs),
             ctypes.addressof(self.config), ctypes.addressof(h))
        self._h = h
        L = _lib.lib()
        self.feat_dim = L.pps_model_feat_dim(h)
        self.math = 'x3' if self.config.math == 0 else 'f32'

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and h.value:
            try:
                _lib.lib().pps_model_destroy(h)
            except Exception:
                pass
            self._h = None

    @property
    def handle(self):
        return self._h

    # -- introspection / tuning table -------------------------------------
    def layers(self, N=64):
        out = []
        for i in range(_lib.lib().pps_model_num_layers(self._h)):
            info = PpsLayerInfo()
            call('pps_model_layer_info', self._h, i, int(N), ctypes.addressof(info))
            out.append(dict(name=info.name.decode(), op=info.op.decode(), tile=info.tile,
                            splitk=info.splitk, planes_in=bool(info.planes_in),
                            planes_out=bool(info.planes_out), gemm=bool(info.gemm),
                            flops=info.flops, bytes=info.bytes,
                            out_shape=tuple(info.out_shape), output=info.output.decode()))
        return out

    def tiles(self):
        return {L['name']: L['tile'] for L in self.layers() if L['op'] in
                ('conv', 'conv_dual', 'heads', 'conv_pps', 'stem_pool')}

    def set_tiles(self, tiles):
        names = {L['name'] for L in self.layers()}
        for k, t in tiles.items():
            if k in names:
                call('pps_model_set_tile', self._h, k.encode(), int(t))

    def plane_edges(self):
        out = []
        for i in range(_lib.lib().pps_model_num_plane_edges(self._h)):
            p, c, on = ctypes.c_char_p(), ctypes.c_char_p(), ctypes.c_int()
            call('pps_model_plane_edge', self._h, i, ctypes.addressof(p), ctypes.addressof(c),
                 ctypes.addressof(on))
            out.append((p.value.decode(), c.value.decode(), bool(on.value)))
        return out

    def planes(self):
        return [p for p, _, on in self.plane_edges() if on]

    def set_planes(self, producers):
        want = set(producers)
        known = {p for p, _, _ in self.plane_edges()}
        if want - known:
            raise ValueError('not a plane-eligible producer: %s' % sorted(want - known)[:3])
        for p in known:
            call('pps_model_set_planes', self._h, p.encode(), int(p in want))

    def splitks(self):
        return {L['name']: L['splitk'] for L in self.layers() if L['splitk'] > 1}

    def set_splitks(self, sks):
        for L in self.layers():
            if L['op'] == 'conv':
                call('pps_model_set_splitk', self._h, L['name'].encode(),
                     int(sks.get(L['name'], 1)))

    def apply_table(self, src):
        """Copy a tuning table from a PPSModel (or a saved tiles dict with
        '__planes__' / '__splitk__' entries)."""
        if isinstance(src, dict):
            tiles, planes, sks = src, src.get('__planes__'), src.get('__splitk__', {})
        else:
            tiles, planes, sks = src.tiles(), src.planes(), src.splitks()
        self.set_tiles({k: v for k, v in tiles.items() if not k.startswith('__')})
        if planes is not None:
            self.set_planes(planes)
        self.set_splitks(sks)

    def autotune(self, x, flags=0):
        N = self._check_x(x)
        call('pps_model_autotune', self._h, x.data_ptr(), N, int(flags), _stream())
        return self.tiles()

    # -- execution ----------------------------------------------------------
    def reserve(self, N):
        call('pps_model_reserve', self._h, int(N))

    def release(self, N=0):
        call('pps_model_release', self._h, int(N))

    def _check_x(self, x):
        c = self.config
        if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()):
            raise RuntimeError('x must be a contiguous float32 device tensor')
        if tuple(x.shape[1:]) != (c.height, c.width, 4):
            raise RuntimeError('x must be NHWC4 [N, %d, %d, 4], got %s'
                               % (c.height, c.width, tuple(x.shape)))
        return int(x.shape[0])

    def _out(self, N, out, device):
        if out is None:
            out = torch.empty((N, self.feat_dim), dtype=torch.float32, device=device)
        if tuple(out.shape) != (N, self.feat_dim) or not out.is_contiguous():
            raise RuntimeError('out must be contiguous [%d, %d]' % (N, self.feat_dim))
        return out

    def forward(self, x, out=None):
        N = self._check_x(x)
        out = self._out(N, out, x.device)
        call('pps_forward', self._h, x.data_ptr(), N, out.data_ptr(), _stream())
        return out

    __call__ = forward

    def forward_layers(self, x, first, last, out=None, keep_amax=False):
        """Layers [first, last).  keep_amax: trust the activation maxima the
        previous call reported (PPS_FWD_KEEP_AMAX; timing a range whose inputs
        are unchanged), else ranges with first > 0 re-measure them."""
        N = self._check_x(x)
        out = self._out(N, out, x.device)
        call('pps_forward_layers_flags', self._h, x.data_ptr(), N, out.data_ptr(), int(first),
             int(last), FWD_KEEP_AMAX if keep_amax else 0, _stream())
        return out

    def forward_nchw(self, x, out=None):
        """The reference's `data` blob as it is (NCHW [N, 3, H, W])."""
        c = self.config
        if tuple(x.shape[1:]) != (3, c.height, c.width) or x.dtype != torch.float32 or \
                not x.is_contiguous() or not x.is_cuda:
            raise RuntimeError('x must be a contiguous float32 device [N, 3, %d, %d]'
                               % (c.height, c.width))
        N = int(x.shape[0])
        out = self._out(N, out, x.device)
        call('pps_forward_nchw', self._h, x.data_ptr(), N, out.data_ptr(), _stream())
        return out

    def forward_bgr(self, img, out=None):
        """uint8 BGR [N, Hi, Wi, 3] device images -> preprocess -> forward."""
        if img.dtype != torch.uint8 or img.dim() != 4 or img.shape[3] != 3 or \
                not img.is_contiguous() or not img.is_cuda:
            raise RuntimeError('img must be a contiguous uint8 device [N, Hi, Wi, 3]')
        N, Hi, Wi, _ = img.shape
        out = self._out(int(N), out, img.device)
        call('pps_forward_bgr', self._h, img.data_ptr(), int(N), int(Hi), int(Wi),
             out.data_ptr(), _stream())
        return out

    def tensor(self, N, blob):
        """Copy of an intermediate tensor of the last forward at batch N
        (f32; bf16x3-plane tensors are summed back to f32 on the host)."""
        p, pl = ctypes.c_void_p(), ctypes.c_int()
        shape = (ctypes.c_int64 * 4)()
        call('pps_model_tensor', self._h, int(N), blob.encode(), ctypes.addressof(p),
             ctypes.addressof(pl), ctypes.addressof(shape))
        n = int(np.prod(list(shape)))
        torch.cuda.synchronize()
        if pl.value == 2:   # f16x2 planes of a PPS_TILE_H2E edge, on the bound's scale
            raw = (ctypes.c_uint16 * (2 * n))()
            _memcpy_d2h(raw, p.value, 4 * n)
            h = np.frombuffer(raw, np.float16).astype(np.float64).reshape(2, n).sum(0)
            inv = h2_inv_scale(self.tensor_amax(N, blob))
            return (h * inv).astype(np.float32).reshape(tuple(shape))
        if pl.value:
            raw = (ctypes.c_uint16 * (3 * n))()
            _memcpy_d2h(raw, p.value, 6 * n)
            u = np.frombuffer(raw, np.uint16).astype(np.uint32) << 16
            f = u.view(np.float32).reshape(3, n).astype(np.float64).sum(0)
            return f.astype(np.float32).reshape(tuple(shape))
        raw = (ctypes.c_float * n)()
        _memcpy_d2h(raw, p.value, 4 * n)
        return np.frombuffer(raw, np.float32).reshape(tuple(shape)).copy()

    def tensor_amax(self, N, blob):
        """max |t| the producer of tensor `blob` reported in the last forward
        at batch N (the f16x2 layers' input scales)."""
        torch.cuda.synchronize()
        v = ctypes.c_float()
        call('pps_model_tensor_amax', self._h, int(N), blob.encode(), ctypes.addressof(v))
        return float(v.value)


def h2_inv_scale(amax):
    """2^-s for the f16x2 scale 2^s the kernels derive from a tensor's max
    (pps_internal.hpp h2_scale_of): s = 15 - (biased exponent - 126), so
    max|x 2^s| lies in [2^14, 2^15); a zero max keeps scale 1, a denormal one
    takes s = 126, and s is clamped to [-126, 126]."""
    a = np.float32(amax)
    ebits = (int(a.view(np.uint32)) >> 23) & 0xff
    if ebits == 0:
        sh = 126 if a > 0 else 0
    else:
        sh = 15 - (ebits - 126)
    sh = max(-126, min(126, sh))
    return 2.0 ** (-sh)


_HIP = None


def _memcpy_d2h(dst, src, nbytes):
    """hipMemcpy device -> host of a buffer torch does not own (debug path)."""
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL('libamdhip64.so')
        _HIP.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_int]
    rc = _HIP.hipMemcpy(ctypes.addressof(dst), ctypes.c_void_p(src), ctypes.c_size_t(nbytes),
                        2)  # hipMemcpyDeviceToHost
    if rc != 0:
        raise RuntimeError('hipMemcpy D2H failed (%d)' % rc)


def _stream():
    return torch.cuda.current_stream().cuda_stream
