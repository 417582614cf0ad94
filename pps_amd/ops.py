"""Device operators over torch CUDA tensors, backed by libpps_hip.so.

torch is used only for device memory and the current HIP stream; every
computation below is a libpps_hip.so kernel.  Each wrapper checks device,
dtype and contiguity, then calls the C ABI on torch's current stream.

Also hosts the operator registry that mirrors the reference's Caffe2 op names
(`model.net.PairWiseDistance(X, Z)`, detectron/modeling/triplet_loss.py:145;
registration detectron/ops/pairwise_distance_op.cu:124-127), so code written
against that registry can look ops up by the same names.
"""
import os

import numpy as np
import torch

from . import _lib
from ._lib import METRICS, call


TILE_P_FIRST = 29  # first pipelined (gemm_x3p.hip) tile id, include/pps_abi.h
TILE_P16_FIRST = 38  # pipelined tiles on 16x16x32 MFMA blocks (their own rounding)
TILE_C16_FIRST = 56  # patch-staged 3x3 tiles (gemm_x3c.hip): K in (channel chunk, tap) order
TILE_B_TILED = 0x100  # PPS_TILE_B_TILED: or-ed into a conv tile, the weights are chunk-tiled
TILE_COL_ORDER = 0x200  # PPS_TILE_COL_ORDER: column-major output tile order (same bits)
TILE_SEAM = 0x400  # PPS_TILE_SEAM (whole-network plan): branch2c + next branch2a in one launch
TILE_H2 = 0x800    # PPS_TILE_H2 (whole-network plan): the layer in f16x2 arithmetic
TILE_H2P = 0x1000  # PPS_TILE_H2P: with TILE_H2, the input split once into f16x2 planes
TILE_H2E = 0x2000  # PPS_TILE_H2E: with TILE_H2, the input arrives as f16x2 planes its
                   # producer wrote on the scale of an output bound (conv2d_bn_act_h2out)
TILE_WS = 54       # the weight-stationary 1x1 tile (gemm_ws.hip)
TILE_H2_WIDE = 60  # 192x128 as 4 x 1 waves: f16x2 only (bf16x3 launches run tile 47)
TILE_FLAGS = TILE_B_TILED | TILE_COL_ORDER | TILE_SEAM | TILE_H2 | TILE_H2P | TILE_H2E   # every or-ed flag
# tiles built with the one-launch split-K epilogue (conv2d_bn_act_x3p(..., counters=))
FIX_TILES = (45, 47, 48, 49, 50)
PPS_FUSE_MAX_COLS = 256  # widest tile the fused part pooling takes (pps_internal.hpp)


def num_tiles():
    return _lib.lib().pps_gemm_num_tiles()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _dev(t, name, dtype=torch.float32):
    if not isinstance(t, torch.Tensor):
        raise TypeError('%s must be a torch.Tensor' % name)
    if not t.is_cuda:
        raise RuntimeError('%s must be a device (HIP) tensor; the product path has no '
                           'CPU implementation' % name)
    if t.dtype != dtype:
        raise RuntimeError('%s must be %s, got %s' % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise RuntimeError('%s must be contiguous' % name)
    return t.data_ptr()


def _dev_rows(t, name, dtype=torch.float32):
    """A 2-D device matrix whose rows may be padded (stride(1) == 1,
    stride(0) >= columns): distance matrices are passed with their row
    stride (ld*) so a [Q, G] view of a wider buffer needs no copy."""
    if not isinstance(t, torch.Tensor) or t.dim() != 2:
        raise RuntimeError('%s must be a 2-D torch.Tensor' % name)
    if not t.is_cuda:
        raise RuntimeError('%s must be a device (HIP) tensor; the product path has no '
                           'CPU implementation' % name)
    if t.dtype != dtype:
        raise RuntimeError('%s must be %s, got %s' % (name, dtype, t.dtype))
    if t.shape[0] > 1 and (t.stride(1) != 1 or t.stride(0) < t.shape[1]):
        raise RuntimeError('%s must have unit column stride and row stride >= columns'
                           % name)
    return t.data_ptr()


def _ld(t):
    return t.stride(0) if t.shape[0] > 1 else t.shape[1]


# ---------------------------------------------------------------------------
# Retrieval
# ---------------------------------------------------------------------------
def default_math():
    """'x3' (f32 products on bf16 matrix cores, f32-level error) unless the
    environment asks for the exact-f32 MFMA kernels with PPS_MATH=f32."""
    m = os.environ.get('PPS_MATH', 'x3')
    if m not in ('x3', 'f32'):
        raise ValueError('PPS_MATH must be x3 or f32, got %r' % m)
    return m


def dist_math():
    """Arithmetic of the distance GEMMs (compute_dist and everything built on
    it): 'h2' (default: f16x2, three f16 MFMA terms per product, f32-level
    error -- csrc/gemm_h2.hip), 'x3' (six bf16 terms) or 'f32' (exact f32
    MFMA), from PPS_DIST_MATH; PPS_MATH=f32 (exact f32 everywhere) also
    selects 'f32' here."""
    m = os.environ.get('PPS_DIST_MATH')
    if m is None:
        return 'f32' if default_math() == 'f32' else 'h2'
    if m not in ('h2', 'x3', 'f32'):
        raise ValueError('PPS_DIST_MATH must be h2, x3 or f32, got %r' % m)
    return m


def h2_num_tiles():
    return int(_lib.lib().pps_h2_num_tiles())


def split_h2_tiled(x):
    """f16x2 split of a [R, D] tensor (D % 32 == 0) for the h2 distance GEMM,
    one read of x: -> (planes, rscale, sqnorm) with planes the two f16 planes
    chunk-tiled as an int16 [2, R16, D] tensor, rscale [R] the per-row
    power-of-two inverse scales, sqnorm [R] = row_sqnorm(x) (same bits)."""
    R, D = x.shape
    r16 = (R + 15) // 16 * 16
    planes = torch.empty((2, r16, D), dtype=torch.int16, device=x.device)
    rs = torch.empty((R,), dtype=torch.float32, device=x.device)
    sq = torch.empty((R,), dtype=torch.float32, device=x.device)
    call('pps_split_f16x2_sqnorm_tiled', _dev(x, 'x'), R, D, D, _dev(planes, 'out2t', torch.int16), _dev(rs, 'rscale'), _dev(sq, 'sqnorm'), _stream())
    return planes, rs, sq


def row_sqnorm(x):
    """Squared L2 norm of every row of a [R, D] tensor (fixed summation order)."""
    R, D = x.shape
    out = torch.empty((R,), dtype=torch.float32, device=x.device)
    call('pps_row_sqnorm', _dev(x, 'x'), R, D, x.stride(0), _dev(out, 'out'), _stream())
    return out


def split_sqnorm(x):
    """(split_bf16x3(x), row_sqnorm(x)) of a [R, D] tensor from one read of x
    (pps_split_bf16x3_sqnorm; same bits as the two calls).  Planes [3, R, D]."""
    R, D = x.shape
    planes = torch.empty((3, R, D), dtype=torch.int16, device=x.device)
    sq = torch.empty((R,), dtype=torch.float32, device=x.device)
    call('pps_split_bf16x3_sqnorm', _dev(x, 'x'), R, D, x.stride(0),
         _dev(planes, 'out3', torch.int16), _dev(sq, 'sqnorm'), _stream())
    return planes, sq


def split_sqnorm_tiled(x):
    """split_sqnorm writing the planes chunk-tiled (tile_planes' layout, as an
    int16 [3, R16, D] tensor) from one read of x; D % 32 == 0.  Same bits."""
    R, D = x.shape
    r16 = (R + 15) // 16 * 16
    planes = torch.empty((3, r16, D), dtype=torch.int16, device=x.device)
    sq = torch.empty((R,), dtype=torch.float32, device=x.device)
    call('pps_split_bf16x3_sqnorm_tiled', _dev(x, 'x'), R, D, x.stride(0),
         _dev(planes, 'out3t', torch.int16), _dev(sq, 'sqnorm'), _stream())
    return planes, sq


class GalleryIndex(object):
    """A gallery prepared once for the distance GEMM; score any number of
    query batches against it with compute_dist(q, index).  math 'h2' (the
    dist_math() default when D % 32 == 0): the f16x2 split (split_h2_tiled:
    two chunk-tiled f16 planes, per-row scales, squared norms); 'x3': the
    features split into three bf16 planes + squared norms, tiled=True in the
    chunk-tiled layout the query-planes GEMM streams (one pass; the row-major
    planes are then split on first use)."""

    def __init__(self, g, tiled=False, math=None):
        if g.dim() != 2:
            raise RuntimeError('gallery must be [G, D], got %s' % (tuple(g.shape),))
        self.feats = g
        self._planes = self._tiled = self.h2 = None
        math = math or dist_math()
        if math == 'f32':
            math = 'x3'   # an index is a split; f32 distances take the features as they are
        if math == 'h2' and not (g.is_contiguous() and g.shape[1] % 32 == 0):
            math = 'x3'   # the f16x2 kernel needs D % 32 == 0 (chunk-tiled planes)
        self.math = math
        if math == 'h2':
            self.h2 = split_h2_tiled(g)   # (planes, rscale, sqnorm)
            self.sqnorm = self.h2[2]
        elif tiled and g.is_contiguous() and g.shape[1] % 32 == 0:
            self._tiled, self.sqnorm = split_sqnorm_tiled(g)
        elif g.is_contiguous() and g.shape[1] % 4 == 0:
            self._planes, self.sqnorm = split_sqnorm(g)
        else:
            self._planes = split_bf16x3(g)
            self.sqnorm = row_sqnorm(g)

    @property
    def shape(self):
        return self.feats.shape

    @property
    def planes(self):
        """Row-major planes [3, G, D]."""
        if self._planes is None:
            self._planes = split_bf16x3(self.feats)
        return self._planes

    @property
    def tiled_planes(self):
        """The planes chunk-tiled (tile_planes' layout), built on first use."""
        if self._tiled is None:
            self._tiled = tile_planes(self.planes)
        return self._tiled


# tiles the symmetric self-distance takes: every pipelined tile (the upper
# triangle is enumerated by lcm(BM, BN) super-blocks); 0 = tile 43
SELF_TILES = (0,) + tuple(range(TILE_P_FIRST, 54)) + (55,)


def dist_buffer(Q, G, device):
    """[Q, G] float32 view of a buffer whose rows are padded to a multiple of
    4 floats: every row starts 16-byte aligned, so the distance epilogue
    stores whole 16-byte vectors and the rank kernels stream 16-byte loads."""
    ld = (G + 3) // 4 * 4
    return torch.empty((Q, ld), dtype=torch.float32, device=device)[:, :G]


def compute_dist(q, g, metric='euclidean', out=None, tile=0, math=None, q_planes=None,
                 symmetric=None, pad_rows=False):
    """[Q,D] x [G,D] -> [Q,G] distance matrix (reid_dataset_evaluator.py:244).
    math: 'h2' / 'x3' / 'f32' (None = dist_math(), or the GalleryIndex's own).
    g may be a GalleryIndex (then the GEMM runs on its prepared split).
    h2: queries split by split_h2_tiled, pps_distmat_h2_tiled (tile = h2 tile
    id, 0 = default); D % 32 != 0 runs x3.
    q_planes (x3): also split the queries into bf16x3 planes first so the
    pipelined GEMM stages both operands by DMA (pps_distmat_x3p; pipelined
    tiles only).  Same bits either way; measured at the Market shape it is
    not faster (scripts/probes/dist_probe.py: the split in the K loop is hidden),
    so None = off.
    pad_rows: return a [Q, G] view of a buffer with 16-byte-aligned rows
    (dist_buffer) instead of a dense matrix.
    symmetric (h2, x3): a self-distance (q and g the same rows, e.g.
    compute_dist(g, g) of re-ranking) computed from the upper-triangle tiles
    and mirrored (pps_distmat_h2_self_tiled / pps_distmat_x3_self, half the
    work); None = whenever q IS g's data, D % 32 == 0 and (x3) the tile is a
    square one (SELF_TILES)."""
    if isinstance(g, GalleryIndex):
        # the index fixes the arithmetic; an explicit request for another one
        # is an error (f32 reads the index's features as they are)
        if math not in (None, 'f32', g.math):
            raise RuntimeError("compute_dist: math=%r but the GalleryIndex holds a %r split"
                               % (math, g.math))
        math = math or g.math
    math = math or dist_math()
    if q.dim() != 2 or len(g.shape) != 2 or q.shape[1] != g.shape[1]:
        raise RuntimeError('compute_dist expects [m1,n] and [m2,n], got %s %s'
                           % (tuple(q.shape), tuple(g.shape)))
    Q, D = q.shape
    G = g.shape[0]
    if out is None:
        out = dist_buffer(Q, G, q.device) if pad_rows else \
            torch.empty((Q, G), dtype=torch.float32, device=q.device)
    if tuple(out.shape) != (Q, G):
        raise RuntimeError('out must be [%d, %d], got %s' % (Q, G, tuple(out.shape)))
    # the mark re_ranking reads: set on every return, so a reused buffer
    # never carries a stale True from an earlier self-distance
    out._pps_symmetric = False
    if math == 'f32':
        gf = g.feats if isinstance(g, GalleryIndex) else g
        call('pps_distmat', _dev(q, 'q'), Q, D, _dev(gf, 'g'), G, D, D, METRICS[metric],
             _dev_rows(out, 'out'), _ld(out), int(tile), _stream())
        return out
    f = g.feats if isinstance(g, GalleryIndex) else g
    same = (f.data_ptr() == q.data_ptr() and tuple(f.shape) == tuple(q.shape) and
            f.stride() == q.stride() and q.is_contiguous() and D % 32 == 0)
    if math == 'h2' and D % 32 == 0 and q.is_contiguous():
        if symmetric is None:
            symmetric = same
        if symmetric:
            x2, xrs, xsq = g.h2 if isinstance(g, GalleryIndex) and g.h2 is not None else \
                split_h2_tiled(q)
            call('pps_distmat_h2_self_tiled', _dev(x2, 'x2t', torch.int16), Q, _dev(xsq, 'xsq'),
                 _dev(xrs, 'xrs'), D, METRICS[metric], _dev_rows(out, 'out'), _ld(out),
                 int(tile), _stream())
            out._pps_symmetric = True   # mirrored tiles: exactly symmetric
            return out
        # a strided raw gallery (e.g. big[:, :D]) is made contiguous first: the
        # f16x2 index needs whole rows
        idx = g if isinstance(g, GalleryIndex) and g.h2 is not None else \
            GalleryIndex(f if f.is_contiguous() else f.contiguous(), math='h2')
        q2, qrs, qsq = split_h2_tiled(q)
        return distmat_h2(q2, qrs, qsq, idx, out, metric, tile, Q=Q)
    if math == 'h2':
        math, tile = 'x3', 0   # D % 32 != 0 (or strided queries): the bf16x3 kernels
    tiled = bool(q_planes) and D % 32 == 0 and (tile == 0 or tile >= TILE_P_FIRST)
    if symmetric is None:
        symmetric = same and tile in SELF_TILES
    if symmetric:
        # one read of x -> chunk-tiled planes + norms; both operands staged
        # from that copy by DMA (pps_distmat_x3_self_tiled)
        if isinstance(g, GalleryIndex) and g._tiled is not None:
            x3t, xsq = g._tiled, g.sqnorm
        else:
            x3t, xsq = split_sqnorm_tiled(q)
        call('pps_distmat_x3_self_tiled', _dev(x3t, 'x3t', torch.int16), Q, _dev(xsq, 'xsq'),
             D, METRICS[metric], _dev_rows(out, 'out'), _ld(out), int(tile), _stream())
        out._pps_symmetric = True   # mirrored tiles: exactly symmetric (re_ranking uses it)
        return out
    idx = g if isinstance(g, GalleryIndex) else GalleryIndex(g, tiled=tiled, math='x3')
    if q_planes:
        if tiled and q.is_contiguous():  # both operands chunk-tiled, queries in one pass
            qt, qsq = split_sqnorm_tiled(q)
            return distmat_planes(None, qsq, idx, out, metric, tile, q_tiled=qt, Q=Q, D=D)
        q3, qsq = split_sqnorm(q) if q.is_contiguous() else (split_bf16x3(q), row_sqnorm(q))
        return distmat_planes(q3, qsq, idx, out, metric, tile)
    qsq = row_sqnorm(q)
    call('pps_distmat_x3', _dev(q, 'q'), Q, D, _dev(qsq, 'qsq'),
         _dev(idx.planes, 'g3', torch.int16), _dev(idx.sqnorm, 'gsq'), G, D, D,
         METRICS[metric], _dev_rows(out, 'out'), _ld(out), int(tile), _stream())
    return out


def distmat_h2(q2, qrs, qsq, idx, out, metric='euclidean', tile=0, Q=None):
    """The h2 distance GEMM alone on queries already split (split_h2_tiled)
    against an h2 GalleryIndex: what compute_dist(math='h2') launches after
    the split (pps_distmat_h2_tiled)."""
    Q = qsq.shape[0] if Q is None else Q
    G, D = idx.shape
    g2, grs, gsq = idx.h2
    call('pps_distmat_h2_tiled', _dev(q2, 'q2t', torch.int16), Q, _dev(qsq, 'qsq'),
         _dev(qrs, 'qrs'), _dev(g2, 'g2t', torch.int16), _dev(gsq, 'gsq'), _dev(grs, 'grs'), G,
         D, METRICS[metric], _dev_rows(out, 'out'), _ld(out), int(tile), _stream())
    return out


def tile_planes(planes):
    """bf16x3 planes [3, R, D] (D % 32 == 0) -> the chunk-tiled layout
    [3][R16 / 16][D / 32][16][32] (R16 = R rounded up to 16, zero rows),
    returned as an int16 [3, R16, D] tensor: a 16-row DMA piece of one
    32-wide K chunk is then one contiguous KiB (pps_tile_planes)."""
    _, R, D = planes.shape
    r16 = (R + 15) // 16 * 16
    out = torch.empty((3, r16, D), dtype=torch.int16, device=planes.device)
    call('pps_tile_planes', _dev(planes, 'planes', torch.int16), R, D, D, R * D,
         _dev(out, 'out', torch.int16), _stream())
    return out


def _tiled_tile(tile):
    """The tile a tiled-plane distance GEMM runs: pipelined ids 29-53 as
    given; ids 54+ (which a distance matrix runs as tile 38) -> 0 (tile 43,
    the same 16x16x32 rounding group)."""
    return int(tile) if TILE_P_FIRST <= tile < 54 else 0


def distmat_planes(q3, qsq, idx, out, metric='euclidean', tile=0, q_tiled=None, Q=None,
                   D=None):
    """The distance GEMM alone on queries already split into bf16x3 planes
    q3 [3, Q, D] with squared norms qsq, against a GalleryIndex: what
    compute_dist(q_planes=True) launches after the split.  With D % 32 == 0
    both operands go chunk-tiled (pps_distmat_x3p_tiled: same bits, Market
    1.98 -> 1.83 ms on tile 52, scripts/probes/dist_tiled_probe.py); q_tiled
    = tile_planes(q3) when the caller has it already (q3 may then be None,
    with Q and D given)."""
    if q3 is not None:
        _, Q, D = q3.shape
    G = idx.shape[0]
    if D % 32 == 0 and (tile == 0 or tile >= TILE_P_FIRST):
        qt = q_tiled if q_tiled is not None else tile_planes(q3)
        call('pps_distmat_x3p_tiled', _dev(qt, 'q3t', torch.int16), Q, _dev(qsq, 'qsq'),
             _dev(idx.tiled_planes, 'g3t', torch.int16), _dev(idx.sqnorm, 'gsq'), G, D,
             METRICS[metric], _dev_rows(out, 'out'), _ld(out), _tiled_tile(tile), _stream())
        return out
    call('pps_distmat_x3p', _dev(q3, 'q3', torch.int16), Q, D, _dev(qsq, 'qsq'),
         _dev(idx.planes, 'g3', torch.int16), _dev(idx.sqnorm, 'gsq'), G, D, D,
         METRICS[metric], _dev_rows(out, 'out'), _ld(out), int(tile), _stream())
    return out


def pairwise_distance(X):
    """Caffe2 PairWiseDistance: squared L2, [N,D] -> [N,N]."""
    if X.dim() != 2:
        raise RuntimeError('[enforce fail] X.dim() == 2 (got %d)' % X.dim())
    N, D = X.shape
    Z = torch.empty((N, N), dtype=torch.float32, device=X.device)
    call('pps_pairwise_distance', _dev(X, 'X'), N, D, _dev(Z, 'Z'), _stream())
    return Z


def argsort_rows(dist, with_values=False):
    """Every row's columns in stable (distance, index) order -> idx [Q, G]
    int32 (and the sorted distances): np.argsort(dist, axis=1,
    kind='stable') -- the reference's full rank list
    (reid_dataset_evaluator.py:319,420).  G <= pps_argsort_rows_cap()."""
    Q, G = dist.shape
    idx = torch.empty((Q, G), dtype=torch.int32, device=dist.device)
    vals = torch.empty((Q, G), dtype=torch.float32, device=dist.device) if with_values else None
    call('pps_argsort_rows', _dev_rows(dist, 'dist'), Q, G, _ld(dist), idx.data_ptr(), G,
         vals.data_ptr() if vals is not None else None, G, _stream())
    return (idx, vals) if with_values else idx


def sgs_groups(order, gid, gcam, qid, qcam, U, separate_camera_set):
    """Steps 1-3 of CMC single_gallery_shot (pps_sgs_keys, pps_argsort_rows,
    pps_sgs_groups) from the stable rank list `order` [Q, G] and dense
    identities (device int32).  Returns (perm, gstart, glen, nids, qt)."""
    Q, G = order.shape
    dev = order.device
    keys = torch.empty((Q, G), dtype=torch.float32, device=dev)
    call('pps_sgs_keys', _dev_rows(order, 'order', torch.int32), Q, G, _ld(order),
         _dev(gid, 'gid', torch.int32), _dev(gcam, 'gcam', torch.int32),
         _dev(qid, 'qid', torch.int32), _dev(qcam, 'qcam', torch.int32),
         1 if separate_camera_set else 0, U, keys.data_ptr(), _stream())
    perm, skeys = argsort_rows(keys, with_values=True)
    del keys
    i32 = lambda *s: torch.empty(s, dtype=torch.int32, device=dev)
    gstart, glen, nids, qt = i32(Q, U), i32(Q, U), i32(Q), i32(Q)
    call('pps_sgs_groups', skeys.data_ptr(), perm.data_ptr(), Q, G, U, _dev(qid, 'qid', torch.int32),
         gstart.data_ptr(), glen.data_ptr(), nids.data_ptr(), qt.data_ptr(), _stream())
    return perm, gstart, glen, nids, qt


def sgs_ranks(perm, gstart, glen, nids, qt, rows, draws):
    """Step 5 of CMC single_gallery_shot (pps_sgs_ranks): draws [nr, repeat,
    ldd] int32 for the query rows `rows` [nr] -> k [nr, repeat] int32."""
    Q, G = perm.shape
    U = gstart.shape[1]
    nr, repeat, ldd = draws.shape
    k = torch.empty((nr, repeat), dtype=torch.int32, device=perm.device)
    call('pps_sgs_ranks', perm.data_ptr(), Q, G, _dev(rows, 'rows', torch.int32), nr,
         gstart.data_ptr(), glen.data_ptr(), nids.data_ptr(), qt.data_ptr(), U, repeat,
         _dev(draws, 'draws', torch.int32), ldd, k.data_ptr(), _stream())
    return k


def topk(dist, k):
    """Stable ascending top-k per row -> (vals [Q,k] f32, idx [Q,k] i32)."""
    Q, G = dist.shape
    vals = torch.empty((Q, k), dtype=torch.float32, device=dist.device)
    idx = torch.empty((Q, k), dtype=torch.int32, device=dist.device)
    call('pps_topk', _dev_rows(dist, 'dist'), Q, G, _ld(dist), k, vals.data_ptr(),
         idx.data_ptr(), _stream())
    return vals, idx


def topk_merge(vals, idx, offsets, k):
    """Merge R per-shard stable top-k lists vals/idx [R, Q, k_in] (local
    indices; list r starts at global index offsets[r]) into the global stable
    top-k [Q, k] (pps_topk_merge; (+inf, -1) past the available entries)."""
    R, Q, kin = vals.shape
    offs = np.ascontiguousarray(np.asarray(offsets, np.int64).reshape(-1))
    if offs.shape[0] != R:
        raise RuntimeError('need one offset per list: %d lists, %d offsets'
                           % (R, offs.shape[0]))
    out_v = torch.empty((Q, k), dtype=torch.float32, device=vals.device)
    out_i = torch.empty((Q, k), dtype=torch.int32, device=vals.device)
    call('pps_topk_merge', _dev(vals, 'vals'), _dev(idx, 'idx', torch.int32), R, Q, kin,
         offs.ctypes.data_as(_lib.ctypes.c_void_p), k, out_v.data_ptr(), out_i.data_ptr(),
         _stream())
    return out_v, out_i


class MatchIndex(object):
    """Per-identity index of a gallery (shard) for one query set, built once
    from the ids (host metadata, O(G log G)): members = local gallery indices
    sorted by (id, index); query q's identity occupies
    members[q_beg[q]:q_end[q]].  `capacity` = the most same-id entries any
    query has = an exact bound for its positive and junk lists."""

    def __init__(self, qid, qcam, gid, gcam, device='cuda'):
        qid, qcam = np.asarray(qid).astype(np.int64), np.asarray(qcam)
        gid, gcam = np.asarray(gid).astype(np.int64), np.asarray(gcam)
        order = np.lexsort((np.arange(len(gid)), gid))
        sid = gid[order]
        beg = np.searchsorted(sid, qid, 'left')
        end = np.searchsorted(sid, qid, 'right')
        self.capacity = max(1, int((end - beg).max()) if len(qid) else 1)
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a).astype(np.int32)).to(device)
        self.members, self.q_beg, self.q_end = i32(order), i32(beg), i32(end)
        self.qcam, self.gcam = i32(qcam), i32(gcam)
        self.Q, self.G = len(qid), len(gid)


def collect_matches(dist, index, g_offset=0, pmax=None):
    """(pos_d, pos_idx, pos_cnt, junk_d, junk_idx, junk_cnt) of every query
    from the MatchIndex (pps_collect_matches)."""
    Q, G = dist.shape
    if (Q, G) != (index.Q, index.G):
        raise RuntimeError('distance matrix %s does not match the index (%d, %d)'
                           % (tuple(dist.shape), index.Q, index.G))
    pmax = pmax or index.capacity
    jmax = index.capacity
    dev = dist.device
    pos_d = torch.empty((Q, pmax), dtype=torch.float32, device=dev)
    pos_idx = torch.empty((Q, pmax), dtype=torch.int32, device=dev)
    pos_cnt = torch.empty((Q,), dtype=torch.int32, device=dev)
    junk_d = torch.empty((Q, jmax), dtype=torch.float32, device=dev)
    junk_idx = torch.empty((Q, jmax), dtype=torch.int32, device=dev)
    junk_cnt = torch.empty((Q,), dtype=torch.int32, device=dev)
    call('pps_collect_matches', _dev_rows(dist, 'dist'), Q, G, _ld(dist),
         _dev(index.qcam, 'qcam', torch.int32), _dev(index.gcam, 'gcam', torch.int32),
         _dev(index.members, 'members', torch.int32), _dev(index.q_beg, 'q_beg', torch.int32),
         _dev(index.q_end, 'q_end', torch.int32), int(g_offset), pmax, pos_d.data_ptr(),
         pos_idx.data_ptr(), pos_cnt.data_ptr(), jmax, junk_d.data_ptr(), junk_idx.data_ptr(),
         junk_cnt.data_ptr(), _stream())
    return pos_d, pos_idx, pos_cnt, (junk_d, junk_idx, junk_cnt)


class SortedPositives(object):
    """Merged, sorted positive lists of a query set (pps_rank_prepare):
    sorted_d / sorted_idx [Q, Ptot], pos_total [Q], bin-lookup cells."""

    def __init__(self, sorted_d, sorted_idx, pos_total, cells):
        self.sorted_d, self.sorted_idx, self.pos_total = sorted_d, sorted_idx, pos_total
        self.cells = cells

    def __iter__(self):   # (sorted_d, sorted_idx, pos_total), as the old triple
        return iter((self.sorted_d, self.sorted_idx, self.pos_total))


def rank_prepare(pos_d, pos_idx, pos_cnt):
    """Merge [R, Q, Pmax] positive lists, sorted -> SortedPositives
    (pps_rank_prepare)."""
    R, Q, Pmax = pos_d.shape
    dev = pos_d.device
    sd = torch.empty((Q, R * Pmax), dtype=torch.float32, device=dev)
    si = torch.empty((Q, R * Pmax), dtype=torch.int32, device=dev)
    tot = torch.empty((Q,), dtype=torch.int32, device=dev)
    cells = torch.empty((Q, _lib.lib().pps_rank_cells()), dtype=torch.int32, device=dev)
    call('pps_rank_prepare', R, Q, Pmax, _dev(pos_d, 'pos_d'), _dev(pos_idx, 'pos_idx',
                                                                   torch.int32),
         _dev(pos_cnt, 'pos_cnt', torch.int32), sd.data_ptr(), si.data_ptr(), tot.data_ptr(),
         cells.data_ptr(), _stream())
    return SortedPositives(sd, si, tot, cells)


def rank_count_stream(dist, g_offset, sp, junk, hist=None, before=None):
    """Additive (hist, before) counts of this shard's rows against the
    SortedPositives sp (pps_rank_count_stream); hist/before accumulate when
    given."""
    Q, G = dist.shape
    sorted_d, sorted_idx, pos_total = sp.sorted_d, sp.sorted_idx, sp.pos_total
    Ptot = sorted_d.shape[1]
    junk_d, junk_idx, junk_cnt = junk
    dev = dist.device
    if hist is None:
        hist = torch.zeros((Q, Ptot), dtype=torch.int32, device=dev)
    if before is None:
        before = torch.zeros((Q,), dtype=torch.int32, device=dev)
    call('pps_rank_count_stream', _dev_rows(dist, 'dist'), Q, G, _ld(dist), int(g_offset),
         Ptot, _dev(sorted_d, 'sorted_d'), _dev(sorted_idx, 'sorted_idx', torch.int32),
         _dev(pos_total, 'pos_total', torch.int32), _dev(sp.cells, 'cells', torch.int32),
         junk_d.shape[1], _dev(junk_d, 'junk_d'),
         _dev(junk_idx, 'junk_idx', torch.int32), _dev(junk_cnt, 'junk_cnt', torch.int32),
         _dev(hist, 'hist', torch.int32), _dev(before, 'before', torch.int32), _stream())
    return hist, before


def cmc_counts(dist, g_offset, sp, junk, index=None, separate_camera_set=False, hist=None):
    """Per-positive exact-rank bins for the reference's general cmc
    (pps_cmc_counts); with separate_camera_set the MatchIndex's qcam / gcam
    drop every same-camera entry.  hist accumulates when given."""
    Q, G = dist.shape
    Ptot = sp.sorted_d.shape[1]
    junk_d, junk_idx, junk_cnt = junk
    if hist is None:
        hist = torch.zeros((Q, Ptot), dtype=torch.int32, device=dist.device)
    qc = gc = 0
    if separate_camera_set:
        qc = _dev(index.qcam, 'qcam', torch.int32)
        gc = _dev(index.gcam, 'gcam', torch.int32)
    call('pps_cmc_counts', _dev_rows(dist, 'dist'), Q, G, _ld(dist), int(g_offset), Ptot,
         _dev(sp.sorted_d, 'sorted_d'), _dev(sp.sorted_idx, 'sorted_idx', torch.int32),
         _dev(sp.pos_total, 'pos_total', torch.int32), qc, gc, junk_d.shape[1],
         _dev(junk_d, 'junk_d'), _dev(junk_idx, 'junk_idx', torch.int32),
         _dev(junk_cnt, 'junk_cnt', torch.int32), _dev(hist, 'hist', torch.int32), _stream())
    return hist


def cmc_finalize(pos_total, hist, topk, first_match_break):
    """(ret [Q, topk] float64 after the reference's cumsum, valid [Q] int32)."""
    Q, Ptot = hist.shape
    ret = torch.empty((Q, topk), dtype=torch.float64, device=hist.device)
    valid = torch.empty((Q,), dtype=torch.int32, device=hist.device)
    call('pps_cmc_finalize', Q, Ptot, _dev(pos_total, 'pos_total', torch.int32),
         _dev(hist, 'hist', torch.int32), int(topk), int(bool(first_match_break)),
         ret.data_ptr(), valid.data_ptr(), _stream())
    return ret, valid


def collect_positives(dist, qid, qcam, gid, gcam, g_offset, Pmax):
    Q, G = dist.shape
    pos_d = torch.empty((Q, Pmax), dtype=torch.float32, device=dist.device)
    pos_idx = torch.empty((Q, Pmax), dtype=torch.int32, device=dist.device)
    pos_cnt = torch.empty((Q,), dtype=torch.int32, device=dist.device)
    call('pps_collect_positives', _dev_rows(dist, 'dist'), Q, G, _ld(dist),
         _dev(qid, 'qid', torch.int32), _dev(qcam, 'qcam', torch.int32),
         _dev(gid, 'gid', torch.int32), _dev(gcam, 'gcam', torch.int32), int(g_offset),
         Pmax, pos_d.data_ptr(), pos_idx.data_ptr(), pos_cnt.data_ptr(), _stream())
    return pos_d, pos_idx, pos_cnt


def rank_counts(dist, qid, qcam, gid, gcam, g_offset, pos_d, pos_idx, pos_cnt,
                hist=None, before=None):
    """pos_* are [R,Q,Pmax] / [R,Q] merged lists.  hist/before accumulate."""
    Q, G = dist.shape
    R, _, Pmax = pos_d.shape
    Ptot = R * Pmax
    dev = dist.device
    sorted_d = torch.empty((Q, Ptot), dtype=torch.float32, device=dev)
    sorted_idx = torch.empty((Q, Ptot), dtype=torch.int32, device=dev)
    pos_total = torch.empty((Q,), dtype=torch.int32, device=dev)
    if hist is None:
        hist = torch.zeros((Q, Ptot), dtype=torch.int32, device=dev)
    if before is None:
        before = torch.zeros((Q,), dtype=torch.int32, device=dev)
    call('pps_rank_counts', _dev_rows(dist, 'dist'), Q, G, _ld(dist),
         _dev(qid, 'qid', torch.int32), _dev(qcam, 'qcam', torch.int32),
         _dev(gid, 'gid', torch.int32), _dev(gcam, 'gcam', torch.int32), int(g_offset),
         R, Pmax, _dev(pos_d, 'pos_d'), _dev(pos_idx, 'pos_idx', torch.int32),
         _dev(pos_cnt, 'pos_cnt', torch.int32), sorted_d.data_ptr(),
         sorted_idx.data_ptr(), pos_total.data_ptr(), _dev(hist, 'hist', torch.int32),
         _dev(before, 'before', torch.int32), _stream())
    return sorted_d, sorted_idx, pos_total, hist, before


def ap_finalize(sorted_d, pos_total, hist, before):
    Q, Ptot = sorted_d.shape
    dev = sorted_d.device
    ap = torch.empty((Q,), dtype=torch.float64, device=dev)
    valid = torch.empty((Q,), dtype=torch.int32, device=dev)
    first = torch.empty((Q,), dtype=torch.int32, device=dev)
    call('pps_ap_finalize', Q, Ptot, _dev(sorted_d, 'sorted_d'),
         _dev(pos_total, 'pos_total', torch.int32), _dev(hist, 'hist', torch.int32),
         _dev(before, 'before', torch.int32), ap.data_ptr(), valid.data_ptr(),
         first.data_ptr(), _stream())
    return ap, valid, first


def re_ranking(q_g, q_q, g_g, k1=20, k2=6, lambda_value=0.3, symmetric=None, whole=False):
    """k-reciprocal re-ranking (reid_dataset_evaluator.py:442-519) -> [Q, G].
    symmetric: q_q and g_g are exactly symmetric (PPS_RERANK_SYMMETRIC: with
    16-byte rows and N >= 16384 the N x N normalised distance is never built,
    pps_re_ranking_ld; else it is built from rows, only q_g^T transposed);
    None = both came from compute_dist's mirrored self-distance (tagged
    `_pps_symmetric`).  Same result either way on symmetric inputs.  Inputs
    may be row-padded views (dist_buffer / compute_dist(pad_rows=True)).
    whole: the three are the blocks of one symmetric [N, N] self-distance
    (self_distance_blocks) -- q_g^T is read in place (PPS_RERANK_WHOLE)."""
    Q, G = q_g.shape
    assert tuple(q_q.shape) == (Q, Q) and tuple(g_g.shape) == (G, G)
    if symmetric is None:
        symmetric = bool(getattr(q_q, '_pps_symmetric', False) and
                         getattr(g_g, '_pps_symmetric', False))
    flags = (RERANK_SYMMETRIC if symmetric else 0) | (RERANK_WHOLE if whole else 0)
    blocks = (_dev_rows(q_g, 'q_g'), _ld(q_g), _dev_rows(q_q, 'q_q'), _ld(q_q),
              _dev_rows(g_g, 'g_g'), _ld(g_g))
    # the size of the path this call takes (in place: no N x N region)
    nbytes = _lib.lib().pps_rerank_workspace_bytes_ld(*blocks, Q, G, k1, k2, flags)
    if nbytes < 0:
        raise RuntimeError('bad re-ranking arguments')
    ws = torch.empty((int(nbytes),), dtype=torch.uint8, device=q_g.device)
    out = torch.empty((Q, G), dtype=torch.float32, device=q_g.device)
    call('pps_re_ranking_ld', *blocks, Q, G, k1, k2, float(lambda_value), flags,
         ws.data_ptr(), int(nbytes), out.data_ptr(), _stream())
    return out


RERANK_SYMMETRIC = 1   # pps_abi.h PPS_RERANK_SYMMETRIC
RERANK_WHOLE = 2       # pps_abi.h PPS_RERANK_WHOLE


def self_distance_blocks(x, Q, metric='euclidean'):
    """Re-ranking's three distance blocks from ONE mirrored self-distance of
    x = [queries; gallery] ([N, D], the first Q rows the queries): -> (M,
    q_g, q_q, g_g), the blocks row-padded views of the exactly symmetric
    [N, N] M (compute_dist(x, x), upper triangle + mirror, one bf16x3 split of
    x).  Pass them to re_ranking(..., whole=True); q_g serves the plain
    ranking as well.  Same values as the three separate compute_dist calls
    on the same tile group."""
    M = compute_dist(x, x, metric=metric, pad_rows=True, symmetric=True)
    return M, M[:Q, Q:], M[:Q, :Q], M[Q:, Q:]


def max_positives(qid, qcam, gid, gcam):
    """Host-side bound on true matches per query (metadata only, exact)."""
    qid = np.asarray(qid, np.int64)
    qcam = np.asarray(qcam, np.int64)
    gid = np.asarray(gid, np.int64)
    gcam = np.asarray(gcam, np.int64)
    if len(qid) == 0 or len(gid) == 0:
        return 0
    ids, inv = np.unique(np.concatenate([qid, gid]), return_inverse=True)
    qi, gi = inv[:len(qid)], inv[len(qid):]
    per_id = np.bincount(gi, minlength=len(ids))
    cams = np.unique(np.concatenate([qcam, gcam]), return_inverse=True)[1]
    qc, gc = cams[:len(qcam)], cams[len(qcam):]
    ncam = int(cams.max()) + 1
    per_idcam = np.bincount(gi * ncam + gc, minlength=len(ids) * ncam)
    cnt = per_id[qi] - per_idcam[qi * ncam + qc]
    return int(cnt.max())


# ---------------------------------------------------------------------------
# Feature extractor
# ---------------------------------------------------------------------------
def _weights(entry, w):
    """f32 weights -> the exact-f32 MFMA entry; int16 (bf16x3 planes from
    split_bf16x3) -> the `_x3` entry (f32 products on bf16 matrix cores)."""
    if isinstance(w, torch.Tensor) and w.dtype == torch.int16:
        return entry + '_x3', _dev(w, 'w', torch.int16)
    return entry, _dev(w, 'w')


def split_bf16x3(x, batched=False):
    """f32 x -> int16 bf16 planes hi, mid, lo with x = hi + mid + lo exactly
    (the weight format of the `_x3` GEMMs): shape (3,) + x.shape, or for
    batched=True (x.shape[0], 3) + x.shape[1:]."""
    nbatch = x.shape[0] if batched else 1
    n = x.numel() // nbatch
    shape = ((nbatch, 3) + tuple(x.shape[1:])) if batched else ((3,) + tuple(x.shape))
    out = torch.empty(shape, dtype=torch.int16, device=x.device)
    call('pps_split_bf16x3', _dev(x, 'x'), n, nbatch, _dev(out, 'out', torch.int16), _stream())
    return out


def conv2d_bn_act(x, cin, w, kpad, k, stride, pad, dil, scale, shift, residual, relu, y,
                  tile=0):
    N, H, W, ldx = x.shape
    _, Ho, Wo, Cout = y.shape
    rp = 0
    if residual is not None:
        if tuple(residual.shape) != tuple(y.shape):
            raise RuntimeError('residual shape %s != output %s'
                               % (tuple(residual.shape), tuple(y.shape)))
        rp = _dev(residual, 'residual')
    fn, wp = _weights('pps_conv2d_bn_act', w)
    call(fn, _dev(x, 'x'), N, H, W, cin, ldx, wp, Cout, kpad,
         k, k, stride, pad, dil, _dev(scale, 'scale'), _dev(shift, 'shift'), rp,
         int(bool(relu)), _dev(y, 'y'), Ho, Wo, Cout, int(tile), _stream())
    return y


def tile_shape(tile, planes=False):
    """(rows, cols) of the tile a pipelined GEMM id launches ((0, 0) if none)."""
    r, c = _lib.ctypes.c_int(0), _lib.ctypes.c_int(0)
    call('pps_x3p_tile_shape', int(tile), int(bool(planes)), _lib.ctypes.addressof(r),
         _lib.ctypes.addressof(c))
    return r.value, c.value


def conv2d_bn_act_pps(x, cin, w3, kpad, k, stride, pad, dil, scale, shift, residual, split,
                      max_ave, pps_out, y=None, tile=0):
    """The last res5 conv (+ BN + residual + ReLU) with the part pooling fused
    into its epilogue (pps_conv2d_bn_act_pps_x3p): pps_out [2^S-1, N, Cout]
    gets what part_power_set would compute from the conv output; y (NHWC, or
    None = not written) the conv output itself.  x: f32 NHWC or bf16x3
    planes (act_planes)."""
    xs = x.shape[1:] if _is_planes(x) else x.shape
    N, H, W, ldx = xs
    nsub, n2, Cout = pps_out.shape
    split = np.ascontiguousarray(split, dtype=np.int32)
    Ho = (H + 2 * pad - dil * (k - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (k - 1) - 1) // stride + 1
    if nsub != (1 << len(split)) - 1 or n2 != N:
        raise RuntimeError('pps_out must be [2^S - 1, N, Cout]')
    if tuple(residual.shape) != (N, Ho, Wo, Cout) or (y is not None and
                                                       tuple(y.shape) != (N, Ho, Wo, Cout)):
        raise RuntimeError('residual / y must be [N, Ho, Wo, Cout]')
    if _is_planes(x):
        xp, x3, xpl = 0, _dev(x, 'x planes', torch.int16), x[0].numel()
    else:
        xp, x3, xpl = _dev(x, 'x'), 0, 0
    call('pps_conv2d_bn_act_pps_x3p', xp, x3, xpl, N, H, W, cin, ldx,
         _dev(w3, 'w3', torch.int16), Cout, kpad, k, k, stride, pad, dil, _dev(scale, 'scale'),
         _dev(shift, 'shift'), _dev(residual, 'residual'), _dev(y, 'y') if y is not None else 0,
         Ho, Wo, split.ctypes.data_as(_lib.ctypes.c_void_p), len(split), int(bool(max_ave)),
         _dev(pps_out, 'pps_out'), int(tile), _stream())
    return pps_out


def act_planes(shape, device):
    """Buffer for a bf16x3 activation tensor: int16 [3, N, H, W, C] holding
    hi, mid, lo planes with x = hi + mid + lo exactly (split as the x3 GEMMs
    split f32 operands, so a consumer reading the planes gets the bits it
    would have computed from the f32 tensor)."""
    return torch.empty((3,) + tuple(shape), dtype=torch.int16, device=device)


def _is_planes(t):
    return isinstance(t, torch.Tensor) and t.dtype == torch.int16 and t.dim() == 5 \
        and t.shape[0] == 3


def conv2d_bn_act_x3p(x, cin, w3, kpad, k, stride, pad, dil, scale, shift, residual, relu,
                      y, tile=0, splitk=1, part=None, counters=None):
    """conv2d_bn_act on the pipelined bf16x3 GEMM where the input and/or the
    output are bf16x3 activation planes (act_planes) instead of f32 NHWC:
    x / y may each be either.  Same bits as the f32-activation call.
    splitk > 1: K slices with raw partials in `part`, summed in slice order by
    a second pass -- or, with `counters` (int32, zero, >= output tiles), by
    the last slice of each tile in the same launch (same bits)."""
    xs = x.shape[1:] if _is_planes(x) else x.shape
    ys = y.shape[1:] if _is_planes(y) else y.shape
    N, H, W, ldx = xs
    _, Ho, Wo, Cout = ys
    if not (isinstance(w3, torch.Tensor) and w3.dtype == torch.int16):
        raise RuntimeError('activation planes need bf16x3 weights (split_bf16x3)')
    rp = 0
    if residual is not None:
        if tuple(residual.shape) != tuple(ys):
            raise RuntimeError('residual shape %s != output %s'
                               % (tuple(residual.shape), tuple(ys)))
        rp = _dev(residual, 'residual')
    if _is_planes(x):
        xp, x3, xpl = 0, _dev(x, 'x planes', torch.int16), x[0].numel()
    else:
        xp, x3, xpl = _dev(x, 'x'), 0, 0
    if _is_planes(y):
        yp, y3, ypl = 0, _dev(y, 'y planes', torch.int16), y[0].numel()
    else:
        yp, y3, ypl = _dev(y, 'y'), 0, 0
    if splitk > 1:
        M = N * Ho * Wo
        if part is None or part.numel() < splitk * M * Cout:
            raise RuntimeError('split-K needs a partials buffer of >= %d floats'
                               % (splitk * M * Cout))
        if counters is not None:
            call('pps_conv2d_bn_act_x3p_splitk_fused', xp, x3, xpl, N, H, W, cin, ldx,
                 _dev(w3, 'w', torch.int16), Cout, kpad, k, k, stride, pad, dil,
                 _dev(scale, 'scale'), _dev(shift, 'shift'), rp, int(bool(relu)), yp, y3, ypl,
                 Ho, Wo, Cout, int(splitk), _dev(part, 'part'),
                 _dev(counters, 'counters', torch.int32), counters.numel(), int(tile),
                 _stream())
            return y
        call('pps_conv2d_bn_act_x3p_splitk', xp, x3, xpl, N, H, W, cin, ldx,
             _dev(w3, 'w', torch.int16), Cout, kpad, k, k, stride, pad, dil,
             _dev(scale, 'scale'), _dev(shift, 'shift'), rp, int(bool(relu)), yp, y3, ypl, Ho,
             Wo, Cout, int(splitk), _dev(part, 'part'), int(tile), _stream())
        return y
    call('pps_conv2d_bn_act_x3p', xp, x3, xpl, N, H, W, cin, ldx, _dev(w3, 'w', torch.int16),
         Cout, kpad, k, k, stride, pad, dil, _dev(scale, 'scale'), _dev(shift, 'shift'), rp,
         int(bool(relu)), yp, y3, ypl, Ho, Wo, Cout, int(tile), _stream())
    return y


def conv1x1_seam(x, w2c3, scale2c, shift2c, residual, trunk, w2a3, scale2a, shift2a, y):
    """branch2c of an identity bottleneck + branch2a of the next one in one
    launch (pps_conv1x1_seam_x3): trunk = relu(x . w2c * s + t + residual),
    y = relu(trunk . w2a * s + t); x [..., K1], trunk / residual [..., N1],
    y [..., N2] NHWC f32, (K1, N1, N2) = (64, 256, 64) or (128, 512, 128);
    w2c3 / w2a3 bf16x3 planes of the packed [Cout][Kpad] weights.  Same bits
    as the two convolutions on a 16x16x32-block tile."""
    K1, N1, N2 = x.shape[-1], trunk.shape[-1], y.shape[-1]
    M = x.numel() // K1
    if residual.shape != trunk.shape or y.numel() // N2 != M or trunk.numel() // N1 != M:
        raise RuntimeError('seam shapes: x %s, residual %s, trunk %s, y %s'
                           % (tuple(x.shape), tuple(residual.shape), tuple(trunk.shape),
                              tuple(y.shape)))
    call('pps_conv1x1_seam_x3', _dev(x, 'x'), M, K1, _dev(w2c3, 'w2c', torch.int16), N1,
         _dev(scale2c, 'scale2c'), _dev(shift2c, 'shift2c'), _dev(residual, 'residual'),
         _dev(trunk, 'trunk'), _dev(w2a3, 'w2a', torch.int16), N2, _dev(scale2a, 'scale2a'),
         _dev(shift2a, 'shift2a'), _dev(y, 'y'), _stream())
    return trunk, y


def conv2d_dual_bn_act(x, cin, k, stride, pad, x2, stride2, w, kpad1, shift, relu, y,
                       tile=0):
    """relu?(conv_k(x) + conv_1x1/stride2(x2) + shift), BN scales folded in w."""
    N, H, W, ldx = x.shape
    _, H2, W2, C2 = x2.shape
    _, Ho, Wo, Cout = y.shape
    fn, wp = _weights('pps_conv2d_dual_bn_act', w)
    call(fn, _dev(x, 'x'), N, H, W, cin, ldx, k, k, stride, pad,
         _dev(x2, 'x2'), H2, W2, C2, C2, stride2, wp, Cout, kpad1, C2,
         _dev(shift, 'shift'), int(bool(relu)), _dev(y, 'y'), Ho, Wo, Cout, int(tile),
         _stream())
    return y


# ---- f16x2 convolutions (include/pps_abi.h "f16x2 convolutions") ----------
def split_weights_h2(w_packed):
    """Packed [Cout, Kpad] f32 conv weights (Kpad % 32 == 0) -> (w2t, wrs):
    the two chunk-tiled f16 planes [2, Cout16, Kpad] (int16) and the
    per-output-channel inverse scales [Cout] the f16x2 conv entries take."""
    planes, rs, _ = split_h2_tiled(w_packed.contiguous())
    return planes, rs


AMAX_SLOT_FLOATS = 1024   # pps_abi.h PPS_AMAX_SLOT_FLOATS: 16 partial maxima, 64 apart


def amax_slot(device='cuda'):
    """A zeroed activation-max slot (the f16x2 entries' amax_x / amax_y)."""
    return torch.zeros((AMAX_SLOT_FLOATS,), dtype=torch.float32, device=device)


def amax_value(slot):
    """The tensor max a slot holds (max of its partial maxima)."""
    return float(slot[::64].max())


def amax(x, out=None):
    """max |x| into an activation-max slot (pps_amax; the slot is zeroed here)."""
    if out is None:
        out = amax_slot(x.device)
    else:
        _amax_arg(out, 'amax')
        out.zero_()
    call('pps_amax', _dev(x, 'x'), x.numel(), _dev(out, 'amax'), _stream())
    return out


def _amax_arg(a, name):
    if a is None:
        return 0
    if a.dtype != torch.float32 or a.numel() < AMAX_SLOT_FLOATS:
        raise RuntimeError('%s must be an activation-max slot of %d float32 (ops.amax_slot)'
                           % (name, AMAX_SLOT_FLOATS))
    return _dev(a, name)


def split_act_h2(x, amax_x, out=None):
    """f16x2 activation planes [2, *x.shape] (int16 storage) of f32 x with the
    scale of the slot amax_x (pps_split_f16x2_act): what the f16x2 kernels
    split after an f32 fragment read, done once per element."""
    n = x.numel()
    if out is None:
        out = torch.empty((2,) + tuple(x.shape), dtype=torch.int16, device=x.device)
    call('pps_split_f16x2_act', _dev(x, 'x'), n, _amax_arg(amax_x, 'amax_x'),
         _dev(out, 'planes', torch.int16), out[0].numel(), _stream())
    return out


def h2_out_bound(w_packed, scale, shift):
    """(bound_w, bound_b) of a conv whose output is written as f16x2 planes
    (pps_h2_out_bound on the packed f32 weights [Cout, Kpad], BN scale / shift):
    max|y| <= bound_w * max|x| + bound_b."""
    Cout, Kpad = w_packed.shape
    out = (_lib.ctypes.c_float * 2)()
    call('pps_h2_out_bound', _dev(w_packed.contiguous(), 'w'), Cout, Kpad,
         _dev(scale, 'scale') if scale is not None else 0, _dev(shift, 'shift'), out, _stream())
    return float(out[0]), float(out[1])


def conv2d_bn_act_h2out(x, cin, w, wrs, kpad, k, stride, pad, dil, scale, shift, y2, amax_x,
                        bound_in, bound, bound_out, tile=0):
    """Conv + BN + ReLU whose output y2 [2, N, Ho, Wo, Cout] (int16) is f16x2
    planes on the scale of the bound bound[0] * max|x| + bound[1] (max|x| from
    the slot bound_in, `bound` from h2_out_bound), the bound written to the slot
    bound_out (pps_conv2d_bn_act_h2out).  w: bf16x3 planes [3, Cout, Kpad] with
    wrs None, or split_weights_h2 output with its wrs (then x may be f16x2
    planes, and amax_x is the f16x2 input slot)."""
    planes = _h2_planes(x)
    N, H, W, ldx = x.shape[1:] if planes else x.shape
    _, _, Ho, Wo, Cout = y2.shape
    call('pps_conv2d_bn_act_h2out', 0 if planes else _dev(x, 'x'),
         _dev(x, 'x planes', torch.int16) if planes else 0, x.stride(0) if planes else 0,
         N, H, W, cin, ldx, _dev(w, 'w', torch.int16), _dev(wrs, 'wrs') if wrs is not None else 0,
         Cout, kpad, k, k, stride, pad, dil, _dev(scale, 'scale'), _dev(shift, 'shift'),
         _dev(y2, 'y2', torch.int16), y2.stride(0), Ho, Wo, Cout,
         _amax_arg(amax_x, 'amax_x') if amax_x is not None else 0,
         _amax_arg(bound_in, 'bound_in'), float(bound[0]), float(bound[1]),
         _amax_arg(bound_out, 'bound_out'), int(tile), _stream())
    return y2


def _h2_planes(x):
    """x is f16x2 activation planes [2, N, H, W, C] (split_act_h2)?"""
    return x.dtype == torch.int16 and x.dim() == 5 and x.shape[0] == 2


def conv2d_bn_act_h2(x, cin, w2, wrs, kpad, k, stride, pad, dil, scale, shift, residual, relu, y,
                     amax_x, amax_y=None, tile=0):
    """conv2d_bn_act in f16x2 arithmetic (pps_conv2d_bn_act_h2): w2 / wrs from
    split_weights_h2, amax_x = max|x| as a device float (amax() or the
    producer's amax_y), amax_y (optional, zeroed by the caller) receives
    max|y|.  x may be f16x2 activation planes (split_act_h2 with amax_x;
    pps_conv2d_bn_act_h2_planes, same bits)."""
    planes = _h2_planes(x)
    N, H, W, ldx = x.shape[1:] if planes else x.shape
    _, Ho, Wo, Cout = y.shape
    rp = 0
    if residual is not None:
        if tuple(residual.shape) != tuple(y.shape):
            raise RuntimeError('residual shape %s != output %s'
                               % (tuple(residual.shape), tuple(y.shape)))
        rp = _dev(residual, 'residual')
    rest = (N, H, W, cin, ldx, _dev(w2, 'w2t', torch.int16), _dev(wrs, 'wrs'), Cout, kpad, k, k,
            stride, pad, dil, _dev(scale, 'scale'), _dev(shift, 'shift'), rp, int(bool(relu)),
            _dev(y, 'y'), Ho, Wo, Cout, _amax_arg(amax_x, 'amax_x'), _amax_arg(amax_y, 'amax_y'),
            int(tile), _stream())
    if planes:
        call('pps_conv2d_bn_act_h2_planes', _dev(x, 'x planes', torch.int16), x.stride(0), *rest)
    else:
        call('pps_conv2d_bn_act_h2', _dev(x, 'x'), *rest)
    return y


def conv2d_dual_bn_act_h2(x, cin, k, stride, pad, x2, stride2, w2, wrs, kpad1, shift, relu, y,
                          amax_x, amax_x2, amax_y=None, tile=0):
    """conv2d_dual_bn_act in f16x2 arithmetic (pps_conv2d_dual_bn_act_h2)."""
    N, H, W, ldx = x.shape
    _, H2, W2, C2 = x2.shape
    _, Ho, Wo, Cout = y.shape
    call('pps_conv2d_dual_bn_act_h2', _dev(x, 'x'), N, H, W, cin, ldx, k, k, stride, pad,
         _dev(x2, 'x2'), H2, W2, C2, C2, stride2, _dev(w2, 'w2t', torch.int16), _dev(wrs, 'wrs'),
         Cout, kpad1, C2, _dev(shift, 'shift'), int(bool(relu)), _dev(y, 'y'), Ho, Wo, Cout,
         _amax_arg(amax_x, 'amax_x'), _amax_arg(amax_x2, 'amax_x2'), _amax_arg(amax_y, 'amax_y'),
         int(tile), _stream())
    return y


def conv2d_bn_act_pps_h2(x, cin, w2, wrs, kpad, k, stride, pad, dil, scale, shift, residual,
                         split, max_ave, pps_out, amax_x, y=None, tile=0):
    """conv2d_bn_act_pps in f16x2 arithmetic (pps_conv2d_bn_act_pps_h2); x may
    be f16x2 activation planes (pps_conv2d_bn_act_pps_h2_planes)."""
    planes = _h2_planes(x)
    N, H, W, ldx = x.shape[1:] if planes else x.shape
    nsub, n2, Cout = pps_out.shape
    split = np.ascontiguousarray(split, dtype=np.int32)
    Ho = (H + 2 * pad - dil * (k - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (k - 1) - 1) // stride + 1
    if nsub != (1 << len(split)) - 1 or n2 != N:
        raise RuntimeError('pps_out must be [2^S - 1, N, Cout]')
    rest = (N, H, W, cin, ldx, _dev(w2, 'w2t', torch.int16), _dev(wrs, 'wrs'), Cout, kpad, k, k,
            stride, pad, dil, _dev(scale, 'scale'), _dev(shift, 'shift'),
            _dev(residual, 'residual'), _dev(y, 'y') if y is not None else 0, Ho, Wo,
            split.ctypes.data_as(_lib.ctypes.c_void_p), len(split), int(bool(max_ave)),
            _dev(pps_out, 'pps_out'), _amax_arg(amax_x, 'amax_x'), int(tile), _stream())
    if planes:
        call('pps_conv2d_bn_act_pps_h2_planes', _dev(x, 'x planes', torch.int16), x.stride(0),
             *rest)
    else:
        call('pps_conv2d_bn_act_pps_h2', _dev(x, 'x'), *rest)
    return pps_out


def gemm_bn_act_batched(x, w, scale, shift, relu, y, tile=0):
    """x [B,M,K], w [B,Cout,K] -> y [M, B*Cout] (PPS head convs)."""
    B, M, K = x.shape
    Cout = w.shape[1]
    call('pps_gemm_bn_act_batched', _dev(x, 'x'), M * K, M, K, _dev(w, 'w'), Cout * K,
         Cout, _dev(scale, 'scale'), _dev(shift, 'shift'), int(bool(relu)), _dev(y, 'y'),
         y.stride(0), B, int(tile), _stream())
    return y


def gemm_splitk_batched(x, w, splitk, part, tile=0):
    """x [B,M,K], w [B,Cout,K] (f32) or [B,3,Cout,K] (bf16x3 planes) -> raw
    partials part [splitk, M, B*Cout]."""
    B, M, K = x.shape
    Cout = w.shape[-2]
    fn, wp = _weights('pps_gemm_splitk_batched', w)
    call(fn, _dev(x, 'x'), M, K, wp, Cout, B, splitk, _dev(part, 'part'), int(tile),
         _stream())
    return part


def splitk_bn_act_normalize(part, scale, shift, relu, normalize, y):
    S, M, N = part.shape
    call('pps_splitk_bn_act_normalize', _dev(part, 'part'), S, M, N, _dev(scale, 'scale'),
         _dev(shift, 'shift'), int(bool(relu)), int(bool(normalize)), _dev(y, 'y'), _stream())
    return y


STEM_WIDTH = 128  # input width the fused stem kernel takes (stem.hip kStemW)


def stem_k():
    return _lib.lib().pps_stem_k()


def stem_variant(v=-1):
    """Select the fused stem kernel (0: ring-staged, the default; 1: whole
    tile staged with an LDS epilogue); returns the previous choice, v < 0
    only queries.  Both give identical bits."""
    return _lib.lib().pps_stem_variant(int(v))


def stem_conv_pool_x3(x, w3, scale, shift, y):
    """Fused conv1 7x7/2 + BN + ReLU + maxpool 3x3/2 (pps_stem_conv_pool_x3):
    x NHWC4 [N, H, 128, 4] -> y NHWC [N, Hp, 32, 64]; w3 = split_bf16x3 of
    model.pack_stem_weight."""
    N, H, W, C = x.shape
    _, Hp, Wp, Co = y.shape
    if C != 4 or Co != 64 or tuple(w3.shape) != (3, 64, stem_k()):
        raise RuntimeError('stem: x must be NHWC4, y 64 channels, w3 [3, 64, %d]' % stem_k())
    call('pps_stem_conv_pool_x3', _dev(x, 'x'), N, H, W, _dev(w3, 'w3', torch.int16),
         _dev(scale, 'scale'), _dev(shift, 'shift'), _dev(y, 'y'), Hp, Wp, _stream())
    return y


def stem_split_h2(w):
    """The f16x2 split of the packed stem weight [64, stem_k()] f32
    (pps_stem_split_h2): (w2 [2, 64, stem_k()] f16 planes as int16, w_inv [64]
    the per-channel 2^-s)."""
    if tuple(w.shape) != (64, stem_k()):
        raise RuntimeError('stem weight must be [64, %d]' % stem_k())
    w = w.contiguous()
    w2 = torch.empty((2, 64, stem_k()), dtype=torch.int16, device=w.device)
    winv = torch.empty(64, dtype=torch.float32, device=w.device)
    call('pps_stem_split_h2', _dev(w, 'w'), _dev(w2, 'w2', torch.int16), _dev(winv, 'w_inv'),
         _stream())
    return w2, winv


def stem_conv_pool_h2(x, w2, winv, amax_x, scale, shift, y):
    """The fused stem in f16x2 arithmetic (pps_stem_conv_pool_h2): as
    stem_conv_pool_x3, the input split on the scale of its max (amax_x: an
    activation-max slot, e.g. amax(x)), stem_split_h2 weights."""
    N, H, W, C = x.shape
    _, Hp, Wp, Co = y.shape
    if C != 4 or Co != 64 or tuple(w2.shape) != (2, 64, stem_k()):
        raise RuntimeError('stem: x must be NHWC4, y 64 channels, w2 [2, 64, %d]' % stem_k())
    _amax_arg(amax_x, 'amax_x')
    call('pps_stem_conv_pool_h2', _dev(x, 'x'), N, H, W, _dev(w2, 'w2', torch.int16),
         _dev(winv, 'w_inv'), _dev(amax_x, 'amax_x'), _dev(scale, 'scale'), _dev(shift, 'shift'),
         _dev(y, 'y'), Hp, Wp, _stream())
    return y


def maxpool2d(x, k, stride, pad, y):
    N, H, W, C = x.shape
    _, Ho, Wo, _ = y.shape
    call('pps_maxpool2d', _dev(x, 'x'), N, H, W, C, k, stride, pad, _dev(y, 'y'), Ho, Wo,
         _stream())
    return y


def part_power_set(x, split, max_ave, out):
    N, H, W, C = x.shape
    split = np.ascontiguousarray(split, dtype=np.int32)
    call('pps_part_power_set', _dev(x, 'x'), N, H, W, C,
         split.ctypes.data_as(_lib.ctypes.c_void_p), len(split), int(bool(max_ave)),
         _dev(out, 'out'), _stream())
    return out


def group_mean(x, groups):
    """x [N,D] device; groups: list of index lists -> [len(groups), D] means."""
    N, D = x.shape
    offs = np.zeros(len(groups) + 1, np.int32)
    offs[1:] = np.cumsum([len(g) for g in groups])
    mem = np.concatenate([np.asarray(g, np.int32) for g in groups]) if groups else \
        np.zeros(0, np.int32)
    d_offs = torch.from_numpy(offs).to(x.device)
    d_mem = torch.from_numpy(mem).to(x.device)
    out = torch.empty((len(groups), D), dtype=torch.float32, device=x.device)
    call('pps_group_mean', _dev(x, 'x'), D, d_offs.data_ptr(), d_mem.data_ptr(), len(groups),
         out.data_ptr(), _stream())
    return out


ELTWISE = {'Sum': 0, 'Add': 0, 'Max': 1, 'Mean': 2, 'Relu': 3}


def spatial_bn(x, s, b, rm, riv, eps=1e-5, relu=False, y=None):
    """Caffe2 SpatialBN (is_test) over the last (channel) axis of an NHWC /
    [M, C] tensor (pps_spatial_bn)."""
    C = x.shape[-1]
    if y is None:
        y = torch.empty_like(x)
    call('pps_spatial_bn', _dev(x, 'x'), x.numel() // C, C, _dev(s, 's'), _dev(b, 'b'),
         _dev(rm, 'rm'), _dev(riv, 'riv'), float(eps), int(bool(relu)), _dev(y, 'y'),
         _stream())
    return y


def eltwise(op, xs, y=None):
    """Sum / Add / Max / Mean / Relu of same-shape tensors (pps_eltwise)."""
    xs = list(xs)
    for t in xs[1:]:
        if tuple(t.shape) != tuple(xs[0].shape):
            raise RuntimeError('%s: input shapes differ: %s vs %s'
                               % (op, tuple(xs[0].shape), tuple(t.shape)))
    if y is None:
        y = torch.empty_like(xs[0])
    ptrs = (_lib.ctypes.c_void_p * len(xs))(*[_dev(t, 'input %d' % i) for i, t in enumerate(xs)])
    call('pps_eltwise', ptrs, len(xs), xs[0].numel(), ELTWISE[op], _dev(y, 'y'), _stream())
    return y


def global_pool(x, mode, y=None):
    """AveragePool (mode 'ave') / MaxPool ('max') with global_pooling over an
    NHWC tensor -> [N, C].  x may be an H-slice view of a taller NHWC tensor
    (a Split strip): per-image blocks contiguous, image stride x.stride(0)."""
    N, H, W, C = x.shape
    if x.stride(3) != 1 or x.stride(2) != C or x.stride(1) != W * C:
        raise RuntimeError('global_pool needs per-image contiguous NHWC blocks')
    if y is None:
        y = torch.empty((N, C), dtype=torch.float32, device=x.device)
    if not x.is_cuda or x.dtype != torch.float32:
        raise RuntimeError('x must be a float32 device tensor')
    call('pps_global_pool', x.data_ptr(), N, H, W, C, x.stride(0) if N > 1 else H * W * C,
         0 if mode == 'ave' else 1, _dev(y, 'y'), _stream())
    return y


def l2_normalize(x, y=None):
    N, D = x.shape
    if y is None:
        y = torch.empty_like(x)
    call('pps_l2_normalize', _dev(x, 'x'), N, D, _dev(y, 'y'), _stream())
    return y


def preprocess_bgr(img_u8, pixel_means, out_hw, y=None):
    """uint8 BGR [N,Hi,Wi,3] (device) -> NHWC4 float32 [N,Ho,Wo,4]."""
    N, Hi, Wi, C = img_u8.shape
    assert C == 3
    Ho, Wo = out_hw
    if y is None:
        y = torch.empty((N, Ho, Wo, 4), dtype=torch.float32, device=img_u8.device)
    m = np.ascontiguousarray(np.asarray(pixel_means, np.float32).ravel()[:3])
    call('pps_preprocess_bgr', _dev(img_u8, 'img', torch.uint8), N, Hi, Wi,
         m.ctypes.data_as(_lib.ctypes.c_void_p), Ho, Wo, _dev(y, 'y'), _stream())
    return y


# ---------------------------------------------------------------------------
# Operator registry (reference Caffe2 op names): pps_amd/net.py
# ---------------------------------------------------------------------------
def run_op(name, inputs, **args):
    """Look up an operator by its reference (Caffe2) name and run it
    (the registry is net.OPS: every op name of the reference's test net)."""
    from .net import run_op as _run
    return _run(name, inputs, **args)


def preprocess_bgr_ragged(blob_u8, offsets, heights, widths, pixel_means, out_hw, y=None):
    """Ragged batch: blob_u8 flat uint8 device tensor; offsets int64 [N],
    heights/widths int32 [N] device tensors -> NHWC4 float32 [N,Ho,Wo,4]."""
    N = offsets.shape[0]
    Ho, Wo = out_hw
    if y is None:
        y = torch.empty((N, Ho, Wo, 4), dtype=torch.float32, device=blob_u8.device)
    m = np.ascontiguousarray(np.asarray(pixel_means, np.float32).ravel()[:3])
    call('pps_preprocess_bgr_ragged', _dev(blob_u8, 'blob', torch.uint8), N,
         _dev(offsets, 'offsets', torch.int64), _dev(heights, 'heights', torch.int32),
         _dev(widths, 'widths', torch.int32), m.ctypes.data_as(_lib.ctypes.c_void_p), Ho, Wo,
         _dev(y, 'y'), _stream())
    return y
