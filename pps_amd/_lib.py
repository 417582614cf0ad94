"""ctypes binding of libpps_hip.so (the C ABI in include/pps_abi.h).

This is the product path's only way to compute: there is no CPU or PyTorch
fallback.  If the shared library is missing, `lib()` raises immediately.
A negative status from any entry point is raised as RuntimeError carrying the
library's ENFORCE-style message, mirroring how Caffe2's CAFFE_ENFORCE surfaced
in Python (reference detectron/tests/test_zero_even_op.py:48-51).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PPS_LIB_PATH: load an alternative build (kernel experiments, scripts/)
LIB_PATH = os.environ.get('PPS_LIB_PATH') or os.path.join(_HERE, 'libpps_hip.so')

c_f32p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_ptr = ctypes.c_void_p

# name -> argtypes (all return int status)
SIGNATURES = {
    'pps_distmat': [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_int, c_int, c_ptr,
                    c_i64, c_int, c_ptr],
    'pps_pairwise_distance': [c_ptr, c_int, c_int, c_ptr, c_ptr],
    'pps_row_sqnorm': [c_ptr, c_i64, c_int, c_i64, c_ptr, c_ptr],
    'pps_split_bf16x3_sqnorm': [c_ptr, c_i64, c_int, c_i64, c_ptr, c_ptr, c_ptr],
    'pps_distmat_x3': [c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_i64, c_int, c_int,
                       c_ptr, c_i64, c_int, c_ptr],
    'pps_distmat_x3p': [c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_i64, c_int, c_int,
                        c_ptr, c_i64, c_int, c_ptr],
    'pps_tile_planes': [c_ptr, c_i64, c_int, c_i64, c_i64, c_ptr, c_ptr],
    'pps_split_bf16x3_sqnorm_tiled': [c_ptr, c_i64, c_int, c_i64, c_ptr, c_ptr, c_ptr],
    'pps_distmat_x3p_tiled': [c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_int, c_int, c_ptr,
                              c_i64, c_int, c_ptr],
    'pps_distmat_x3_self': [c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_int, c_int, c_ptr, c_i64,
                            c_int, c_ptr],
    'pps_distmat_x3_self_tiled': [c_ptr, c_i64, c_ptr, c_int, c_int, c_ptr, c_i64, c_int,
                                  c_ptr],
    'pps_split_f16x2_sqnorm_tiled': [c_ptr, c_i64, c_int, c_i64, c_ptr, c_ptr, c_ptr, c_ptr],
    'pps_distmat_h2_tiled': [c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_int,
                             c_int, c_ptr, c_i64, c_int, c_ptr],
    'pps_distmat_h2_self_tiled': [c_ptr, c_i64, c_ptr, c_ptr, c_int, c_int, c_ptr, c_i64, c_int,
                                  c_ptr],
    'pps_conv2d_bn_act_h2': [c_ptr, c_int, c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_int, c_int,
                             c_int, c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_int, c_ptr,
                             c_int, c_int, c_int, c_ptr, c_ptr, c_int, c_ptr],
    'pps_conv2d_dual_bn_act_h2': [c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_int, c_ptr, c_int, c_int, c_int, c_int, c_int, c_ptr, c_ptr,
                                  c_int, c_int, c_int, c_ptr, c_int, c_ptr, c_int, c_int, c_int,
                                  c_ptr, c_ptr, c_ptr, c_int, c_ptr],
    'pps_conv2d_bn_act_pps_h2': [c_ptr, c_int, c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_int,
                                 c_int, c_int, c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr,
                                 c_ptr, c_int, c_int, c_ptr, c_int, c_int, c_ptr, c_ptr, c_int,
                                 c_ptr],
    'pps_amax': [c_ptr, c_i64, c_ptr, c_ptr],
    'pps_split_f16x2_act': [c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_ptr],
    'pps_h2_out_bound': [c_ptr, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr],
    'pps_conv2d_bn_act_h2out': [c_ptr, c_ptr, c_i64, c_int, c_int, c_int, c_int, c_int, c_ptr,
                                c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ptr,
                                c_ptr, c_ptr, c_i64, c_int, c_int, c_int, c_ptr, c_ptr,
                                ctypes.c_float, ctypes.c_float, c_ptr, c_int, c_ptr],
    'pps_conv2d_bn_act_h2_planes': [c_ptr, c_i64, c_int, c_int, c_int, c_int, c_int, c_ptr,
                                    c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_int, c_int, c_int,
                                    c_ptr, c_ptr, c_int, c_ptr],
    'pps_conv2d_bn_act_pps_h2_planes': [c_ptr, c_i64, c_int, c_int, c_int, c_int, c_int, c_ptr,
                                        c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                        c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_int, c_ptr, c_int,
                                        c_int, c_ptr, c_ptr, c_int, c_ptr],
    'pps_collect_positives': [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr,
                              c_i64, c_int, c_ptr, c_ptr, c_ptr, c_ptr],
    'pps_rank_counts': [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_i64,
                        c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                        c_ptr, c_ptr],
    'pps_collect_matches': [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                            c_i64, c_int, c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_ptr, c_ptr,
                            c_ptr],
    'pps_rank_prepare': [c_int, c_i64, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                         c_ptr],
    'pps_rank_count_stream': [c_ptr, c_i64, c_i64, c_i64, c_i64, c_int, c_ptr, c_ptr, c_ptr,
                              c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr],
    'pps_ap_finalize': [c_i64, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                        c_ptr],
    'pps_topk': [c_ptr, c_i64, c_i64, c_i64, c_int, c_ptr, c_ptr, c_ptr],
    'pps_conv1x1_seam_x3': [c_ptr, c_i64, c_int, c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr,
                            c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr],
    'pps_argsort_rows': [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr],
    'pps_sgs_keys': [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_int, c_ptr,
                     c_ptr],
    'pps_sgs_groups': [c_ptr, c_ptr, c_i64, c_i64, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                       c_ptr],
    'pps_sgs_ranks': [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_int,
                      c_ptr, c_i64, c_ptr, c_ptr],
    'pps_cmc_counts': [c_ptr, c_i64, c_i64, c_i64, c_i64, c_int, c_ptr, c_ptr, c_ptr, c_ptr,
                       c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr],
    'pps_cmc_finalize': [c_i64, c_int, c_ptr, c_ptr, c_int, c_int, c_ptr, c_ptr, c_ptr],
    'pps_topk_merge': [c_ptr, c_ptr, c_int, c_i64, c_int, c_ptr, c_int, c_ptr, c_ptr, c_ptr],
    'pps_conv2d_bn_act': [c_ptr, c_int, c_int, c_int, c_int, c_int, c_ptr, c_int, c_int,
                          c_int, c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_int,
                          c_ptr, c_int, c_int, c_int, c_int, c_ptr],
    'pps_conv2d_dual_bn_act': [c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                               c_int, c_ptr, c_int, c_int, c_int, c_int, c_int, c_ptr,
                               c_int, c_int, c_int, c_ptr, c_int, c_ptr, c_int, c_int,
                               c_int, c_int, c_ptr],
    'pps_gemm_bn_act_batched': [c_ptr, c_i64, c_int, c_int, c_ptr, c_i64, c_int, c_ptr,
                                c_ptr, c_int, c_ptr, c_int, c_int, c_int, c_ptr],
    'pps_gemm_splitk_batched': [c_ptr, c_int, c_int, c_ptr, c_int, c_int, c_int, c_ptr, c_int,
                                c_ptr],
    'pps_split_bf16x3': [c_ptr, c_i64, c_int, c_ptr, c_ptr],
    'pps_conv2d_bn_act_x3': [c_ptr, c_int, c_int, c_int, c_int, c_int, c_ptr, c_int, c_int,
                             c_int, c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_int,
                             c_ptr, c_int, c_int, c_int, c_int, c_ptr],
    'pps_conv2d_bn_act_x3p': [c_ptr, c_ptr, c_i64, c_int, c_int, c_int, c_int, c_int, c_ptr,
                              c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ptr, c_ptr,
                              c_ptr, c_int, c_ptr, c_ptr, c_i64, c_int, c_int, c_int, c_int,
                              c_ptr],
    'pps_conv2d_bn_act_pps_x3p': [c_ptr, c_ptr, c_i64, c_int, c_int, c_int, c_int, c_int,
                                  c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_int, c_ptr, c_int,
                                  c_int, c_ptr, c_int, c_ptr],
    'pps_x3p_tile_shape': [c_int, c_int, c_ptr, c_ptr],
    'pps_conv2d_bn_act_x3p_splitk': [c_ptr, c_ptr, c_i64, c_int, c_int, c_int, c_int, c_int,
                                     c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_ptr, c_i64, c_int,
                                     c_int, c_int, c_int, c_ptr, c_int, c_ptr],
    'pps_conv2d_bn_act_x3p_splitk_fused': [c_ptr, c_ptr, c_i64, c_int, c_int, c_int, c_int,
                                           c_int, c_ptr, c_int, c_int, c_int, c_int, c_int,
                                           c_int, c_int, c_ptr, c_ptr, c_ptr, c_int, c_ptr,
                                           c_ptr, c_i64, c_int, c_int, c_int, c_int, c_ptr,
                                           c_ptr, c_i64, c_int, c_ptr],
    'pps_conv2d_dual_bn_act_x3': [c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_int, c_int, c_ptr, c_int, c_int, c_int, c_int, c_int,
                                  c_ptr, c_int, c_int, c_int, c_ptr, c_int, c_ptr, c_int,
                                  c_int, c_int, c_int, c_ptr],
    'pps_gemm_splitk_batched_x3': [c_ptr, c_int, c_int, c_ptr, c_int, c_int, c_int, c_ptr,
                                   c_int, c_ptr],
    'pps_splitk_bn_act_normalize': [c_ptr, c_int, c_int, c_int, c_ptr, c_ptr, c_int, c_int,
                                    c_ptr, c_ptr],
    'pps_re_ranking': [c_ptr, c_ptr, c_ptr, c_i64, c_i64, c_int, c_int, ctypes.c_double,
                       c_ptr, c_i64, c_ptr, c_ptr],
    'pps_re_ranking_flags': [c_ptr, c_ptr, c_ptr, c_i64, c_i64, c_int, c_int, ctypes.c_double,
                             c_int, c_ptr, c_i64, c_ptr, c_ptr],
    'pps_re_ranking_ld': [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_int, c_int,
                          ctypes.c_double, c_int, c_ptr, c_i64, c_ptr, c_ptr],
    'pps_stem_conv_pool_x3': [c_ptr, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_int,
                              c_int, c_ptr],
    'pps_stem_split_h2': [c_ptr, c_ptr, c_ptr, c_ptr],
    'pps_stem_conv_pool_h2': [c_ptr, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                              c_ptr, c_int, c_int, c_ptr],
    'pps_maxpool2d': [c_ptr, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_ptr,
                      c_int, c_int, c_ptr],
    'pps_part_power_set': [c_ptr, c_int, c_int, c_int, c_int, c_ptr, c_int, c_int, c_ptr,
                           c_ptr],
    'pps_l2_normalize': [c_ptr, c_i64, c_int, c_ptr, c_ptr],
    'pps_group_mean': [c_ptr, c_int, c_ptr, c_ptr, c_int, c_ptr, c_ptr],
    'pps_spatial_bn': [c_ptr, c_i64, c_int, c_ptr, c_ptr, c_ptr, c_ptr, ctypes.c_float, c_int,
                       c_ptr, c_ptr],
    'pps_eltwise': [c_ptr, c_int, c_i64, c_int, c_ptr, c_ptr],
    'pps_global_pool': [c_ptr, c_int, c_int, c_int, c_int, c_i64, c_int, c_ptr, c_ptr],
    'pps_preprocess_bgr': [c_ptr, c_int, c_int, c_int, c_ptr, c_int, c_int, c_ptr, c_ptr],
    'pps_preprocess_bgr_ragged': [c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_int,
                                  c_ptr, c_ptr],
    # whole network (pps_amd/native.py); struct arguments by address
    'pps_model_config_default': [c_ptr],
    'pps_model_create': [c_ptr, c_int, c_ptr, c_ptr],
    'pps_model_destroy': [c_ptr],
    'pps_model_layer_info': [c_ptr, c_int, c_int, c_ptr],
    'pps_model_set_tile': [c_ptr, ctypes.c_char_p, c_int],
    'pps_model_set_splitk': [c_ptr, ctypes.c_char_p, c_int],
    'pps_model_plane_edge': [c_ptr, c_int, c_ptr, c_ptr, c_ptr],
    'pps_model_set_planes': [c_ptr, ctypes.c_char_p, c_int],
    'pps_model_autotune': [c_ptr, c_ptr, c_int, c_int, c_ptr],
    'pps_model_reserve': [c_ptr, c_int],
    'pps_model_release': [c_ptr, c_int],
    'pps_model_tensor': [c_ptr, c_int, ctypes.c_char_p, c_ptr, c_ptr, c_ptr],
    'pps_model_tensor_amax': [c_ptr, c_int, ctypes.c_char_p, c_ptr],
    'pps_forward': [c_ptr, c_ptr, c_int, c_ptr, c_ptr],
    'pps_forward_layers': [c_ptr, c_ptr, c_int, c_ptr, c_int, c_int, c_ptr],
    'pps_forward_layers_flags': [c_ptr, c_ptr, c_int, c_ptr, c_int, c_int, c_int, c_ptr],
    'pps_forward_nchw': [c_ptr, c_ptr, c_int, c_ptr, c_ptr],
    'pps_forward_bgr': [c_ptr, c_ptr, c_int, c_int, c_int, c_ptr, c_ptr],
}
EXTRA = {
    'pps_abi_version': ([], ctypes.c_int),
    'pps_gemm_num_tiles': ([], ctypes.c_int),
    'pps_h2_num_tiles': ([], ctypes.c_int),
    'pps_rank_cells': ([], ctypes.c_int),
    'pps_argsort_rows_cap': ([], ctypes.c_int),
    'pps_stem_k': ([], ctypes.c_int),
    'pps_stem_variant': ([ctypes.c_int], ctypes.c_int),
    'pps_rerank_workspace_bytes': ([c_i64, c_i64, c_int, c_int], ctypes.c_int64),
    'pps_rerank_workspace_bytes_ld': ([c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_int,
                                       c_int, c_int], ctypes.c_int64),
    'pps_last_error': ([], ctypes.c_char_p),
    'pps_registered_ops': ([], ctypes.c_char_p),
    'pps_model_feat_dim': ([c_ptr], ctypes.c_int),
    'pps_model_num_layers': ([c_ptr], ctypes.c_int),
    'pps_model_num_plane_edges': ([c_ptr], ctypes.c_int),
}

METRICS = {'euclidean': 0, 'sqeuclidean': 1, 'cosine': 2}

_LIB = None


def lib():
    """Load (once) and return the configured CDLL. Raises if it is absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            'libpps_hip.so not found at %s: build it with `make` or '
            '`python -c "import __graft_entry__ as g; g.build()"`. There is no '
            'CPU fallback on the product path.' % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    for name, (argtypes, res) in EXTRA.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = res
    _LIB = L
    return L


def call(name, *args):
    """Invoke an entry point; raise RuntimeError on a negative status."""
    L = lib()
    status = getattr(L, name)(*args)
    if status != 0:
        msg = L.pps_last_error().decode('utf-8', 'replace')
        raise RuntimeError('%s failed (status %d): %s' % (name, status, msg))
    return status


def exported_symbols():
    return sorted(list(SIGNATURES) + list(EXTRA))
