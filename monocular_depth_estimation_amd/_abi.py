"""ctypes binding of libmde_hip.so (the C ABI declared in include/mde_abi.h).

This is the only place the shared library is loaded.  There is no fallback:
if the library is missing, or a GPU op is called on a CPU tensor, the call
raises.  torch must be imported first so that the HIP runtime torch ships
(SONAME libamdhip64.so.7) is the one the library binds to — the library then
shares torch's device context and streams.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads torch's libamdhip64 before ours)

# MDE_HIP_LIB: another build of the same library (interleaved A/B runs in tools/).
LIB_PATH = os.environ.get("MDE_HIP_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libmde_hip.so")

MDE_F32 = 0
MDE_BF16 = 1

_c = ctypes
_vp = _c.c_void_p
_i64 = _c.c_int64
_f32 = _c.c_float
_int = _c.c_int
_sz = _c.c_size_t
_fp = _c.POINTER(_c.c_float)

# name -> (restype, argtypes); mirrors include/mde_abi.h exactly.
SIGNATURES = {
    "mde_abi_version": (_int, []),
    "mde_status_string": (_c.c_char_p, [_int]),
    "mde_bilinear_fwd": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _f32, _int, _int, _vp]),
    "mde_bilinear_bwd": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _f32, _int, _int, _vp]),
    "mde_bilinear_bwd2_supported": (_int, [_i64, _i64, _i64, _i64, _i64, _i64, _f32, _f32, _int]),
    "mde_bilinear_bwd2": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _f32, _int,
                                 _int, _vp]),
    "mde_nearest_fwd": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _f32, _int, _vp]),
    "mde_nearest_bwd": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _f32, _f32, _int, _vp]),
    "mde_nearest_pyramid_supported": (_int, [_i64, _i64, _i64, _i64]),
    "mde_nearest_pyramid": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_se_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64]),
    "mde_se_fwd": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                          _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_se_bwd": (_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp,
                          _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_se_bn_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64]),
    "mde_se_bn_fwd": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                             _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_se_bn_bwd": (_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _int, _vp, _vp, _i64,
                             _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp,
                             _int, _vp]),
    "mde_skip_reduce_fwd": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_skip_reduce_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64]),
    "mde_skip_reduce_bwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64,
                                   _vp, _int, _vp]),
    "mde_skip_reduce_bn_supported": (_int, [_i64, _i64, _i64, _i64, _int]),
    "mde_skip_reduce_bn_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64]),
    "mde_skip_reduce_bn_fwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64,
                                      _int, _vp]),
    "mde_skip_reduce_bn_bwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64,
                                      _i64, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_minmax_workspace": (_sz, [_i64]),
    "mde_minmax": (_int, [_vp, _i64, _vp, _vp, _int, _vp]),
    "mde_depthnorm_apply": (_int, [_vp, _vp, _vp, _i64, _int, _vp]),
    "mde_ssim3_l1_workspace": (_sz, [_i64, _i64, _i64]),
    "mde_ssim3_l1_fwd": (_int, [_vp, _vp, _vp, _f32, _f32, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_depth_loss_workspace": (_sz, [_i64, _i64, _i64]),
    "mde_depth_loss_fwd": (_int, [_vp, _vp, _f32, _f32, _f32, _f32, _vp, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_depth_loss_bwd": (_int, [_vp, _vp, _f32, _f32, _f32, _f32, _vp, _vp, _vp, _i64, _i64, _i64,
                                  _vp, _int, _vp]),
    "mde_batchnorm_workspace": (_sz, [_i64, _i64, _i64, _i64]),
    "mde_batchnorm_fwd_train": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _vp, _vp, _vp,
                                       _vp, _i64, _i64, _i64, _i64, _int, _vp, _int, _vp]),
    "mde_batchnorm_fwd_eval": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp,
                                      _i64, _i64, _i64, _i64, _int, _int, _vp]),
    "mde_batchnorm_bwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _int, _vp, _vp, _vp, _vp, _vp,
                                 _i64, _i64, _i64, _i64, _int, _vp, _int, _vp]),
    "mde_batchnorm_bwd_apply": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _int, _vp, _vp, _vp, _vp,
                                       _vp, _vp, _i64, _i64, _i64, _i64, _int, _int, _vp]),
    "mde_window_attn_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64, _i64]),
    "mde_window_attn_fwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64,
                                   _i64, _int, _vp]),
    "mde_window_attn_bwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64,
                                   _i64, _i64, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_se_gate_fwd": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _int, _vp, _vp, _vp,
                               _vp, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_se_gate_bwd": (_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _int, _vp, _vp, _vp,
                               _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_pointwise_supported": (_int, [_i64, _i64, _i64, _i64]),
    "mde_pointwise_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64]),
    "mde_pointwise_fwd": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_pointwise_bwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64,
                                 _vp, _int, _vp]),
    "mde_pointwise_stats_blocks": (_int, [_i64, _i64, _i64, _i64, _i64]),
    "mde_pointwise_fwd_stats": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64,
                                       _int, _vp]),
    "mde_conv3x3_stats_blocks": (_int, [_i64, _i64, _i64, _i64, _i64, _int]),
    "mde_conv3x3_fwd_stats": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_batchnorm_fwd_train_stats": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _vp,
                                             _vp, _vp, _vp, _i64, _i64, _i64, _i64, _int, _vp,
                                             _i64, _vp, _int, _vp]),
    "mde_batchnorm_fwd_coef_stats": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _vp,
                                            _vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _i64, _vp,
                                            _int, _vp]),
    "mde_pointwise_bwd_bn": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64,
                                    _i64, _i64, _vp, _int, _vp]),
    "mde_batchnorm_fwd_coef": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _int, _vp, _vp,
                                      _vp, _vp, _i64, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_conv3x3_supported": (_int, [_i64, _i64, _int, _int]),
    "mde_conv3x3_fwd": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_conv3x3_bwd_data": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_conv3x3_wgrad_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64, _int]),
    "mde_conv3x3_wgrad": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_conv3x3s2_supported": (_int, [_i64, _i64, _int]),
    "mde_conv3x3s2_wgrad_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64, _int]),
    "mde_conv3x3s2_wgrad": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_dwconv_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64, _i64, _i64]),
    "mde_dwconv_fwd": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_dwconv_bwd": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
                              _vp, _int, _vp]),
    "mde_layernorm_workspace": (_sz, [_i64, _i64]),
    "mde_layernorm_fwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _f32, _int, _vp]),
    "mde_layernorm_bwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _int,
                                 _vp]),
    "mde_layernorm_add_fwd": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _f32,
                                      _int, _vp]),
    "mde_layernorm_bwd_res": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64,
                                      _vp, _int, _vp]),
    "mde_transpose": (_int, [_vp, _vp, _i64, _i64, _i64, _int, _vp]),
    "mde_nyu_augment": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_eval_workspace": (_sz, [_i64, _i64, _i64]),
    "mde_eval_sums": (_int, [_vp, _vp, _i64, _i64, _i64, _f32, _f32, _int, _c.POINTER(_c.c_int32), _vp,
                             _vp, _int, _vp]),
    "mde_colsum_workspace": (_sz, [_i64, _i64]),
    "mde_colsum": (_int, [_vp, _vp, _i64, _i64, _vp, _int, _vp]),
    "mde_head_conv_supported": (_int, [_i64, _i64, _i64, _i64]),
    "mde_head_conv_fwd": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_head_conv_dgrad": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_head_conv_wgrad_workspace": (_sz, [_i64, _i64, _i64, _i64]),
    "mde_head_conv_wgrad": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_chansum_workspace": (_sz, [_i64, _i64, _i64]),
    "mde_chansum": (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_linear_wgrad_workspace": (_sz, [_i64, _i64, _i64]),
    "mde_linear_wgrad": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _int, _vp]),
    "mde_gelu_bwd_colsum": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _vp, _int, _vp]),
    "mde_conv1x1_supported": (_int, [_i64, _i64, _i64, _i64, _int, _int]),
    "mde_conv1x1_fwd": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _int, _vp]),
    "mde_conv1x1_bwd_data": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _int, _vp]),
    "mde_conv1x1_wgrad_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64, _int, _int]),
    "mde_conv1x1_wgrad": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp, _int,
                                 _vp]),
    "mde_conv3x3s2_fwd_supported": (_int, [_i64, _i64, _i64, _i64, _int]),
    "mde_conv3x3s2_dgrad_supported": (_int, [_i64, _i64, _i64, _i64, _int]),
    "mde_conv3x3s2_fwd": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_conv3x3s2_bwd_data": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_conv3x3_wide_supported": (_int, [_i64, _i64, _i64, _i64, _int, _int]),
    "mde_conv3x3_wide_fwd": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_conv3x3_wide_bwd_data": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _vp]),
    "mde_wino_mode": (_int, [_int]),
    "mde_wino_supported": (_int, [_i64, _i64, _i64, _i64, _int]),
    "mde_wino_weight_bytes": (_sz, [_i64, _i64]),
    "mde_wino_weight": (_int, [_vp, _vp, _i64, _i64, _int, _vp]),
    "mde_wino_weight2": (_int, [_vp, _vp, _vp, _i64, _i64, _vp]),
    "mde_wino_weight_blocks": (_i64, [_i64, _i64, _int]),
    "mde_wino_weight_table": (_int, [_vp, _int, _i64, _i64, _vp]),
    "mde_wino_conv": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _int, _vp]),
    "mde_wino_conv_acc": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _int, _vp]),
    "mde_wino_conv_stats": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _int,
                                   _vp]),
    "mde_wino_stats_blocks": (_int, [_i64, _i64, _i64, _i64, _i64]),
    "mde_batchnorm_stats_route": (_int, [_i64, _i64, _i64, _i64, _i64, _int]),
    "mde_bn_chan_mode": (_int, [_int]),
    "mde_convbf_supported": (_int, [_i64, _i64, _i64, _i64, _int, _int, _int]),
    "mde_convbf_supported_n": (_int, [_i64, _i64, _i64, _i64, _i64, _int, _int, _int]),
    "mde_convbf_flops": (_c.c_double, [_i64, _i64, _i64, _i64, _i64, _int, _int, _int]),
    "mde_stem_bf16_supported": (_int, [_i64, _i64, _i64, _i64]),
    "mde_stem_bf16_fwd": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp]),
    "mde_stem_bf16_wgrad_workspace": (_sz, [_i64, _i64, _i64, _i64]),
    "mde_stem_bf16_wgrad": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp]),
    "mde_conv3x3_guide_bf16_wgrad_workspace": (_sz, [_i64, _i64, _i64, _i64]),
    "mde_conv3x3_guide_bf16_wgrad": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp]),
    "mde_convbf_pack_elems": (_sz, [_i64, _i64, _int, _int]),
    "mde_convbf_pack": (_int, [_vp, _vp, _i64, _i64, _int, _int, _vp]),
    "mde_convbf_pack_both": (_int, [_vp, _vp, _vp, _i64, _i64, _int, _vp]),
    "mde_convbf_pack_table": (_int, [_vp, _int, _i64, _i64, _vp]),
    "mde_convbf_stats_blocks": (_int, [_i64, _i64, _i64, _i64, _i64, _int, _int]),
    "mde_convbf_fwd": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _int, _vp]),
    "mde_convbf_bwd_data": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _int, _vp]),
    "mde_convbf_wgrad_workspace": (_sz, [_i64, _i64, _i64, _i64, _i64, _int, _int]),
    "mde_convbf_wgrad": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _int, _int, _vp, _vp]),
    "mde_conv3x3_guide_bf16_stats_blocks": (_int, [_i64, _i64, _i64, _i64]),
    "mde_conv3x3_guide_bf16_fwd": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp]),
    "mde_graph_count_memsets": (_int, [_vp, _c.POINTER(_i64)]),
    "mde_graph_replace_memsets": (_int, [_vp, _c.POINTER(_i64)]),
    "mde_graph_node_counts": (_int, [_vp, _c.POINTER(_i64)]),
    "mde_graph_node_types": (_int, [_vp, _c.POINTER(_i64)]),
    "mde_graph_dot": (_int, [_vp, _c.c_char_p]),
    "mde_timing_enable": (_int, [_int]),
    "mde_timing_reset": (_int, []),
    "mde_timing_collect": (_int, []),
    "mde_kernel_count": (_int, []),
    "mde_kernel_name": (_c.c_char_p, [_int]),
    "mde_timing_query": (_int, [_int, _c.POINTER(_c.c_double), _c.POINTER(_c.c_int64),
                                _c.POINTER(_c.c_double)]),
    "mde_timing_query_flops": (_int, [_int, _c.POINTER(_c.c_double)]),
}


class MdeError(RuntimeError):
    """A non-zero status from libmde_hip.so."""


_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and return the library; raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C monocular_depth_estimation_amd/csrc). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = load().mde_status_string(status).decode()
        raise MdeError(f"{what} failed with status {status}: {msg}")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def query(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))


def ptr(t) -> int | None:
    """Device pointer of a tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_of(t) -> int:
    """Handle of torch's current stream on t's device (the launch stream)."""
    return torch.cuda.current_stream(t.device).cuda_stream


def dtype_code(t) -> int:
    if t.dtype == torch.float32:
        return MDE_F32
    if t.dtype == torch.bfloat16:
        return MDE_BF16
    raise TypeError(f"unsupported dtype {t.dtype} (the HIP kernels take float32)")


# ---------------------------------------------------------------------- graphs
def graph_count_memsets(raw_graph: int) -> int:
    n = ctypes.c_int64()
    check(load().mde_graph_count_memsets(raw_graph, ctypes.byref(n)), "mde_graph_count_memsets")
    return n.value


def graph_node_counts(raw_graph: int) -> dict:
    """Node census of a captured (uninstantiated, keep_graph=True) hipGraph."""
    c = (ctypes.c_int64 * 6)()
    check(load().mde_graph_node_counts(raw_graph, c), "mde_graph_node_counts")
    return dict(zip(("total", "kernel", "memcpy", "memset", "event", "other"), list(c)))


GRAPH_NODE_TYPES = ("kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event",
                    "event_record", "sem_signal", "sem_wait", "mem_alloc", "mem_free",
                    "memcpy_from_symbol", "memcpy_to_symbol", "batch_mem_op", "other")


def graph_node_types(raw_graph: int) -> dict:
    """Nodes per hipGraphNodeType of a captured (uninstantiated) hipGraph, zero
    counts omitted."""
    c = (ctypes.c_int64 * 16)()
    check(load().mde_graph_node_types(raw_graph, c), "mde_graph_node_types")
    return {k: v for k, v in zip(GRAPH_NODE_TYPES, list(c)) if v}


def graph_dot(raw_graph: int, path: str) -> None:
    call("mde_graph_dot", raw_graph, path.encode())


def graph_replace_memsets(raw_graph: int) -> int:
    """Swap the memset nodes of a captured, uninstantiated hipGraph for fill
    kernels (captured memsets are wrong from the second replay on; graph.hip)."""
    n = ctypes.c_int64()
    check(load().mde_graph_replace_memsets(raw_graph, ctypes.byref(n)),
          "mde_graph_replace_memsets")
    return n.value


_DOT_SEQ = [0]


def default_capture_mode() -> str:
    """"thread_local" when a torch.distributed process group is initialised
    (its watchdog thread queries events during our captures), else "global"."""
    import torch.distributed as dist
    return "thread_local" if dist.is_available() and dist.is_initialized() else "global"


def capture_graph(fn, stream, pool=None, capture_error_mode: str | None = None):
    """Capture fn() on `stream` into a torch CUDAGraph, repair its memset nodes
    and instantiate it.  Returns (graph, fn's result, memset nodes replaced).

    Capture mode: "thread_local" once a torch.distributed group exists, else
    "global".  ProcessGroupNCCL's watchdog thread polls the completion event of
    every collective issued eagerly before the capture (the warm-up steps' and
    the per-step BN broadcast's) with hipEventQuery; while ANY thread holds a
    global-mode capture that query fails with hipErrorStreamCaptureUnsupported,
    the watchdog throws and the process aborts (SIGABRT, the round-3/4
    captured-RCCL aborts: gpurun_out/r04w/suite.log).  A thread-local capture
    only restricts the capturing thread, and every GPU call of the step is
    issued from it.

    Diagnostics (environment): MDE_GRAPH_CAPTURE_MODE overrides the capture
    mode, MDE_GRAPH_DOT_DIR dumps every captured graph as
    hipGraphDebugDotPrint output before and after the memset repair."""
    mode = capture_error_mode or os.environ.get("MDE_GRAPH_CAPTURE_MODE") or default_capture_mode()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=stream, pool=pool, capture_error_mode=mode):
        out = fn()
    raw = g.raw_cuda_graph()
    dot_dir = os.environ.get("MDE_GRAPH_DOT_DIR")
    if dot_dir:
        os.makedirs(dot_dir, exist_ok=True)
        _DOT_SEQ[0] += 1
        graph_dot(raw, os.path.join(dot_dir, f"graph{_DOT_SEQ[0]:02d}_captured.dot"))
    g.node_types = graph_node_types(raw)
    n = graph_replace_memsets(raw)
    if dot_dir:
        graph_dot(raw, os.path.join(dot_dir, f"graph{_DOT_SEQ[0]:02d}_repaired.dot"))
    g.node_counts = graph_node_counts(raw)
    g.instantiate()
    return g, out, n


# --------------------------------------------------------------------- timing
def timing_enable(on: bool) -> None:
    call("mde_timing_enable", 1 if on else 0)


def timing_reset() -> None:
    call("mde_timing_reset")


def timing_collect(resolve: bool = True) -> dict:
    """Resolve pending events (resolve=True; once per graph replay when the
    events were captured) and return {kernel: (total_ms, launches, bytes, flops)}."""
    lib = load()
    if resolve:
        check(lib.mde_timing_collect(), "mde_timing_collect")
    out = {}
    for k in range(lib.mde_kernel_count()):
        ms, n, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        check(lib.mde_timing_query(k, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(by)),
              "mde_timing_query")
        fl = ctypes.c_double()
        check(lib.mde_timing_query_flops(k, ctypes.byref(fl)), "mde_timing_query_flops")
        if n.value:
            out[lib.mde_kernel_name(k).decode()] = (ms.value, n.value, by.value, fl.value)
    return out
