"""The C ABI library loads and exports exactly what include/mde_abi.h declares (CPU only).

No compute runs here: argument-validation paths return before any HIP call,
and the workspace queries are host arithmetic.
"""
import ctypes
import os
import re

import pytest

from tests.conftest import REPO

HEADER = os.path.join(REPO, "include", "mde_abi.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(?:int64_t|int|size_t|double|const char\*)\s+(mde_\w+)\s*\(([^)]*)\)\s*;", text):
        args = m.group(2).strip()
        n = 0 if args in ("", "void") else args.count(",") + 1
        decls[m.group(1)] = n
    return decls


def test_header_declares_the_hot_path_ops():
    d = declared_functions()
    for op in ("mde_bilinear_fwd", "mde_bilinear_bwd", "mde_nearest_fwd", "mde_se_fwd",
               "mde_se_bwd", "mde_skip_reduce_fwd", "mde_skip_reduce_bwd", "mde_minmax",
               "mde_ssim3_l1_fwd", "mde_depth_loss_fwd", "mde_depth_loss_bwd"):
        assert op in d


def test_library_exports_every_declared_symbol():
    from monocular_depth_estimation_amd import _abi
    lib = _abi.load()
    d = declared_functions()
    assert d, "no declarations parsed"
    for name, nargs in d.items():
        assert hasattr(lib, name), f"{name} not exported by {_abi.LIB_PATH}"
        assert name in _abi.SIGNATURES, f"{name} missing from the ctypes table"
        assert len(_abi.SIGNATURES[name][1]) == nargs, f"{name}: ctypes arity != header arity"
    assert set(_abi.SIGNATURES) == set(d), "ctypes table and header disagree"


def test_version_and_status_strings():
    from monocular_depth_estimation_amd import _abi
    lib = _abi.load()
    assert lib.mde_abi_version() == 1
    assert lib.mde_status_string(0) == b"ok"
    assert b"invalid" in lib.mde_status_string(-1)
    assert b"unsupported" in lib.mde_status_string(-2)


def test_invalid_arguments_are_rejected_before_launch():
    from monocular_depth_estimation_amd import _abi
    lib = _abi.load()
    assert lib.mde_bilinear_fwd(None, None, 1, 1, 4, 4, 8, 8, 0.5, 0.5, 0, 0, None) == -1
    # bf16 storage: the exact x2 resize has it (null pointers -> invalid), nearest does not
    assert lib.mde_bilinear_fwd(None, None, 1, 1, 4, 4, 8, 8, 0.5, 0.5, 0, 1, None) == -1
    assert lib.mde_nearest_fwd(None, None, 1, 1, 4, 4, 8, 8, 0.5, 0.5, 1, None) == -2
    assert lib.mde_bilinear_fwd(None, None, 1, 1, 4, 4, 8, 8, 0.5, 0.5, 0, 7, None) == -2
    assert lib.mde_nearest_fwd(None, None, 1, 1, 0, 4, 8, 8, 0.5, 0.5, 0, None) == -1
    assert lib.mde_skip_reduce_fwd(None, None, None, None, None, 1, 65, 1, 4, 4, 0, None) == -1
    assert lib.mde_ssim3_l1_fwd(None, None, None, 1.0, 0.1, None, None, None, 1, 1, 8, None, 0,
                                None) == -1
    assert lib.mde_minmax(None, 0, None, None, 0, None) == -1
    # token-major reductions: widths must be multiples of 4, fp32 only
    assert lib.mde_colsum_workspace(100, 6) == 0
    assert lib.mde_colsum_workspace(100, 8) > 0
    assert lib.mde_colsum(None, None, 100, 8, None, 0, None) == -1
    assert lib.mde_gelu_bwd_colsum(None, None, None, None, 100, 8, None, 1, None) == -2
    with pytest.raises(_abi.MdeError, match="invalid argument"):
        _abi.call("mde_depthnorm_apply", None, None, None, 0, 0, None)


def test_workspace_queries():
    from monocular_depth_estimation_amd import _abi
    lib = _abi.load()
    # SE: partial slab per (n, c, 16384-element chunk) + three per-sample vectors
    assert lib.mde_se_workspace(32, 16, 16, 480, 640) >= 4 * 32 * 16 * 19
    # SSIM: one (ssim, l1) pair per block of 4 waves, sized for the larger of
    # the two kernels' plans: the two-column kernel's 108-column strips x
    # 30-row chunks (6 x 16 per 480x640 image) and the one-column kernel's
    # 60-column strips x 30-row chunks (11 x 16)
    assert lib.mde_ssim3_l1_workspace(32, 480, 640) == 4 * 2 * (32 * 11 * 16 // 4)
    assert lib.mde_minmax_workspace(10) >= 8
    assert lib.mde_skip_reduce_workspace(32, 64, 32, 120, 160) >= 4 * (64 * 32 + 32)
    assert lib.mde_depth_loss_workspace(2, 24, 32) >= 4 * 3 * 2 * 24 * 32


def test_timing_registry_names():
    from monocular_depth_estimation_amd import _abi
    lib = _abi.load()
    names = [lib.mde_kernel_name(k).decode() for k in range(lib.mde_kernel_count())]
    assert "bilinear_bwd" in names and "ssim3_l1" in names and len(set(names)) == len(names)
    _abi.timing_reset()
    assert _abi.timing_collect() == {}


def test_convbf_flops_are_algorithmic():
    """The registry prices every convbf pass at the convolution's own MACs over
    the forward output plane -- the stride-2 data gradient too (it used to be
    credited with its full-resolution gx plane: 4x the true count)."""
    from monocular_depth_estimation_amd import _abi
    lib = _abi.load()
    n, cin, cout, h, w = 32, 32, 64, 240, 320
    for ks in (1, 3):
        for stride in (1, 2):
            ho, wo = (h + 2 * (ks // 2) - ks) // stride + 1, (w + 2 * (ks // 2) - ks) // stride + 1
            want = 2.0 * n * ho * wo * cin * cout * ks * ks
            for pass_ in (0, 1, 2):
                assert lib.mde_convbf_flops(n, cin, cout, h, w, ks, stride, pass_) == want, \
                    (ks, stride, pass_)
    assert lib.mde_convbf_flops(n, 30, cout, h, w, 3, 2, 1) == 0.0  # unsupported shape


def test_convbf_supported_at_batch():
    """mde_convbf_supported_n refuses a batch whose launch would be refused
    (n x patches >= 2^22), where the batch-free query still says yes."""
    from monocular_depth_estimation_amd import _abi
    lib = _abi.load()
    args = (64, 64, 60, 80, 3, 1)
    for p in (0, 1, 2):
        assert lib.mde_convbf_supported(*args, p) == 1
        assert lib.mde_convbf_supported_n(32, *args, p) == 1
        assert lib.mde_convbf_supported_n(1 << 22, *args, p) == 0
    assert lib.mde_convbf_supported_n(0, *args, 0) == 0


def test_round6_shape_queries():
    """Host-side shape rules of the round-6 entries (no GPU needed): the Linear
    weight gradient (t % 16, m and n % 128), the per-channel sum (hw % 4), the
    one-output-channel head conv (w % 4), the padded 1x1 / wide-wgrad shapes."""
    from monocular_depth_estimation_amd import _abi
    lib = _abi.load()
    assert lib.mde_linear_wgrad_workspace(307200, 128, 512) > 0
    for t, m, n in ((100, 128, 128), (160, 96, 128), (160, 128, 200), (0, 128, 128)):
        assert lib.mde_linear_wgrad_workspace(t, m, n) == 0
    assert lib.mde_chansum_workspace(16, 128, 19200) > 0
    assert lib.mde_chansum_workspace(16, 128, 19202) == 0
    assert lib.mde_head_conv_supported(16, 128, 120, 160) == 1
    assert lib.mde_head_conv_supported(16, 128, 120, 162) == 0
    assert lib.mde_conv1x1_supported(24, 72, 120, 160, 1, 0) == 1  # MobileNetV3, padded
    assert lib.mde_conv1x1_supported(12, 72, 120, 160, 1, 0) == 0
    assert lib.mde_conv3x3_wgrad_workspace(2, 24, 128, 120, 160, 0) > 0  # padded to 32
    assert lib.mde_conv3x3_wgrad_workspace(2, 24, 128, 120, 48, 0) == 0  # not a strip width
    assert lib.mde_layernorm_workspace(307200, 128) > 0
