"""MI355X-native (gfx950) dense-depth training hot path.

Mirrors the Python API of LuizGuzzo/Monocular_Depth_Estimation on the path
src/train.py -> GuideDepth -> SSIM + L1 (plus Depth_Loss), with the
bandwidth-bound ops on hand-written HIP kernels (libmde_hip.so, C ABI in
include/mde_abi.h).  Importing the package loads the library and fails
loudly if it has not been built.
"""
from . import _abi

_abi.load()

from . import functional  # noqa: E402,F401
from .GuideDepth.model.GuideDepth import GuideDepth  # noqa: E402,F401
from .loss import SSIM, SSIML1, Silog_loss_variance  # noqa: E402,F401
from .utils import AverageMeter, DepthNorm  # noqa: E402,F401

__version__ = "0.1.0"
