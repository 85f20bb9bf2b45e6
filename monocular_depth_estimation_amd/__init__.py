"""MI355X-native (gfx950) dense-depth training hot path.

Mirrors the Python API of LuizGuzzo/Monocular_Depth_Estimation on the path
src/train.py -> GuideDepth -> SSIM + L1 (plus Depth_Loss), with the
bandwidth-bound ops on hand-written HIP kernels (libmde_hip.so, C ABI in
include/mde_abi.h).  Importing the package loads the library and fails
loudly if it has not been built.
"""
import os as _os

# MIOpen compiles each convolution kernel on first use (~3 minutes for
# GuideDepth's ~100 conv configurations on a fresh box).  A kernel cache /
# find-db collected on an MI355X ships next to the package (git-ignored,
# travels with the working tree); use it unless the caller chose their own.
_MIOPEN_DIR = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), ".miopen")
if _os.path.isdir(_MIOPEN_DIR):
    _os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", _os.path.join(_MIOPEN_DIR, "cache"))
    _os.environ.setdefault("MIOPEN_USER_DB_PATH", _os.path.join(_MIOPEN_DIR, "db"))

from . import _abi  # noqa: E402

_abi.load()

from . import functional  # noqa: E402,F401
from .GuideDepth.model.GuideDepth import GuideDepth  # noqa: E402,F401
from .loss import SSIM, SSIML1, Silog_loss_variance  # noqa: E402,F401
from .nn import BatchNorm2d  # noqa: E402,F401
from .utils import AverageMeter, DepthNorm  # noqa: E402,F401

__version__ = "0.1.0"
