from .GuideDepth import GuideDepth  # noqa: F401
from .modules import Guided_Upsampling_Block, SELayer  # noqa: F401
from .DDRNet_23_slim import DualResNet_Backbone  # noqa: F401
