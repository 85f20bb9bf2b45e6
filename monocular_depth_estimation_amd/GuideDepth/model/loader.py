"""Model builder by name (mirror of src/GuideDepth/model/loader.py:6-22)."""
from __future__ import annotations

from .GuideDepth import GuideDepth

_CONFIGS = {
    "GuideDepth": dict(up_features=[64, 32, 16], inner_features=[64, 32, 16]),
    "GuideDepth-S": dict(up_features=[32, 8, 4], inner_features=[32, 8, 4]),
}


def model_builder(model_name, pretrained=True):
    """Build 'GuideDepth' or 'GuideDepth-S'.

    The reference prints and exit(0)s on an unknown name; a library must not
    exit the interpreter, so this raises ValueError instead.
    """
    if model_name not in _CONFIGS:
        raise ValueError(f"Invalid model {model_name!r}; choose one of {sorted(_CONFIGS)}")
    return GuideDepth(pretrained, **_CONFIGS[model_name])


def load_model(model_name, weights_pth, device="cuda"):
    """Build and load a {'model': state_dict} or plain state_dict checkpoint (weights_only)."""
    import torch
    model = model_builder(model_name, pretrained=False)
    if weights_pth is not None:
        state = torch.load(weights_pth, map_location="cpu", weights_only=True)
        if isinstance(state, dict) and "model" in state:
            state = state["model"]
        model.load_state_dict(state)
    return model.to(device)
