"""CPU oracle of the NYU batch augmentation (test infrastructure only).

Restates src/data.py's per-sample chain for one decoded sample:
RandomHorizontalFlip (:16-31: both maps mirrored), RandomChannelSwap
(:33-46: image channels reordered by permutations(range(3))[k]) and ToTensor
(:100-155: uint8 -> float32 / 255, HWC -> CHW; 'I;16' depth as int16, not
scaled).  Pinned to tests/golden/golden_data.npz (the reference's own
transforms run on seeded `random` draws, tests/golden/make_golden.py).
"""
from __future__ import annotations

from itertools import permutations

import numpy as np

PERMS = list(permutations(range(3), 3))


def augment(img: np.ndarray, dep: np.ndarray, flip: int, k: int):
    """img uint8 [h, w, 3], dep uint8 / int16 [h, w] -> (float32 [3, h, w], float32 [1, h, w])."""
    if flip:
        img = img[:, ::-1]
        dep = dep[:, ::-1]
    if k >= 0:
        img = img[..., list(PERMS[k])]
    image = np.ascontiguousarray(img.transpose(2, 0, 1)).astype(np.float32) / np.float32(255)
    depth = dep.astype(np.float32)[None]
    if dep.dtype == np.uint8:
        depth = depth / np.float32(255)
    return image, np.ascontiguousarray(depth)
