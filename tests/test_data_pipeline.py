"""NYU data pipeline host side (CPU): the oracle and the host transform API
against the reference's own transforms (golden_data.npz), loadZipToMem's
shuffled rows, decoding and the augmentation draws."""
import random

import numpy as np
import pytest
import torch

from oracle import data as od
from tests.golden.make_golden import _nyu_zip


def test_oracle_matches_reference_transforms(golden):
    from monocular_depth_estimation_amd.data import draw_augment
    g = golden("golden_data.npz")
    for i, sd in enumerate(g["data::seeds"]):
        random.seed(int(sd))
        flip, k = draw_augment(random)
        image, depth = od.augment(g["data::img"][i % 2], g["data::dep"][i % 2], flip, k)
        np.testing.assert_array_equal(image, g[f"data::train{i}::image"])
        np.testing.assert_array_equal(depth, g[f"data::train{i}::depth"])
    image, depth = od.augment(g["data::img"][0], g["data::dep"][0], 0, -1)
    np.testing.assert_array_equal(image, g["data::test::image"])
    np.testing.assert_array_equal(depth, g["data::test::depth"])


def test_host_transforms_match_reference(golden):
    from PIL import Image

    from monocular_depth_estimation_amd import data as md
    g = golden("golden_data.npz")
    for i, sd in enumerate(g["data::seeds"][:6]):
        random.seed(int(sd))
        s = md.getDefaultTrainTransform()({"image": Image.fromarray(g["data::img"][i % 2]),
                                           "depth": Image.fromarray(g["data::dep"][i % 2])})
        np.testing.assert_array_equal(s["image"].numpy(), g[f"data::train{i}::image"])
        np.testing.assert_array_equal(s["depth"].numpy(), g[f"data::train{i}::depth"])
    with pytest.raises(TypeError, match="PIL Image"):
        md.RandomHorizontalFlip()({"image": np.zeros((2, 2, 3)), "depth": None})


def test_load_zip_rows_match_reference(golden, tmp_path, capsys):
    from monocular_depth_estimation_amd.data import loadZipToMem
    g = golden("golden_data.npz")
    path = tmp_path / "CSVdata.zip"
    _nyu_zip(str(path))
    data, train, test = loadZipToMem(str(path))
    assert [",".join(r) for r in train] == list(g["data::zip_train"])
    assert [",".join(r) for r in test] == list(g["data::zip_test"])
    assert "Loaded (12) to train and (5) to validate." in capsys.readouterr().out
    img, dep = __import__("monocular_depth_estimation_amd.data", fromlist=["x"]).decode_sample(data, train[0])
    assert img.shape == (6, 10, 3) and img.dtype == np.uint8 and dep.shape == (6, 10)


def test_draw_augment_follows_reference_sequence():
    """flip draw, swap draw, randint only when swapping (data.py:27,43,45)."""
    from monocular_depth_estimation_amd.data import draw_augment
    r1, r2 = random.Random(3), random.Random(3)
    for _ in range(50):
        flip, k = draw_augment(r1)
        f = r2.random() < 0.5
        kk = r2.randint(0, 5) if r2.random() < 0.5 else -1
        assert (flip, k) == (int(f), kk)


def test_int16_depth_oracle():
    """'I;16' depth: ToTensor's integer path (int16 view, no scaling)."""
    d = np.array([[0, 1000], [40000, 65535]], dtype=np.uint16).view(np.int16)
    img = np.zeros((2, 2, 3), np.uint8)
    _, depth = od.augment(img, d, 1, -1)
    np.testing.assert_array_equal(depth[0], np.array([[1000, 0], [-1, -25536]], np.float32))


def test_gpu_ops_refuse_cpu_tensors():
    from monocular_depth_estimation_amd.data import nyu_augment
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        nyu_augment(torch.zeros(1, 2, 2, 3, dtype=torch.uint8), torch.zeros(1, 2, 2, dtype=torch.uint8),
                    torch.zeros(1, 2, dtype=torch.int32))
