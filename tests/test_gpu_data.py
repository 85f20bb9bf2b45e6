"""NYU batch augmentation on MI355X (mde_nyu_augment) vs the reference's
transforms (golden_data.npz) and the oracle: bit-exact (integer flips /
permutations, IEEE fp32 division by 255)."""
import random

import numpy as np
import pytest
import torch

from oracle import data as od
from tests.golden.make_golden import _nyu_zip

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")


def test_batch_kernel_matches_reference(golden):
    from monocular_depth_estimation_amd.data import draw_augment, nyu_augment
    g = golden("golden_data.npz")
    seeds = g["data::seeds"]
    flags = []
    for sd in seeds:
        random.seed(int(sd))
        flags.append(draw_augment(random))
    n = len(seeds)
    img = torch.from_numpy(np.stack([g["data::img"][i % 2] for i in range(n)])).to(DEV)
    dep = torch.from_numpy(np.stack([g["data::dep"][i % 2] for i in range(n)])).to(DEV)
    image, depth = nyu_augment(img, dep, torch.tensor(flags, dtype=torch.int32).to(DEV))
    for i in range(n):
        np.testing.assert_array_equal(image[i].cpu().numpy(), g[f"data::train{i}::image"])
        np.testing.assert_array_equal(depth[i].cpu().numpy(), g[f"data::train{i}::depth"])


@pytest.mark.parametrize("bits", [8, 16])
def test_full_size_batch_vs_oracle(bits):
    """A cfg2 batch (32 x 480 x 640) with every flip / permutation combination."""
    from monocular_depth_estimation_amd.data import nyu_augment
    rng = np.random.default_rng(bits)
    n, h, w = 32, 480, 640
    img = rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)
    dep = (rng.integers(0, 256, (n, h, w), dtype=np.uint8) if bits == 8
           else rng.integers(0, 65536, (n, h, w), dtype=np.uint16).view(np.int16))
    flags = np.array([(i % 2, (i // 2) % 7 - 1) for i in range(n)], dtype=np.int32)
    image, depth = nyu_augment(torch.from_numpy(img).to(DEV), torch.from_numpy(dep).to(DEV),
                               torch.from_numpy(flags).to(DEV))
    image, depth = image.cpu().numpy(), depth.cpu().numpy()
    for i in range(n):
        ri, rd = od.augment(img[i], dep[i], int(flags[i, 0]), int(flags[i, 1]))
        np.testing.assert_array_equal(image[i], ri)
        np.testing.assert_array_equal(depth[i], rd)


def test_loader_end_to_end(tmp_path):
    """Zip -> worker decode -> pinned uint8 upload -> GPU augment, against the
    oracle applied to the same rows with the same draws."""
    from monocular_depth_estimation_amd.data import NYUBatchLoader, decode_sample, loadZipToMem
    path = tmp_path / "CSVdata.zip"
    _nyu_zip(str(path))
    data, train, test = loadZipToMem(str(path))
    loader = NYUBatchLoader(data, train, batch_size=5, train=True, shuffle=True, num_workers=2,
                            rng=random.Random(0))
    seen = 0
    for batch in loader:
        assert batch["image"].is_cuda and batch["image"].dtype == torch.float32
        torch.cuda.synchronize()
        for j, idx in enumerate(loader.last_indices.tolist()):
            img, dep = decode_sample(data, train[idx])
            f, k = loader.last_flags[j].tolist()
            ri, rd = od.augment(img, dep, f, k)
            np.testing.assert_array_equal(batch["image"][j].cpu().numpy(), ri)
            np.testing.assert_array_equal(batch["depth"][j].cpu().numpy(), rd)
            seen += 1
    assert seen == len(train)
    tl = NYUBatchLoader(data, test, batch_size=4, train=False, shuffle=False, num_workers=0)
    b = next(iter(tl))
    img, dep = decode_sample(data, test[0])
    ri, _ = od.augment(img, dep, 0, -1)
    np.testing.assert_array_equal(b["image"][0].cpu().numpy(), ri)


def test_train_cli_on_nyu_zip(tmp_path):
    """The drop-in train.py CLI with --data: one epoch over a miniature zip
    (64 x 96 RGB + 8-bit depth), checkpoint written."""
    from monocular_depth_estimation_amd.train import main
    path = tmp_path / "CSVdata.zip"
    _nyu_zip(str(path), n_train=8, n_test=2, h=64, w=96)
    ckpt = tmp_path / "ckpt.pth"
    main(["--epochs", "1", "--bs", "4", "--data", str(path), "--workers", "0",
          "--checkpoint", str(ckpt)])
    state = torch.load(str(ckpt), map_location="cpu", weights_only=True)
    assert state["epoch"] == 0 and "model_state_dict" in state
    assert bool(torch.isfinite(state["loss"]).all())
