"""NYU-Depth-V2 input pipeline of src/data.py on MI355X.

Reference (src/data.py): the CSV-in-zip is read whole into memory
(loadZipToMem :48-74), samples are PIL-decoded one at a time in the training
process (depthDatasetMemory :77-98, DataLoader with num_workers=0 :179) and
each sample is flipped / channel-swapped / converted to fp32 on the host
(:16-46, :100-168), then copied to the GPU as fp32 (train.py:89-90).

Here:
  * loadZipToMem / loadTest / depthDatasetMemory and the transform classes
    keep the reference's names, return values and TypeErrors (host API);
  * NYUBatchLoader decodes in DataLoader worker processes to uint8 arrays
    only, draws each sample's flip / channel-swap decision in the main process
    with the reference's `random` call sequence (so seeding `random`
    reproduces the reference's augmentation), copies the uint8 batch
    host -> device from pinned memory on a side stream (4 B per RGB-D pixel
    instead of 16) and runs one HIP kernel (mde_nyu_augment) that flips,
    permutes and converts the whole batch into the fp32 NCHW tensors the
    model takes -- bit-exact with the reference's ToTensor.
  * getTrainingTestingData / getTestingData return NYUBatchLoaders yielding
    {'image': cuda [n,3,h,w], 'depth': cuda [n,1,h,w]} (the reference's
    `.cuda()` on them is a no-op).
"""
from __future__ import annotations

import random
from io import BytesIO
from itertools import permutations

import numpy as np
import torch
from PIL import Image
from torch.utils.data import DataLoader, Dataset

from . import _abi
from .functional import _gpu

_PERMS = list(permutations(range(3), 3))


def _pil(x) -> bool:
    return isinstance(x, Image.Image)


def _ndarray_image(x) -> bool:
    return isinstance(x, np.ndarray) and x.ndim in (2, 3)


def _require_pil(sample, what):
    """Both entries of a sample must be PIL images (TypeError otherwise, as the
    reference transforms raise)."""
    for key in ("image", "depth"):
        if not _pil(sample[key]):
            raise TypeError(f"{what}: sample[{key!r}] must be a PIL Image, got {type(sample[key])}")
    return sample["image"], sample["depth"]


# ------------------------------------------------------------------ host API
class RandomHorizontalFlip:
    """data.py:16-31 (host, PIL): one random.random() draw per sample; < 0.5
    mirrors image and depth together."""

    def __call__(self, sample):
        image, depth = _require_pil(sample, "RandomHorizontalFlip")
        flip = random.random() < 0.5
        if flip:
            image, depth = (im.transpose(Image.FLIP_LEFT_RIGHT) for im in (image, depth))
        return {"image": image, "depth": depth}


class RandomChannelSwap:
    """data.py:33-46 (host, PIL): a random.random() draw against `probability`,
    then (only when it hits) a random.randint over the 6 RGB permutations."""

    def __init__(self, probability):
        self.probability = probability
        self.indices = list(_PERMS)

    def __call__(self, sample):
        image, depth = _require_pil(sample, "RandomChannelSwap")
        if random.random() < self.probability:
            perm = self.indices[random.randint(0, len(self.indices) - 1)]
            image = Image.fromarray(np.asarray(image)[..., list(perm)])
        return {"image": image, "depth": depth}


class ToTensor:
    """data.py:100-155 (host): uint8 -> float / 255, CHW; 'I' / 'I;16' keep their integers."""

    def __init__(self, is_test=False):
        self.is_test = is_test

    def __call__(self, sample):
        return {"image": self.to_tensor(sample["image"]),
                "depth": self.to_tensor(sample["depth"]).float()}

    def to_tensor(self, pic):
        if not (_pil(pic) or _ndarray_image(pic)):
            raise TypeError("pic should be PIL Image or ndarray. Got {}".format(type(pic)))
        if isinstance(pic, np.ndarray):
            return torch.from_numpy(pic.transpose((2, 0, 1))).float().div(255)
        a = _pil_array(pic)
        t = torch.from_numpy(a.reshape(pic.size[1], pic.size[0], -1).copy())
        t = t.permute(2, 0, 1).contiguous()
        return t.float().div(255) if t.dtype == torch.uint8 else t


class _Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, sample):
        for t in self.transforms:
            sample = t(sample)
        return sample


def getNoTransform(is_test=False):  # noqa: N802  (reference name)
    return _Compose([ToTensor(is_test=is_test)])


def getDefaultTrainTransform():  # noqa: N802  (reference name)
    return _Compose([RandomHorizontalFlip(), RandomChannelSwap(0.5), ToTensor()])


def _read_zip(zip_file):
    from zipfile import ZipFile
    z = ZipFile(zip_file)
    return {name: z.read(name) for name in z.namelist()}


def _csv_rows(blob: bytes):
    return list(row.split(",") for row in blob.decode("utf-8").split("\n") if len(row) > 0)


def loadZipToMem(zip_file):  # noqa: N802  (reference name)
    """data.py:48-74: every member in memory, train / test rows shuffled (random_state=0)."""
    from sklearn.utils import shuffle
    print("Loading dataset zip file...", end="")
    data = _read_zip(zip_file)
    nyu2_train = shuffle(_csv_rows(data["data/nyu2_train.csv"]), random_state=0)
    nyu2_test = shuffle(_csv_rows(data["data/nyu2_test.csv"]), random_state=0)
    print("Loaded ({0}) to train and ({1}) to validate.".format(len(nyu2_train), len(nyu2_test)))
    return data, nyu2_train, nyu2_test


def loadTest(zip_file):  # noqa: N802  (reference name)
    """data.py:186-200."""
    from sklearn.utils import shuffle
    print("Loading TEST zip file...", end="")
    data = _read_zip(zip_file)
    nyu2_test = shuffle(_csv_rows(data["data/nyu2_test.csv"]), random_state=0)
    print("Loaded ({}) to test.".format(len(nyu2_test)))
    return data, nyu2_test


class depthDatasetMemory(Dataset):  # noqa: N801  (reference name)
    """data.py:77-98: PIL samples, the reference's transform applied when given."""

    def __init__(self, data, nyu2_train, transform=None):
        self.data, self.nyu_dataset = data, nyu2_train
        self.transform = transform

    def __getitem__(self, idx):
        sample = self.nyu_dataset[idx]
        image = Image.open(BytesIO(self.data[sample[0]]))
        depth = Image.open(BytesIO(self.data[sample[1]]))
        sample = {"image": image, "depth": depth}
        if self.transform:
            sample = self.transform(sample)
        return sample

    def __len__(self):
        return len(self.nyu_dataset)


# ------------------------------------------------------------------ GPU path
def _pil_array(pic) -> np.ndarray:
    """Raw pixels as ToTensor reads them: uint8 for 8-bit modes, int32 for 'I',
    int16 for 'I;16' (the reference views the uint16 PNG as np.int16)."""
    if pic.mode == "I":
        return np.array(pic, np.int32)
    if pic.mode == "I;16":
        return np.array(pic, np.uint16).view(np.int16)
    return np.frombuffer(pic.tobytes(), dtype=np.uint8)


def decode_sample(data, row):
    """(image uint8 [h, w, 3], depth uint8 [h, w] or int16 [h, w]) of one CSV row."""
    image = Image.open(BytesIO(data[row[0]]))
    depth = Image.open(BytesIO(data[row[1]]))
    if image.mode != "RGB":
        raise TypeError(f"NYU images are RGB, got mode {image.mode!r} ({row[0]})")
    img = _pil_array(image).reshape(image.size[1], image.size[0], 3)
    if depth.mode == "L":
        dep = _pil_array(depth).reshape(depth.size[1], depth.size[0])
    elif depth.mode == "I;16":
        dep = _pil_array(depth).reshape(depth.size[1], depth.size[0])
    else:
        raise TypeError(f"depth PNGs are 'L' or 'I;16', got mode {depth.mode!r} ({row[1]})")
    return img, dep


def draw_augment(rng=random, swap_probability=0.5):
    """One sample's (flip, k) with the reference's draws, in its order:
    RandomHorizontalFlip's random() < 0.5, then RandomChannelSwap's
    random() < p and, when taken, randint(0, 5) (k = -1: no swap)."""
    flip = rng.random() < 0.5
    k = rng.randint(0, len(_PERMS) - 1) if rng.random() < swap_probability else -1
    return int(flip), int(k)


def nyu_augment(image_u8: torch.Tensor, depth_raw: torch.Tensor, flags: torch.Tensor):
    """mde_nyu_augment on device tensors: image [n,h,w,3] uint8, depth [n,dh,dw]
    uint8 or int16, flags int32 [n,2] -> (image [n,3,h,w], depth [n,1,dh,dw]) fp32."""
    _gpu(image_u8, depth_raw, flags)
    n, h, w, c = image_u8.shape
    if c != 3 or image_u8.dtype != torch.uint8 or flags.dtype != torch.int32 or flags.shape != (n, 2):
        raise ValueError("image [n,h,w,3] uint8 and flags int32 [n,2] expected")
    if depth_raw.dim() != 3 or depth_raw.shape[0] != n:
        raise ValueError(f"depth [n,h,w] expected, got {tuple(depth_raw.shape)}")
    bits = {torch.uint8: 8, torch.int16: 16}.get(depth_raw.dtype)
    if bits is None:
        raise TypeError(f"depth dtype {depth_raw.dtype}: uint8 ('L') or int16 ('I;16')")
    dh, dw = depth_raw.shape[1], depth_raw.shape[2]
    img = torch.empty((n, 3, h, w), dtype=torch.float32, device=image_u8.device)
    dep = torch.empty((n, 1, dh, dw), dtype=torch.float32, device=image_u8.device)
    # contiguous copies (if any) stay referenced until the launch is enqueued
    src, draw, flg = image_u8.contiguous(), depth_raw.contiguous(), flags.contiguous()
    _abi.call("mde_nyu_augment", _abi.ptr(src), _abi.ptr(draw), _abi.ptr(flg), _abi.ptr(img),
              _abi.ptr(dep), n, h, w, dh, dw, bits, _abi.stream_of(image_u8))
    return img, dep


class _DecodeDataset(Dataset):
    def __init__(self, data, rows):
        self.data, self.rows = data, rows

    def __len__(self):
        return len(self.rows)

    def __getitem__(self, idx):
        img, dep = decode_sample(self.data, self.rows[idx])
        return idx, img, dep


def _collate(batch):
    idx = torch.tensor([b[0] for b in batch], dtype=torch.int64)
    img = torch.from_numpy(np.stack([b[1] for b in batch]))
    dep = torch.from_numpy(np.stack([b[2] for b in batch]))
    return idx, img, dep


class NYUBatchLoader:
    """Batches of {'image': fp32 [n,3,h,w], 'depth': fp32 [n,1,h,w]} on `device`.

    train=True applies the reference's training augmentation (flip, channel
    swap with p=0.5) with decisions drawn from `rng` (Python's `random` by
    default, as the reference); train=False is getNoTransform.  The decisions
    of the last batch are kept in `last_flags` ([n, 2] int32, CPU) and its
    sample indices (into `rows`) in `last_indices`."""

    def __init__(self, data, rows, batch_size, train=True, shuffle=True, num_workers=4,
                 device="cuda", rng=None, drop_last=False):
        self.train = train
        self.rng = rng if rng is not None else random
        self.device = torch.device(device)
        self.loader = DataLoader(_DecodeDataset(data, rows), batch_size=batch_size, shuffle=shuffle,
                                 num_workers=num_workers, collate_fn=_collate,
                                 pin_memory=self.device.type == "cuda", drop_last=drop_last,
                                 persistent_workers=num_workers > 0)
        self.last_flags = None
        self.last_indices = None
        self._stream = None

    def __len__(self):
        return len(self.loader)

    def _flags(self, n):
        if self.train:
            f = [draw_augment(self.rng) for _ in range(n)]
        else:
            f = [(0, -1)] * n
        return torch.tensor(f, dtype=torch.int32)

    def __iter__(self):
        if self._stream is None and self.device.type == "cuda":
            self._stream = torch.cuda.Stream(device=self.device)
        for idx, img, dep in self.loader:
            flags = self._flags(img.shape[0])
            self.last_flags, self.last_indices = flags, idx
            cur = torch.cuda.current_stream(self.device)
            with torch.cuda.stream(self._stream):
                img_d = img.to(self.device, non_blocking=True)
                dep_d = dep.to(self.device, non_blocking=True)
                flg_d = flags.to(self.device, non_blocking=True)
                image, depth = nyu_augment(img_d, dep_d, flg_d)
            cur.wait_stream(self._stream)
            for t in (image, depth):
                t.record_stream(cur)
            yield {"image": image, "depth": depth}


def getTrainingTestingData(batch_size, zip_file="CSVdata.zip", num_workers=4,  # noqa: N802
                           device="cuda"):
    """data.py:171-179 on the GPU path (train: shuffled + augmented; test: in order)."""
    data, nyu2_train, nyu2_test = loadZipToMem(zip_file)
    return (NYUBatchLoader(data, nyu2_train, batch_size, train=True, shuffle=True,
                           num_workers=num_workers, device=device),
            NYUBatchLoader(data, nyu2_test, batch_size, train=False, shuffle=False,
                           num_workers=num_workers, device=device))


def getTestingData(batch_size, zip_file="testData.zip", num_workers=4, device="cuda"):  # noqa: N802
    """data.py:203-206 (the reference shuffles its test loader; kept)."""
    data, nyu2_test = loadTest(zip_file)
    return NYUBatchLoader(data, nyu2_test, batch_size, train=False, shuffle=True,
                          num_workers=num_workers, device=device)
