"""NYU input-pipeline throughput on a synthetic CSVdata.zip.

    python tools/data_bench.py [--samples 256] [--bs 32] [--workers 8]

Builds a zip shaped like NYU's (640x480 JPEG RGB + 8-bit PNG depth, CSV
rows) in a temp dir, then times
  gpu     NYUBatchLoader: worker decode -> pinned uint8 upload -> mde_nyu_augment
  host    the reference's path: depthDatasetMemory + getDefaultTrainTransform,
          DataLoader(num_workers=0), then .cuda() of the fp32 batch (data.py:171-179,
          train.py:89-90)
and prints one JSON line (images/s each; the training step consumes ~690 img/s
at cfg2).
"""
from __future__ import annotations

import argparse
import io
import json
import os
import sys
import tempfile
import time
import zipfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_zip(path, n, h=480, w=640):
    from PIL import Image
    rng = np.random.default_rng(0)
    base = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    rows = []
    with zipfile.ZipFile(path, "w") as z:
        for i in range(n):
            img = np.roll(base, i, axis=1)
            dep = img[..., 0]
            a, b = f"data/nyu2_train/s/{i}.jpg", f"data/nyu2_train/s/{i}.png"
            bi, bd = io.BytesIO(), io.BytesIO()
            Image.fromarray(img).save(bi, format="JPEG", quality=95)
            Image.fromarray(dep).save(bd, format="PNG")
            z.writestr(a, bi.getvalue())
            z.writestr(b, bd.getvalue())
            rows.append(f"{a},{b}")
        z.writestr("data/nyu2_train.csv", "\n".join(rows) + "\n")
        z.writestr("data/nyu2_test.csv", "\n".join(rows[:8]) + "\n")


def time_epoch(loader):
    """images/s of one whole epoch, from creating the iterator (workers start
    decoding then) to the last batch on the device."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for b in loader:
        n += b["image"].shape[0]
    torch.cuda.synchronize()
    return n / (time.perf_counter() - t0)


def time_batches(it, nbatches):
    it = iter(it)
    next(it)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for _ in range(nbatches):
        n += next(it)["image"].shape[0]
    torch.cuda.synchronize()
    return n / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--host-batches", type=int, default=2)
    a = ap.parse_args()
    from monocular_depth_estimation_amd import data as md
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "CSVdata.zip")
        make_zip(path, a.samples)
        data, train, _ = md.loadZipToMem(path)
        loader = md.NYUBatchLoader(data, train, a.bs, train=True, shuffle=True,
                                   num_workers=a.workers, drop_last=True)
        time_epoch(loader)  # first epoch: worker start-up
        gpu = time_epoch(loader)
        ref = torch.utils.data.DataLoader(md.depthDatasetMemory(data, train, md.getDefaultTrainTransform()),
                                          a.bs, shuffle=True)

        def host_iter():
            for b in ref:
                yield {"image": b["image"].cuda(), "depth": b["depth"].cuda()}
        host = time_batches(host_iter(), a.host_batches)
    print(json.dumps({"metric": "NYU input pipeline images/s (640x480 JPEG+PNG, bs %d)" % a.bs,
                      "gpu_pipeline": round(gpu, 1), "workers": a.workers,
                      "reference_host_path": round(host, 1), "samples": a.samples}), flush=True)


if __name__ == "__main__":
    main()
