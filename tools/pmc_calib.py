"""Calibration factors of rocprofv3's FETCH_SIZE / WRITE_SIZE per access width.

    python tools/pmc_calib.py DIR_FETCH DIR_WRITE [-o profiles/r03_pmc_calib.json]

DIR_* are the rocprofv3 --pmc output directories of tools/calib/pmc_calib
(one pass per counter).  Every calibration kernel moves a known byte count
once (1 GiB, beyond the Infinity Cache): read_w{4,8,16} read 2^30 bytes,
write_w* write 2^30, copy_w* read and write 2^30 each.  The factor of a
width is true bytes / (counter KiB * 1024), the median over the repetitions:
tools/pmc_traffic.py multiplies each kernel's counter by the factor of the
kernel's access width.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics

GIB = float(1 << 30)


def rows(d, counter):
    out = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") == counter:
                out.append(r)
    return out


def per_kernel(d, counter):
    agg = {}
    for r in rows(d, counter):
        m = re.search(r"(read|write|copy)_kernel<(\d+)>", r["Kernel_Name"])
        if not m:
            continue
        key = f"{m.group(1)}_w{m.group(2)}"
        # one row per dispatch (summed over instances/dimensions when split)
        agg.setdefault(key, {}).setdefault(r.get("Dispatch_Id", r.get("Correlation_Id")), 0.0)
        agg[key][r.get("Dispatch_Id", r.get("Correlation_Id"))] += float(r["Counter_Value"])
    return {k: sorted(v.values()) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("-o", "--out", default="")
    a = ap.parse_args()
    f = per_kernel(a.fetch_dir, "FETCH_SIZE")
    w = per_kernel(a.write_dir, "WRITE_SIZE")
    out = {"fetch": {}, "write": {}, "raw_kib": {"FETCH_SIZE": f, "WRITE_SIZE": w}}
    for k, v in f.items():
        if k.startswith(("read", "copy")):
            out["fetch"][k] = round(GIB / (statistics.median(v) * 1024.0), 4)
    for k, v in w.items():
        if k.startswith(("write", "copy")):
            out["write"][k] = round(GIB / (statistics.median(v) * 1024.0), 4)
    txt = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
