"""Per-kernel PMC traffic / algorithmic bytes for one workload: the bench
JSON's hip_kernels (algorithmic bytes = GBps x ms per launch) against the
FETCH / WRITE traffic file of the same tree (tools/pmc_traffic.py output).

    python tools/traffic_ratios.py profiles/r05_bench_gd_fp32.json profiles/r05_pmc_traffic_guidedepth_fp32.json
"""
import json
import sys


def main():
    bench = json.load(open(sys.argv[1]))
    pmc = json.load(open(sys.argv[2]))
    hk = bench["hip_kernels"]
    rows = []
    for key, t in pmc.items():
        ids = key.split("+")
        algo = sum(hk[i]["GBps"] * 1e9 * hk[i]["ms_total"] * 1e-3 for i in ids if i in hk)
        nl = sum(hk[i]["launches"] for i in ids if i in hk)
        if not nl or not algo:
            continue
        per_launch = algo / nl
        rows.append((key, t["bytes_per_launch"] / per_launch, per_launch, t["bytes_per_launch"],
                     sum(hk[i]["ms_per_step"] for i in ids if i in hk)))
    print(f"{'kernel id':36s} {'traffic/algo':>12s} {'algo MB/launch':>15s} {'PMC MB/launch':>14s} {'ms/step':>8s}")
    for key, r, a, p, ms in sorted(rows, key=lambda x: -x[4]):
        print(f"{key:36s} {r:12.3f} {a / 1e6:15.1f} {p / 1e6:14.1f} {ms:8.3f}")


if __name__ == "__main__":
    main()
