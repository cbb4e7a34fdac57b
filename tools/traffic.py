#!/usr/bin/env python3
"""Summarise a tools/gpu_prof.sh run into profiles/ (the files the judge and bench.py read).

  python tools/traffic.py gpurun_out/prof_r01 --tag r01 [--mode min --groups 65536]

Writes profiles/<tag>/ (the rocprofv3 kernel stats + the PMC counter CSVs of the profiled
kernel) and profiles/traffic_<tag>.json:
  bytes_per_launch = (FETCH_SIZE x 2 + WRITE_SIZE) x 1024, averaged over the kernel's dispatches.
FETCH_SIZE / WRITE_SIZE are KiB per dispatch. The x2 on FETCH_SIZE is the gfx950 correction of
MI355X_MICROARCH.md (HBM section): FETCH_SIZE tallies 128-B requests of wide coalesced reads at
64 B. The kernel's loads are 16-B (replies, instance state) and 8-B (keys, values, tables) per
lane, coalesced; the 1-B opcode loads (1/57 of the bytes) are not calibrated separately.
"""
import argparse
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(path, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"]]
    return statistics.mean(vals) if vals else None, len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--kernel", default="k_group_fast")
    ap.add_argument("--mode", default="min")
    ap.add_argument("--groups", type=int, default=65536)
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(a.prof_dir, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, "kernel_stats.csv"))
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if a.kernel in r["Name"]:
            avg_ns = float(r["AverageNs"])
    res = {"kernel": a.kernel, "mode": a.mode, "groups": a.groups, "avg_duration_ns": avg_ns,
           "fetch_correction": 2.0}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(a.prof_dir, f"pmc_{c}", "pmc_counter_collection.csv")
        v, n = pmc(p, a.kernel)
        res[c.lower() + "_kib"] = v
        res[c.lower() + "_dispatches"] = n
        with open(os.path.join(out, f"pmc_{c}.csv"), "w", newline="") as f:
            rows = [r for r in csv.DictReader(open(p)) if a.kernel in r["Kernel_Name"]]
            if rows:
                w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)
    if res["fetch_size_kib"] is not None and res["write_size_kib"] is not None:
        res["bytes_per_launch"] = (res["fetch_size_kib"] * 2 + res["write_size_kib"]) * 1024
    else:
        res["bytes_per_launch"] = None
    bench = os.path.join(a.prof_dir, "bench.log")
    if os.path.exists(bench):
        shutil.copy(bench, os.path.join(out, "bench.log"))
    json.dump(res, open(os.path.join(ROOT, "profiles", f"traffic_{a.tag}.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
