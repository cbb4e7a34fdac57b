#!/usr/bin/env python3
"""Per-kernel HBM-side traffic of the apply pipeline from tools/apply_pmc.sh's PMC passes.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (median over the timed calls; the first call fills
the table and runs the two-pass bins). FETCH_SIZE is shown raw and x2 (the gfx950 correction of
MI355X_MICROARCH.md for wide coalesced reads; the gathers and byte loads here are uncalibrated,
so the true figure lies between). Writes a JSON summary next to the CSVs."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]


def load(sub, counter):
    out = {}
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = r["Kernel_Name"].split("(")[0]
            out.setdefault(k, []).append(float(r["Counter_Value"]))
    return out


fe, wr = load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE")
rows, tf, tw = [], 0.0, 0.0
for k in sorted(set(fe) | set(wr)):
    if "k_ap_" not in k and "k_apply" not in k:  # the call's kernels (not export / fill)
        continue
    f = statistics.median(fe.get(k, [0])) * 1024
    w = statistics.median(wr.get(k, [0])) * 1024
    tf += f
    tw += w
    rows.append({"kernel": k, "fetch_raw_B": f, "write_B": w, "calls": len(fe.get(k, []))})
    print(f"{k:28s} fetch {f/1e6:9.1f} MB (x2 {2*f/1e6:9.1f})  write {w/1e6:9.1f} MB")
print(f"{'pipeline':28s} fetch {tf/1e6:9.1f} MB (x2 {2*tf/1e6:9.1f})  write {tw/1e6:9.1f} MB")
json.dump({"kernels": rows, "fetch_raw_B": tf, "fetch_x2_B": 2 * tf, "write_B": tw},
          open(os.path.join(d, "apply_traffic.json"), "w"), indent=1)
