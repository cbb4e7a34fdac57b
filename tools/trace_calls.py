#!/usr/bin/env python3
"""Per-call kernel durations from a rocprofv3 kernel trace: for every kernel whose name matches,
the duration of each of its launches in order (us), so the first (table-filling) call of an
apply bench can be told from the steady-state ones.

  python tools/trace_calls.py gpurun_out/x/t_kernel_trace.csv [substring ...]
"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
pats = sys.argv[2:] or ["k_ap"]
d = defaultdict(list)
for r in csv.DictReader(open(path)):
    nm = r["Kernel_Name"]
    if any(p in nm for p in pats):
        d[nm.split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = None
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[:40]:40s} " + " ".join(f"{x:7.1f}" for x in v))
    tot = [a + b for a, b in zip(tot, v)] if tot else list(v)
print(f"{'sum':40s} " + " ".join(f"{x:7.1f}" for x in tot))
