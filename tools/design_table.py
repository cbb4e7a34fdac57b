#!/usr/bin/env python3
"""Print DESIGN.md's measurement table from a directory of bench lines (<name>_bench.json), e.g.
  python tools/design_table.py profiles/r03/configs
HBM figures come from roofline (or roofline.hbm for the issue-bound rows), the issue bound from
roofline.bound / frac when it is not "hbm"."""
import json
import os
import sys


def main(d):
    rows = []
    for f in sorted(os.listdir(d)):
        if not f.endswith("_bench.json"):
            continue
        x = json.loads(open(os.path.join(d, f)).read())
        rf, cb, par = x.get("roofline") or {}, x.get("cpu_baseline") or {}, x.get("parity", {})
        hbm = rf.get("hbm") or rf
        bound = rf.get("bound", "hbm")
        if bound == "hbm":
            issue = "-"
        elif rf.get("frac"):
            issue = "%.3f of %s issue" % (rf["frac"], bound)
        else:
            issue = "%s (no counter pass)" % bound
        cpu = ("%.3g (%s core)" % (cb["value"], cb.get("cores", "?"))) if cb.get("value") else "-"
        rows.append("| %s | %s | %.3g %s | %.3f | %.0f | %.3f | %s | %s | %s |" % (
            f[:-len("_bench.json")], x["config"]["workload"], x["value"], x["unit"],
            x["ms_per_step"], hbm.get("achieved") or 0.0, hbm.get("frac") or 0.0, issue, cpu,
            par.get("bit_exact")))
    print("| workload | shape | value | ms / launch | GB/s | frac of 8 TB/s | issue bound | CPU port "
          "| bit-exact |")
    print("|---|---|---|---|---|---|---|---|---|")
    print("\n".join(rows))


if __name__ == "__main__":
    main(sys.argv[1])
