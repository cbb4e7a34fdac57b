#!/usr/bin/env python3
"""Print DESIGN.md's measurement table from a directory of bench lines (<name>_bench.json), e.g.
  python tools/design_table.py profiles/r03/configs
HBM figures come from roofline (or roofline.hbm for the issue-bound rows), the issue bound from
roofline.bound / frac when it is not "hbm"."""
import json
import os
import sys


def bound_label(rf):
    """the table's bound column: '-' for HBM-graded rows; the issue fraction for VALU / LDS-bound
    rows; for latency / issue-stall rows the SQ wave-cycle split that put them there"""
    bound = rf.get("bound", "hbm")
    if bound == "hbm":
        return "-"
    if bound in ("valu", "lds"):
        return ("%.3f of %s issue" % (rf["frac"], bound.upper())) if rf.get("frac") else \
            "%s (no counter pass)" % bound
    w = rf.get("wave_cycle_split") or {}
    if not w:
        return "%s (no counter pass)" % bound
    wa, wi, ac = (w.get(k, 0.0) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))
    bound = "latency" if wa >= max(wi, ac) else "issue-stall" if wi >= ac else "issue (mixed)"
    return "%s: waves parked %.0f %%, issue-stalled %.0f %%, %.1f per CU" % (
        bound, 100 * wa, 100 * wi, w.get("mean_waves_per_cu", 0))


def main(d):
    rows = []
    for f in sorted(os.listdir(d)):
        if not f.endswith("_bench.json"):
            continue
        x = json.loads(open(os.path.join(d, f)).read())
        rf, cb, par = x.get("roofline") or {}, x.get("cpu_baseline") or {}, x.get("parity", {})
        hbm = rf.get("hbm") or rf
        issue = bound_label(rf)
        cpu = ("%.3g (%s core)" % (cb["value"], cb.get("cores", "?"))) if cb.get("value") else "-"
        rows.append("| %s | %s | %.3g %s | %.3f | %.0f | %.3f | %s | %s | %s |" % (
            f[:-len("_bench.json")], x["config"]["workload"], x["value"], x["unit"],
            x["ms_per_step"], hbm.get("achieved") or 0.0, hbm.get("frac") or 0.0, issue, cpu,
            par.get("bit_exact")))
    print("| workload | shape | value | ms / launch | GB/s | frac of 8 TB/s | bound (SQ counters) | "
          "CPU port | bit-exact |")
    print("|---|---|---|---|---|---|---|---|---|")
    print("\n".join(rows))


if __name__ == "__main__":
    main(sys.argv[1])
