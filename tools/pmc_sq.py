#!/usr/bin/env python3
"""Per-kernel SQ / LDS counters of a bench.py line, one rocprofv3 --pmc pass per counter group
(each group within one pass's limits: at most 8 SQ_ counters), each pass its own process:

  python tools/pmc_sq.py --out gpurun_out/sq/resolve.json --match k_ap_resolve \
      "--workload apply --dist uniform --steps 3 --warmup 1"

Prints, per matching kernel, the median over its dispatches of every counter and the derived
fractions: WAIT_ANY (parked at s_waitcnt / barrier), WAIT_INST_ANY (issue stalls), ACTIVE_INST_ANY
over WAVE_CYCLES (MI355X_MICROARCH.md: the three are disjoint and sum to WAVE_CYCLES); VALU and
LDS instructions per wave. The tool never touches the GPU itself: rocprofv3 starts each bench.
"""
import argparse
import csv
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GROUPS = [
    "SQ_WAVES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,"
    "SQ_INSTS_VALU,SQ_INSTS_LDS",
    "SQ_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_ACTIVE_INST_VALU,"
    "SQ_ACTIVE_INST_LDS,SQ_INSTS_SALU,GRBM_GUI_ACTIVE",
]


def run_pass(args, counters, d):
    cmd = ["timeout", "-s", "KILL", "400", "rocprofv3", "--pmc", *counters.split(","),
           "--output-format", "csv", "-d", d, "-o", "pmc", "--", sys.executable,
           os.path.join(ROOT, "bench.py"), *args.split(), "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
    if r.returncode:
        print(f"pmc {counters}: rc {r.returncode}\n{r.stderr[-1500:]}", file=sys.stderr, flush=True)
        return None
    for dp, _, fs in os.walk(d):
        for f in fs:
            if f.endswith("counter_collection.csv"):
                return os.path.join(dp, f)
    print(f"no counter csv under {d}", file=sys.stderr, flush=True)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sets", nargs="+")
    ap.add_argument("--out", required=True)
    ap.add_argument("--match", default="", help="comma list of kernel-name substrings")
    ap.add_argument("--groups", default="", help="';'-separated counter groups (default: two)")
    a = ap.parse_args()
    groups = a.groups.split(";") if a.groups else GROUPS
    pats = [p for p in a.match.split(",") if p]
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    res = {}
    for i, args in enumerate(a.sets):
        per = {}
        for j, grp in enumerate(groups):
            path = run_pass(args, grp, os.path.join(os.path.dirname(a.out), f"sq{i}_{j}"))
            if path is None:
                per.setdefault("_failed_groups", []).append(grp)
                continue
            vals = {}
            for r in csv.DictReader(open(path)):
                name = r["Kernel_Name"]
                if pats and not any(p in name for p in pats):
                    continue
                vals.setdefault((name, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
            for (name, c), v in vals.items():
                per.setdefault(name[:100], {})[c] = statistics.median(v)
        for name, c in per.items():
            if name.startswith("_"):
                continue
            wc = c.get("SQ_WAVE_CYCLES")
            if wc:
                for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                          "SQ_WAIT_INST_LDS"):
                    if k in c:
                        c["frac_" + k[3:].lower()] = c[k] / wc
            wv = c.get("SQ_WAVES")
            if wv:
                for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM"):
                    if k in c:
                        c[k[3:].lower() + "_per_wave"] = c[k] / wv
        res[args] = per
        json.dump(res, open(a.out, "w"), indent=1)
        print(json.dumps({args: per}), flush=True)


if __name__ == "__main__":
    main()
