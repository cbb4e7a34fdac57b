#!/usr/bin/env python3
"""HBM traffic of bench.py's measured call, per exact configuration, into a counter database
(profiles/traffic_r03.json after copying): for every bench argument set, the line itself (its
roofline.traffic_key / traffic_kernels / launches_in_process), then one rocprofv3 --pmc pass
per counter (FETCH_SIZE, WRITE_SIZE: they do not fit one pass), each in its own process.

  bytes_per_launch = sum over the call's kernels (names matching traffic_kernels) of
                     (FETCH_SIZE x 2 + WRITE_SIZE) x 1024 x (dispatches per launch),
  taking each kernel's median over its dispatches (first-call outliers such as apply's
  table-filling call drop out). FETCH_SIZE x 2 is MI355X_MICROARCH.md's gfx950 correction for
  wide coalesced reads (HBM section); narrower accesses are uncalibrated.

  python tools/pmc_collect.py --out gpurun_out/pmc/traffic.json "--workload tally --mode min" ...
This tool never touches the GPU itself: rocprofv3 starts every bench process.
"""
import argparse
import csv
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_line(args, extra=()):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args.split(),
                        "--no-cpu-baseline", *extra], capture_output=True, text=True, timeout=600,
                       cwd=ROOT)
    if r.returncode:
        raise SystemExit(f"bench {args}: rc {r.returncode}\n{r.stderr[-2000:]}")
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


def pmc_pass(args, counter, d, steps):
    # counter: one name, or a comma group collected in one pass (within one pass's limits)
    cmd = ["timeout", "-s", "KILL", "300", "rocprofv3", "--pmc", *counter.split(","),
           "--output-format", "csv",
           "-d", d, "-o", "pmc", "--", sys.executable, os.path.join(ROOT, "bench.py"),
           *args.split(), "--no-cpu-baseline", "--steps", str(steps), "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
    if r.returncode:
        raise SystemExit(f"pmc {counter} {args}: rc {r.returncode}\n{r.stderr[-2000:]}")
    for dp, _, fs in os.walk(d):
        for f in fs:
            if f.endswith("counter_collection.csv"):
                return os.path.join(dp, f)
    raise SystemExit(f"no counter csv under {d}")


def per_kernel(path, pats, counter=None):
    vals = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if counter and r["Counter_Name"] != counter:
            continue
        if any(p in name for p in pats):
            vals.setdefault(name, []).append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sets", nargs="+", help="bench.py argument strings")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc", "traffic.json"))
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--instr", default="",
                    help="SQ counters (e.g. SQ_INSTS_VALU,SQ_INSTS_LDS) to add to the entries "
                         "instead of the FETCH/WRITE passes: per launch, summed over the call's "
                         "kernels; ',' separates passes, '+' joins counters into one pass "
                         "(e.g. SQ_WAVE_CYCLES+SQ_WAIT_ANY+SQ_WAIT_INST_ANY)")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    db = {"entries": []}
    if os.path.exists(a.out):
        db = json.load(open(a.out))
    for i, args in enumerate(a.sets):
        line = bench_line(args, ("--steps", str(a.steps), "--warmup", "1"))
        rf = line["roofline"]
        key, pats = rf["traffic_key"], rf["traffic_kernels"]
        launches = line["launches_in_process"]
        d = os.path.join(os.path.dirname(a.out), f"set{i}")
        if a.instr:
            old = [e for e in db["entries"] if e["key"] == key]
            ent = old[0] if old else {"key": key, "kernels": pats, "bytes_per_launch": None,
                                      "alg_bytes_per_launch": rf["alg_bytes_per_launch"]}
            ins = ent.setdefault("instr", {})
            for grp in a.instr.split(","):
                names = grp.split("+")
                path = pmc_pass(args, ",".join(names), os.path.join(d, names[0]), a.steps)
                for c in names:
                    vals = per_kernel(path, pats, c)
                    tot = 0.0
                    for name, v in vals.items():
                        tot += statistics.median(v) * max(1, round(len(v) / launches))
                    ins[c] = tot
            ent["instr_source"] = (f"rocprofv3 --pmc passes ({a.instr}) of bench.py {args} "
                                   f"(tools/pmc_collect.py --instr)")
            db["entries"] = [e for e in db["entries"] if e["key"] != key] + [ent]
            json.dump(db, open(a.out, "w"), indent=1)
            print(json.dumps({"key": key, "instr": ins}), flush=True)
            continue
        got = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            got[c] = per_kernel(pmc_pass(args, c, os.path.join(d, c), a.steps), pats)
        per, dropped = {}, {}
        total = 0.0
        for name in sorted(set(got["FETCH_SIZE"]) & set(got["WRITE_SIZE"])):
            f, w = got["FETCH_SIZE"][name], got["WRITE_SIZE"][name]
            if 2 * len(f) < launches:  # a one-off kernel of the process (table fill, the
                # parity check's export), not part of the measured call: listed, not counted
                dropped[name[:120]] = {"dispatches": len(f), "launches": launches,
                                       "fetch_kib_median": statistics.median(f),
                                       "write_kib_median": statistics.median(w)}
                continue
            k = max(1, round(len(f) / launches))  # dispatches of this kernel per launch
            b = (statistics.median(f) * 2 + statistics.median(w)) * 1024 * k
            per[name[:120]] = {"fetch_kib_median": statistics.median(f),
                               "write_kib_median": statistics.median(w), "per_launch": k,
                               "bytes": b}
            total += b
        old = [e for e in db["entries"] if e["key"] == key]
        ent = dict(old[0]) if old else {}
        ent.update({"key": key, "kernels": pats, "bytes_per_launch": total,
               "alg_bytes_per_launch": rf["alg_bytes_per_launch"],
               "ratio_to_alg": total / rf["alg_bytes_per_launch"], "per_kernel": per,
               "dropped_one_off": dropped,
               "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py {args} "
                         f"(tools/pmc_collect.py)"})
        db["entries"] = [e for e in db["entries"] if e["key"] != key] + [ent]
        json.dump(db, open(a.out, "w"), indent=1)
        print(json.dumps({"key": key, "bytes_per_launch": total,
                          "ratio_to_alg": round(ent["ratio_to_alg"], 3)}), flush=True)


if __name__ == "__main__":
    main()
