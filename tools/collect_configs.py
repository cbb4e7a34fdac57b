"""Copy a tools/gpu_prof_configs.sh run into profiles/ and print the DESIGN.md measurement table.

usage: python tools/collect_configs.py gpurun_out/profcfg_<tag> profiles/r01/configs
Per workload it keeps the bench JSON line (<name>_bench.json) and the rocprofv3 kernel stats
(<name>_kernel_stats.csv); the table has a row per bench line kept in the destination.
"""
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from design_table import bound_label  # noqa: E402


def main(src: str, dst: str) -> None:
    os.makedirs(dst, exist_ok=True)
    rows = []
    for name in sorted(os.listdir(src)):
        log = os.path.join(src, name + ".log")
        if not os.path.isdir(os.path.join(src, name)) or not os.path.exists(log):
            continue
        lines = [ln for ln in open(log) if ln.startswith("{")]
        if not lines:
            continue
        with open(os.path.join(dst, name + "_bench.json"), "w") as f:
            f.write(lines[-1] if lines[-1].endswith("\n") else lines[-1] + "\n")
        stats = os.path.join(src, name, name + "_kernel_stats.csv")
        if os.path.exists(stats):
            shutil.copy(stats, os.path.join(dst, name + "_kernel_stats.csv"))
    for f in sorted(os.listdir(dst)):  # the table covers every row kept in dst
        if not f.endswith("_bench.json"):
            continue
        name = f[:-len("_bench.json")]
        d = json.loads(open(os.path.join(dst, f)).read())
        rf, cb = d.get("roofline") or {}, d.get("cpu_baseline") or {}
        par = d.get("parity", {})
        hbm = rf.get("hbm") or rf  # issue-bound rows keep their HBM figures under "hbm"
        issue = bound_label(rf)
        cpu = ("%.3g (%s core)" % (cb["value"], cb.get("cores", "?"))) if cb.get("value") else "-"
        rows.append("| %s | %s | %.3g %s | %.3f | %.0f | %.3f | %s | %s | %s |" % (
            name, d["config"]["workload"], d["value"], d["unit"], d["ms_per_step"],
            hbm.get("achieved") or 0.0, hbm.get("frac") or 0.0, issue, cpu, par.get("bit_exact")))
    print("| workload | shape | value | ms / launch | GB/s | frac of 8 TB/s | bound (SQ counters) | CPU port | bit-exact |")
    print("|---|---|---|---|---|---|---|---|---|")
    print("\n".join(rows))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
