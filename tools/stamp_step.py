#!/usr/bin/env python3
"""Per-phase cycle breakdown of the fused group-step kernel (diagnostic build, -DMPX_STAMPS=1).

  make -C minpaxos_amd libmpx_stamp.so && python tools/stamp_step.py [--groups 65536]
Prints the average s_memtime cycles per workgroup for each barrier-delimited phase.
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MPX_LIB"] = os.path.join(ROOT, "minpaxos_amd", "libmpx_stamp.so")
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from minpaxos_amd import _lib, synth  # noqa: E402
from minpaxos_amd import records as R  # noqa: E402
from minpaxos_amd.engine import Engine  # noqa: E402

PHASES = ["loads (B1)", "heads+table (B2)", "tally (B3)", "lookup+chunk scan (B4)", "instance outputs",
          "resolve (B7)", "outputs"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--mode", default="min")
    a = ap.parse_args()
    lib = _lib.load()
    lib.mpx_debug_stamps.restype = C.c_int
    lib.mpx_debug_stamps.argtypes = [C.c_void_p, C.c_int]
    buf = (C.c_ulonglong * 16)()
    b = synth.group_batch(a.groups, 256, 5, 4, 256, seed=45)
    e = Engine(0, 5, a.mode, kv_per_group=512)
    w = e.group_step(b)  # fills the tables
    lib.mpx_debug_stamps(C.cast(buf, C.c_void_p), 1)
    e.group_step(b, w["kv_cnt"], w["kv_key"], w["kv_val"])
    lib.mpx_debug_stamps(C.cast(buf, C.c_void_p), 1)
    tot = sum(buf[:len(PHASES)])
    for i, name in enumerate(PHASES):
        print(f"{name:18s} {buf[i] / a.groups:10.0f} cycles/WG  {100.0 * buf[i] / max(tot, 1):5.1f}%")
    print(f"{'total':18s} {tot / a.groups:10.0f} cycles/WG")


if __name__ == "__main__":
    main()
