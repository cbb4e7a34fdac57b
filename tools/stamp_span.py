#!/usr/bin/env python3
"""Workgroup rounds of the fused group-step kernel (diagnostic build, -DMPX_STAMPS=2):

  make -C minpaxos_amd libmpx_span.so && python tools/stamp_span.py --groups 8192

Runs the step on the per-rank shape of a P-GPU job (8,192 groups = 65,536 / 8) and reads every
fast workgroup's start and end on the chip-wide 100 MHz clock. Workgroups are grouped into
rounds by start time (round r = the r-th batch of resident slots to start), and per round the
script prints how many ran, their median duration and the span the round covered - so the last,
partial round can be compared with the full ones (does it run faster per workgroup, as HBM frees
up, or not).
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MPX_LIB"] = os.path.join(ROOT, "minpaxos_amd", "libmpx_span.so")
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from minpaxos_amd import _lib, synth  # noqa: E402
from minpaxos_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=8192)
    ap.add_argument("--mode", default="min")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--resident", type=int, default=1536, help="resident workgroup slots")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    lib = _lib.load()
    lib.mpx_debug_spans.restype = C.c_int
    lib.mpx_debug_spans.argtypes = [C.c_void_p, C.c_uint]
    G = a.groups
    b = synth.group_batch(G, 256, 5, 4, 256, seed=45)
    e = Engine(0, 5, a.mode, kv_per_group=256, max_groups=max(G, 1024))
    w = e.group_step(b)  # fills the tables
    out = []
    for rep in range(a.reps):
        e.group_step(b, w["kv_cnt"], w["kv_key"], w["kv_val"])
        buf = np.zeros((G, 2), np.uint64)
        assert lib.mpx_debug_spans(buf.ctypes.data_as(C.c_void_p), G) == 0
        st, en = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64)
        t0 = st.min()
        st, en = st - t0, en - t0
        order = np.argsort(st, kind="stable")
        dur = (en - st)[order]
        R = a.resident
        rounds = []
        for r in range((G + R - 1) // R):
            sl = order[r * R:(r + 1) * R]
            d = (en - st)[sl]
            rounds.append({"round": r, "workgroups": int(len(sl)),
                           "median_us": float(np.median(d)) / 100.0,
                           "start_us": float(st[sl].min()) / 100.0,
                           "end_us": float(en[sl].max()) / 100.0})
        rec = {"rep": rep, "kernel_span_us": float(en.max()) / 100.0, "rounds": rounds}
        out.append(rec)
        print(json.dumps(rec))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
