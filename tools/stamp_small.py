#!/usr/bin/env python3
"""Per-phase time of the replica-batch apply's one-workgroup kernel for LONG lists (k_apply_small,
diagnostic build -DMPX_SMALL_STAMP=1); it does work only when a call puts more than 16 commands
on a key (e.g. --keys 64), else every phase reads 0:
  make -C minpaxos_amd variant_of FILE=apply_small NAME=sstamp DEFS=-DMPX_SMALL_STAMP=1
  python tools/stamp_small.py minpaxos_amd/ab/libmpx_sstamp.so [--commands 5000] [--keys 64]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ["load", "-", "flags", "-", "ids", "rank / radix", "groups+commit"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--commands", type=int, default=5000)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--keys", type=int, default=1 << 20)
    a = ap.parse_args()
    os.environ["MPX_LIB"] = os.path.abspath(a.lib)
    from minpaxos_amd import _lib, synth
    from minpaxos_amd.engine import Engine
    lib = _lib.load()
    lib.mpx_debug_small_stamps.restype = C.c_int
    lib.mpx_debug_small_stamps.argtypes = [C.c_void_p, C.c_int]
    buf = (C.c_ulonglong * 16)()
    e = Engine(0, 5, "min", kv_capacity=a.keys)
    op, key, val = synth.commands(a.commands, a.keys, 0.5, "uniform", seed=44)
    for _ in range(3):
        e.apply(op, key, val)
    lib.mpx_debug_small_stamps(C.cast(buf, C.c_void_p), 1)
    for _ in range(a.calls):
        e.apply(op, key, val)
    lib.mpx_debug_small_stamps(C.cast(buf, C.c_void_p), 1)
    tot = 0.0
    for i, name in enumerate(PHASES):
        us = buf[i] / a.calls / 100.0  # 100 MHz ticks -> us
        tot += us
        print(f"{name:14s} {us:8.2f} us")
    print(f"{'total':14s} {tot:8.2f} us")
    if buf[9]:
        print(f"shader clock during the resolve kernel: {buf[8] / (buf[9] / 100.0) / 1e3:.2f} GHz")


if __name__ == "__main__":
    main()
