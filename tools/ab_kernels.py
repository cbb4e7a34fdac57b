#!/usr/bin/env python3
"""Interleaved same-process A/B of engine builds (cdna_hip_programming.md §5.4): every build is
loaded as its own shared object (one HIP runtime, so device pointers are shared), opens its own
engine, and the builds' *_dev calls on the same HBM-resident inputs are timed round-robin with
HIP events on their engine streams. Outputs of every build are compared with the first one.

  python tools/ab_kernels.py --work tally_min,tally_classic,prepare LIB_A LIB_B ...
work: tally_min tally_classic prepare apply_uniform apply_zipf apply_small step
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from minpaxos_amd import _lib, synth  # noqa: E402
from minpaxos_amd import records as R  # noqa: E402


def load(path):
    lib = C.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    return lib


class Eng:
    def __init__(self, lib, mode, **cfg):
        self.lib = lib
        c = _lib.MpxConfig(5, mode, cfg.get("kv_capacity", 0), cfg.get("kv_per_group", 0), 0,
                           cfg.get("max_groups", 0), 0, cfg.get("apply_path", 0), 0, 0, 0)
        h = C.c_void_p()
        rc = lib.mpx_open(0, C.byref(c), C.byref(h))
        assert rc == 0, rc
        self.h = h
        self.s = lib.mpx_stream(h)

    def ck(self, rc, what):
        if rc:
            raise RuntimeError(f"{what}: {rc} {self.lib.mpx_last_error(self.h)}")

    def ev(self):
        e = C.c_void_p()
        self.ck(self.lib.mpx_event_create(self.h, 1, C.byref(e)), "event")
        return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--work", default="tally_min")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    libs = [load(p) for p in a.libs]
    for work in a.work.split(","):
        run(work, libs, a)


def run(work, libs, a):
    mode = R.MODE_CLASSIC if work in ("tally_classic", "prepare") else R.MODE_MIN
    cfg = {}
    if work.startswith("apply"):
        cfg = dict(kv_capacity=1 << 20)
    engs = [Eng(l, mode, **cfg) for l in libs]
    e0 = engs[0]
    bufs = []

    def put(x):
        arr = np.ascontiguousarray(x)
        p = C.c_void_p()
        e0.ck(e0.lib.mpx_dev_alloc(e0.h, max(arr.nbytes, 1), C.byref(p)), "alloc")
        e0.ck(e0.lib.mpx_memcpy_async(e0.h, p, arr.ctypes.data, arr.nbytes, 1, None), "h2d")
        e0.lib.mpx_synchronize(e0.h)
        bufs.append(p)
        return p.value

    def empty(nbytes):
        p = C.c_void_p()
        e0.ck(e0.lib.mpx_dev_alloc(e0.h, max(nbytes, 1), C.byref(p)), "alloc")
        bufs.append(p)
        return p.value

    def get(ptr, nbytes):
        out = np.zeros(nbytes, np.uint8)
        e0.ck(e0.lib.mpx_memcpy_async(e0.h, out.ctypes.data, ptr, nbytes, 2, None), "d2h")
        e0.ck(e0.lib.mpx_synchronize(e0.h), "sync")
        return out

    outs = []  # per engine: (ptr, nbytes) of the outputs compared across builds
    launch = []
    pre = {}  # per engine: untimed work before each launch (scalar resets)
    if work.startswith("tally"):
        I = 1 << 24
        recs, st = synth.accept_replies(I, 5, 0.7, seed=42)
        d_recs, d_st = put(recs), put(st)
        for e in engs:
            d_out, d_sc, d_dec = empty(I * 16), empty(24), empty(I)
            sc0 = put(np.array([-1, 0, 0, 0, 0, 0], np.int32))
            outs.append([(d_out, I * 16), (d_sc, 24), (d_dec, I)])
            pre[len(launch)] = lambda e=e, sc=d_sc, s0=sc0: e.lib.mpx_memcpy_async(
                e.h, sc, s0, 24, 3, e.s)
            launch.append(lambda e=e, o=d_out, sc=d_sc, dd=d_dec: e.ck(
                e.lib.mpx_accept_tally_dev(e.h, d_recs, len(recs), d_st, o, I, 0, sc, dd, e.s),
                "tally"))
        alg = len(recs) * 16 + I * 32
    elif work == "prepare":
        I = 1 << 24
        recs, st = synth.prepare_replies(I, 5, 0.8, seed=43)
        d_recs, d_st = put(recs), put(st)
        for e in engs:
            d_out, d_db, d_p = empty(I * 32), empty(4), empty(I)
            db0 = put(np.array([-1], np.int32))
            outs.append([(d_out, I * 32), (d_db, 4), (d_p, I)])
            pre[len(launch)] = lambda e=e, db=d_db, b0=db0: e.lib.mpx_memcpy_async(
                e.h, db, b0, 4, 3, e.s)
            launch.append(lambda e=e, o=d_out, db=d_db, dp=d_p: e.ck(
                e.lib.mpx_prepare_select_dev(e.h, d_recs, len(recs), d_st, o, I, 0, db, dp, e.s),
                "prepare"))
        alg = len(recs) * 16 + I * 64
    elif work.startswith("apply"):
        if work == "apply_small":
            M, K = 5000, 1 << 20
            op, key, val = synth.commands(M, K, 0.5, "uniform", seed=44)
        else:
            M, K = 1 << 26, 1 << 20
            op, key, val = synth.commands(M, K, 0.5, work.split("_")[1], seed=44)
        d_op, d_key, d_val = put(op), put(key), put(val)
        for e in engs:
            e.ck(e.lib.mpx_apply_reserve(e.h, M), "reserve")
            d_ret, d_conf = empty(M * 8), empty(M)
            outs.append([(d_ret, M * 8), (d_conf, M)])
            launch.append(lambda e=e, r=d_ret, c=d_conf: e.ck(
                e.lib.mpx_apply_dev(e.h, d_op, d_key, d_val, M, r, c, e.s), "apply"))
            launch[-1]()  # the table holds every key from here on
            e.lib.mpx_synchronize(e.h)
        alg = M * 26 + K * 32
    else:
        raise SystemExit(f"unknown work {work}")

    ms = [[] for _ in engs]
    for i, e in enumerate(engs):  # warm-up
        for _ in range(2):
            if i in pre:
                pre[i]()
            launch[i]()
        e.ck(e.lib.mpx_synchronize(e.h), "sync")
    for _ in range(a.rounds):
        for i, e in enumerate(engs):
            evs = [(e.ev(), e.ev()) for _ in range(a.iters)]
            for e_0, e_1 in evs:
                if i in pre:
                    pre[i]()
                e.lib.mpx_event_record(e.h, e_0, e.s)
                launch[i]()
                e.lib.mpx_event_record(e.h, e_1, e.s)
            e.ck(e.lib.mpx_synchronize(e.h), "sync")
            for e_0, e_1 in evs:
                f = C.c_float()
                e.lib.mpx_event_elapsed_ms(e.h, e_0, e_1, C.byref(f))
                ms[i].append(f.value)
                e.lib.mpx_event_destroy(e.h, e_0)
                e.lib.mpx_event_destroy(e.h, e_1)
    ref = [get(p, n) for p, n in outs[0]]
    for i, path in enumerate(a.libs):
        same = all(np.array_equal(get(p, n), r) for (p, n), r in zip(outs[i], ref))
        med = float(np.median(ms[i]))
        print(f"{work:14s} {os.path.basename(path):24s} median {med:.4f} ms  min "
              f"{min(ms[i]):.4f}  frac {alg / (med * 1e-3) / 8e12:.3f}  same_as_first {same}",
              flush=True)
    for p in bufs:
        e0.lib.mpx_dev_free(e0.h, p)
    for e in engs:
        e.lib.mpx_close(e.h)


if __name__ == "__main__":
    main()
