#!/usr/bin/env python3
"""Interleaved A/B timing of several builds of the engine on the same data, in ONE process
(cdna_hip_programming.md §5.4 rule 24): each build is loaded as its own shared object, and the
fused group step of every build is timed round-robin with HIP events on its engine stream.

  python tools/ab_step.py minpaxos_amd/libmpx.so /tmp/libmpx_old.so [--rounds 5 --iters 10]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from minpaxos_amd import _lib, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--kv", type=int, default=512, help="kv_per_group (256: FastBase, the bench's)")
    ap.add_argument("--totals", action="store_true",
                    help="time mpx_group_step_totals_dev (the bench's step) instead of _dev")
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    G, ipg, N, K = a.groups, 256, 5, a.kv
    b = synth.group_batch(G, ipg, N, 4, 256, seed=45)

    def dt(x):
        arr = np.ascontiguousarray(x)
        if arr.dtype.names:
            arr = arr.view(np.uint8)
        return torch.from_numpy(arr).to(dev)

    m = len(b["op"])
    d = dict(recs=dt(b["recs"]), off=dt(b["grp_rec_off"]), st_in=dt(b["st_in"]),
             st_out=torch.empty(G * ipg * 16, dtype=torch.uint8, device=dev),
             ci=dt(b["committed_in"]), ei=dt(b["executed_in"]), pi=dt(b["peer_in"]),
             po=torch.empty(G * N, dtype=torch.int32, device=dev),
             co=torch.empty(G, dtype=torch.int32, device=dev),
             eo=torch.empty(G, dtype=torch.int32, device=dev),
             op=dt(b["op"]), key=dt(b["key"]), val=dt(b["val"]), coff=dt(b["cmd_off"]),
             ret=torch.zeros(m, dtype=torch.int64, device=dev),
             conf=torch.zeros(m, dtype=torch.uint8, device=dev),
             nd=torch.zeros(G, dtype=torch.int32, device=dev),
             tot=torch.zeros(3, dtype=torch.int64, device=dev))
    p = lambda t: t.data_ptr()  # noqa: E731

    def tables():  # each engine gets its own table buffers (its warm-up fills them)
        return {k + s: torch.zeros(G * (K if k != "kc" else 1),
                                   dtype=torch.int32 if k == "kc" else torch.int64, device=dev)
                for k in ("kc", "kk", "kv") for s in ("0", "1")}

    def batch(tb, i, o):
        return _lib.MpxGroupBatch(G, ipg, p(d["recs"]), p(d["off"]), p(d["st_in"]), p(d["st_out"]),
                                  p(d["ci"]), p(d["co"]), p(d["ei"]), p(d["eo"]), p(d["pi"]),
                                  p(d["po"]), p(d["op"]), p(d["key"]), p(d["val"]), p(d["coff"]),
                                  None, p(d["ret"]), p(d["conf"]), p(tb["kc" + i]), p(tb["kk" + i]),
                                  p(tb["kv" + i]), p(tb["kc" + o]), p(tb["kk" + o]),
                                  p(tb["kv" + o]), None, p(d["nd"]) if a.totals else None)

    engines = []
    for path in a.libs:
        lib = C.CDLL(os.path.abspath(path))
        for name, (res, args) in _lib.SIGNATURES.items():
            f = getattr(lib, name, None)  # (an older build lacks the newer entry points)
            if f is not None:
                f.restype, f.argtypes = res, args
        cfg = _lib.MpxConfig(N, a.mode, 0, K, 0, 0)
        h = C.c_void_p()
        assert lib.mpx_open(0, C.byref(cfg), C.byref(h)) == 0
        stream = lib.mpx_stream(h)
        tb = tables()
        engines.append((path, lib, h, stream, tb, batch(tb, "0", "1")))
        assert lib.mpx_group_step_dev(h, C.byref(batch(tb, "1", "0")), stream) == 0  # warm-up
        rc = lib.mpx_synchronize(h)  # ablation builds may flag errors (their results are wrong)
        if rc:
            print(f"{os.path.basename(path)}: warm-up returned {rc}")
    times = {e[0]: [] for e in engines}
    outs = {}
    for r in range(a.rounds):
        for path, lib, h, s, tb, step in engines:
            ts = torch.cuda.ExternalStream(s, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(ts)
            for _ in range(a.iters):
                if a.totals:
                    lib.mpx_group_step_totals_dev(h, C.byref(step), C.c_void_p(p(d["tot"])), s)
                else:
                    lib.mpx_group_step_dev(h, C.byref(step), s)
            e1.record(ts)
            lib.mpx_synchronize(h)
            times[path].append(e0.elapsed_time(e1) / a.iters)
            if r == 0:
                outs[path] = (d["ret"].sum().item(), d["co"].sum().item(), tb["kv1"].sum().item(),
                              d["tot"].tolist() if a.totals else None)
    ref = None
    for path, ts in times.items():
        same = "" if ref is None else ("  outputs " + ("==" if outs[path] == ref else "DIFFER"))
        ref = ref or outs[path]
        print(f"{os.path.basename(path):28s} median {np.median(ts):.4f} ms  min {np.min(ts):.4f} ms{same}")


if __name__ == "__main__":
    main()
