#!/usr/bin/env python3
"""Generates the committed golden fixtures (tests/golden/*.npz + MANIFEST.sha256).

The reference path (Go) cannot be built or run here (no Go toolchain) and its own
tests hold no vectors for this path, so the fixtures are produced by the CPU oracle
(oracle/oracle.cpp, a line-by-line restatement of the cited Go) on seeded synthetic inputs.
They freeze the oracle's outputs: tests/test_golden.py checks that the oracle still reproduces
them bit for bit (CPU) and that the HIP engine does too (GPU).

  python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

import gen_cases  # noqa: E402
from oracle_lib import Oracle  # noqa: E402
from minpaxos_amd import records as R  # noqa: E402
from minpaxos_amd import synth  # noqa: E402


def cases():
    """name -> (kind, params, inputs); outputs are computed by the oracle"""
    out = {}
    rec, st = synth.accept_replies(2048, 5, 0.7, seed=42)
    for mode, mname in ((R.MODE_MIN, "min"), (R.MODE_CLASSIC, "classic")):
        out[f"accept_config2_{mname}"] = ("accept", dict(n=5, mode=mode, base=0, cu=-1),
                                          dict(recs=rec, st=st, pc=np.zeros(5, np.int32)))
    rng = np.random.default_rng(777)
    for mode, mname in ((R.MODE_MIN, "min"), (R.MODE_CLASSIC, "classic")):
        r2, s2 = gen_cases.ragged_accept(rng, 1500, 7, max_r=9, long_every=499, long_len=150,
                                         base=5)
        out[f"accept_ragged_n7_{mname}"] = ("accept", dict(n=7, mode=mode, base=5, cu=20),
                                            dict(recs=r2, st=s2,
                                                 pc=np.arange(7, dtype=np.int32)))
    prec, pst = synth.prepare_replies(2048, 5, 0.8, seed=43)
    out["prepare_config3"] = ("prepare", dict(n=5, base=0, db=-1), dict(recs=prec, st=pst))
    r3, s3 = gen_cases.ragged_prepare(np.random.default_rng(778), 1500, 5, max_r=9,
                                      long_every=307, long_len=120)
    out["prepare_ragged"] = ("prepare", dict(n=5, base=0, db=100), dict(recs=r3, st=s3))
    mrec, moff, mgst = synth.prepare_replies_min(1024, 5, seed=46)
    out["prepare_min"] = ("prepare_min", dict(n=5), dict(recs=mrec, off=moff, gst=mgst))
    for dist in ("uniform", "zipf"):
        op, key, val = synth.commands(1 << 15, 1 << 11, 0.5, dist, seed=44)
        out[f"apply_config4_{dist}"] = ("apply", dict(), dict(op=op, key=key, val=val))
    op, key, val = gen_cases.commands_mixed(np.random.default_rng(779), 20000, 900)
    out["apply_mixed_ops"] = ("apply", dict(), dict(op=op, key=key, val=val))
    sizes = np.random.default_rng(780).integers(0, 7, 3000)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    cop, ckey, _ = gen_cases.commands_mixed(np.random.default_rng(781), int(off[-1]), 1500,
                                            neg_keys=False)
    out["conflict_batch"] = ("conflict", dict(), dict(op=cop, key=ckey, off=off))
    gb = synth.group_batch(24, 256, 5, 4, 256, seed=45)
    for mode, mname in ((R.MODE_MIN, "min"), (R.MODE_CLASSIC, "classic")):
        out[f"group_step_config5_{mname}"] = ("group", dict(n=5, mode=mode, kv=512),
                                              {k: v for k, v in gb.items()
                                               if isinstance(v, np.ndarray)})
    drec, _ = synth.accept_replies(750, 5, 0.7, seed=48)
    out["decode_mixed"] = ("decode", dict(), dict(buf=synth.peer_stream(
        drec, seed=49, p_beacon=0.02, p_prepare=0.01, p_commit_short=0.01, p_unknown=0.03,
        tail=bytes([R.PEER_ACCEPT_REPLY, 7, 0, 0]))))
    head = synth.peer_stream(drec[:1000], seed=50, p_beacon=0.01)
    var = np.array([R.PEER_PREPARE_REPLY, 1, 0, 0, 0], np.uint8)
    out["decode_variable_stop"] = ("decode", dict(), dict(buf=np.concatenate(
        [head, var, synth.peer_stream(drec[1000:], seed=51)])))
    out["fanout_replies"] = ("fanout", dict(n_clients=37, ok=1, leader=3),
                             dict(recs=synth.replies(5000, 37, seed=54)))
    lrec, loff, lop, lkey, lval = synth.log_records(3000, 4, seed=57, ragged=True)
    for fmt, fname in ((R.LOG_CATCHUP, "catchup"), (R.LOG_DURABLE, "durable")):
        out[f"log_{fname}"] = ("log", dict(fmt=fmt),
                               dict(recs=lrec, cmd_off=loff, op=lop, key=lkey, val=lval))
    # durable log read back (getDataFromStableStore): 1-command records, repeated instNos, both
    # statuses, written by the oracle's durable encoder
    rrec, roff, rop, rkey, rval = synth.log_records(2000, 1, seed=61)
    rrec = rrec.copy()
    rng = np.random.default_rng(62)
    rrec["inst_no"] = rng.integers(0, 1500, 2000)
    rrec["status"] = np.where(rng.random(2000) < 0.6, R.COMMITTED, R.ACCEPTED)
    rlog, _ = Oracle(5, R.MODE_MIN).encode_log(R.LOG_DURABLE, rrec, roff, rop, rkey, rval)
    out["replay_durable"] = ("replay", dict(cap=1500, db=7, cu=-1), dict(log=rlog))
    return out


def run_case(kind, p, x, backend_mk):
    """returns dict of outputs (numpy arrays) for one case"""
    if kind == "accept":
        b = backend_mk(p["n"], p["mode"])
        st, cu, pc, dec = b.accept_tally(x["recs"], x["st"], p["base"], p["cu"], x["pc"])
        return dict(st=st, cu=np.array([cu], np.int32), pc=pc, decided=dec)
    if kind == "prepare":
        b = backend_mk(p["n"], R.MODE_CLASSIC)
        st, db, prep = b.prepare_select(x["recs"], x["st"], p["base"], p["db"])
        return dict(st=st, db=np.array([db], np.int32), prepared=prep)
    if kind == "prepare_min":
        b = backend_mk(p["n"], R.MODE_MIN)
        gst, pc, eff = b.prepare_select_min(x["recs"], x["off"], x["gst"])
        return dict(gst=gst, pc=pc, eff=eff)
    if kind == "apply":
        b = backend_mk(5, R.MODE_MIN)
        ret, conf = b.apply(x["op"], x["key"], x["val"])
        k, v = b.kv_export()
        return dict(ret=ret, conf=conf, kv_key=k, kv_val=v)
    if kind == "conflict":
        b = backend_mk(5, R.MODE_MIN)
        return dict(out=b.conflict_batch(x["op"], x["key"], x["off"]))
    if kind == "group":
        b = backend_mk(p["n"], p["mode"], kv_per_group=p["kv"])
        gbat = dict(x, n_groups=len(x["committed_in"]), ipg=len(x["st_in"]) // len(x["committed_in"]))
        o = b.group_step(gbat)
        return {k: v for k, v in o.items() if v is not None}
    if kind == "decode":
        b = backend_mk(5, R.MODE_MIN)
        ar, oth, res = b.decode_peer_stream(x["buf"])
        return dict(ar=ar, other=oth, res=np.array([res], R.DECODE_RESULT))
    if kind == "fanout":
        b = backend_mk(5, R.MODE_MIN)
        out, off = b.encode_replies(x["recs"], p["n_clients"], p["ok"], p["leader"])
        return dict(out=out, client_off=off)
    if kind == "log":
        b = backend_mk(5, R.MODE_MIN)
        out, ro = b.encode_log(p["fmt"], x["recs"], x["cmd_off"], x["op"], x["key"], x["val"])
        return dict(out=out, rec_off=ro)
    if kind == "replay":
        b = backend_mk(5, R.MODE_MIN)
        rc, op, key, val, last, db, cu = b.replay_durable(x["log"], p["cap"], p["db"], p["cu"])
        return dict(recs=rc, op=op, key=key, val=val, last_rec=last,
                    scalars=np.array([db, cu], np.int32))
    raise ValueError(kind)


def main():
    lines = []
    for name, (kind, p, x) in cases().items():
        y = run_case(kind, p, x, lambda n, mode, **kw: Oracle(n, mode, **kw))
        path = os.path.join(HERE, name + ".npz")
        arrs = {"in_" + k: v for k, v in x.items()}
        arrs.update({"out_" + k: v for k, v in y.items()})
        arrs["meta_kind"] = np.array(kind)
        for k, v in p.items():
            arrs["param_" + k] = np.array(v)
        np.savez_compressed(path, **arrs)
        lines.append(f"{hashlib.sha256(open(path, 'rb').read()).hexdigest()}  {name}.npz")
        print(name, os.path.getsize(path))
    open(os.path.join(HERE, "MANIFEST.sha256"), "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
