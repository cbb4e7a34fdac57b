"""Extended randomised sweeps, run on demand: the partitioned apply pipeline (apply_fast.hip),
(MPX_FUZZ_EXT=<seeds>, e.g. 120; skipped otherwise so the default GPU suite keeps its time):
larger calls than test_gpu_fuzz.py's (up to 2^21 commands, so a bin's batches cross the run
window of the resolve several times), table sizes from 4 bins to super-bins, chunked calls, and
key mixes that leave most tiles' runs of a bin empty (the skewed cases) or long (tiny key spaces).
Every call's results and the final table against the oracle.

References: Command.Execute / executeCommands (state.go:77-103, bareminpaxos.go:1066-1098),
state.Conflict (state.go:53-60)."""
import os

import numpy as np
import pytest

from oracle_lib import Oracle
from minpaxos_amd import records as R
from test_gpu_fuzz import _commands

pytestmark = pytest.mark.gpu

_N = int(os.environ.get("MPX_FUZZ_EXT", "0") or 0)


@pytest.mark.skipif(_N == 0, reason="set MPX_FUZZ_EXT=<seeds> to run the extended sweep")
@pytest.mark.parametrize("seed", range(max(_N, 1)))
def test_fuzz_apply_partitioned_ext(mk_engine, seed):
    rng = np.random.default_rng(91000 + seed)
    cap = 1 << int(rng.integers(10, 23))
    chunk = int(rng.choice([0, 0, 0, 200000, 1 << 20]))
    e = mk_engine(5, R.MODE_MIN, kv_capacity=cap, apply_path=R.APPLY_PARTITIONED,
                  apply_chunk=chunk)
    o = Oracle(5, R.MODE_MIN)
    for call in range(3):
        m = int(rng.integers(20000, 1 << 21))
        space = int(rng.integers(1, cap // 2 + 1))
        if rng.random() < 0.15:
            space = int(rng.integers(1, 64))  # long runs per tile and bin
        kind = ["uniform", "zipf", "hot", "special"][int(rng.integers(0, 4))]
        op, key, val = _commands(rng, m, space, kind)
        gr, gc = e.apply(op, key, val)
        wr, wc = o.apply(op, key, val)
        tag = (seed, call, cap, chunk, m, space, kind)
        assert np.array_equal(gr, wr), (tag, np.nonzero(gr != wr)[0][:5])
        assert np.array_equal(gc, wc), (tag, np.nonzero(gc != wc)[0][:5])
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv), seed


@pytest.mark.skipif(_N == 0, reason="set MPX_FUZZ_EXT=<seeds> to run the extended sweep")
@pytest.mark.parametrize("seed", range(max(_N // 4, 1)))
def test_fuzz_conflict_batch_ext(mk_engine, seed):
    """ConflictBatch (state.go:62-71) over ragged instances - empty ones, instances past the
    register path's 4 commands, workgroup ranges past the LDS staging - with the key and op
    arrays at every alignment the device form allows (the kernel stages from the 16-byte
    boundary below each workgroup's range)"""
    from minpaxos_amd.devbuf import Arena
    import gen_cases
    rng = np.random.default_rng(93000 + seed)
    e, o = mk_engine(5, R.MODE_MIN), Oracle(5, R.MODE_MIN)
    n_inst = int(rng.integers(2, 40000))
    hi = int(rng.choice([3, 5, 9, 17]))
    sizes = rng.integers(0, hi, n_inst)
    if rng.random() < 0.3:
        sizes[rng.integers(0, n_inst, 8)] = rng.integers(20, 3000, 8)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    m = int(off[-1])
    op, key, _ = gen_cases.commands_mixed(rng, max(m, 1), int(rng.integers(1, 5000)),
                                          neg_keys=bool(rng.random() < 0.5))
    op, key = op[:m], key[:m]
    want = o.conflict_batch(op, key, off)
    ks, os_ = int(rng.integers(0, 2)), int(rng.integers(0, 16))
    with Arena(e) as ar:
        d_key = ar.put(np.concatenate([np.zeros(ks, np.int64), key]))
        d_op = ar.put(np.concatenate([np.zeros(os_, np.uint8), op]))
        d_off = ar.put(off)
        d_out = ar.full(n_inst, np.uint8, 0xEE)
        e.conflict_batch_dev(d_op.at(os_), d_key.at(ks), d_off.ptr, n_inst, d_out.ptr)
        e.stream_synchronize(None)
        got = ar.get(d_out, n_inst - 1)
    assert np.array_equal(got, want), (seed, np.nonzero(got != want)[0][:5])


def _var_dense(rng, n):
    """bytes from a small alphabet of variable-message codes, zeros and small even numbers: most
    positions parse as frame starts, catch-up logs run deep over the zeros, and a wave's chunks
    hold far more than the framing DP's task window (256 positions)"""
    alpha = np.array([9, 10, 12, 0, 0, 0, 2, 4, 6, 13, 0x80, 1], np.uint8)
    return alpha[rng.integers(0, len(alpha), n)].tobytes()


@pytest.mark.skipif(_N == 0, reason="set MPX_FUZZ_EXT=<seeds> to run the extended sweep")
@pytest.mark.parametrize("seed", range(max(_N // 4, 1)))
def test_fuzz_stream_decode_ext(mk_engine, seed):
    """The full peer-stream decode (replicaListener + every Unmarshal, genericsmr.go:402-446,
    minpaxosprotomarsh.go:352-387 / :470-507 / :648-672) on streams built to stress the framing
    DP's variable-message pass: var-dense byte soups, leader streams whose instance numbers
    carry 9 / 10 / 12 bytes (ballot 0: zero-rich payload), random frame mixes with most frames
    variable, pieces of each concatenated, cut at random places, both wire formats"""
    from minpaxos_amd import wire as W
    from minpaxos_amd import synth
    rng = np.random.default_rng(95000 + seed)
    for proto in (R.MODE_MIN, R.MODE_CLASSIC):
        e, o = mk_engine(5, proto), Oracle(5, proto)
        parts = []
        for _ in range(int(rng.integers(1, 5))):
            k = int(rng.integers(0, 4))
            if k == 0:
                parts.append(_var_dense(rng, int(rng.integers(1, 1 << 20))))
            elif k == 1:
                n = int(rng.integers(1, 1 << 16))
                base = int(rng.choice([0x0A00, 0x090000, 0x0C0C00, int(rng.integers(0, 1 << 24))]))
                recs, _ = synth.accept_replies(n, 5, 0.7, seed=int(rng.integers(0, 1 << 30)),
                                               inst_base=base, ballot=int(rng.choice([0, 16, 10])))
                parts.append(bytes(W.leader_stream(proto, recs, prepare_every=int(rng.integers(1, 300)),
                                                   n_cmds=int(rng.integers(0, 3)))))
            elif k == 2:
                parts.append(W.random_stream(proto, rng, int(rng.integers(1, 20000)),
                                             p_var=float(rng.uniform(0.5, 0.95)), max_cmds=3,
                                             p_big=0.0, max_log=6, p_unknown=0.02))
            else:
                parts.append(rng.integers(0, 256, int(rng.integers(1, 1 << 18)), dtype=np.uint8).tobytes())
        b = b"".join(parts)
        for cut in (len(b), int(rng.integers(0, len(b) + 1))):
            got, want = e.decode_stream(b[:cut]), o.decode_stream(b[:cut])
            for g, w, name in zip(got[:4], want[:4], ("ar", "prep", "var", "other")):
                assert len(g) == len(w) and g.tobytes() == w.tobytes(), (seed, proto, cut, name)
            for f in ("consumed", "next", "n_accept_replies", "n_prepare_replies", "n_var", "n_other",
                      "stop_reason", "stop_code"):
                assert int(got[4][f]) == int(want[4][f]), (seed, proto, cut, f)


_DUR = np.dtype([("ballot", "<i4"), ("status", "<i4"), ("inst", "<i4"), ("op", "u1"),
                 ("key", "<i8"), ("val", "<i8")])  # 29 packed bytes (getDataFromStableStore)


@pytest.mark.skipif(_N == 0, reason="set MPX_FUZZ_EXT=<seeds> to run the extended sweep")
@pytest.mark.parametrize("seed", range(max(_N // 4, 1)))
def test_fuzz_replay_binned_ext(mk_engine, seed):
    """durable-log replay (bareminpaxos.go:122-161) through the binned slot maximum (the
    reserved scratch: chunk-sorted runs, one LDS slice per 32768 slots) against the oracle:
    random record counts (ragged last chunk), instance spaces from one slot to 2^24 (ragged
    last bin), permutations, uniform repeats, repeats packed into one bin, rec_base offsets
    with slots carried from earlier chunks"""
    from minpaxos_amd.devbuf import Arena
    assert _DUR.itemsize == R.DURABLE_REC_BYTES
    rng = np.random.default_rng(95000 + seed)
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    n = int(rng.integers(1, 1 << 21))
    cap = int(rng.choice([int(rng.integers(1, 1 << 12)), int(rng.integers(1, 1 << 24)),
                          32768 * int(rng.integers(1, 64)) + int(rng.integers(-2, 3))]))
    cap = max(cap, 1)
    kind = ["perm", "uniform", "one_bin", "hot"][int(rng.integers(0, 4))]
    if kind == "perm" and n <= cap:
        inst = rng.permutation(cap)[:n]
    elif kind == "one_bin":
        b0 = int(rng.integers(0, (cap + 32767) // 32768)) * 32768
        inst = rng.integers(b0, min(cap, b0 + 32768), n)
    elif kind == "hot":
        inst = rng.integers(0, min(cap, 16), n)
    else:
        inst = rng.integers(0, cap, n)
    recs = np.zeros(n, _DUR)
    recs["ballot"] = rng.integers(-50, 50, n)
    recs["status"] = rng.integers(0, 5, n)
    recs["inst"] = inst
    recs["op"] = rng.integers(0, 3, n)
    recs["key"] = rng.integers(-(1 << 40), 1 << 40, n)
    recs["val"] = rng.integers(-(1 << 40), 1 << 40, n)
    log = recs.view(np.uint8).copy()
    base = int(rng.integers(0, 1000)) if rng.random() < 0.5 else 0
    last0 = rng.integers(-1, base, cap).astype(np.int32) if base else np.full(cap, -1, np.int32)
    want = o.replay_durable(log, cap, 7, -1, rec_base=base, last_rec=last0)
    with Arena(e) as hip:
        e.replay_durable_reserve(len(log), cap)
        d_log = hip.put(log)
        d = [hip.put(np.zeros_like(w)) for w in want[:4]]
        d_last = hip.put(last0)
        d_sc = hip.put(np.array([7, -1], np.int32))
        e.replay_durable_dev(d_log.ptr, len(log), cap, *[x.ptr for x in d], d_last.ptr,
                             d_sc.ptr, rec_base=base)
        e.synchronize()
        tag = (seed, n, cap, kind, base)
        for x, w in zip(d, want[:4]):
            assert np.array_equal(hip.get(x), w), tag
        got = hip.get(d_last)
        assert np.array_equal(got, want[4]), (tag, np.nonzero(got != want[4])[0][:5])
        assert hip.get(d_sc).tolist() == [want[5], want[6]], tag
