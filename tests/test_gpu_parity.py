"""HIP engine vs the CPU oracle, bit-exact, through the C ABI (host-pointer entry points).

Sizes are chosen so the oracle finishes in seconds; the full BASELINE sizes are covered by
test_gpu_full.py.
"""
import numpy as np
import pytest

import gen_cases
import kat_cases
from oracle_lib import Oracle, OracleError
from minpaxos_amd import _lib
from minpaxos_amd import records as R
from minpaxos_amd import synth
from minpaxos_amd.engine import MpxError

pytestmark = pytest.mark.gpu


def eq_struct(a, b):
    assert a.dtype == b.dtype
    for f in a.dtype.names:
        if f == "pad":
            continue
        bad = np.nonzero(a[f] != b[f])[0]
        assert len(bad) == 0, f"field {f} differs at {bad[:10]}: {a[f][bad[:5]]} vs {b[f][bad[:5]]}"


@pytest.mark.parametrize("case", kat_cases.ALL, ids=lambda f: f.__name__)
def test_engine_kat(case, mk_engine):
    case(mk_engine)


# ---- A1 / A2 ----------------------------------------------------------------------------------
@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC])
@pytest.mark.parametrize("n_rep", [1, 2, 3, 5, 7, 16])
def test_accept_tally_ragged(mk_engine, mode, n_rep):
    rng = np.random.default_rng(1000 + 17 * n_rep + mode)
    for trial in range(3):
        rec, st = gen_cases.ragged_accept(rng, 3000, n_rep, max_r=9, long_every=997,
                                          long_len=200 + 70 * trial, base=trial * 50)
        e, o = mk_engine(n_rep, mode), Oracle(n_rep, mode)
        cu0 = int(rng.integers(-1, 60))
        pc0 = rng.integers(-1, 10, n_rep).astype(np.int32)
        got = e.accept_tally(rec, st, trial * 50, cu0, pc0)
        want = o.accept_tally(rec, st, trial * 50, cu0, pc0)
        eq_struct(got[0], want[0])
        assert got[1] == want[1], (got[1], want[1])
        assert np.array_equal(got[2], want[2])
        assert np.array_equal(got[3], want[3])


@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC])
def test_accept_tally_config2_shape(mk_engine, mode):
    rec, st = synth.accept_replies(1 << 16, 5, 0.7, seed=42)
    e, o = mk_engine(5, mode), Oracle(5, mode)
    got = e.accept_tally(rec, st, 0, -1, np.zeros(5, np.int32))
    want = o.accept_tally(rec, st, 0, -1, np.zeros(5, np.int32))
    eq_struct(got[0], want[0])
    assert got[1:3][0] == want[1] and np.array_equal(got[2], want[2])
    assert np.array_equal(got[3], want[3])


@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC])
def test_accept_tally_gaps(mk_engine, mode):
    """sparse replies: instances without replies before the first, between (gaps of 1 to 9000
    instances, longer than a wave and than a tile) and after the last one. Their decided flags
    are 0 (the kernel writes them in its gap pass; nothing is memset) and, CLASSIC, the
    committedUpTo scan (updateCommittedUpTo, paxos.go:259-264) runs through them: most input
    statuses are COMMITTED, so the first non-committed instance lies deep in a gap or past
    every record, or does not exist (all committed)."""
    rng = np.random.default_rng(77 + mode)
    for trial in range(6):
        n_inst = 30000
        picks = np.unique(np.concatenate([rng.integers(3000, 26000, 40), [3000, 26000]]))
        if trial == 5:
            picks = np.array([n_inst - 1])  # one instance, at the window's end
        counts = rng.integers(1, 6, len(picks))
        rec = np.zeros(int(counts.sum()), R.ACCEPT_REPLY)
        rec["instance"] = np.repeat(picks.astype(np.int32), counts) + trial
        rec["id"] = rng.integers(0, 5, len(rec))
        rec["ok"] = (rng.random(len(rec)) < 0.8).astype(np.uint8)
        rec["ballot"] = rng.integers(0, 300, len(rec))
        st = kat_cases.inst_states(n_inst, R.COMMITTED)
        st["status"][picks] = R.PREPARED  # the replied-to instances can commit now
        if trial in (1, 2):  # one non-committed instance inside a long gap / after the records
            st["status"][[12345, 28000][trial - 1]] = R.ACCEPTED
        if trial == 3:
            st["status"][:] = R.COMMITTED  # nothing to decide, nothing bad: watermark stays
        e, o = mk_engine(5, mode), Oracle(5, mode)
        # a dense call first leaves decided = 1 almost everywhere in the engine's staging buffer
        dense = kat_cases.acc(0, [(1, 1, 16), (2, 1, 16)])
        dense = np.concatenate([dense] * n_inst)
        dense["instance"] = np.repeat(np.arange(n_inst, dtype=np.int32), 2) + trial
        assert e.accept_tally(dense, kat_cases.inst_states(n_inst), trial, -1)[3].all()
        for cu0 in (-1, 2999 + trial, 20000):
            got = e.accept_tally(rec, st, trial, cu0, np.zeros(5, np.int32))
            want = o.accept_tally(rec, st, trial, cu0, np.zeros(5, np.int32))
            eq_struct(got[0], want[0])
            assert got[1] == want[1], (trial, cu0, got[1], want[1])
            assert np.array_equal(got[2], want[2])
            assert np.array_equal(got[3], want[3])


def test_prepare_classic_gaps(mk_engine):
    """CLASSIC prepare with sparse replies: the prepared flags of instances without replies are
    0 and defaultBallot is the max over the prepared ones (one launch, no memset)"""
    rng = np.random.default_rng(5)
    rec, st = gen_cases.ragged_prepare(rng, 20000, 5, max_r=6)
    keep = np.isin(rec["instance"], np.unique(rng.integers(0, 20000, 300)))
    rec = rec[keep]
    e, o = mk_engine(5, R.MODE_CLASSIC), Oracle(5, R.MODE_CLASSIC)
    full_rec, full_st = gen_cases.ragged_prepare(np.random.default_rng(6), 20000, 5, max_r=6)
    e.prepare_select(full_rec, full_st, 0, -1)  # leaves prepared flags in the staging buffer
    for db in (-1, 100, 1 << 20):
        got = e.prepare_select(rec, st, 0, db)
        want = o.prepare_select(rec, st, 0, db)
        eq_struct(got[0], want[0])
        assert got[1] == want[1] and np.array_equal(got[2], want[2])


def test_accept_tally_edges(mk_engine):
    e = mk_engine(5, R.MODE_MIN)
    # empty batch
    st = kat_cases.inst_states(4)
    got = e.accept_tally(np.zeros(0, R.ACCEPT_REPLY), st, 0, 3, np.arange(5, dtype=np.int32))
    assert got[1] == 3 and list(got[2]) == [0, 1, 2, 3, 4] and not got[3].any()
    # one instance with 5000 replies (MAX_BATCH-sized fan-in) spanning many waves
    rec = kat_cases.acc(2, [(1 + (k % 4), int(k % 3 != 0), 16) for k in range(5000)])
    o = Oracle(5, R.MODE_MIN)
    g = e.accept_tally(rec, kat_cases.inst_states(3), 0, -1)
    w = o.accept_tally(rec, kat_cases.inst_states(3), 0, -1)
    eq_struct(g[0], w[0])
    assert g[1] == w[1] and np.array_equal(g[2], w[2])


def test_accept_tally_errors(mk_engine):
    e = mk_engine(5, R.MODE_MIN)
    # out-of-window instance -> E_NIL_INSTANCE (the reference indexes past instanceSpace)
    with pytest.raises(MpxError) as ei:
        e.accept_tally(kat_cases.acc(9, [(1, 0, 16)]), kat_cases.inst_states(4), 0, -1)
    assert ei.value.code == R.E_NIL_INSTANCE
    # MIN: a NACK for a nil instance is harmless, an OK dereferences it
    st = kat_cases.inst_states(2)
    st[1]["status"] = R.STATUS_NIL
    e.accept_tally(kat_cases.acc(1, [(1, 0, 16)]), st, 0, -1)
    with pytest.raises(MpxError) as ei:
        e.accept_tally(kat_cases.acc(1, [(1, 1, 16)]), st, 0, -1)
    assert ei.value.code == R.E_NIL_INSTANCE
    # CLASSIC reads status for every reply
    c = mk_engine(5, R.MODE_CLASSIC)
    with pytest.raises(MpxError) as ei:
        c.accept_tally(kat_cases.acc(1, [(1, 0, 16)]), st, 0, -1)
    assert ei.value.code == R.E_NIL_INSTANCE
    # peer id outside peerCommits, reached only past the quorum test
    e.accept_tally(kat_cases.acc(0, [(9, 1, 16)]), kat_cases.inst_states(1), 0, -1)
    with pytest.raises(MpxError) as ei:
        e.accept_tally(kat_cases.acc(0, [(1, 1, 16), (9, 1, 16)]), kat_cases.inst_states(1), 0, -1)
    assert ei.value.code == R.E_BAD_ID
    # records out of ascending instance order
    rec = np.concatenate([kat_cases.acc(1, [(1, 1, 16)]), kat_cases.acc(0, [(1, 1, 16)])])
    with pytest.raises(MpxError) as ei:
        e.accept_tally(rec, kat_cases.inst_states(2), 0, -1)
    assert ei.value.code == R.E_INVAL


def test_committed_prefix(mk_engine):
    rng = np.random.default_rng(7)
    e, o = mk_engine(5, R.MODE_CLASSIC), Oracle(5, R.MODE_CLASSIC)
    for trial in range(20):
        n = int(rng.integers(1, 5000))
        st = kat_cases.inst_states(n, R.COMMITTED)
        if trial % 3:
            bad = rng.integers(0, n, int(rng.integers(1, 4)))
            st["status"][bad] = rng.choice([R.PREPARED, R.STATUS_NIL], len(bad))
        base = int(rng.integers(-3, 3))
        cu = int(rng.integers(base - 2, base + n // 2))
        assert e.committed_prefix(st, base, cu) == o.committed_prefix(st, base, cu)


# ---- A4 ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("n_rep", [1, 3, 5, 9])
def test_prepare_classic_ragged(mk_engine, n_rep):
    rng = np.random.default_rng(2000 + n_rep)
    for trial in range(3):
        rec, st = gen_cases.ragged_prepare(rng, 3000, n_rep, max_r=9, long_every=611,
                                           long_len=150 + 80 * trial, base=-trial)
        e, o = mk_engine(n_rep, R.MODE_CLASSIC), Oracle(n_rep, R.MODE_CLASSIC)
        db = int(rng.integers(-1, 400))
        got = e.prepare_select(rec, st, -trial, db)
        want = o.prepare_select(rec, st, -trial, db)
        eq_struct(got[0], want[0])
        assert got[1] == want[1] and np.array_equal(got[2], want[2])


def test_prepare_classic_config3_shape(mk_engine):
    rec, st = synth.prepare_replies(1 << 16, 5, 0.8, seed=43)
    e, o = mk_engine(5, R.MODE_CLASSIC), Oracle(5, R.MODE_CLASSIC)
    got = e.prepare_select(rec, st, 0, -1)
    want = o.prepare_select(rec, st, 0, -1)
    eq_struct(got[0], want[0])
    assert got[1] == want[1] and np.array_equal(got[2], want[2])


# ---- A3 ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("r", [1, 4, 9])
def test_prepare_min(mk_engine, r):
    rec, off, gst = synth.prepare_replies_min(5000, 5, seed=46 + r, replies_per_group=r)
    e, o = mk_engine(5, R.MODE_MIN), Oracle(5, R.MODE_MIN)
    pc = np.random.default_rng(r).integers(-1, 50, 5000 * 5).astype(np.int32)
    got = e.prepare_select_min(rec, off, gst, pc)
    want = o.prepare_select_min(rec, off, gst, pc)
    eq_struct(got[0], want[0])
    assert np.array_equal(got[1], want[1])
    eq_struct(got[2], want[2])


# ---- A5 / A6 ----------------------------------------------------------------------------------
@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_apply_config4_shape(mk_engine, dist):
    op, key, val = synth.commands(1 << 18, 1 << 12, 0.5, dist, seed=44)
    e, o = mk_engine(5, R.MODE_MIN), Oracle(5, R.MODE_MIN)
    for part in range(3):  # the table persists across calls
        sl = slice(part * (1 << 16), (part + 1) * (1 << 16) + part * 999)
        gr, gc = e.apply(op[sl], key[sl], val[sl])
        wr, wc = o.apply(op[sl], key[sl], val[sl])
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc)
        gk, gv = e.kv_export()
        wk, wv = o.kv_export()
        assert np.array_equal(gk, wk) and np.array_equal(gv, wv)


def test_apply_mixed_ops_and_special_keys(mk_engine):
    rng = np.random.default_rng(5)
    e, o = mk_engine(5, R.MODE_MIN), Oracle(5, R.MODE_MIN)
    for trial in range(4):
        op, key, val = gen_cases.commands_mixed(rng, 50000, 300 + 3000 * trial)
        gr, gc = e.apply(op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc)
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)
    # empty call, import/clear
    e.apply(np.zeros(0, np.uint8), np.zeros(0, np.int64), np.zeros(0, np.int64))
    e.kv_clear()
    assert e.kv_size() == 0
    e.kv_import(np.array([3, -7], np.int64), np.array([30, 70], np.int64))
    r, _ = e.apply(np.array([R.OP_GET, R.OP_GET, R.OP_GET], np.uint8),
                   np.array([3, -7, 4], np.int64), np.zeros(3, np.int64))
    assert list(r) == [30, 70, 0]


@pytest.mark.parametrize("chunk", [1, 7, 777, 4096])
def test_apply_chunked(mk_engine, chunk):
    """the apply pipeline cuts a call into chunks (mpx_config.apply_chunk commands): slot state
    and conflicts carry across chunk boundaries and calls; a GET in one chunk on a key that is
    only PUT in a later chunk still conflicts with that PUT"""
    rng = np.random.default_rng(77 + chunk)
    e = mk_engine(5, R.MODE_MIN, apply_chunk=chunk, apply_path=R.APPLY_SORTED)
    o = Oracle(5, R.MODE_MIN)
    handmade = (np.array([R.OP_GET, R.OP_DELETE, R.OP_GET, R.OP_PUT, R.OP_GET, R.OP_PUT, R.OP_GET],
                         np.uint8),
                np.array([5, 6, 5, 5, 7, 6, 6], np.int64), np.arange(7, dtype=np.int64) + 100)
    calls = [handmade] + [gen_cases.commands_mixed(rng, 5000 if chunk > 1 else 300, 40 + 400 * t)
                          for t in range(3)] + [handmade]
    for op, key, val in calls:
        gr, gc = e.apply(op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc)
        gk, gv = e.kv_export()
        wk, wv = o.kv_export()
        assert np.array_equal(gk, wk) and np.array_equal(gv, wv)


def _apply_form(e, form, op, key, val):
    """one apply call through the host-pointer form (the replica-batch kernels' three-launch
    form over pinned host memory) or the device-pointer form (their one-launch form)"""
    if form == "host":
        return e.apply(op, key, val)
    from minpaxos_amd.devbuf import Arena
    m = len(op)
    e.apply_reserve(m)
    with Arena(e) as ar:
        d_op, d_key, d_val = ar.put(op), ar.put(key), ar.put(val)
        d_ret, d_conf = ar.empty(m, np.int64), ar.empty(m, np.uint8)
        e.apply_dev(d_op.ptr, d_key.ptr, d_val.ptr, m, d_ret.ptr, d_conf.ptr, e.stream)
        e.stream_synchronize(e.stream)
        return ar.get(d_ret), ar.get(d_conf)


@pytest.mark.parametrize("path,form", [(R.APPLY_SMALL, "host"), (R.APPLY_SMALL, "dev"),
                                       (R.APPLY_AUTO, "host"), (R.APPLY_AUTO, "dev"),
                                       (R.APPLY_SORTED, "host")])
def test_apply_small_calls(mk_engine, path, form):
    """replica-sized calls (one drained executeCommands batch, MAX_BATCH = 5000 commands,
    bareminpaxos.go:22,1071-1089): sizes around the wave (64), the workgroup (1024) and the
    small kernels' limit (16384: up to three drained MAX_BATCH batches), mixed ops, the
    special keys, a hot key, GETs of absent keys
    before their first PUT, and one table carried through all calls; every call's results,
    the table and its size bit-exact. AUTO and SMALL run the one-launch kernel (apply_small.hip)
    here, SORTED the multi-launch pipeline; "dev" runs every call through mpx_apply_dev (the
    replica-batch kernels' one-launch form: hash partitions, one workgroup each, up to 64 of
    them at 16384 commands)"""
    rng = np.random.default_rng(91 + path)
    e, o = mk_engine(5, R.MODE_MIN, kv_capacity=1 << 16, apply_path=path), Oracle(5, R.MODE_MIN)
    sizes = [1, 2, 63, 64, 65, 1000, 1023, 1024, 1025, 4095, 5000, 8191, 8192, 8193, 9000,
             12000, 16383, 16384]
    for i, m in enumerate(sizes):
        op, key, val = gen_cases.commands_mixed(rng, m, 50 + 37 * i)
        key = np.where(key > 0, key + (i % 3) * 1_000_003, key)  # fresh keys every third call
        if i % 4 == 1:
            key[rng.random(m) < 0.5] = 424242  # a hot key
        gr, gc = _apply_form(e, form, op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr), (m, np.nonzero(gr != wr)[0][:5])
        assert np.array_equal(gc, wc), (m, np.nonzero(gc != wc)[0][:5])
        gk, gv = e.kv_export()
        wk, wv = o.kv_export()
        assert np.array_equal(gk, wk) and np.array_equal(gv, wv), m
        assert e.kv_size() == len(wk)
    # wide key spaces: almost every command alone on its key (the sort sees a few dozen shared
    # ones), and one call where exactly 1024 / 1025 commands share keys (the rank / radix switch)
    for m, kr, seed in ((8192, 1 << 40, 95), (5000, 1 << 20, 96), (16384, 1 << 20, 97)):
        op, key, val = synth.commands(m, kr, 0.5, "uniform", seed=seed)
        gr, gc = _apply_form(e, form, op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc), m
    for n_sh in (1024, 1025):
        op, key, val = synth.commands(6000, 1 << 40, 0.5, "uniform", seed=n_sh)
        op[:] = R.OP_PUT  # every command gets a slot: exactly n_sh are shared
        key = key + (1 << 41)  # fresh, distinct
        key[:n_sh // 2] = key[n_sh // 2:n_sh // 2 * 2]  # n_sh // 2 pairs share a key ...
        if n_sh % 2:
            key[n_sh - 1] = key[0]  # ... and one triple
        gr, gc = _apply_form(e, form, op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc), n_sh
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)
    # the device-pointer form, one MAX_BATCH call
    from minpaxos_amd.devbuf import Arena
    op, key, val = synth.commands(5000, 1 << 12, 0.5, "uniform", seed=92)
    e.apply_reserve(5000)
    with Arena(e) as ar:
        d_op, d_key, d_val = ar.put(op), ar.put(key), ar.put(val)
        d_ret, d_conf = ar.empty(5000, np.int64), ar.empty(5000, np.uint8)
        e.apply_dev(d_op.ptr, d_key.ptr, d_val.ptr, 5000, d_ret.ptr, d_conf.ptr, e.stream)
        e.stream_synchronize(e.stream)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(ar.get(d_ret), wr) and np.array_equal(ar.get(d_conf), wc)


def test_apply_staged(mk_engine):
    """the zero-copy replica-batch form (mpx_apply_buffers + mpx_apply_staged): batches written
    straight into the engine's pinned arrays, mixed with host-pointer calls on the same table,
    every call and the final table bit-exact; sizes past the arrays are rejected"""
    rng = np.random.default_rng(94)
    e, o = mk_engine(5, R.MODE_MIN, kv_capacity=1 << 16), Oracle(5, R.MODE_MIN)
    io = e.apply_buffers(6000)
    assert io["cap"] >= 6000
    for i, m in enumerate([5000, 1, 6000, 4096, 333]):
        op, key, val = gen_cases.commands_mixed(rng, m, 700 + 13 * i)
        if i % 2:
            gr, gc = e.apply(op, key, val)
        else:
            io["op"][:m], io["key"][:m], io["val"][:m] = op, key, val
            e.apply_staged(m)
            gr, gc = io["ret"][:m].copy(), io["conf"][:m].copy()
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc), m
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)
    with pytest.raises(MpxError):
        e.apply_staged(io["cap"] + 1)


def test_apply_small_then_pipelines(mk_engine):
    """the one-launch kernel neither reads nor advances the call epoch: calls on it between
    calls of the partitioned and sorted pipelines (which tag slots with the epoch) leave
    every later call bit-exact"""
    rng = np.random.default_rng(93)
    e, o = mk_engine(5, R.MODE_MIN, kv_capacity=1 << 14), Oracle(5, R.MODE_MIN)
    for i, m in enumerate([20000, 3000, 30000, 100, 9000, 8000, 40000]):
        op, key, val = gen_cases.commands_mixed(rng, m, 2000)
        gr, gc = e.apply(op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc), m
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)


@pytest.mark.parametrize("path", [R.APPLY_PARTITIONED, R.APPLY_SORTED])
@pytest.mark.parametrize("hot_min", [R.APPLY_NO_HOT, 2, 8])
def test_apply_paths(mk_engine, hot_min, path):
    """the partitioned pipeline with no hot keys (every key through the bins), with as many hot
    keys as fit (apply_hot_min=2), with the sampled default, and the sort-based pipeline:
    every call bit-exact, table state carried across calls. Fresh key ranges per call put GETs
    of absent keys before their first PUT in the same bin (the two-pass bins); the small table
    (32 buckets of 256 slots) is driven to ~70% occupancy"""
    rng = np.random.default_rng(31 + hot_min % 97 + 10 * path)
    e = mk_engine(5, R.MODE_MIN, kv_capacity=4096, apply_path=path, apply_hot_min=hot_min)
    o = Oracle(5, R.MODE_MIN)
    calls = []
    for t in range(3):
        op, key, val = gen_cases.commands_mixed(rng, 30000, 1500)
        calls.append((op, np.where(key > 0, key + t * 1_000_003, key), val))
    calls.append(synth.commands(50000, 300, 0.5, "zipf", seed=5))
    calls.append(synth.commands(9000, 1 << 40, 0.2, "uniform", seed=6))  # mostly absent GETs
    calls.append(synth.commands(70000, 1200, 0.6, "uniform", seed=7))
    calls.append((np.full(5000, R.OP_GET, np.uint8), np.full(5000, 9, np.int64),
                  np.arange(5000, dtype=np.int64)))  # one hot key, GETs only
    for op, key, val in calls:
        gr, gc = e.apply(op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc)
        gk, gv = e.kv_export()
        wk, wv = o.kv_export()
        assert np.array_equal(gk, wk) and np.array_equal(gv, wv)
        assert e.kv_size() == len(wk)


def _bucket_keys(lgnb, bucket, n, start=1):
    """n keys whose hash (kvtab.hpp hash64) puts them in `bucket` of a table of 2^lgnb buckets"""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    x = np.arange(start, start + 64 * n * (1 << lgnb), dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = x ^ (x >> np.uint64(30))
        h = (h * np.uint64(0xBF58476D1CE4E5B9)) & M
        h ^= h >> np.uint64(27)
        h = (h * np.uint64(0x94D049BB133111EB)) & M
        h ^= h >> np.uint64(31)
    sel = x[(h >> np.uint64(64 - lgnb)) == np.uint64(bucket)]
    assert len(sel) >= n
    return sel[:n].astype(np.int64)


@pytest.mark.parametrize("path,form", [(R.APPLY_SMALL, "host"), (R.APPLY_SMALL, "dev"),
                                       (R.APPLY_PARTITIONED, "host"), (R.APPLY_SORTED, "host")])
def test_apply_full_bucket_lookups(mk_engine, path, form):
    """a bucket filled exactly (256 PUT keys in one of the 4 buckets of a 1024-slot table):
    GETs and other ops of keys absent from that full bucket return NIL and leave the table
    unchanged, on every pipeline (mpx.h: only keys PUT at some point occupy the table); a PUT of
    a new key in the full bucket is MPX_E_KV_FULL"""
    e = mk_engine(5, R.MODE_MIN, kv_capacity=512, apply_path=path)  # 1024 slots, 4 buckets
    o = Oracle(5, R.MODE_MIN)
    full = _bucket_keys(2, 1, 256 + 64)
    fill, absent = full[:256], full[256:]
    op = np.full(256, R.OP_PUT, np.uint8)
    gr, gc = e.apply(op, fill, fill * 7)
    wr, wc = o.apply(op, fill, fill * 7)
    assert np.array_equal(gr, wr) and np.array_equal(gc, wc)
    rng = np.random.default_rng(17 + path)
    other = _bucket_keys(2, 2, 100, start=1 << 30)
    key = np.concatenate([absent, absent[:10], fill[:50], other])
    op = np.concatenate([np.full(74, R.OP_GET, np.uint8), np.full(50, R.OP_GET, np.uint8),
                         np.full(100, R.OP_PUT, np.uint8)])
    op[rng.random(len(op)) < 0.1] = R.OP_DELETE
    op[:len(absent) + 10] = np.where(op[:len(absent) + 10] == R.OP_PUT, R.OP_GET,
                                     op[:len(absent) + 10])
    perm = rng.permutation(len(key))
    key, op = key[perm], op[perm]
    val = np.arange(len(key), dtype=np.int64) + 1000
    gr, gc = _apply_form(e, form, op, key, val)
    wr, wc = o.apply(op, key, val)
    assert np.array_equal(gr, wr), np.nonzero(gr != wr)[0][:5]
    assert np.array_equal(gc, wc)
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)
    assert e.kv_size() == len(wk)
    with pytest.raises(MpxError) as ei:
        e.apply(np.array([R.OP_PUT], np.uint8), absent[:1], np.array([5], np.int64))
    assert ei.value.code == R.E_KV_FULL


@pytest.mark.parametrize("path", [R.APPLY_SMALL, R.APPLY_PARTITIONED, R.APPLY_SORTED])
def test_apply_bucket_full(mk_engine, path):
    """more distinct PUT keys than a table of 4 buckets x 256 slots holds: MPX_E_KV_FULL (the
    oracle's Go map never fills; the engine's capacity is documented in mpx.h); a call that fits
    still matches the oracle afterwards on a fresh engine"""
    e = mk_engine(5, R.MODE_MIN, kv_capacity=512, apply_path=path)  # 1024 slots
    keys = np.arange(1, 1501, dtype=np.int64)
    with pytest.raises(MpxError) as ei:
        e.apply(np.full(len(keys), R.OP_PUT, np.uint8), keys, keys * 3)
    assert ei.value.code == R.E_KV_FULL
    e2, o = mk_engine(5, R.MODE_MIN, kv_capacity=512, apply_path=path), Oracle(5, R.MODE_MIN)
    rng = np.random.default_rng(3)
    op, key, val = gen_cases.commands_mixed(rng, 20000, 400)
    gr, gc = e2.apply(op, key, val)
    wr, wc = o.apply(op, key, val)
    assert np.array_equal(gr, wr) and np.array_equal(gc, wc)


def test_apply_size_dispatch(mk_engine):
    """with apply_path AUTO the call size picks the pipeline: the replica-batch kernels up to
    16384 commands, the sort-based pipeline below apply_fast_min (here 20000), the partitioned
    one from there: calls on both sides of both switches carry one table, bit-exact. The
    device-pointer entry point reserved for the largest call also runs the smaller calls, which
    take the other pipelines with their own scratch layouts (mpx_apply_reserve covers all)"""
    from minpaxos_amd.devbuf import Arena
    rng = np.random.default_rng(57)
    e = mk_engine(5, R.MODE_MIN, kv_capacity=1 << 16, apply_fast_min=20000)
    o = Oracle(5, R.MODE_MIN)
    sizes = [40000, 19999, 20000, 37, 16384, 16385, 25000, 1]
    e.apply_reserve(max(sizes))
    with Arena(e) as ar:
        for i, m in enumerate(sizes):
            op, key, val = gen_cases.commands_mixed(rng, m, 3000)
            if i % 2:
                gr, gc = e.apply(op, key, val)
            else:
                d_op, d_key, d_val = ar.put(op), ar.put(key), ar.put(val)
                d_ret, d_conf = ar.empty(m, np.int64), ar.empty(m, np.uint8)
                e.apply_dev(d_op.ptr, d_key.ptr, d_val.ptr, m, d_ret.ptr, d_conf.ptr, e.stream)
                e.stream_synchronize(e.stream)
                gr, gc = ar.get(d_ret), ar.get(d_conf)
            wr, wc = o.apply(op, key, val)
            assert np.array_equal(gr, wr) and np.array_equal(gc, wc), m
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)


@pytest.mark.parametrize("path", [R.APPLY_PARTITIONED, R.APPLY_SORTED])
def test_apply_epoch_wrap(mk_engine, path):
    """the call epoch tags every slot a call touched (state.Conflict against the same call's
    earlier commands); 2^30 calls wrap it to 1 after clearing every tag. Calls at epochs 1..3
    tag the slots of key set A; the epoch then moves to three calls before the wrap
    (mpx_debug_kv_set_epoch, slots untouched); two calls on a disjoint key set B run at
    2^30-2 and 2^30-1, and three calls on A at the wrapped epochs 1..3: without the wrap sweep
    A's slots would still carry tags 1..3 and read as touched earlier in the same call. Every
    call and the final table bit-exact; after the wrap no slot carries a pre-wrap tag."""
    rng = np.random.default_rng(71 + path)
    e, o = mk_engine(5, R.MODE_MIN, kv_capacity=4096, apply_path=path), Oracle(5, R.MODE_MIN)

    def call(key_lo):
        op, key, val = gen_cases.commands_mixed(rng, 20000, 700)
        key = np.where(key > 0, key % 700 + key_lo, key)
        gr, gc = e.apply(op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc)

    for _ in range(3):
        call(1)                       # epochs 1, 2, 3 on key set A
    e.debug_kv_set_epoch((1 << 30) - 3)
    for _ in range(2):
        call(1_000_000)               # epochs 2^30-2, 2^30-1 on key set B
    for _ in range(3):
        call(1)                       # the wrap: epochs 1, 2, 3 on A again
    tags = e.debug_kv_state() >> 2
    assert tags.max() <= 3 and set(np.unique(tags)) <= {0, 1, 2, 3}
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)
    with pytest.raises(MpxError):
        e.debug_kv_set_epoch(1 << 30)  # outside [1, 2^30)


@pytest.mark.parametrize("form", ["host", "dev"])
def test_apply_small_lists_and_tag_wrap(mk_engine, form):
    """replica-sized calls resolve each key's commands by walking the key's list of the call
    (apply_small.hip steps 1-3) and leave lists longer than 16 to the one-workgroup sort: calls
    whose key ranges put 1 .. ~100 commands on a key mix both in one call. The list heads are
    tagged with the call (18 bits); at the wrap the heads are cleared: calls on key set A at tags
    1..3, the tag moved to three calls before the wrap (mpx_debug_kv_set_small_tag), two calls on
    a disjoint set B, then calls on A at the wrapped tags 1..3 - without the clear A's heads would
    still carry tags 1..3 and link stale positions. Every call and the table bit-exact; "dev":
    the one-launch form, whose partitions resolve their own LONG lists."""
    e = mk_engine(5, R.MODE_MIN, kv_capacity=1 << 16, apply_path=R.APPLY_SMALL)
    o = Oracle(5, R.MODE_MIN)

    def call(m, kr, lo, seed):
        op, key, val = synth.commands(m, kr, 0.5, "uniform", seed=seed, other_ops=0.1)
        key = key + lo
        gr, gc = _apply_form(e, form, op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr), (m, kr, np.nonzero(gr != wr)[0][:5])
        assert np.array_equal(gc, wc), (m, kr, np.nonzero(gc != wc)[0][:5])

    for i, kr in enumerate((20000, 2000, 600, 300, 250, 40, 1)):
        call(5000, kr, 1, 300 + i)
    for i in range(3):
        call(3000, 500, 10_000_000, 310 + i)          # key set A
    e.debug_kv_set_small_tag((1 << 18) - 3)
    for i in range(2):
        call(3000, 500, 20_000_000, 320 + i)          # key set B, tags 2^18-2, 2^18-1
    for i in range(3):
        call(3000, 500, 10_000_000, 330 + i)          # A again at the wrapped tags 1..3
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)
    assert e.kv_size() == len(wk)
    with pytest.raises(MpxError):
        e.debug_kv_set_small_tag(1 << 18)


def _part_keys(n, lgnp, part, start):
    """n distinct keys whose partition hash (apply_small.hip part_of) is `part` of 2^lgnp"""
    x = np.arange(start, start + (n << lgnp) * 4, dtype=np.uint64)
    f = ((x & np.uint64(0xFFFFFFFF)) ^ (x >> np.uint64(32))) * np.uint64(0x9E3779B1)
    sel = x[((f & np.uint64(0xFFFFFFFF)) >> np.uint64(32 - lgnp)) == np.uint64(part)]
    assert len(sel) >= n
    return sel[:n].astype(np.int64)


def test_apply_small_partition_skew(mk_engine):
    """the one-launch form (mpx_apply_dev, at most 16384 commands) splits a call into 2^k hash
    partitions, one workgroup each; a partition of at most 1024 commands whose keys each carry at
    most 16 of them resolves in LDS, any other takes the list phases. Calls that put 2000-3000
    commands on distinct keys into one partition (the list phases without LONG lists), a hot key
    in the same partition (LONG lists), GETs of absent keys before and after their first PUT, the
    sentinel key, calls whose every command is on one key: every call and the table bit-exact"""
    rng = np.random.default_rng(99)
    e, o = mk_engine(5, R.MODE_MIN, kv_capacity=1 << 16, apply_path=R.APPLY_SMALL), \
        Oracle(5, R.MODE_MIN)
    def lg_parts(m, per=128, cap=256):  # apply_small.hip launch_apply_small (MPX_SMALL_PART_CMDS)
        n = 1
        while n < cap and n * per < m:
            n <<= 1
        return n.bit_length() - 1

    for i, m in enumerate((16384, 5000, 8000)):
        lgnp = lg_parts(m)
        op, key, val = gen_cases.commands_mixed(rng, m, 400 + 100 * i)
        skew = _part_keys(2000 + 500 * i, lgnp, 3 + i, start=10_000_000 * (i + 1))
        at = rng.choice(m, size=len(skew), replace=False)
        key[at] = skew
        if i == 1:
            key[at[:200]] = skew[0]  # a hot key inside the skewed partition
        if i == 2:
            key[rng.random(m) < 0.01] = np.iinfo(np.int64).min  # the sentinel key
        gr, gc = _apply_form(e, "dev", op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr), (m, np.nonzero(gr != wr)[0][:5])
        assert np.array_equal(gc, wc), (m, np.nonzero(gc != wc)[0][:5])
        gk, gv = e.kv_export()
        wk, wv = o.kv_export()
        assert np.array_equal(gk, wk) and np.array_equal(gv, wv), m
        assert e.kv_size() == len(wk)
    # every command on one key (one partition, one LONG list of the whole call): a fresh key, the
    # sentinel key, a key present in the table
    for m, k in ((5000, 77_000_001), (16384, np.iinfo(np.int64).min), (3000, int(key[0]))):
        op = rng.choice([R.OP_PUT, R.OP_GET, R.OP_DELETE], m, p=[0.4, 0.5, 0.1]).astype(np.uint8)
        kk = np.full(m, k, np.int64)
        vv = rng.integers(-(1 << 62), 1 << 62, m).astype(np.int64)
        gr, gc = _apply_form(e, "dev", op, kk, vv)
        wr, wc = o.apply(op, kk, vv)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc), (m, k)
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)


@pytest.mark.parametrize("cap_lg", [22, 23, 25, 26])
def test_apply_large_table(mk_engine, cap_lg):
    """tables past the partition's 1024 bins: kv_capacity 2^22 / 2^23 / 2^25 / 2^26 keys
    (2^23..2^27 slots) split the log into 1024 super-bins of 2 / 4 / 16 / 32 bins, which the
    resolve workgroup takes one after another (partitioned pipeline forced for the smaller
    tables, AUTO's pick - the same pipeline - for 2^27 slots). Every call and the final table
    bit-exact, across calls, with GETs of new keys before their first PUT (the two-pass bins)
    and a zipf call (hot keys)"""
    rng = np.random.default_rng(41 + cap_lg)
    path = R.APPLY_PARTITIONED if cap_lg < 26 else R.APPLY_AUTO
    e = mk_engine(5, R.MODE_MIN, kv_capacity=1 << cap_lg, apply_path=path)
    o = Oracle(5, R.MODE_MIN)
    calls = [gen_cases.commands_mixed(rng, 60000, 20000) for _ in range(2)]
    calls.append(synth.commands(200000, 1 << 40, 0.5, "uniform", seed=cap_lg))
    calls.append(synth.commands(100000, 5000, 0.5, "zipf", seed=cap_lg + 1))
    for op, key, val in calls:
        gr, gc = e.apply(op, key, val)
        wr, wc = o.apply(op, key, val)
        assert np.array_equal(gr, wr) and np.array_equal(gc, wc)
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv)
    assert e.kv_size() == len(wk)


def test_conflict_batch(mk_engine):
    rng = np.random.default_rng(9)
    e, o = mk_engine(5, R.MODE_MIN), Oracle(5, R.MODE_MIN)
    # LDS-staged workgroups (with a few big instances), then ranges too long to stage
    for every, big in ((500, 700), (90, 400)):
        sizes = rng.integers(0, 12, 4000)
        sizes[::every] = big
        off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        op, key, _ = gen_cases.commands_mixed(rng, int(off[-1]), 2000, neg_keys=False)
        assert np.array_equal(e.conflict_batch(op, key, off), o.conflict_batch(op, key, off))


@pytest.mark.gpu
@pytest.mark.parametrize("kshift,oshift", [(0, 0), (1, 3), (1, 15), (0, 7)])
def test_conflict_batch_dev_misaligned(mk_engine, kshift, oshift):
    """the device form with key / op pointers off their 16-byte alignment: the kernel stages
    each workgroup's range by 16-byte vectors from the aligned address at or below it"""
    from minpaxos_amd.devbuf import Arena
    rng = np.random.default_rng(11 + kshift * 16 + oshift)
    e, o = mk_engine(5, R.MODE_MIN), Oracle(5, R.MODE_MIN)
    sizes = rng.integers(0, 9, 3000)
    sizes[::700] = 40
    sizes[5:9] = 0  # empty instances
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    m = int(off[-1])
    op, key, _ = gen_cases.commands_mixed(rng, m, 300, neg_keys=True)
    want = o.conflict_batch(op, key, off)
    n_inst = len(off) - 1
    with Arena(e) as ar:
        d_key = ar.put(np.concatenate([np.zeros(kshift, np.int64), key]))
        d_op = ar.put(np.concatenate([np.zeros(oshift, np.uint8), op]))
        d_off = ar.put(off)
        d_out = ar.full(n_inst, np.uint8, 0xEE)
        e.conflict_batch_dev(d_op.at(oshift), d_key.at(kshift), d_off.ptr, n_inst, d_out.ptr)
        e.stream_synchronize(None)
        got = ar.get(d_out, n_inst - 1)
    assert np.array_equal(got, want)


# ---- fused group step (config 5 shape) ----------------------------------------------------------
def _cmp_group(got, want, G, K):
    for f in ("committed_out", "executed_out", "peer_out", "ret", "conf_prev", "kv_cnt",
              "decided", "n_decided"):
        a, b = got[f], want[f]
        bad = np.nonzero(a != b)[0]
        assert len(bad) == 0, f"{f} differs at {bad[:8]}: {a[bad[:5]]} vs {b[bad[:5]]}"
    eq_struct(got["st_out"], want["st_out"])
    cnt = want["kv_cnt"]
    for g in range(G):
        n = int(cnt[g])
        assert np.array_equal(got["kv_key"][g * K:g * K + n], want["kv_key"][g * K:g * K + n]), g
        assert np.array_equal(got["kv_val"][g * K:g * K + n], want["kv_val"][g * K:g * K + n]), g


@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC])
def test_group_step_config5_shape(mk_engine, mode):
    G, ipg, K = 96, 256, 512
    b = synth.group_batch(G, ipg, 5, 4, 256, seed=45)
    e, o = mk_engine(5, mode, kv_per_group=K), Oracle(5, mode, kv_per_group=K)
    got = e.group_step(b)
    want = o.group_step(b)
    _cmp_group(got, want, G, K)
    # second step from the produced tables and watermarks, new replies/commands
    b2 = synth.group_batch(G, ipg, 5, 4, 256, seed=46)
    b2["committed_in"] = want["committed_out"]
    b2["executed_in"] = np.minimum(want["executed_out"], 100).astype(np.int32)
    b2["peer_in"] = want["peer_out"]
    got2 = e.group_step(b2, want["kv_cnt"], want["kv_key"], want["kv_val"])
    want2 = o.group_step(b2, want["kv_cnt"], want["kv_key"], want["kv_val"])
    _cmp_group(got2, want2, G, K)


def test_group_step_ragged(mk_engine):
    """variable replies per instance, nil Cmds, big groups (multi-chunk apply), skewed keys"""
    rng = np.random.default_rng(31)
    G, ipg, K = 40, 512, 600
    recs, offs, sts, ops, keys, vals, coff = [], [0], [], [], [], [], [0]
    for g in range(G):
        rec, st = gen_cases.ragged_accept(rng, ipg, 5, max_r=6, random_state=False, p_ok=0.75)
        rec["id"] = rng.integers(0, 5, len(rec))
        recs.append(rec)
        offs.append(offs[-1] + len(rec))
        sts.append(st)
        nc = rng.integers(0, 9, ipg)
        m = int(nc.sum())
        op, key, val = gen_cases.commands_mixed(rng, m, 20 if g % 3 == 0 else 700, neg_keys=True)
        ops.append(op); keys.append(key); vals.append(val)
        coff.extend((coff[-1] + np.cumsum(nc)).tolist())
    b = dict(n_groups=G, ipg=ipg, recs=np.concatenate(recs),
             grp_rec_off=np.array(offs, np.uint64), st_in=np.concatenate(sts),
             committed_in=rng.integers(-1, 5, G).astype(np.int32),
             executed_in=rng.integers(-1, 3, G).astype(np.int32),
             peer_in=np.zeros(G * 5, np.int32), op=np.concatenate(ops), key=np.concatenate(keys),
             val=np.concatenate(vals), cmd_off=np.array(coff, np.uint32),
             has_cmds=(rng.random(G * ipg) > 0.002).astype(np.uint8))
    for mode in (R.MODE_MIN, R.MODE_CLASSIC):
        e, o = mk_engine(5, mode, kv_per_group=K), Oracle(5, mode, kv_per_group=K)
        ret0 = np.full(len(b["op"]), 12345, np.int64)
        got = e.group_step(b, ret=ret0)
        want = o.group_step(b, ret=ret0)
        _cmp_group(got, want, G, K)


@pytest.mark.parametrize("shape", [
    dict(N=5, ipg=256, K=256, keys=256, B=4),      # FastBase
    dict(N=7, ipg=256, K=256, keys=256, B=4),      # FastRecs (6 x 256 replies)
    dict(N=9, ipg=256, K=256, keys=200, B=3),      # FastRecs, 8 replies per instance
    dict(N=5, ipg=256, K=1024, keys=1024, B=4),    # FastKeys (tables of up to 1024 keys)
    dict(N=5, ipg=512, K=512, keys=256, B=4),      # FastWide (512 instances per group)
    dict(N=5, ipg=512, K=256, keys=256, B=4),      # FastWide256 (512 instances, 256-key tables)
    dict(N=3, ipg=400, K=256, keys=240, B=5),      # FastWide256, partial space, fuller tables
    dict(N=5, ipg=384, K=512, keys=400, B=5),      # FastWide with a partial instance space
    dict(N=3, ipg=128, K=1024, keys=5000, B=9),    # FastKeys -> general (1152 commands)
], ids=lambda d: "N{N}_ipg{ipg}_K{K}_keys{keys}_B{B}".format(**d))
@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC])
def test_group_step_variants(mk_engine, shape, mode):
    """every fast-path capacity variant (and its run-time fallback to the general kernel),
    two steps: from empty tables, then from the tables the first step produced"""
    G, N, ipg, K = 128, shape["N"], shape["ipg"], shape["K"]
    b = synth.group_batch(G, ipg, N, shape["B"], shape["keys"], seed=90 + N + ipg)
    e, o = mk_engine(N, mode, kv_per_group=K), Oracle(N, mode, kv_per_group=K)
    try:
        want = o.group_step(b)
    except OracleError:
        pytest.skip("oracle: table full for this shape")
    _cmp_group(e.group_step(b), want, G, K)
    b2 = synth.group_batch(G, ipg, N, shape["B"], shape["keys"], seed=91 + N + ipg)
    try:
        want2 = o.group_step(b2, want["kv_cnt"], want["kv_key"], want["kv_val"])
    except OracleError:
        return
    _cmp_group(e.group_step(b2, want["kv_cnt"], want["kv_key"], want["kv_val"]), want2, G, K)


def _dev_group_batch(ar, b, N, K, with_nd):
    """the device-pointer mpx_group_batch of a host batch dict (empty input tables)"""
    G, ipg, m = b["n_groups"], b["ipg"], len(b["op"])
    d = dict(recs=ar.put(b["recs"]), off=ar.put(b["grp_rec_off"]), st_in=ar.put(b["st_in"]),
             st_out=ar.put(b["st_in"]), ci=ar.put(b["committed_in"]),
             co=ar.empty(G, np.int32), ei=ar.put(b["executed_in"]), eo=ar.empty(G, np.int32),
             pi=ar.put(b["peer_in"]), po=ar.empty(G * N, np.int32), op=ar.put(b["op"]),
             key=ar.put(b["key"]), val=ar.put(b["val"]), coff=ar.put(b["cmd_off"]),
             hc=ar.put(b["has_cmds"]) if b.get("has_cmds") is not None else None,
             ret=ar.full(m, np.int64, 0), conf=ar.full(m, np.uint8, 0),
             kc0=ar.full(G, np.uint32, 0), kk0=ar.full(G * K, np.int64, 0),
             kv0=ar.full(G * K, np.int64, 0), kc1=ar.full(G, np.uint32, 0),
             kk1=ar.full(G * K, np.int64, 0), kv1=ar.full(G * K, np.int64, 0),
             nd=ar.full(G, np.uint32, 0) if with_nd else None)
    p = lambda x: x.ptr if x is not None else None  # noqa: E731
    gb = _lib.MpxGroupBatch(
        G, ipg, p(d["recs"]), p(d["off"]), p(d["st_in"]), p(d["st_out"]), p(d["ci"]), p(d["co"]),
        p(d["ei"]), p(d["eo"]), p(d["pi"]), p(d["po"]), p(d["op"]), p(d["key"]), p(d["val"]),
        p(d["coff"]), p(d["hc"]), p(d["ret"]), p(d["conf"]), p(d["kc0"]), p(d["kk0"]),
        p(d["kv0"]), p(d["kc1"]), p(d["kk1"]), p(d["kv1"]), None, p(d["nd"]))
    return gb, d


def _want_totals(b, want):
    """decided instances, executed instances, executed commands of one step (oracle outputs)"""
    G, ipg = b["n_groups"], b["ipg"]
    coff = b["cmd_off"].astype(np.int64)
    xi = xc = 0
    for g in range(G):
        lo, eo = max(int(b["executed_in"][g]) + 1, 0), int(want["executed_out"][g])
        if lo <= eo < ipg:
            xi += eo - lo + 1
            xc += int(coff[g * ipg + eo + 1] - coff[g * ipg + lo])
    return [int(want["decided"].sum()), xi, xc]


@pytest.mark.parametrize("kind", ["fast", "general"])
def test_group_step_fused_totals(mk_engine, kind):
    """mpx_group_step_totals_dev: the step totals reduced by the step's second kernel (an empty
    work list: slices of the fast kernel's outputs; a full one: its last workgroup over every
    group) equal the oracle's and mpx_step_totals_dev's over repeated steps (the accumulators
    and tickets reset themselves) and after a plain mpx_group_step_dev; without n_decided the
    call is rejected"""
    from minpaxos_amd.devbuf import Arena
    if kind == "fast":
        N, K = 5, 256
        b = synth.group_batch(300, 256, N, 4, 256, seed=77)
    else:  # > 1024 commands per group: every group goes through the work list
        N, K = 3, 1024
        b = synth.group_batch(64, 128, N, 9, 800, seed=78)
    b.setdefault("has_cmds", None)
    e, o = mk_engine(N, R.MODE_MIN, kv_per_group=K), Oracle(N, R.MODE_MIN, kv_per_group=K)
    want = _want_totals(b, o.group_step(b))
    with Arena(e) as ar:
        for with_nd in (True, False):
            gb, d = _dev_group_batch(ar, b, N, K, with_nd)
            tot = ar.full(3, np.int64, 0x55)
            e.group_step_dev(gb, e.stream)  # leaves no partials behind
            if not with_nd:
                with pytest.raises(MpxError):
                    e.group_step_totals_dev(gb, tot.ptr, e.stream)
                continue
            for _ in range(3):
                e.group_step_totals_dev(gb, tot.ptr, e.stream)
                e.stream_synchronize(e.stream)
                assert ar.get(tot).tolist() == want
            if with_nd:
                tot2 = ar.full(3, np.int64, 0x55)
                e.step_totals_dev(gb, tot2.ptr, e.stream)
                e.stream_synchronize(e.stream)
                assert ar.get(tot2).tolist() == want


def test_group_step_events_destroyed_unregister(mk_engine):
    """destroying a registered timing event unregisters the pair, so later group
    steps record nothing (no use of a destroyed event) and stay correct"""
    from minpaxos_amd.devbuf import Arena
    N, K = 5, 256
    b = synth.group_batch(40, 256, N, 4, 256, seed=81)
    b.setdefault("has_cmds", None)
    e, o = mk_engine(N, R.MODE_MIN, kv_per_group=K), Oracle(N, R.MODE_MIN, kv_per_group=K)
    want = _want_totals(b, o.group_step(b))
    with Arena(e) as ar:
        gb, d = _dev_group_batch(ar, b, N, K, True)
        ev0, ev1 = e.event_create(), e.event_create()
        e.group_step_events(ev0, ev1)
        tot = ar.full(3, np.int64, 0x55)
        e.group_step_totals_dev(gb, tot.ptr, e.stream)
        e.stream_synchronize(e.stream)
        assert e.event_elapsed_ms(ev0, ev1) >= 0.0
        e.event_destroy(ev1)  # the pair is unregistered here
        e.event_destroy(ev0)
        for _ in range(2):
            e.group_step_totals_dev(gb, tot.ptr, e.stream)
            e.stream_synchronize(e.stream)
            assert ar.get(tot).tolist() == want


def test_group_step_totals_many_groups(mk_engine):
    """the step totals of a batch of more groups than 256 workgroups x 1024 groups (ADVICE r4:
    the old empty-list reduction covered only the first 262,144): 300,000 groups, three steps
    in a row (the partial slots reset themselves), against the oracle's outputs"""
    from minpaxos_amd.devbuf import Arena
    N, K, G = 5, 256, 300000
    b = synth.group_batch(G, 2, N, 2, 64, seed=79)
    b.setdefault("has_cmds", None)
    e = mk_engine(N, R.MODE_MIN, kv_per_group=K, max_groups=G)
    o = Oracle(N, R.MODE_MIN, kv_per_group=K)
    want = _want_totals(b, o.group_step(b))
    assert want[0] > 0 and want[2] > 0
    with Arena(e) as ar:
        gb, d = _dev_group_batch(ar, b, N, K, True)
        tot = ar.full(3, np.int64, 0x55)
        for _ in range(3):
            e.group_step_totals_dev(gb, tot.ptr, e.stream)
            e.stream_synchronize(e.stream)
            assert ar.get(tot).tolist() == want


@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC])
@pytest.mark.parametrize("G", [1, 17, 64, 65, 300, 4099, 64 * 70 + 1])
def test_group_step_one_launch(mk_engine, mode, G):
    """MPX_FLAG_STEP_ONE_LAUNCH: the group step is the fast kernel alone, its last workgroup
    folding the packed totals: ceil(G / 64) slots, group g adding into slot g % ceil(G / 64),
    so a slot holds at most 64 groups and, when 64 does not divide G, the slots hold unequal
    counts (G = 65: 33 and 32; G = 64 * 70 + 1: 71 slots, the first 8 with 64 groups, the rest
    with 63 - slot s expects (G - 1 - s) / nslots + 1). Outputs and totals equal the oracle's over repeated
    steps (the slots reset themselves), also replayed from a captured graph; a shape no fast
    variant takes is rejected at the call; a group past the fast kernel's capacity fails the
    step"""
    from minpaxos_amd.devbuf import Arena
    N, K = 5, 256
    b = synth.group_batch(G, 256, N, 4, 256, seed=300 + G)
    b.setdefault("has_cmds", None)
    e = mk_engine(N, mode, kv_per_group=K, step_one_launch=True)
    o = Oracle(N, mode, kv_per_group=K)
    want = o.group_step(b)
    want_tot = _want_totals(b, want)
    with Arena(e) as ar:
        gb, d = _dev_group_batch(ar, b, N, K, True)
        tot = ar.full(3, np.int64, 0x55)
        for _ in range(3):
            e.group_step_totals_dev(gb, tot.ptr, e.stream)
            e.synchronize()
            assert ar.get(tot).tolist() == want_tot
            assert np.array_equal(ar.get(d["co"]), want["committed_out"])
            assert np.array_equal(ar.get(d["eo"]), want["executed_out"])
            assert np.array_equal(ar.get(d["po"]), want["peer_out"].reshape(-1))
            assert np.array_equal(ar.get(d["st_out"]).view(np.int32),
                                  want["st_out"].view(np.int32))
            assert np.array_equal(ar.get(d["nd"]), want["n_decided"])
        e.group_step_dev(gb, e.stream)  # no totals: no slot is touched
        e.synchronize()
        s = e.stream_create()
        e.graph_begin(s)
        e.group_step_totals_dev(gb, tot.ptr, s)
        g = e.graph_end(s)
        try:
            for _ in range(2):
                e.memset(tot.ptr, 0x55, 24, s)
                e.graph_launch(g, s)
                e.stream_synchronize(s)
                assert ar.get(tot).tolist() == want_tot
        finally:
            e.graph_destroy(g)
            e.stream_destroy(s)
    if G != 300:
        return
    # ipg 1024: no fast variant; rejected at the call
    e2 = mk_engine(3, R.MODE_MIN, kv_per_group=K, step_one_launch=True)
    b2 = synth.group_batch(4, 1024, 3, 2, 64, seed=5)
    b2.setdefault("has_cmds", None)
    with Arena(e2) as ar:
        gb2, _ = _dev_group_batch(ar, b2, 3, K, True)
        with pytest.raises(MpxError):
            e2.group_step_dev(gb2, e2.stream)
    # groups of more than 1024 commands (the work list's, on a two-launch handle): the step
    # fails, and the next step on fitting groups runs clean (the slots were all taken)
    e3 = mk_engine(3, R.MODE_MIN, kv_per_group=1024, step_one_launch=True)
    b3 = synth.group_batch(64, 128, 3, 9, 800, seed=78)
    b3.setdefault("has_cmds", None)
    o3 = Oracle(3, R.MODE_MIN, kv_per_group=1024)
    b4 = synth.group_batch(64, 128, 3, 2, 100, seed=79)
    b4.setdefault("has_cmds", None)
    want4 = _want_totals(b4, o3.group_step(b4))
    with Arena(e3) as ar:
        gb3, _ = _dev_group_batch(ar, b3, 3, 1024, True)
        tot = ar.full(3, np.int64, 0)
        e3.group_step_totals_dev(gb3, tot.ptr, e3.stream)
        with pytest.raises(MpxError):
            e3.synchronize()
        gb4, _ = _dev_group_batch(ar, b4, 3, 1024, True)
        e3.group_step_totals_dev(gb4, tot.ptr, e3.stream)
        e3.synchronize()
        assert ar.get(tot).tolist() == want4


@pytest.mark.gpu
def test_group_step_graph_replay(mk_engine):
    """mpx_graph_begin / _end / _launch: a group step (+ its totals) captured on a stream and
    replayed from the graph three times gives the oracle's outputs and totals every time (the
    captured kernels' control words reset themselves, so replays are independent); what
    bench.py's one-process line replays"""
    from minpaxos_amd.devbuf import Arena
    N, K = 5, 256
    b = synth.group_batch(300, 256, N, 4, 256, seed=91)
    b.setdefault("has_cmds", None)
    e, o = mk_engine(N, R.MODE_MIN, kv_per_group=K), Oracle(N, R.MODE_MIN, kv_per_group=K)
    want = o.group_step(b)
    want_tot = _want_totals(b, want)
    # the commands the step executes (the rest keep whatever ret / conf held)
    G, ipg = b["n_groups"], b["ipg"]
    coff = b["cmd_off"].astype(np.int64)
    ex = np.zeros(len(b["op"]), bool)
    for g in range(G):
        lo, eo = max(int(b["executed_in"][g]) + 1, 0), int(want["executed_out"][g])
        if lo <= eo < ipg:
            ex[coff[g * ipg + lo]:coff[g * ipg + eo + 1]] = True
    assert ex.any()
    s = e.stream_create()
    with Arena(e) as ar:
        gb, d = _dev_group_batch(ar, b, N, K, True)
        tot = ar.full(3, np.int64, 0x55)
        e.graph_begin(s)
        e.group_step_totals_dev(gb, tot.ptr, s)
        g = e.graph_end(s)
        try:
            for _ in range(3):
                for x in ("co", "eo", "ret", "conf"):  # poison what the replay must rewrite
                    e.memset(d[x].ptr, 0x77, d[x].nbytes, s)
                e.graph_launch(g, s)
                e.stream_synchronize(s)
                assert ar.get(tot).tolist() == want_tot
                assert np.array_equal(ar.get(d["co"]), want["committed_out"])
                assert np.array_equal(ar.get(d["eo"]), want["executed_out"])
                ret, conf = ar.get(d["ret"]), ar.get(d["conf"])
                assert np.array_equal(ret[ex], want["ret"][ex])
                assert np.array_equal(conf[ex], want["conf_prev"][ex])
                assert (ret[~ex] == 0x7777777777777777).all() and (conf[~ex] == 0x77).all()
                assert np.array_equal(ar.get(d["st_out"]).view(np.int32),
                                      want["st_out"].view(np.int32))
        finally:
            e.graph_destroy(g)
            e.stream_destroy(s)
