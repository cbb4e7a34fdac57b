"""Randomised parity sweeps on the GPU: many seeded shapes per test, every result against the
oracle (oracle/oracle.cpp through tests/oracle_lib.py). The fixed-shape tests elsewhere pin the
cases the reference's handlers branch on; these draw the shape itself - call sizes, key ranges
and distributions, table sizes, pipelines, fan-in, replica counts, group shapes - so a build
parameter that only some shapes reach (a batch boundary, a heavy slot, a partition past its LDS
capacity) meets them. Seeds are fixed: a failure names its seed and reproduces.

References: Command.Execute / executeCommands (state.go:77-103, bareminpaxos.go:1066-1098),
handleAcceptReply (bareminpaxos.go:1014-1064, paxos.go:631-673), the fused group step
(bareminpaxos.go:1014-1098 per group)."""
import numpy as np
import pytest

import gen_cases
from oracle_lib import Oracle, OracleError
from minpaxos_amd import records as R
from minpaxos_amd import synth
from test_gpu_parity import _apply_form, _cmp_group, eq_struct

pytestmark = pytest.mark.gpu

_PATHS = [R.APPLY_AUTO, R.APPLY_SMALL, R.APPLY_PARTITIONED, R.APPLY_SORTED]


def _commands(rng, m, space, kind):
    """m commands over `space` keys: uniform, zipf-like, one hot key mixed in, or the sentinel
    and the extremes sprinkled in"""
    op, key, val = gen_cases.commands_mixed(rng, m, space, neg_keys=kind == "special")
    if kind == "zipf":
        key = (rng.zipf(1.3, m) % space).astype(np.int64)
    elif kind == "hot":
        key[rng.random(m) < rng.uniform(0.05, 0.9)] = int(rng.integers(0, space))
    return op, key, val


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_apply(mk_engine, seed):
    """apply: a random pipeline and table size, four calls of random size (replica-sized ones
    through the host and the device-pointer forms), random key distributions; every call's
    results and the final table bit-exact"""
    rng = np.random.default_rng(5000 + seed)
    path = _PATHS[seed % len(_PATHS)]
    cap = 1 << int(rng.integers(12, 18))
    chunk = int(rng.choice([0, 0, 5000, 33333]))  # multi-chunk calls: every PUT key inserted first
    e = mk_engine(5, R.MODE_MIN, kv_capacity=cap, apply_path=path, apply_chunk=chunk)
    o = Oracle(5, R.MODE_MIN)
    for call in range(4):
        small = path == R.APPLY_SMALL or rng.random() < 0.5
        m = int(rng.integers(1, R.APPLY_SMALL_MAX + 1)) if small else int(rng.integers(1, 120000))
        space = int(rng.integers(1, cap // 2 + 1))
        kind = ["uniform", "zipf", "hot", "special"][int(rng.integers(0, 4))]
        op, key, val = _commands(rng, m, space, kind)
        form = "dev" if (m <= R.APPLY_SMALL_MAX and rng.random() < 0.5) else "host"
        gr, gc = _apply_form(e, form, op, key, val)
        wr, wc = o.apply(op, key, val)
        tag = (seed, call, path, chunk, m, space, kind, form)
        assert np.array_equal(gr, wr), (tag, np.nonzero(gr != wr)[0][:5])
        assert np.array_equal(gc, wc), (tag, np.nonzero(gc != wc)[0][:5])
    gk, gv = e.kv_export()
    wk, wv = o.kv_export()
    assert np.array_equal(gk, wk) and np.array_equal(gv, wv), seed
    assert e.kv_size() == len(wk)


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_accept_tally(mk_engine, seed):
    """accept tally: random replica count, fan-in (with gaps and long instances), window base
    and starting watermarks, both modes"""
    rng = np.random.default_rng(6000 + seed)
    n_rep = int(rng.integers(1, 10))
    n_inst = int(rng.integers(1, 40000))
    rec, st = gen_cases.ragged_accept(rng, n_inst, n_rep, max_r=int(rng.integers(1, 12)),
                                      long_every=int(rng.integers(0, 3000)),
                                      long_len=int(rng.integers(20, 400)),
                                      base=int(rng.integers(0, 1000)))
    base = int(rec["instance"][0]) if len(rec) else 0
    for mode in (R.MODE_MIN, R.MODE_CLASSIC):
        e, o = mk_engine(n_rep, mode), Oracle(n_rep, mode)
        cu0 = int(rng.integers(-1, 50))
        pc0 = rng.integers(-1, 10, n_rep).astype(np.int32)
        got = e.accept_tally(rec, st, base, cu0, pc0)
        want = o.accept_tally(rec, st, base, cu0, pc0)
        eq_struct(got[0], want[0])
        assert got[1] == want[1], (seed, mode, got[1], want[1])
        assert np.array_equal(got[2], want[2]), (seed, mode)
        assert np.array_equal(got[3], want[3]), (seed, mode)


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_group_step(mk_engine, seed):
    """the fused group step: random replica count, instances per group, commands per instance,
    key range and table capacity (so every fast variant and the work list are drawn), two
    chained steps, both modes"""
    rng = np.random.default_rng(7000 + seed)
    N = int(rng.integers(3, 10))
    ipg = int(rng.choice([64, 128, 200, 256, 384, 512]))
    K = int(rng.choice([64, 256, 512, 1024]))
    B = int(rng.integers(1, 6))
    keys = int(rng.integers(8, K + 1))
    G = int(rng.integers(1, 200))
    for mode in (R.MODE_MIN, R.MODE_CLASSIC):
        b = synth.group_batch(G, ipg, N, B, keys, p_ok=float(rng.uniform(0.3, 0.95)),
                              seed=int(rng.integers(0, 1 << 30)))
        e, o = mk_engine(N, mode, kv_per_group=K), Oracle(N, mode, kv_per_group=K)
        try:
            want = o.group_step(b)
        except OracleError:
            continue  # a table past kv_per_group: the engine's MPX_E_KV_FULL, tested elsewhere
        _cmp_group(e.group_step(b), want, G, K)
        b2 = synth.group_batch(G, ipg, N, B, keys, seed=int(rng.integers(0, 1 << 30)))
        b2["committed_in"] = want["committed_out"]
        b2["executed_in"] = np.minimum(want["executed_out"], ipg // 2).astype(np.int32)
        b2["peer_in"] = want["peer_out"]
        try:
            want2 = o.group_step(b2, want["kv_cnt"], want["kv_key"], want["kv_val"])
        except OracleError:
            continue
        got2 = e.group_step(b2, want["kv_cnt"], want["kv_key"], want["kv_val"])
        _cmp_group(got2, want2, G, K)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_stream_decode(mk_engine, seed):
    """the full peer-stream decode (replicaListener + every Unmarshal): random frame mixes of
    random length - up to several 4 MB tile groups - with variable frames of random size, cut
    at random places, both wire formats"""
    from minpaxos_amd import wire as W
    rng = np.random.default_rng(8000 + seed)
    for proto in (R.MODE_MIN, R.MODE_CLASSIC):
        e, o = mk_engine(5, proto), Oracle(5, proto)
        n = int(rng.integers(1, 12)) * int(10 ** rng.integers(1, 5))
        b = W.random_stream(proto, rng, n, p_var=float(rng.uniform(0, 0.4)),
                            p_big=float(rng.uniform(0, 0.03)), p_unknown=float(rng.uniform(0, 0.1)))
        if seed % 3 == 0:  # a long AcceptReply run: past a tile group (4 MB)
            recs, _ = synth.accept_replies(int(rng.integers(1 << 18, 1 << 19)), 5, 0.7,
                                           seed=int(rng.integers(0, 1 << 30)))
            b = b + bytes(W.leader_stream(proto, recs, prepare_every=int(rng.integers(1, 5000)),
                                          n_cmds=int(rng.integers(0, 3)))) + b
        for cut in (len(b), int(rng.integers(0, len(b) + 1))):
            got, want = e.decode_stream(b[:cut]), o.decode_stream(b[:cut])
            for g, w, name in zip(got[:4], want[:4], ("ar", "prep", "var", "other")):
                assert len(g) == len(w) and g.tobytes() == w.tobytes(), (seed, proto, cut, name)
            for f in ("consumed", "n_accept_replies", "n_prepare_replies", "n_var", "n_other",
                      "stop_reason", "stop_code"):
                assert int(got[4][f]) == int(want[4][f]), (seed, proto, cut, f)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_peer_decode(mk_engine, seed):
    """the fixed-frame decoder: AcceptReplies with random mixes of the other fixed frames and
    unknown codes, random lengths (a tile is ~1170 AcceptReplies, a group 256 tiles), cut at
    random places"""
    rng = np.random.default_rng(9000 + seed)
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    n = int(rng.integers(1, 1 << int(rng.integers(1, 20))))
    recs, _ = synth.accept_replies(n, 5, 0.7, seed=int(rng.integers(0, 1 << 30)))
    buf = synth.peer_stream(recs, seed=int(rng.integers(0, 1 << 30)),
                            p_beacon=float(rng.uniform(0, 0.1)), p_prepare=float(rng.uniform(0, 0.05)),
                            p_commit_short=float(rng.uniform(0, 0.05)),
                            p_unknown=float(rng.uniform(0, 0.05)))
    for cut in (len(buf), int(rng.integers(0, len(buf) + 1))):
        ga, go, gr = e.decode_peer_stream(buf[:cut])
        wa, wo, wr = o.decode_peer_stream(buf[:cut])
        assert gr.tobytes() == wr.tobytes(), (seed, cut)
        assert ga.tobytes() == wa.tobytes() and go.tobytes() == wo.tobytes(), (seed, cut)


def _log_uniform(rng, lo, hi):
    """an integer in [lo, hi], log-uniformly"""
    return int(min(hi, max(lo, round(float(np.exp(rng.uniform(np.log(lo), np.log(hi))))))))


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_prepare(mk_engine, seed):
    """CLASSIC prepare (random fan-in, gaps, long instances, window base, defaultBallot) and MIN
    prepare (random groups and replies per group, peer commits)"""
    rng = np.random.default_rng(10000 + seed)
    n_rep = int(rng.integers(1, 10))
    rec, st = gen_cases.ragged_prepare(rng, _log_uniform(rng, 1, 60000), n_rep,
                                       max_r=int(rng.integers(1, 10)),
                                       long_every=int(rng.integers(0, 2000)),
                                       long_len=int(rng.integers(20, 300)), base=-int(rng.integers(0, 5)))
    base = int(rec["instance"][0]) if len(rec) else 0
    e, o = mk_engine(n_rep, R.MODE_CLASSIC), Oracle(n_rep, R.MODE_CLASSIC)
    db = int(rng.integers(-1, 400))
    got, want = e.prepare_select(rec, st, base, db), o.prepare_select(rec, st, base, db)
    eq_struct(got[0], want[0])
    assert got[1] == want[1] and np.array_equal(got[2], want[2]), seed
    G = _log_uniform(rng, 1, 100000)
    rec, off, gst = synth.prepare_replies_min(G, 5, seed=int(rng.integers(0, 1 << 30)),
                                              replies_per_group=int(rng.integers(1, 10)))
    e, o = mk_engine(5, R.MODE_MIN), Oracle(5, R.MODE_MIN)
    pc = rng.integers(-1, 50, G * 5).astype(np.int32)
    got, want = e.prepare_select_min(rec, off, gst, pc), o.prepare_select_min(rec, off, gst, pc)
    eq_struct(got[0], want[0])
    assert np.array_equal(got[1], want[1]), seed
    eq_struct(got[2], want[2])


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_fanout(mk_engine, seed):
    """client reply fan-out: random batch sizes, connection counts (the counting-sort and the
    radix path), a hot connection, OK / leader fields"""
    rng = np.random.default_rng(11000 + seed)
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    n = _log_uniform(rng, 1, 3_000_000)
    c = _log_uniform(rng, 1, 70000)
    rec = synth.replies(n, c, seed=int(rng.integers(0, 1 << 30)))
    if seed % 2:
        rec["client"][rng.random(n) < rng.uniform(0.1, 0.9)] = int(rng.integers(0, c))
    ok, leader = int(rng.integers(0, 2)), int(rng.integers(0, 9))
    got, want = e.encode_replies(rec, c, ok, leader), o.encode_replies(rec, c, ok, leader)
    assert np.array_equal(got[1], want[1]), (seed, n, c)
    assert got[0].tobytes() == want[0].tobytes(), (seed, n, c)


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_logenc(mk_engine, seed):
    """durable and catch-up log encoding: random instance counts and commands per instance
    (ragged, empty instances, one very long instance)"""
    rng = np.random.default_rng(12000 + seed)
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    n = _log_uniform(rng, 1, 200000)
    recs, off, op, key, val = synth.log_records(n, int(rng.integers(1, 9)),
                                                seed=int(rng.integers(0, 1 << 30)), ragged=True)
    if seed % 3 == 0 and n > 2:  # one instance with many commands (multi-byte varint, big blocks)
        big = np.array(off, np.int64)
        extra = int(rng.integers(100, 3000))
        big[n // 2:] += extra
        op, key, val = synth.commands(int(big[-1]), 1 << 12, 0.5, "uniform",
                                      seed=int(rng.integers(0, 1 << 30)))
        off = big.astype(np.uint64)
    for fmt in (R.LOG_CATCHUP, R.LOG_DURABLE):
        got, want = e.encode_log(fmt, recs, off, op, key, val), o.encode_log(fmt, recs, off, op, key, val)
        assert np.array_equal(got[1], want[1]), (seed, fmt, n)
        assert got[0].tobytes() == want[0].tobytes(), (seed, fmt, n)


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_replay(mk_engine, seed):
    """durable-log replay: random record counts, instance spaces (dense, sparse, with repeats),
    starting watermarks"""
    from test_replay import durable_log
    rng = np.random.default_rng(13000 + seed)
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    n = _log_uniform(rng, 1, 400000)
    cap = _log_uniform(rng, max(1, n // 4), 2 * n + 1)
    dup = bool(seed % 2) or cap < n
    log = durable_log(n, cap, int(rng.integers(0, 1 << 30)), dup=dup)
    db, cu = int(rng.integers(-1, 1000)), int(rng.integers(-1, 1 << 20))
    got, want = e.replay_durable(log, cap, db, cu), o.replay_durable(log, cap, db, cu)
    assert np.array_equal(got[0], want[0]), (seed, n, cap)
    for g, w in zip(got[1:5], want[1:5]):
        assert np.array_equal(g, w), (seed, n, cap)
    assert got[5:] == want[5:], (seed, n, cap)


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_apply_sequence(mk_engine, seed):
    """one table through a random sequence of every way to reach it: apply calls of every size
    through the host, device-pointer and staged forms (so the replica-batch kernels, the
    sort-based and the partitioned pipelines take turns on the same slots and call tags),
    imports of present keys, clears, exports; bit-exact after every step"""
    from minpaxos_amd.devbuf import Arena  # noqa: F401  (through _apply_form)
    rng = np.random.default_rng(14000 + seed)
    cap = 1 << int(rng.integers(13, 18))
    e = mk_engine(5, R.MODE_MIN, kv_capacity=cap, apply_fast_min=int(rng.choice([0, 20000, 50000])))
    o = Oracle(5, R.MODE_MIN)
    io = e.apply_buffers(R.APPLY_SMALL_MAX)
    space = int(rng.integers(16, cap // 3))
    for stepno in range(14):
        act = ["host", "dev", "staged", "host", "dev", "import", "clear"][int(rng.integers(0, 7))]
        if act == "clear":
            e.kv_clear()
            o = Oracle(5, R.MODE_MIN)
            continue
        if act == "import":
            n = int(rng.integers(0, space // 4 + 1))
            keys = rng.choice(space * 4, n, replace=False).astype(np.int64) - space
            vals = rng.integers(-(1 << 62), 1 << 62, n).astype(np.int64)
            e.kv_import(keys, vals)
            o.kv_import(keys, vals)
        else:
            m = (int(rng.integers(1, R.APPLY_SMALL_MAX + 1)) if act == "staged" or rng.random() < 0.6
                 else int(rng.integers(R.APPLY_SMALL_MAX, 90000)))
            op, key, val = _commands(rng, m, space, ["uniform", "zipf", "hot", "special"][int(rng.integers(0, 4))])
            if act == "staged":
                io["op"][:m], io["key"][:m], io["val"][:m] = op, key, val
                e.apply_staged(m)
                gr, gc = io["ret"][:m].copy(), io["conf"][:m].copy()
            else:
                gr, gc = _apply_form(e, act, op, key, val)
            wr, wc = o.apply(op, key, val)
            assert np.array_equal(gr, wr), (seed, stepno, act, m, np.nonzero(gr != wr)[0][:5])
            assert np.array_equal(gc, wc), (seed, stepno, act, m, np.nonzero(gc != wc)[0][:5])
        gk, gv = e.kv_export()
        wk, wv = o.kv_export()
        assert np.array_equal(gk, wk) and np.array_equal(gv, wv), (seed, stepno, act)
        assert e.kv_size() == len(wk)


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_conflict_and_prefix(mk_engine, seed):
    """ConflictBatch over every consecutive instance pair (random sizes, empty and very large
    instances, key ranges) and updateCommittedUpTo over random status windows"""
    import kat_cases
    rng = np.random.default_rng(15000 + seed)
    e, o = mk_engine(5, R.MODE_CLASSIC), Oracle(5, R.MODE_CLASSIC)
    n_inst = _log_uniform(rng, 1, 200000)
    sizes = rng.integers(0, int(rng.integers(1, 20)), n_inst)
    if seed % 2:
        sizes[rng.random(n_inst) < 0.002] = int(rng.integers(200, 3000))
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    op, key, _ = gen_cases.commands_mixed(rng, int(off[-1]), _log_uniform(rng, 1, 1 << 20),
                                          neg_keys=bool(seed % 3 == 0))
    assert np.array_equal(e.conflict_batch(op, key, off), o.conflict_batch(op, key, off)), seed
    n = _log_uniform(rng, 1, 300000)
    st = kat_cases.inst_states(n, R.COMMITTED)
    bad = rng.integers(0, n, int(rng.integers(0, 6)))
    st["status"][bad] = rng.choice([R.PREPARED, R.STATUS_NIL, R.ACCEPTED], len(bad))
    base = int(rng.integers(-3, 3))
    cu = int(rng.integers(base - 2, base + n))
    assert e.committed_prefix(st, base, cu) == o.committed_prefix(st, base, cu), seed
