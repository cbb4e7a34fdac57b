"""Parity backstop: the CPU oracle (oracle/oracle.cpp) against a second, independent restatement
of A1–A5 (tests/go_translit.py, a literal transliteration of the Go over Go-shaped objects).

Both restate the same cited Go text; no reference vectors exist for this path, so
agreement between two differently shaped readings is what guards against a misreading. Checked on
every golden fixture of A1–A6, the hand-traced known-answer cases, and seeded random batches
(ragged reply counts, every N, mixed statuses, nil instances, panicking inputs).
"""
import numpy as np
import pytest

import gen_cases
import kat_cases
from go_translit import GoBackend, GoPanic
from oracle_lib import Oracle, OracleError
from test_golden import FILES, check, load
from golden.make_golden import run_case
from minpaxos_amd import records as R
from minpaxos_amd import synth

KINDS = {"accept", "prepare", "prepare_min", "apply", "conflict", "group"}
A_FILES = [f for f in FILES if load(f)[0] in KINDS]


def go_mk(n, mode, **kw):
    return GoBackend(n, mode, **kw)


@pytest.mark.parametrize("path", A_FILES, ids=lambda p: p.rsplit("/", 1)[-1][:-4])
def test_translit_reproduces_golden(path):
    kind, p, x, y = load(path)
    check(run_case(kind, p, x, go_mk), y)


@pytest.mark.parametrize("case", kat_cases.ALL, ids=lambda f: f.__name__)
def test_translit_kat(case):
    case(go_mk)


def both(fn):
    """run fn on the oracle and the transliteration; both succeed or both refuse"""
    res = []
    for mk in (lambda n, m, **kw: Oracle(n, m, **kw), go_mk):
        try:
            res.append(("ok", fn(mk)))
        except (OracleError, GoPanic) as e:
            res.append(("err", e.code))
    assert res[0][0] == res[1][0], res
    return res


def eq_any(a, b):
    if isinstance(a, dict):
        for k in a:
            if a[k] is not None:
                eq_any(a[k], b[k])
        return
    if isinstance(a, tuple):
        for u, v in zip(a, b):
            eq_any(u, v)
        return
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.names:
        a, b = a.view(np.uint8), b.view(np.uint8)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 16])
@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC], ids=["min", "classic"])
def test_accept_random(n, mode):
    rng = np.random.default_rng(1000 + n + 50 * mode)
    for trial in range(6):
        recs, st = gen_cases.ragged_accept(rng, 300, n, max_r=n + 3, long_every=97, long_len=40,
                                           base=trial)
        st = st.copy()
        # mixed statuses (COMMITTED ones and, for MIN, nil ones that only get NACKs)
        st["status"] = rng.choice([R.PREPARED, R.ACCEPTED, R.COMMITTED, R.PREPARING], len(st),
                                  p=[0.5, 0.2, 0.2, 0.1])
        st["accept_oks"] = rng.integers(0, 3, len(st))
        if trial == 5:
            recs = recs.copy()
            recs["id"][rng.integers(0, len(recs))] = n  # out of peerCommits
        cu = int(rng.integers(-1, 20))
        pc = rng.integers(-1, 50, n).astype(np.int32)
        res = both(lambda mk: mk(n, mode).accept_tally(recs, st, trial, cu, pc))
        if res[0][0] == "ok":
            eq_any(res[0][1], res[1][1])
        else:
            assert res[0][1] == res[1][1]


def test_accept_nil_instances():
    n = 5
    rng = np.random.default_rng(7)
    recs, st = gen_cases.ragged_accept(rng, 200, n, max_r=6, long_every=0, long_len=0, base=0)
    st = st.copy()
    nil = rng.random(len(st)) < 0.1
    st["status"][nil] = R.STATUS_NIL
    for mode in (R.MODE_MIN, R.MODE_CLASSIC):
        for only_nacks in (False, True):
            r = recs.copy()
            if only_nacks:  # MIN tolerates NACKs to a nil instance; CLASSIC dereferences it
                r["ok"][nil[r["instance"]]] = 0
            res = both(lambda mk: mk(n, mode).accept_tally(r, st, 0, -1, np.zeros(n, np.int32)))
            if res[0][0] == "ok":
                eq_any(res[0][1], res[1][1])
            else:
                assert res[0][1] == res[1][1] == R.E_NIL_INSTANCE


@pytest.mark.parametrize("n", [1, 3, 5, 9])
def test_prepare_classic_random(n):
    rng = np.random.default_rng(2000 + n)
    for trial in range(6):
        recs, st = gen_cases.ragged_prepare(rng, 300, n, max_r=n + 3, long_every=61,
                                            long_len=30)
        st = st.copy()
        st["status"] = rng.choice([R.PREPARING, R.PREPARED, R.ACCEPTED], len(st),
                                  p=[0.8, 0.1, 0.1])
        st["flags"] = rng.integers(0, 8, len(st))
        db = int(rng.integers(-1, 400))
        res = both(lambda mk: mk(n, R.MODE_CLASSIC).prepare_select(recs, st, 0, db))
        assert res[0][0] == "ok"
        eq_any(res[0][1], res[1][1])


@pytest.mark.parametrize("n", [1, 3, 5, 7])
def test_prepare_min_random(n):
    for seed in range(4):
        recs, off, gst = synth.prepare_replies_min(200, n, seed=300 + seed,
                                                   replies_per_group=None if seed else 2 * n)
        pc = np.random.default_rng(seed).integers(-1, 9, 200 * n).astype(np.int32)
        res = both(lambda mk: mk(n, R.MODE_MIN).prepare_select_min(recs, off, gst, pc))
        if res[0][0] == "ok":
            eq_any(res[0][1], res[1][1])
        else:  # N = 1: reply ids 1..N-1 index outside peerCommits
            assert n == 1 and res[0][1] == res[1][1] == R.E_BAD_ID


def test_apply_and_conflict_random():
    rng = np.random.default_rng(3000)
    for trial in range(4):
        op, key, val = gen_cases.commands_mixed(rng, 5000, 300 if trial else 20)
        o, g = Oracle(5, R.MODE_MIN), GoBackend(5, R.MODE_MIN)
        for call in range(2):  # the table persists across calls
            eq_any(o.apply(op, key, val), g.apply(op, key, val))
            eq_any(o.kv_export(), g.kv_export())
        sizes = rng.integers(0, 9, 500)
        off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        cop, ckey, _ = gen_cases.commands_mixed(rng, int(off[-1]), 60, neg_keys=False)
        eq_any(o.conflict_batch(cop, ckey, off), g.conflict_batch(cop, ckey, off))


@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC], ids=["min", "classic"])
@pytest.mark.parametrize("n", [3, 5, 7])
def test_group_step_random(mode, n):
    G, ipg, K = 6, 64, 128
    b = synth.group_batch(G, ipg, n, 3, 100, seed=400 + n)
    rng = np.random.default_rng(n)
    b["st_in"] = b["st_in"].copy()
    b["st_in"]["status"][rng.random(G * ipg) < 0.02] = R.COMMITTED
    b["has_cmds"] = (rng.random(G * ipg) > 0.01).astype(np.uint8)
    o, g = Oracle(n, mode, kv_per_group=K), GoBackend(n, mode, kv_per_group=K)
    w1 = o.group_step(b)
    eq_any(w1, g.group_step(b))
    # second step from the tables the first left
    w2 = o.group_step(b, w1["kv_cnt"], w1["kv_key"], w1["kv_val"])
    eq_any(w2, g.group_step(b, w1["kv_cnt"], w1["kv_key"], w1["kv_val"]))
    # a table too small for the keys the step PUTs: both refuse
    res = both(lambda mk: mk(n, mode, kv_per_group=8).group_step(b))
    assert res[0] == ("err", R.E_KV_FULL) and res[1] == ("err", R.E_KV_FULL)
