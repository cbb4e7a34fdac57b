"""Durable-log replay (read side): getDataFromStableStore.

CPU: the oracle against the Go loop restated with struct.unpack (bareminpaxos.go:122-161:
12 metadata bytes, one Command.Unmarshal, the two watermark updates, instanceSpace[instNo] = the
record), the durable encoder -> replay round trip for 1-command records (the only shape the
reference's replay reads back), and the error paths (partial trailing record, instNo outside the
instance space).
GPU: mpx_replay_durable and mpx_replay_durable_dev vs the oracle, bit for bit, across the
engine's 256-record tiles (duplicate instNos, so the last-record-wins slot is exercised).
"""
import struct

import numpy as np
import pytest

from oracle_lib import Oracle, OracleError
from minpaxos_amd import records as R
from minpaxos_amd import synth


def durable_log(n, inst_cap, seed, dup=True):
    """n random 29-byte records; instNos drawn with repeats when dup, any status/ballot."""
    rng = np.random.default_rng(seed)
    recs = np.zeros(n, R.LOG_REC)
    recs["ballot"] = rng.integers(-(1 << 31), 1 << 31, n, dtype=np.int64).astype(np.int32)
    small = rng.random(n) < 0.5  # ballots near 0 as well as the full int32 range
    recs["ballot"][small] = rng.integers(-2, 64, int(small.sum()))
    recs["status"] = rng.integers(-1, 5, n)
    hi = max(1, inst_cap // 2) if dup else inst_cap
    recs["inst_no"] = rng.integers(0, hi, n) if dup else rng.permutation(inst_cap)[:n]
    op, key, val = synth.commands(n, 1 << 12, 0.5, "uniform", seed=seed + 1)
    key = key.copy()
    key[rng.random(n) < 0.01] = np.iinfo(np.int64).min
    w = bytearray()
    for i in range(n):
        w += struct.pack("<IIIBqq", int(recs["ballot"][i]) & 0xFFFFFFFF,
                         int(recs["status"][i]) & 0xFFFFFFFF, int(recs["inst_no"][i]) & 0xFFFFFFFF,
                         int(op[i]), int(key[i]), int(val[i]))
    return np.frombuffer(bytes(w), np.uint8).copy()


def go_replay(log, inst_cap, default_ballot, committed_up_to):
    """The loop of bareminpaxos.go:122-161 record by record."""
    b = bytes(log)
    recs, cmds, space = [], [], [-1] * inst_cap
    for i in range(len(b) // R.DURABLE_REC_BYTES):
        ballot, status, inst = struct.unpack_from("<iii", b, 29 * i)
        op, k, v = struct.unpack_from("<Bqq", b, 29 * i + 12)
        if ballot > default_ballot:
            default_ballot = ballot
        if inst > committed_up_to and status == 3:  # minpaxosproto.COMMITTED
            committed_up_to = inst
        space[inst] = i
        recs.append((ballot, status, inst))
        cmds.append((op, k, v))
    return recs, cmds, space, default_ballot, committed_up_to


def test_oracle_matches_go_loop():
    o = Oracle()
    for n, cap, seed in ((0, 4, 1), (1, 1, 2), (50, 64, 3), (700, 300, 4)):
        log = durable_log(n, cap, seed)
        for db, cu in ((0, -1), (1 << 30, 1 << 30), (-5, 7)):
            recs, op, key, val, last, b2, c2 = o.replay_durable(log, cap, db, cu)
            wr, wc, ws, wb, wcu = go_replay(log, cap, db, cu)
            assert [tuple(int(x) for x in r)[:3] for r in recs] == wr
            assert list(zip(op.tolist(), key.tolist(), val.tolist())) == wc
            assert last.tolist() == ws and (b2, c2) == (wb, wcu)


def test_encode_replay_round_trip():
    o = Oracle()
    recs, off, op, key, val = synth.log_records(1000, 1, seed=5, ragged=False)
    recs = recs.copy()
    recs["inst_no"] = np.arange(1000)
    log, _ = o.encode_log(R.LOG_DURABLE, recs, off, op, key, val)
    r2, op2, k2, v2, last, _, cu = o.replay_durable(log, 1000)
    assert np.array_equal(r2[["ballot", "status", "inst_no"]], recs[["ballot", "status", "inst_no"]])
    assert np.array_equal(op2, op) and np.array_equal(k2, key) and np.array_equal(v2, val)
    assert np.array_equal(last, np.arange(1000))
    com = recs["inst_no"][recs["status"] == 3]
    assert cu == (int(com.max()) if len(com) else -1)


def test_oracle_errors():
    o = Oracle()
    log = durable_log(10, 16, 6)
    with pytest.raises(OracleError):
        o.replay_durable(log[:-1], 16)  # partial trailing record
    with pytest.raises(OracleError):
        o.replay_durable(log, 4)  # instNo outside instanceSpace


@pytest.mark.gpu
def test_replay_parity(mk_engine):
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    cases = [(0, 8), (1, 1), (255, 300), (256, 100), (257, 1000), (4097, 64), (100003, 50000)]
    for n, cap in cases:
        log = durable_log(n, cap, n + cap, dup=n > 300 or cap < n)
        for db, cu in ((0, -1), (123, 1 << 20)):
            got = e.replay_durable(log, cap, db, cu)
            want = o.replay_durable(log, cap, db, cu)
            assert np.array_equal(got[0], want[0]), n
            for g, w in zip(got[1:5], want[1:5]):
                assert np.array_equal(g, w), n
            assert got[5:] == want[5:], n


@pytest.mark.gpu
def test_replay_round_trip_engine(mk_engine):
    """The engine's durable encoder, then its replay: records, commands and slots come back."""
    e = mk_engine(5, R.MODE_MIN)
    n = 1 << 20
    recs, off, op, key, val = synth.log_records(n, 1, seed=7, ragged=False)
    recs = recs.copy()
    recs["inst_no"] = np.random.default_rng(8).permutation(n)
    log, _ = e.encode_log(R.LOG_DURABLE, recs, off, op, key, val)
    assert len(log) == 29 * n
    r2, op2, k2, v2, last, _, cu = e.replay_durable(log, n)
    assert np.array_equal(r2[["ballot", "status", "inst_no"]], recs[["ballot", "status", "inst_no"]])
    assert np.array_equal(op2, op) and np.array_equal(k2, key) and np.array_equal(v2, val)
    assert np.array_equal(last[recs["inst_no"]], np.arange(n))


class _Hip:
    """Device buffers through the HIP runtime libmpx.so is bound to in this process (its
    libamdhip64.so.7, already loaded with the engine: /opt/rocm's, or torch's when torch came
    first). torch.cuda cannot be used here: once the engine has initialised a runtime that is not
    torch's, torch finds no device."""

    def __init__(self):
        import ctypes as C
        import os
        self.C = C
        self.h = C.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
        self.live = []

    def put(self, a):
        C = self.C
        a = np.ascontiguousarray(a)
        p = C.c_void_p()
        assert self.h.hipMalloc(C.byref(p), C.c_size_t(max(a.nbytes, 16))) == 0
        self.live.append(p)
        if a.nbytes:
            assert self.h.hipMemcpy(p, a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes), 1) == 0
        return p.value

    def get(self, ptr, like):
        C = self.C
        out = np.empty_like(like)
        if out.nbytes:
            assert self.h.hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(ptr),
                                    C.c_size_t(out.nbytes), 2) == 0
        return out

    def free(self):
        for p in self.live:
            self.h.hipFree(p)


@pytest.mark.gpu
def test_replay_errors_and_dev(mk_engine):
    from minpaxos_amd.engine import MpxError
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    log = durable_log(1000, 600, 11)
    with pytest.raises(MpxError):
        e.replay_durable(log[:-3], 600)
    with pytest.raises(MpxError):
        e.replay_durable(log, 100)
    # device form: caller-initialised slots, scalars in HBM
    n, cap = 1000, 600
    want = o.replay_durable(log, cap)
    hip = _Hip()
    try:
        d_log = hip.put(log)
        d = [hip.put(np.zeros_like(w)) for w in want[:4]]
        d_last = hip.put(np.full(cap, -1, np.int32))
        d_sc = hip.put(np.array([0, -1], np.int32))
        e.replay_durable_dev(d_log, len(log), cap, *d, d_last, d_sc)
        e.synchronize()
        for ptr, w in zip(d, want[:4]):
            assert np.array_equal(hip.get(ptr, w), w)
        assert np.array_equal(hip.get(d_last, want[4]), want[4])
        assert hip.get(d_sc, np.zeros(2, np.int32)).tolist() == [want[5], want[6]]
        with pytest.raises(MpxError):  # misaligned device log
            e.replay_durable_dev(d_log + 1, 29, cap, *d, d_last, d_sc)
    finally:
        hip.free()
