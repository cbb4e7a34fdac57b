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
from minpaxos_amd.devbuf import Arena


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


def test_oracle_chunked_replay_matches_whole():
    """rec_base + carried last_rec: chunked replay == one pass (the ADVICE r1 'last record wins
    across chunks' case)"""
    o = Oracle()
    log = durable_log(900, 120, 31)
    whole = o.replay_durable(log, 120)
    last, db, cu = None, 0, -1
    for a, b in ((0, 300), (300, 301), (301, 900)):
        r = o.replay_durable(log[a * 29:b * 29], 120, db, cu, rec_base=a, last_rec=last)
        last, db, cu = r[4], r[5], r[6]
    assert np.array_equal(last, whole[4]) and (db, cu) == tuple(whole[5:])
    assert np.array_equal(last, np.array(go_replay(log, 120, 0, -1)[2], np.int32))


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


@pytest.mark.gpu
def test_replay_errors_and_dev(mk_engine):
    from minpaxos_amd.engine import MpxError
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    log = durable_log(1000, 600, 11)
    with pytest.raises(MpxError):
        e.replay_durable(log[:-3], 600)
    with pytest.raises(MpxError):
        e.replay_durable(log, 100)
    # no instance space at all: the first record is already a panic in the reference
    with pytest.raises(MpxError) as ei:
        e.replay_durable(log, 0)
    assert ei.value.code == R.E_NIL_INSTANCE
    # device form: caller-initialised slots, scalars in HBM (buffers from the engine's runtime)
    cap = 600
    want = o.replay_durable(log, cap)
    with Arena(e) as hip:
        d_log = hip.put(log)
        d = [hip.put(np.zeros_like(w)) for w in want[:4]]
        d_last = hip.put(np.full(cap, -1, np.int32))
        d_sc = hip.put(np.array([0, -1], np.int32))
        e.replay_durable_dev(d_log.ptr, len(log), cap, *[x.ptr for x in d], d_last.ptr, d_sc.ptr)
        e.synchronize()
        for x, w in zip(d, want[:4]):
            assert np.array_equal(hip.get(x), w)
        assert np.array_equal(hip.get(d_last), want[4])
        assert hip.get(d_sc).tolist() == [want[5], want[6]]
        with pytest.raises(MpxError):  # misaligned device log
            e.replay_durable_dev(d_log.ptr + 1, 29, cap, *[x.ptr for x in d], d_last.ptr, d_sc.ptr)
        with pytest.raises(MpxError) as ei:  # inst_cap 0 with records: E_NIL_INSTANCE, any history
            e.replay_durable_dev(d_log.ptr, 29, 0, *[x.ptr for x in d], d_last.ptr, d_sc.ptr)
        assert ei.value.code == R.E_NIL_INSTANCE


@pytest.mark.gpu
def test_replay_chunked(mk_engine):
    """a store replayed in chunks (rec_base = the chunk's first file record, last_rec carried):
    the same slots and watermarks as one call over the whole file, so a later chunk's record
    wins its instance even where an earlier chunk named it at a higher in-chunk index"""
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    n, cap = 5000, 700
    log = durable_log(n, cap, 21)
    whole = o.replay_durable(log, cap, 3, -1)
    for cuts in ((0, 1, 257, 2600, n), (0, 4096, n), (0, 999, 1000, n)):
        last, db, cu = None, 3, -1
        for a, b in zip(cuts[:-1], cuts[1:]):
            part = log[a * 29:b * 29]
            got = e.replay_durable(part, cap, db, cu, rec_base=a, last_rec=last)
            want = o.replay_durable(part, cap, db, cu, rec_base=a, last_rec=last)
            assert np.array_equal(got[4], want[4]) and got[5:] == want[5:]
            last, db, cu = got[4], got[5], got[6]
        assert np.array_equal(last, whole[4]) and (db, cu) == tuple(whole[5:])


@pytest.mark.gpu
def test_replay_dev_binned_and_atomic(mk_engine):
    """mpx_replay_durable_dev with the reserved scratch (the binned slot maximum: pairs, each
    chunk's pairs sorted by bin in LDS with its run starts, one LDS slice per 32768 slots) and without it (one
    device atomicMax per record): the same slots as the oracle - a ragged last bin, every record
    in one bin, heavy repeats, a space past the binned limit (2^25 slots: the atomic form),
    rec_base offsets"""
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    cases = [(100003, 50000, 0), (70001, 3 * 32768 + 5, 17), (1 << 18, 1000, 5),
             (4099, 8192, 0), (1000, (1 << 25) + 1, 3),
             # 64 chunks x 129 bins (a ragged last bin): the chunk-sorted runs
             ((1 << 20) + 77, (1 << 22) + 3, 11)]
    with Arena(e) as hip:
        for n, cap, base in cases:
            log = durable_log(n, cap, n ^ cap, dup=True)
            # slots from earlier chunks: below this call's rec_base (chunks replay in file order)
            last0 = np.random.default_rng(n).integers(-1, max(base, 0) + 0, cap).astype(np.int32) \
                if base else np.full(cap, -1, np.int32)
            want = o.replay_durable(log, cap, 7, -1, rec_base=base, last_rec=last0)
            for reserve in (True, False):
                if reserve:
                    e.replay_durable_reserve(len(log), cap)
                d_log = hip.put(log)
                d = [hip.put(np.zeros_like(w)) for w in want[:4]]
                d_last = hip.put(last0)
                d_sc = hip.put(np.array([7, -1], np.int32))
                e.replay_durable_dev(d_log.ptr, len(log), cap, *[x.ptr for x in d], d_last.ptr,
                                     d_sc.ptr, rec_base=base)
                e.synchronize()
                for x, w in zip(d, want[:4]):
                    assert np.array_equal(hip.get(x), w), (n, cap, reserve)
                assert np.array_equal(hip.get(d_last), want[4]), (n, cap, reserve)
                assert hip.get(d_sc).tolist() == [want[5], want[6]], (n, cap, reserve)
        # an instNo outside the space through the binned form: E_NIL_INSTANCE
        from minpaxos_amd.engine import MpxError
        log = durable_log(5000, 600, 99)  # instNos in [0, 300)
        e.replay_durable_reserve(len(log), 100)
        d_log = hip.put(log)
        want = o.replay_durable(log, 600)
        d = [hip.put(np.zeros_like(w)) for w in want[:4]]
        d_last = hip.put(np.full(100, -1, np.int32))
        d_sc = hip.put(np.array([0, -1], np.int32))
        with pytest.raises(MpxError) as ei:
            e.replay_durable_dev(d_log.ptr, len(log), 100, *[x.ptr for x in d], d_last.ptr,
                                 d_sc.ptr)
            e.synchronize()
        assert ei.value.code == R.E_NIL_INSTANCE
