"""Instance-log encoding.

CPU: the oracle against Instance.Marshal / recordInstanceMetadata + recordCommands restated
with struct.pack (minpaxosprotomarsh.go:100-124, bareminpaxos.go:164-188, statemarsh.go:8-19),
including multi-byte varints and empty (nil) command slices; bcastAccept's per-peer CatchUpLog is
a suffix of one encoded run (bareminpaxos.go:488-513).
GPU: mpx_encode_log vs the oracle, bit for bit, across the engine's 4 KB output blocks.
"""
import struct

import numpy as np
import pytest

from oracle_lib import Oracle
from minpaxos_amd import records as R
from minpaxos_amd import synth


def put_varint(x):  # encoding/binary.PutVarint
    ux = (x << 1) ^ (-1 if x < 0 else 0)
    ux &= (1 << 64) - 1
    b = bytearray()
    while ux >= 0x80:
        b.append((ux & 0x7F) | 0x80)
        ux >>= 7
    b.append(ux)
    return bytes(b)


def cmd_bytes(op, key, val):
    return struct.pack("<Bqq", op, key, val)


def expected(fmt, recs, off, op, key, val):
    w, ro = bytearray(), []
    for i, r in enumerate(recs):
        ro.append(len(w))
        w += struct.pack("<ii", int(r["ballot"]), int(r["status"]))
        c0, c1 = int(off[i]), int(off[i + 1])
        w += put_varint(c1 - c0) if fmt == R.LOG_CATCHUP else struct.pack("<i", int(r["inst_no"]))
        for j in range(c0, c1):
            w += cmd_bytes(int(op[j]), int(key[j]), int(val[j]))
    ro.append(len(w))
    return bytes(w), ro


def sample():
    recs = np.zeros(4, R.LOG_REC)
    recs["ballot"] = [16, 16, -1, 33]
    recs["status"] = [R.COMMITTED, R.ACCEPTED, R.COMMITTED, R.PREPARED]
    recs["inst_no"] = [7, 8, 9, 10]
    cnt = [1, 0, 64, 3]  # 64 commands -> a 2-byte varint (zigzag 128)
    off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64)
    m = int(off[-1])
    rng = np.random.default_rng(3)
    op = rng.integers(0, 6, m).astype(np.uint8)
    key = rng.integers(-(1 << 62), 1 << 62, m).astype(np.int64)
    val = rng.integers(-(1 << 62), 1 << 62, m).astype(np.int64)
    key[0] = np.iinfo(np.int64).min
    return recs, off, op, key, val


@pytest.mark.parametrize("fmt", [R.LOG_CATCHUP, R.LOG_DURABLE])
def test_kat_formats(fmt):
    recs, off, op, key, val = sample()
    out, ro = Oracle().encode_log(fmt, recs, off, op, key, val)
    want, wro = expected(fmt, recs, off, op, key, val)
    assert out.tobytes() == want and list(ro) == wro
    if fmt == R.LOG_CATCHUP:
        assert out[int(ro[2]) + 8:int(ro[2]) + 10].tobytes() == bytes([0x80, 0x01])


def test_kat_catchup_suffix_per_peer():
    recs, off, op, key, val = synth.log_records(50, 4, ragged=True)
    out, ro = Oracle().encode_log(R.LOG_CATCHUP, recs, off, op, key, val)
    peer_commits = [-1, 10, 48]  # bcastAccept: from = 0 if peercommits < 0 else pc + 1
    for pc in peer_commits:
        frm = 0 if pc < 0 else pc + 1
        sub = Oracle().encode_log(R.LOG_CATCHUP, recs[frm:], off[frm:] - off[frm],
                                  op[int(off[frm]):], key[int(off[frm]):], val[int(off[frm]):])[0]
        assert out[int(ro[frm]):].tobytes() == sub.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [R.LOG_CATCHUP, R.LOG_DURABLE])
def test_logenc_parity(mk_engine, fmt):
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    cases = [sample()]
    for n, c, ragged in ((1, 1, False), (10, 4, True), (4000, 4, True), (100000, 4, False),
                         (300, 40, True)):
        cases.append(synth.log_records(n, c, seed=n + c, ragged=ragged))
    recs, off, op, key, val = synth.log_records(600, 2, seed=9, ragged=True)
    big = np.array(off, np.int64)
    big[300:] += 900  # one instance with 900 commands (many 4 KB blocks, 2-byte varint)
    m = int(big[-1])
    bop, bkey, bval = synth.commands(m, 1 << 10, 0.5, "uniform", seed=10)
    cases.append((recs, big.astype(np.uint64), bop, bkey, bval))
    empty = np.zeros(0, R.LOG_REC)
    cases.append((empty, np.zeros(1, np.uint64), np.zeros(0, np.uint8), np.zeros(0, np.int64),
                  np.zeros(0, np.int64)))
    for recs, off, op, key, val in cases:
        got = e.encode_log(fmt, recs, off, op, key, val)
        want = o.encode_log(fmt, recs, off, op, key, val)
        assert np.array_equal(got[1], want[1]), len(recs)
        assert got[0].tobytes() == want[0].tobytes(), len(recs)
