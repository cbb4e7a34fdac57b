"""Client reply fan-out.

CPU: the oracle's byte runs against ProposeReplyTS.Marshal restated with struct.pack
(gsmrprotomarsh.go:702-732: OK u8, CommandId i32, Value i64, Timestamp i64, Leader i32, LE),
one run per client connection in execution order (ReplyProposeTS, genericsmr.go:529-535).
GPU: mpx_encode_replies vs the oracle, bit for bit.
"""
import struct

import numpy as np
import pytest

from oracle_lib import Oracle, OracleError
from minpaxos_amd import records as R
from minpaxos_amd import synth


def marshal(ok, cid, value, ts, leader):
    return struct.pack("<BiqqiB", ok, cid, value, ts, leader, 0)[:25]


def test_kat_two_clients_in_execution_order():
    rec = np.zeros(4, R.REPLY_REC)
    rec["client"] = [1, 0, 1, 1]
    rec["command_id"] = [10, 20, 11, -1]
    rec["value"] = [0, -5, 7, 1 << 40]
    rec["timestamp"] = [100, 200, 300, -400]
    out, off = Oracle().encode_replies(rec, 3, ok=1, leader=2)
    assert list(off) == [0, 25, 100, 100]
    assert out[0:25].tobytes() == marshal(1, 20, -5, 200, 2)
    assert out[25:100].tobytes() == (marshal(1, 10, 0, 100, 2) + marshal(1, 11, 7, 300, 2) +
                                     marshal(1, -1, 1 << 40, -400, 2))


def test_kat_empty_and_bad_client():
    out, off = Oracle().encode_replies(np.zeros(0, R.REPLY_REC), 4)
    assert len(out) == 0 and list(off) == [0, 0, 0, 0, 0]
    rec = np.zeros(1, R.REPLY_REC)
    rec["client"] = 4
    with pytest.raises(OracleError):
        Oracle().encode_replies(rec, 4)


@pytest.mark.gpu
def test_fanout_parity(mk_engine):
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    # counting-sort path (<= 1024 connections; 5M replies = several tiles per workgroup) and the
    # radix path (65536 connections)
    for n, c in ((1, 1), (255, 2), (256, 7), (257, 7), (1000, 1024), (4099, 3),
                 (300000, 1024), (200000, 65536), (70000, 1), (5000000, 1000), (4500001, 2)):
        rec = synth.replies(n, c, seed=n + c)
        for ok, leader in ((1, 0), (0, 7)):
            got = e.encode_replies(rec, c, ok, leader)
            want = o.encode_replies(rec, c, ok, leader)
            assert np.array_equal(got[1], want[1]), (n, c)
            assert got[0].tobytes() == want[0].tobytes(), (n, c)


@pytest.mark.gpu
def test_fanout_empty_and_bad_client(mk_engine):
    from minpaxos_amd.engine import MpxError
    e = mk_engine(5, R.MODE_MIN)
    out, off = e.encode_replies(np.zeros(0, R.REPLY_REC), 5)
    assert len(out) == 0 and list(off) == [0] * 6
    rec = synth.replies(100, 4)
    rec["client"][50] = 9
    with pytest.raises(MpxError):
        e.encode_replies(rec, 4)
    rec["client"][50] = 1  # the handle stays usable
    got = e.encode_replies(rec, 4)
    want = Oracle().encode_replies(rec, 4)
    assert got[0].tobytes() == want[0].tobytes() and np.array_equal(got[1], want[1])


@pytest.mark.gpu
def test_fanout_skewed_and_unaligned_output(mk_engine):
    """one hot connection among many, into output buffers at every address mod 4"""
    from minpaxos_amd.devbuf import Arena
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    n, c = 600000, 1024
    rec = synth.replies(n, c, seed=5)
    rec["client"][np.random.default_rng(6).random(n) < 0.7] = 517
    want = o.encode_replies(rec, c, 1, 3)
    e.encode_replies_reserve(n)
    with Arena(e) as ar:
        d_rec = ar.put(rec)
        d_out = ar.empty(25 * n + 8, np.uint8)
        d_off = ar.empty(c + 1, np.uint64)
        for mis in range(4):
            e.encode_replies_dev(d_rec.ptr, n, c, 1, 3, d_out.ptr + mis, d_off.ptr)
            e.synchronize()
            got = ar.get(d_out)[mis:mis + 25 * n]
            assert got.tobytes() == want[0].tobytes(), mis
            assert np.array_equal(ar.get(d_off), want[1])
