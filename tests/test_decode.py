"""Peer-stream framing + AcceptReply decode.

CPU: hand-built known-answer streams against the oracle (oracle/wire.cpp), each derived from
the cited Go: replicaListener's frame loop (genericsmr.go:402-446) and the Unmarshal()s it
dispatches to (minpaxosprotomarsh.go, gsmrprotomarsh.go).
GPU: mpx_decode_peer_stream vs the oracle, bit for bit, on streams that cross the engine's
chunk (128 B), tile (16 KB) and group (4 MB) boundaries, junk, partial tails, variable-length
stops and short output capacities.
"""
import struct

import numpy as np
import pytest

from oracle_lib import Oracle
from minpaxos_amd import records as R
from minpaxos_amd import synth


def ar_frame(inst, ok, ballot, rid):
    # AcceptReply.Marshal  minpaxosprotomarsh.go:545-566: Instance, OK, Ballot, Id (LE)
    return bytes([R.PEER_ACCEPT_REPLY]) + struct.pack("<iBii", inst, ok, ballot, rid)


def test_kat_single_accept_reply():
    ar, oth, res = Oracle().decode_peer_stream(ar_frame(-5, 1, 0x12345678, 3))
    assert len(ar) == 1 and len(oth) == 0
    assert (ar[0]["instance"], ar[0]["ok"], ar[0]["ballot"], ar[0]["id"]) == (-5, 1, 0x12345678, 3)
    assert res["consumed"] == 14 and res["stop_reason"] == R.DECODE_END and res["stop_code"] == -1


def test_kat_mixed_frames_in_order():
    beacon = bytes([R.PEER_BEACON]) + struct.pack("<Q", 99)           # Beacon{Timestamp}
    prep = bytes([R.PEER_PREPARE]) + struct.pack("<iii", 1, 16, 7)      # Prepare (12 B)
    cs = bytes([R.PEER_COMMIT_SHORT]) + struct.pack("<iiii", 0, 4, 2, 16)  # CommitShort (16 B)
    unknown = bytes([200])                                               # logged, skipped
    s = ar_frame(1, 1, 16, 1) + beacon + unknown + prep + ar_frame(2, 0, 32, 2) + cs
    ar, oth, res = Oracle().decode_peer_stream(s)
    assert list(ar["instance"]) == [1, 2] and list(ar["ok"]) == [1, 0]
    assert [(int(f["offset"]), int(f["code"])) for f in oth] == [
        (14, R.PEER_BEACON), (23, 200), (24, R.PEER_PREPARE), (51, R.PEER_COMMIT_SHORT)]
    assert res["consumed"] == len(s) and res["stop_reason"] == R.DECODE_END


@pytest.mark.parametrize("code,body", [(R.PEER_ACCEPT_REPLY, 13), (R.PEER_BEACON, 8),
                                       (R.PEER_BEACON_REPLY, 8), (R.PEER_PREPARE, 12),
                                       (R.PEER_COMMIT_SHORT, 16)])
def test_kat_partial_frame_at_end(code, body):
    head = ar_frame(9, 1, 16, 4)
    for cut in range(0, body):
        s = head + bytes([code]) + bytes(cut)
        ar, oth, res = Oracle().decode_peer_stream(s)
        assert len(ar) == 1 and len(oth) == 0
        assert res["consumed"] == 14 and res["stop_reason"] == R.DECODE_PARTIAL
        assert res["stop_code"] == code


@pytest.mark.parametrize("code", [R.PEER_ACCEPT, R.PEER_COMMIT, R.PEER_PREPARE_REPLY])
def test_kat_variable_length_frame_stops(code):
    s = ar_frame(1, 1, 16, 1) + bytes([code, 0, 0, 0]) + ar_frame(2, 1, 16, 1)
    ar, oth, res = Oracle().decode_peer_stream(s)
    assert len(ar) == 1 and res["consumed"] == 14
    assert res["stop_reason"] == R.DECODE_VARIABLE and res["stop_code"] == code


def test_kat_empty_and_capacity():
    ar, oth, res = Oracle().decode_peer_stream(b"")
    assert res["consumed"] == 0 and res["stop_reason"] == R.DECODE_END and len(ar) == 0
    s = b"".join(ar_frame(i, 1, 16, 1) for i in range(10))
    ar, _, res = Oracle().decode_peer_stream(s, ar_cap=4)
    assert len(ar) == 4 and res["n_accept_replies"] == 10 and list(ar["instance"]) == [0, 1, 2, 3]


def test_synth_round_trip():
    rec, _ = synth.accept_replies(500, 5, 0.7, seed=42)
    buf = synth.peer_stream(rec, p_beacon=0.05, p_prepare=0.02, p_commit_short=0.02,
                            p_unknown=0.05)
    ar, oth, res = Oracle().decode_peer_stream(buf)
    for f in ("instance", "ballot", "id", "ok"):
        assert np.array_equal(ar[f], rec[f]), f
    assert res["consumed"] == len(buf) and res["stop_reason"] == R.DECODE_END


# ---- GPU parity --------------------------------------------------------------------------------
def _eq(got, want):
    ga, go, gr = got
    wa, wo, wr = want
    assert gr.tobytes() == wr.tobytes(), (gr, wr)
    assert ga.tobytes() == wa.tobytes()
    assert go.tobytes() == wo.tobytes()


def _streams():
    rng = np.random.default_rng(31)
    rec, _ = synth.accept_replies(1 << 17, 5, 0.7, seed=42)
    out = {}
    for n in (1, 3, 4, 5, 37, 585, 1170, 1171, 1172, 2000):  # 1170 frames ~ one 16 KB tile
        out[f"ar_only_{n}"] = synth.peer_stream(rec[:n])
    out["mixed_small"] = synth.peer_stream(rec[:3000], p_beacon=0.05, p_prepare=0.03,
                                           p_commit_short=0.03, p_unknown=0.1)
    out["mixed_groups"] = synth.peer_stream(rec, seed=5, p_beacon=0.01, p_prepare=0.01,
                                            p_commit_short=0.01, p_unknown=0.01)  # > 4 MB
    out["unknown_heavy"] = synth.peer_stream(rec[:20000], seed=6, p_unknown=0.6)
    junk = rng.integers(0, 256, 300000).astype(np.uint8)
    junk[np.isin(junk, [R.PEER_ACCEPT, R.PEER_COMMIT, R.PEER_PREPARE_REPLY])] = 200
    out["junk_no_variable"] = junk
    out["junk_raw"] = rng.integers(0, 256, 5000).astype(np.uint8)
    for cut in (1, 5, 13):
        out[f"partial_{cut}"] = synth.peer_stream(rec[:2000], tail=bytes([13] + [0] * cut))
    base = synth.peer_stream(rec[:40000], seed=7, p_beacon=0.01)
    starts = _frame_starts(base)
    for at in (0, 13, 16384 * 3 + 5, len(base) // 2):
        # a variable-length frame spliced in at the first frame boundary at or after `at`
        pos = int(starts[min(int(np.searchsorted(starts, at)), len(starts) - 1)])
        out[f"variable_at_{at}"] = np.concatenate(
            [base[:pos], np.array([R.PEER_COMMIT, 3], np.uint8), base[pos:]])
    return out


def _frame_starts(buf):
    p, starts = 0, []
    body = {R.PEER_BEACON: 8, R.PEER_BEACON_REPLY: 8, R.PEER_PREPARE: 12,
            R.PEER_COMMIT_SHORT: 16, R.PEER_ACCEPT_REPLY: 13}
    b = buf.tobytes()
    while p < len(b):
        starts.append(p)
        p += 1 + body.get(b[p], 0)
    return np.array(starts, np.int64)


STREAMS = None


def streams():
    global STREAMS
    if STREAMS is None:
        STREAMS = _streams()
    return STREAMS


@pytest.mark.gpu
def test_decode_parity(mk_engine):
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    for name, buf in streams().items():
        got = e.decode_peer_stream(buf)
        want = o.decode_peer_stream(buf)
        try:
            _eq(got, want)
        except AssertionError as ex:
            raise AssertionError(f"stream {name} (len {len(buf)}): {ex}")


@pytest.mark.gpu
def test_decode_empty_and_short_capacity(mk_engine):
    e, o = mk_engine(5, R.MODE_MIN), Oracle()
    _eq(e.decode_peer_stream(np.zeros(0, np.uint8)), o.decode_peer_stream(np.zeros(0, np.uint8)))
    rec, _ = synth.accept_replies(3000, 5, 0.7, seed=42)
    buf = synth.peer_stream(rec, p_beacon=0.05, p_unknown=0.05)
    for cap in (0, 1, 100, 11999):
        _eq(e.decode_peer_stream(buf, ar_cap=cap, other_cap=cap // 3),
            o.decode_peer_stream(buf, ar_cap=cap, other_cap=cap // 3))
