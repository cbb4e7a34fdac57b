"""Full peer-stream decode: fixed AND variable-length frames, MIN and
CLASSIC wire formats (mpx_decode_stream).

CPU: the oracle (oracle/wire.cpp) against a second, independent restatement written here as a
literal Python transliteration of replicaListener (genericsmr.go:402-446) and the Unmarshal
methods it dispatches to (minpaxosprotomarsh.go / paxosprotomarsh.go, binary.ReadVarint),
on hand-built known-answer streams, on every truncation point of a stream, on malformed
varints / negative lengths, and on random streams.
GPU: the engine against the oracle, bit for bit, on random streams, leader-side streams (dense
AcceptReplies with PrepareReplies mixed in) and streams with frames longer than the engine's
in-map window (each such frame is one MPX_DECODE_LONG resume of the _dev form).
"""
import struct

import numpy as np
import pytest

from oracle_lib import Oracle
from minpaxos_amd import records as R
from minpaxos_amd import synth
from minpaxos_amd import wire as W

MIN, CLASSIC = R.MODE_MIN, R.MODE_CLASSIC


# ---- second restatement: the Go loop, literally ----------------------------------------------
class _Short(Exception):
    """a read past the end of the bytes (on the socket: Unmarshal blocks for more)"""


class _Reader:
    def __init__(self, b, pos):
        self.b, self.pos = b, pos

    def read(self, n):  # io.ReadAtLeast / io.ReadFull
        if self.pos + n > len(self.b):
            raise _Short()
        x = self.b[self.pos:self.pos + n]
        self.pos += n
        return x

    def read_byte(self):
        return self.read(1)[0]


def _read_varint(r):
    """binary.ReadVarint -> (value, error)"""
    x, s = 0, 0
    for i in range(10):
        b = r.read_byte()
        if b < 0x80:
            if i == 9 and b > 1:
                return 0, "overflow"
            x |= b << s
            v = x >> 1
            if x & 1:
                v = ~v
            return v, None
        x |= (b & 0x7F) << s
        s += 7
    return 0, "overflow"


def _slice(r, n, elem):
    if n < 0:
        raise ValueError("makeslice: len out of range")  # Go panics
    if n > len(r.b):
        raise _Short()
    return [elem(r) for _ in range(n)]


def _command(r):
    op, k, v = struct.unpack("<Bqq", r.read(17))
    return op, k, v


def _instance(r):
    r.read(8)
    k, err = _read_varint(r)
    if err:
        raise OverflowError(err)
    return _slice(r, k, _command)


def go_listener(proto, b):
    """-> (frames, stop_reason, consumed, stop_code); frames = [(offset, code, fields)]"""
    frames, p = [], 0
    hdr = {MIN: {R.PEER_ACCEPT: 16, R.PEER_COMMIT: 12, R.PEER_PREPARE_REPLY: 17},
           CLASSIC: {R.PEER_ACCEPT: 12, R.PEER_COMMIT: 12, R.PEER_PREPARE_REPLY: 9}}[proto]
    body = R.PEER_BODY if proto == MIN else R.PEER_BODY_CLASSIC
    while p < len(b):
        code = b[p]
        r = _Reader(b, p + 1)
        try:
            if code in hdr:
                h = r.read(hdr[code])
                n, err = _read_varint(r)
                if err:
                    raise OverflowError(err)
                cmds_off = r.pos
                cmds = _slice(r, n, _command)
                log_off, log = r.pos, []
                if proto == MIN and code != R.PEER_COMMIT:
                    m, err = _read_varint(r)
                    if err:
                        raise OverflowError(err)
                    log_off = r.pos
                    log = _slice(r, m, _instance)
                frames.append((p, code, dict(hdr=h, n_cmds=len(cmds), cmds_off=cmds_off,
                                             n_log=len(log), log_off=log_off, length=r.pos - p)))
            elif code in body:
                frames.append((p, code, dict(hdr=r.read(body[code]))))
            else:
                frames.append((p, code, None))  # "unknown message type": 1 byte
        except _Short:
            return frames, R.DECODE_PARTIAL, p, code
        except (OverflowError, ValueError):
            return frames, R.DECODE_MALFORMED, p, code
        p = r.pos
    return frames, R.DECODE_END, p, -1


def check_against_go(proto, got, b):
    ar, pr, var, oth, res = got
    frames, why, consumed, code = go_listener(proto, b)
    assert (int(res["stop_reason"]), int(res["consumed"]), int(res["stop_code"])) == \
        (why, consumed, code)
    ia = ip = iv = io = 0
    for off, c, f in frames:
        if c == R.PEER_ACCEPT_REPLY:
            h = f["hdr"]
            inst, ok, bal = struct.unpack_from("<iBi", h)
            rid = struct.unpack_from("<i", h, 9)[0] if proto == MIN else -1
            assert tuple(int(x) for x in ar[ia][["instance", "ok", "ballot", "id"]]) == \
                (inst, ok, bal, rid)
            ia += 1
        elif f is not None and "n_cmds" in f:
            v = var[iv]
            assert (int(v["offset"]), int(v["code"]), int(v["length"]), int(v["n_cmds"]),
                    int(v["cmds_off"]), int(v["n_log"]), int(v["log_off"])) == \
                (off, c, f["length"], f["n_cmds"], f["cmds_off"], f["n_log"], f["log_off"])
            if c == R.PEER_PREPARE_REPLY:
                h = f["hdr"]
                if proto == MIN:
                    rid, inst, ok, bal, lc = struct.unpack("<iiBii", h)
                    want = (rid, inst, bal, lc, ok, iv)
                    got_p = tuple(int(x) for x in pr[ip][["id", "instance", "ballot",
                                                          "last_committed", "ok", "value_id"]])
                else:
                    inst, ok, bal = struct.unpack("<iBi", h)
                    want = (inst, bal, ok, iv)
                    got_p = tuple(int(x) for x in pr[ip][["instance", "ballot", "ok", "value_id"]])
                assert got_p == want
                ip += 1
            iv += 1
        else:
            assert (int(oth[io]["offset"]), int(oth[io]["code"])) == (off, c)
            io += 1
    assert (ia, ip, iv, io) == (len(ar), len(pr), len(var), len(oth))


# ---- CPU: oracle vs the Go loop ------------------------------------------------------------------
def kat_stream(proto):
    return b"".join([
        W.accept_reply(proto, 7, 1, 16, 2),
        W.prepare_reply(proto, 9, 1, 33, [(1, -5, 50)], 3, 8,
                        [(16, 3, [(1, 1, 1), (2, 1, 0)])]),
        W.fixed(proto, R.PEER_BEACON, 0x1122334455667788),
        W.accept(proto, 0, 10, 33, [], 9, []),
        W.commit(0, 10, 33, [(1, 2, 3)] * 3),
        bytes([250]),  # unknown code: 1 byte
        W.fixed(proto, R.PEER_COMMIT_SHORT, 12345),
        W.prepare_reply(proto, -1, 0, -1, []),
        W.fixed(proto, R.PEER_PREPARE, 99),
        W.accept_reply(proto, 8, 0, 48, 4),
    ])


@pytest.mark.parametrize("proto", [MIN, CLASSIC], ids=["min", "classic"])
def test_oracle_kat(proto):
    b = kat_stream(proto)
    got = Oracle(5, proto).decode_stream(b)
    ar, pr, var, oth, res = got
    assert int(res["stop_reason"]) == R.DECODE_END and int(res["consumed"]) == len(b)
    assert len(ar) == 2 and len(pr) == 2 and len(var) == 4 and len(oth) == 4
    assert [int(x) for x in ar["instance"]] == [7, 8]
    assert [int(x) for x in var["code"]] == [12, 9, 10, 12]
    assert int(var[2]["n_cmds"]) == 3  # the Commit
    assert int(pr[0]["value_id"]) == 0 and int(pr[1]["value_id"]) == 3
    if proto == MIN:
        assert int(var[0]["n_log"]) == 1 and int(pr[0]["last_committed"]) == 8
    check_against_go(proto, got, b)


@pytest.mark.parametrize("proto", [MIN, CLASSIC], ids=["min", "classic"])
def test_oracle_every_truncation(proto):
    b = kat_stream(proto)
    o = Oracle(5, proto)
    for cut in range(len(b) + 1):
        check_against_go(proto, o.decode_stream(b[:cut]), b[:cut])


@pytest.mark.parametrize("proto", [MIN, CLASSIC], ids=["min", "classic"])
def test_oracle_malformed(proto):
    o = Oracle(5, proto)
    good = W.accept_reply(proto, 1, 1, 16, 1)
    hdr = W.prepare_reply(proto, 1, 1, 16, [])[:1 + (17 if proto == MIN else 9)]
    for bad in (bytes([0xFF] * 9 + [0x02]),         # 10th byte > 1: overflow
                bytes([0x80] * 10),                  # never terminates within 10 bytes
                W.put_varint(-1),                    # negative slice length: make panics
                W.put_varint(-(1 << 40))):
        b = good + hdr + bad + good
        got = o.decode_stream(b)
        assert int(got[4]["stop_reason"]) == R.DECODE_MALFORMED
        assert int(got[4]["consumed"]) == len(good)
        check_against_go(proto, got, b)
    # a length whose Commands have not arrived: partial, not malformed
    b = good + hdr + W.put_varint(1 << 40)
    got = o.decode_stream(b)
    assert int(got[4]["stop_reason"]) == R.DECODE_PARTIAL
    check_against_go(proto, got, b)


@pytest.mark.parametrize("proto", [MIN, CLASSIC], ids=["min", "classic"])
def test_oracle_random_streams(proto):
    rng = np.random.default_rng(70 + proto)
    o = Oracle(5, proto)
    for trial in range(6):
        b = W.random_stream(proto, rng, 400, p_var=0.1 + 0.15 * trial)
        check_against_go(proto, o.decode_stream(b), b)
        cut = int(rng.integers(0, len(b)))
        check_against_go(proto, o.decode_stream(b[:cut]), b[:cut])


@pytest.mark.parametrize("proto", [MIN, CLASSIC], ids=["min", "classic"])
def test_leader_stream_generator(proto):
    recs, _ = synth.accept_replies(3000, 5, 0.7, seed=42)
    buf = W.leader_stream(proto, recs, prepare_every=97, n_cmds=2, p_beacon=0.01)
    got = Oracle(5, proto).decode_stream(buf)
    check_against_go(proto, got, bytes(buf))
    ar = got[0]
    assert len(ar) == len(recs) and np.array_equal(ar["instance"], recs["instance"])
    assert len(got[1]) == len(range(0, len(recs), 97)) and (got[2]["n_cmds"] == 2).all()


# ---- GPU: engine vs oracle -------------------------------------------------------------------------
def _eq_decode(got, want):
    for g, w, name in zip(got[:4], want[:4], ("ar", "prep", "var", "other")):
        assert len(g) == len(w), name
        assert g.tobytes() == w.tobytes(), name
    for f in ("consumed", "n_accept_replies", "n_prepare_replies", "n_var", "n_other",
              "stop_reason", "stop_code"):
        assert int(got[4][f]) == int(want[4][f]), f


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [MIN, CLASSIC], ids=["min", "classic"])
def test_stream_decode_parity_random(mk_engine, proto):
    rng = np.random.default_rng(80 + proto)
    e, o = mk_engine(5, proto), Oracle(5, proto)
    for trial in range(8):
        b = W.random_stream(proto, rng, 3000 + 2000 * trial, p_var=0.05 * trial,
                            p_big=0.01 * (trial % 3))
        for cut in (len(b), int(rng.integers(0, len(b)))):
            _eq_decode(e.decode_stream(b[:cut]), o.decode_stream(b[:cut]))
    _eq_decode(e.decode_stream(b""), o.decode_stream(b""))
    _eq_decode(e.decode_stream(kat_stream(proto)), o.decode_stream(kat_stream(proto)))


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [MIN, CLASSIC], ids=["min", "classic"])
def test_stream_decode_parity_leader(mk_engine, proto):
    e, o = mk_engine(5, proto), Oracle(5, proto)
    recs, _ = synth.accept_replies(1 << 18, 5, 0.7, seed=42)
    for every, k in ((4096, 1), (7, 1), (1, 3), (50, 0)):
        buf = W.leader_stream(proto, recs, prepare_every=every, n_cmds=k)
        _eq_decode(e.decode_stream(buf), o.decode_stream(buf))


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [MIN, CLASSIC], ids=["min", "classic"])
def test_stream_decode_long_frames_and_malformed(mk_engine, proto):
    """frames far longer than the in-map window (catch-up logs, 5000-command batches), back to
    back and between short frames; a malformed varint after them"""
    rng = np.random.default_rng(90 + proto)
    e, o = mk_engine(5, proto), Oracle(5, proto)
    parts = []
    for k in range(40):
        parts.append(W.random_stream(proto, rng, int(rng.integers(0, 60)), p_var=0.2))
        n = [0, 5, 60, 5000][k % 4]
        cmds = [(1, i, -i) for i in range(n)]
        parts.append(W.accept(proto, 0, k, 16, cmds, k - 1,
                              [(16, 3, cmds[:7])] * (k % 5)) if k % 2 else
                     W.prepare_reply(proto, k, 1, 16, cmds, 1, k - 2, [(16, 3, cmds[:3])] * (k % 3)))
    b = b"".join(parts)
    _eq_decode(e.decode_stream(b), o.decode_stream(b))
    b2 = b + W.prepare_reply(proto, 1, 1, 16, [])[:1 + (17 if proto == MIN else 9)] + \
        bytes([0xFF] * 9 + [0x03]) + b
    _eq_decode(e.decode_stream(b2), o.decode_stream(b2))


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [MIN, CLASSIC], ids=["min", "classic"])
def test_stream_decode_tile_edges(mk_engine, proto):
    """buffers ending exactly at, one byte before and one byte after 16 KB tile boundaries (the
    framing pass's extra tile, a stop in a TileEnt tile's group 0 or past it), tiny buffers,
    and leader streams whose instance numbers put a variable-message code byte in every frame
    (var-dense framing-DP waves)"""
    e, o = mk_engine(5, proto), Oracle(5, proto)
    recs, _ = synth.accept_replies(1 << 15, 5, 0.7, seed=7, inst_base=0x0A0A00)
    buf = bytes(W.leader_stream(proto, recs, prepare_every=97, n_cmds=1))
    for cut in [1, 2, 13, 127, 128, 129, 1023] + [k * 16384 + d for k in (1, 2, 7) for d in (-1, 0, 1)] + \
               [8 * 128 + d for d in (-1, 0, 1)] + [len(buf)]:
        b = buf[:cut]
        _eq_decode(e.decode_stream(b), o.decode_stream(b))
