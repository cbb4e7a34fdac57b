"""Peer-connection byte streams as the reference's Marshal() methods write them (synthetic input
for mpx_decode_stream; the decoder itself is native code).

Layouts, little endian (MIN = minpaxosproto, minpaxosprotomarsh.go; CLASSIC = paxosproto,
paxosprotomarsh.go), each frame = [code u8][body]:
  Beacon / BeaconReply (6/7)  Timestamp u64                               genericsmrproto
  Prepare (8)      MIN LeaderId, Ballot, LastCommitted (12)               :237-257
                   CLASSIC LeaderId, Instance, Ballot, ToInfinity (13)    :53-74
  Accept (9)       MIN LeaderId, Instance, Ballot, LastCommitted, V(n), n Commands, V(m),
                   m Instances                                            :425-468
                   CLASSIC LeaderId, Instance, Ballot, V(n), n Commands   :214-242
  Commit (10)      LeaderId, Instance, Ballot, V(n), n Commands           :618-646 / :373-401
  CommitShort (11) LeaderId, Instance, Count, Ballot                      :710-735 / :465-490
  PrepareReply(12) MIN Id, Instance, OK, Ballot, LastCommitted, V(n), n Commands, V(m),
                   m Instances                                            :308-350
                   CLASSIC Instance, OK, Ballot, V(n), n Commands         :126-150
  AcceptReply (13) MIN Instance, OK, Ballot, Id (13)                      :545-566
                   CLASSIC Instance, OK, Ballot (9)                       :306-322
  Instance         Ballot, Status, V(k), k Commands                       :100-124
  Command          Op u8, K i64, V i64                                    statemarsh.go:8-20
V(x) = binary.PutVarint (zig-zag + base-128 groups).
"""
import struct

import numpy as np

from . import records as R
from . import synth

MIN, CLASSIC = R.MODE_MIN, R.MODE_CLASSIC


def put_varint(x):
    """binary.PutVarint"""
    ux = ((x << 1) ^ (x >> 63)) & 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while ux >= 0x80:
        out.append((ux & 0x7F) | 0x80)
        ux >>= 7
    out.append(ux)
    return bytes(out)


def command(op, k, v):
    return struct.pack("<Bqq", op, k, v)


def commands(cmds):
    return put_varint(len(cmds)) + b"".join(command(*c) for c in cmds)


def instance(ballot, status, cmds):
    return struct.pack("<ii", ballot, status) + commands(cmds)


def catchup(log):
    """log: [(ballot, status, cmds)]"""
    return put_varint(len(log)) + b"".join(instance(*x) for x in log)


def accept_reply(proto, inst, ok, ballot, rid=0):
    if proto == MIN:
        return bytes([R.PEER_ACCEPT_REPLY]) + struct.pack("<iBii", inst, ok, ballot, rid)
    return bytes([R.PEER_ACCEPT_REPLY]) + struct.pack("<iBi", inst, ok, ballot)


def prepare_reply(proto, inst, ok, ballot, cmds, rid=0, last_committed=0, log=()):
    if proto == MIN:
        return (bytes([R.PEER_PREPARE_REPLY]) +
                struct.pack("<iiBii", rid, inst, ok, ballot, last_committed) + commands(cmds) +
                catchup(log))
    return bytes([R.PEER_PREPARE_REPLY]) + struct.pack("<iBi", inst, ok, ballot) + commands(cmds)


def accept(proto, leader, inst, ballot, cmds, last_committed=0, log=()):
    if proto == MIN:
        return (bytes([R.PEER_ACCEPT]) + struct.pack("<iiii", leader, inst, ballot, last_committed)
                + commands(cmds) + catchup(log))
    return bytes([R.PEER_ACCEPT]) + struct.pack("<iii", leader, inst, ballot) + commands(cmds)


def commit(leader, inst, ballot, cmds):
    return bytes([R.PEER_COMMIT]) + struct.pack("<iii", leader, inst, ballot) + commands(cmds)


def fixed(proto, code, payload):
    """a fixed-size frame of `code` with body bytes taken from `payload` (an int)"""
    body = {R.PEER_BEACON: 8, R.PEER_BEACON_REPLY: 8, R.PEER_COMMIT_SHORT: 16,
            R.PEER_PREPARE: 12 if proto == MIN else 13}[code]
    return bytes([code]) + (payload & ((1 << (8 * body)) - 1)).to_bytes(body, "little")


def random_stream(proto, rng, n_frames, p_var=0.3, max_cmds=6, p_big=0.02, big_cmds=300,
                  max_log=3, p_unknown=0.03):
    """n_frames random frames of every kind; variable ones with 0..max_cmds Commands (a few
    with big_cmds), MIN ones with CatchUpLogs of 0..max_log Instances. Returns bytes."""
    out = []
    for _ in range(n_frames):
        u = rng.random()

        def cmds(k=None):
            if k is None:
                k = big_cmds if rng.random() < p_big else int(rng.integers(0, max_cmds + 1))
            return [(int(rng.integers(0, 6)), int(rng.integers(-(1 << 62), 1 << 62)),
                     int(rng.integers(-(1 << 62), 1 << 62))) for _ in range(k)]

        def log():
            if proto != MIN:
                return ()
            return [(int(rng.integers(-2, 300)), int(rng.integers(0, 4)),
                     cmds(int(rng.integers(0, 4)))) for _ in range(int(rng.integers(0, max_log + 1)))]
        i32 = lambda: int(rng.integers(-(1 << 31), 1 << 31))  # noqa: E731
        if u < p_var:
            kind = int(rng.integers(0, 3))
            if kind == 0:
                out.append(prepare_reply(proto, i32(), int(rng.integers(0, 2)), i32(), cmds(),
                                         int(rng.integers(0, 5)), i32(), log()))
            elif kind == 1:
                out.append(accept(proto, i32(), i32(), i32(), cmds(), i32(), log()))
            else:
                out.append(commit(i32(), i32(), i32(), cmds()))
        elif u < p_var + p_unknown:
            c = int(rng.integers(0, 256))
            out.append(bytes([c if not 6 <= c <= 13 else 200]))
        elif u < 0.75:
            out.append(accept_reply(proto, i32(), int(rng.integers(0, 3)), i32(),
                                    int(rng.integers(0, 5))))
        else:
            code = [R.PEER_BEACON, R.PEER_BEACON_REPLY, R.PEER_PREPARE,
                    R.PEER_COMMIT_SHORT][int(rng.integers(0, 4))]
            out.append(fixed(proto, code, int(rng.integers(0, 1 << 62)) * 7919 + 13))
    return b"".join(out)


def leader_stream(proto, recs, seed=61, prepare_every=4096, n_cmds=1, p_beacon=1.0 / 4096):
    """What a leader reads from one follower during recovery + steady state: every AcceptReply
    of `recs` (MIN 14-byte / CLASSIC 10-byte frames), a PrepareReply carrying n_cmds Commands
    (MIN: empty CatchUpLog) before every `prepare_every`-th AcceptReply, and Beacons.
    Vectorised (the bench builds ~1 GB with it). Returns a uint8 array."""
    n = len(recs)
    ar_len = 14 if proto == MIN else 10
    pr_hdr = 17 if proto == MIN else 9
    vn = put_varint(n_cmds)
    pr_len = 1 + pr_hdr + len(vn) + 17 * n_cmds + (1 if proto == MIN else 0)
    u = synth.stream(seed, 30, 0, n)
    has_pr = (np.arange(n) % max(prepare_every, 1) == 0) if prepare_every else np.zeros(n, bool)
    has_bc = (u & np.uint64(0xFFFFFF)) < np.uint64(int(p_beacon * (1 << 24)))
    pre = has_pr * pr_len + has_bc * 9
    off = np.zeros(n + 1, np.int64)
    np.cumsum(pre + ar_len, out=off[1:])
    buf = np.zeros(int(off[-1]), np.uint8)

    def put32(at, v):
        vb = np.ascontiguousarray(v.astype("<i4")).view(np.uint8).reshape(len(at), 4)
        for j in range(4):
            buf[at + j] = vb[:, j]

    # beacons first in the gap, then the PrepareReply, then the AcceptReply
    bat = off[:-1][has_bc]
    buf[bat] = R.PEER_BEACON
    ts = synth.stream(seed, 31, 0, int(has_bc.sum()))
    for j in range(8):
        buf[bat + 1 + j] = ((ts >> np.uint64(8 * j)) & np.uint64(0xFF)).astype(np.uint8)
    pat = off[:-1][has_pr] + has_bc[has_pr] * 9
    k = len(pat)
    pu = synth.stream(seed, 32, 0, k)
    buf[pat] = R.PEER_PREPARE_REPLY
    inst = recs["instance"][has_pr]
    bal = recs["ballot"][has_pr]
    ok = (pu & np.uint64(1)).astype(np.uint8)
    if proto == MIN:
        put32(pat + 1, recs["id"][has_pr])
        put32(pat + 5, inst)
        buf[pat + 9] = ok
        put32(pat + 10, bal)
        put32(pat + 14, inst - 1)  # LastCommitted
    else:
        put32(pat + 1, inst)
        buf[pat + 5] = ok
        put32(pat + 6, bal)
    c0 = pat + 1 + pr_hdr
    for j, b in enumerate(vn):
        buf[c0 + j] = b
    c0 = c0 + len(vn)
    for c in range(n_cmds):
        at = c0 + 17 * c
        buf[at] = R.OP_PUT
        kv = synth.stream(seed, 33 + c, 0, k)
        for j in range(8):
            buf[at + 1 + j] = ((kv >> np.uint64(8 * j)) & np.uint64(0xFF)).astype(np.uint8)
            buf[at + 9 + j] = ((kv >> np.uint64(8 * ((j + 3) % 8))) & np.uint64(0xFF)).astype(np.uint8)
    if proto == MIN:
        buf[c0 + 17 * n_cmds] = 0  # V(0): empty CatchUpLog
    at = off[1:] - ar_len
    buf[at] = R.PEER_ACCEPT_REPLY
    put32(at + 1, recs["instance"])
    buf[at + 5] = recs["ok"]
    put32(at + 6, recs["ballot"])
    if proto == MIN:
        put32(at + 10, recs["id"])
    return buf
