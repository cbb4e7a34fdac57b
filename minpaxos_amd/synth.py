"""Counter-based synthetic reply / command streams.

Every value is a pure function of (seed, stream, index) through splitmix64, so any
sub-range of a workload can be regenerated exactly: the bench times the GPU on the full
stream and the CPU baseline on a bounded prefix of the same stream.
Shapes follow the reference's own knobs: replies come from acceptors 1..N-1 (the leader,
replica 0, never messages itself: bareminpaxos.go:471-475), ballots are
makeUniqueBallot(b) = (b<<4)|id (bareminpaxos.go:383-385), client ops are PUT with
probability -w (client.go:22,88-92), keys uniform or Zipf (client.go:30-31,46),
val = command index (client.go:164).
"""
import numpy as np

from . import records as R

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix(z):
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def stream(seed, tag, start, count):
    """u64 draws [start, start+count) of stream `tag` under `seed` (splitmix64)."""
    with np.errstate(over="ignore"):
        s = _mix(np.array([(seed * 0x100000001B3 + tag * 0x632BE59BD9B4E019) & 0xFFFFFFFFFFFFFFFF],
                          dtype=np.uint64))[0]
        idx = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        return _mix(s + idx * GOLDEN)


def _bern(u, p):
    return (u & np.uint64(0xFFFFFF)) < np.uint64(int(p * (1 << 24)))


def accept_replies(n_inst, n_replicas=5, p_ok=0.7, seed=42, inst_base=0, ballot=16):
    """Config 2: per instance R = N-1 AcceptReplyRec, grouped by instance, slot s holding
    acceptor perm_i[s] of {1..N-1}; ok ~ Bern(p_ok); ballot = makeUniqueBallot(1) = 16."""
    r = n_replicas - 1
    n = n_inst * r
    rec = np.zeros(n, dtype=R.ACCEPT_REPLY)
    rec["instance"] = np.repeat(np.arange(inst_base, inst_base + n_inst, dtype=np.int32), r)
    if r > 0:
        keys = stream(seed, 1, 0, n).reshape(n_inst, r)
        rec["id"] = (np.argsort(keys, axis=1, kind="stable") + 1).astype(np.int32).reshape(-1)
        rec["ok"] = _bern(stream(seed, 2, 0, n), p_ok)
    rec["ballot"] = ballot
    st = np.zeros(n_inst, dtype=R.INST_STATE)
    st["status"] = R.PREPARED
    return rec, st


def prepare_replies(n_inst, n_replicas=5, p_ok=0.8, seed=43, inst_base=0):
    """Config 3: per instance R = N-1 PrepareReplyRec; ballot = (U[0,16)<<4)|U[0,5) with 1/16
    forced to -1; value_id unique per reply, 1/32 the shared empty command (handle 0).
    Initial state {ballot 256, PREPARING, 0, 0, maxRecvBallot 0, own value, proposals}."""
    r = n_replicas - 1
    n = n_inst * r
    u = stream(seed, 3, 0, n)
    rec = np.zeros(n, dtype=R.PREPARE_REPLY)
    rec["instance"] = np.repeat(np.arange(inst_base, inst_base + n_inst, dtype=np.int32), r)
    rec["ok"] = _bern(u, p_ok)
    b = (((u >> np.uint64(24)) & np.uint64(15)) << np.uint64(4)) | ((u >> np.uint64(28)) % np.uint64(5))
    b = b.astype(np.int32)
    b[((u >> np.uint64(32)) & np.uint64(15)) == 0] = -1
    rec["ballot"] = b
    vid = np.arange(1, n + 1, dtype=np.uint32)
    vid[((u >> np.uint64(36)) & np.uint64(31)) == 0] = 0
    rec["value_id"] = vid
    st = np.zeros(n_inst, dtype=R.PREP_STATE)
    st["ballot"] = 256
    st["status"] = R.PREPARING
    st["value_id"] = np.uint32(0x80000000) | np.arange(n_inst, dtype=np.uint32)
    st["flags"] = R.PF_HAS_PROPOSALS
    return rec, st


def prepare_replies_min(n_groups, n_replicas=5, seed=46, replies_per_group=None):
    """MIN prepare: one PrepareBookkeeping per group. Ballots equal / below / above the
    group's defaultBallot (3/4, 1/8, 1/8), instances and lastCommitted scattered around the
    group's committedUpTo so that selection, catch-up and the trigger all fire."""
    r = (n_replicas - 1) if replies_per_group is None else replies_per_group
    n = n_groups * r
    ug = stream(seed, 4, 0, n_groups)
    u = stream(seed, 5, 0, n)
    gst = np.zeros(n_groups, dtype=R.GROUP_PREP_STATE)
    dball = ((((ug & np.uint64(7)) + np.uint64(1)) << np.uint64(4))).astype(np.int32)
    cu = ((ug >> np.uint64(8)) % np.uint64(100)).astype(np.int32)
    gst["default_ballot"] = dball
    gst["max_recv_ballot"] = dball
    gst["highest_instance"] = cu
    gst["committed_upto"] = cu
    gst["value_id"] = np.uint32(0x80000000) | np.arange(n_groups, dtype=np.uint32)
    rec = np.zeros(n, dtype=R.PREPARE_REPLY_MIN)
    gidx = np.repeat(np.arange(n_groups), r)
    sel = (u & np.uint64(7)).astype(np.int64)
    db = dball[gidx]
    rec["ballot"] = np.where(sel == 0, db - 16, np.where(sel == 1, db + 16, db))
    rec["instance"] = cu[gidx] + ((u >> np.uint64(8)) % np.uint64(4)).astype(np.int32) - 1
    rec["last_committed"] = cu[gidx] + ((u >> np.uint64(16)) % np.uint64(4)).astype(np.int32) - 2
    rec["ok"] = _bern(u >> np.uint64(24), 0.9)
    ids = (np.argsort(stream(seed, 6, 0, n).reshape(n_groups, r), axis=1, kind="stable") % max(1, n_replicas - 1) + 1)
    rec["id"] = ids.reshape(-1).astype(np.int32)
    rec["value_id"] = np.arange(1, n + 1, dtype=np.uint32)
    off = (np.arange(n_groups + 1, dtype=np.uint64) * np.uint64(r))
    return rec, off, gst


def zipf_cdf(n_keys, s=2.0, v=1.0):
    w = 1.0 / np.power(np.arange(n_keys, dtype=np.float64) + v, s)
    c = np.cumsum(w)
    return c / c[-1]


def commands(m, n_keys, p_put=0.5, dist="uniform", seed=44, start=0, other_ops=0.0,
             zipf_s=2.0, zipf_v=1.0):
    """Config 4: op = PUT w.p. p_put else GET (other_ops > 0 mixes in NONE/DELETE/RLOCK/
    WLOCK), key uniform or Zipf(s, v) over [0, n_keys), val = command index."""
    u = stream(seed, 7, start, m)
    uk = stream(seed, 8, start, m)
    fr = (u & np.uint64(0xFFFFFF)).astype(np.float64) / float(1 << 24)
    op = np.where(fr < p_put, R.OP_PUT, R.OP_GET).astype(np.uint8)
    if other_ops > 0:
        fr2 = ((u >> np.uint64(24)) & np.uint64(0xFFFFFF)).astype(np.float64) / float(1 << 24)
        alt = np.array([R.OP_NONE, R.OP_DELETE, R.OP_RLOCK, R.OP_WLOCK], dtype=np.uint8)
        op = np.where(fr2 < other_ops, alt[((u >> np.uint64(48)) & np.uint64(3)).astype(np.int64)], op)
    if dist == "uniform":
        key = (uk % np.uint64(n_keys)).astype(np.int64)
    elif dist == "zipf":
        cdf = zipf_cdf(n_keys, zipf_s, zipf_v)
        x = (uk >> np.uint64(11)).astype(np.float64) * (1.0 / float(1 << 53))
        key = np.minimum(np.searchsorted(cdf, x, side="right"), n_keys - 1).astype(np.int64)
    else:
        raise ValueError(dist)
    val = np.arange(start, start + m, dtype=np.int64)
    return op, key, val


def group_batch(n_groups, ipg=256, n_replicas=5, cmds_per_inst=4, keys_per_group=256,
                p_ok=0.7, p_put=0.5, seed=45, first_group=0):
    """Config 5: G groups x ipg instances x (N-1) replies + cmds_per_inst commands per
    instance; per-group keys uniform on [0, keys_per_group). Groups are generated from
    their global index, so a rank's block [first_group, first_group+n_groups) is identical
    to the same block of the whole job."""
    r = n_replicas - 1
    n_inst = n_groups * ipg
    g0 = first_group * ipg
    n = n_inst * r
    rec = np.zeros(n, dtype=R.ACCEPT_REPLY)
    rec["instance"] = np.tile(np.repeat(np.arange(ipg, dtype=np.int32), r), n_groups)
    if r > 0:
        keys = stream(seed, 9, g0 * r, n).reshape(n_inst, r)
        rec["id"] = (np.argsort(keys, axis=1, kind="stable") + 1).astype(np.int32).reshape(-1)
        rec["ok"] = _bern(stream(seed, 10, g0 * r, n), p_ok)
    rec["ballot"] = 16
    grp_rec_off = np.arange(n_groups + 1, dtype=np.uint64) * np.uint64(ipg * r)
    st = np.zeros(n_inst, dtype=R.INST_STATE)
    st["status"] = R.PREPARED
    m = n_inst * cmds_per_inst
    c0 = g0 * cmds_per_inst
    u = stream(seed, 11, c0, m)
    op = np.where((u & np.uint64(0xFFFFFF)) < np.uint64(int(p_put * (1 << 24))),
                  R.OP_PUT, R.OP_GET).astype(np.uint8)
    key = ((u >> np.uint64(32)) % np.uint64(keys_per_group)).astype(np.int64)
    val = np.arange(c0, c0 + m, dtype=np.int64)
    cmd_off = (np.arange(n_inst + 1, dtype=np.uint64) * np.uint64(cmds_per_inst)).astype(np.uint32)
    return dict(
        n_groups=n_groups, ipg=ipg, n_replicas=n_replicas, recs=rec, grp_rec_off=grp_rec_off,
        st_in=st, committed_in=np.full(n_groups, -1, np.int32),
        executed_in=np.full(n_groups, -1, np.int32),
        peer_in=np.zeros(n_groups * n_replicas, np.int32), op=op, key=key, val=val,
        cmd_off=cmd_off)


def peer_stream(recs, seed=47, p_beacon=0.0, p_prepare=0.0, p_commit_short=0.0, p_unknown=0.0,
                tail=None):
    """A peer connection's bytes: every AcceptReply of `recs` (mpx_accept_reply, arrival order)
    framed as [13][Instance i32][OK u8][Ballot i32][Id i32] (minpaxosprotomarsh.go:545-566),
    with other fixed-size frames interleaved before AcceptReply k with the given per-frame
    probabilities: Beacon [6][ts u64], Prepare [8][12 B], CommitShort [11][16 B], or one byte
    of an unregistered code. `tail`: bytes appended at the end (e.g. a partial frame or the
    start of a variable-length one). Returns a uint8 array."""
    n = len(recs)
    u = stream(seed, 20, 0, n)
    lim = lambda p: np.uint64(int(p * (1 << 24)))  # noqa: E731
    r = u & np.uint64(0xFFFFFF)
    kind = np.zeros(n, np.int8)  # 0 none, 1 beacon, 2 prepare, 3 commit short, 4 unknown
    a = lim(p_beacon)
    b = a + lim(p_prepare)
    c = b + lim(p_commit_short)
    d = c + lim(p_unknown)
    kind[r < a] = 1
    kind[(r >= a) & (r < b)] = 2
    kind[(r >= b) & (r < c)] = 3
    kind[(r >= c) & (r < d)] = 4
    pre = np.array([0, 9, 13, 17, 1], np.int64)[kind]
    size = pre + 14
    off = np.zeros(n + 1, np.int64)
    np.cumsum(size, out=off[1:])
    extra = b"" if tail is None else bytes(tail)
    buf = np.zeros(int(off[-1]) + len(extra), np.uint8)
    pay = stream(seed, 21, 0, n)  # payload bytes of the interleaved frames
    for k, code, body in ((1, R.PEER_BEACON, 8), (2, R.PEER_PREPARE, 12),
                          (3, R.PEER_COMMIT_SHORT, 16)):
        at = off[:-1][kind == k]
        buf[at] = code
        pk = pay[kind == k]
        for j in range(body):
            buf[at + 1 + j] = ((pk >> np.uint64((8 * j) % 64)) & np.uint64(0xFF)).astype(np.uint8)
    unk = off[:-1][kind == 4]
    codes = (pay[kind == 4] % np.uint64(251)).astype(np.int64)
    codes = np.where((codes >= 6) & (codes <= 13), codes + 20, codes)  # never a registered code
    buf[unk] = codes.astype(np.uint8)
    at = off[:-1] + pre
    buf[at] = R.PEER_ACCEPT_REPLY
    fields = ((1, recs["instance"].astype("<i4")), (6, recs["ballot"].astype("<i4")),
              (10, recs["id"].astype("<i4")))
    for o, v in fields:
        vb = v.view(np.uint8).reshape(n, 4)
        for j in range(4):
            buf[at + o + j] = vb[:, j]
    buf[at + 5] = recs["ok"]
    if extra:
        buf[int(off[-1]):] = np.frombuffer(extra, np.uint8)
    return buf


def replies(m, n_clients, seed=53, value=None):
    """Client replies for m executed commands, in execution order: client connection uniform on
    [0, n_clients), CommandId = the client's own running counter (client.go sends ids 0..q-1
    per client), Timestamp a nanosecond clock, Value = `value` (e.g. apply's ret) or index."""
    rec = np.zeros(m, R.REPLY_REC)
    c = (stream(seed, 30, 0, m) % np.uint64(n_clients)).astype(np.uint32)
    rec["client"] = c
    order = np.argsort(c, kind="stable")
    cnt = np.bincount(c, minlength=n_clients)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    ids = np.empty(m, np.int64)
    ids[order] = np.arange(m) - np.repeat(start, cnt)
    rec["command_id"] = ids.astype(np.int32)
    rec["timestamp"] = (1_700_000_000_000_000_000 + np.arange(m, dtype=np.int64) * 37)
    rec["value"] = np.arange(m, dtype=np.int64) if value is None else value
    return rec


def log_records(n_inst, cmds_per_inst=4, seed=56, ragged=False, first_inst=0):
    """A run of committed log records for the instance-log encoders: ballot makeUniqueBallot(1)
    = 16 (a few re-proposed at 32), status COMMITTED, instNo = first_inst + i, and
    cmds_per_inst commands each (ragged: 0..2*cmds_per_inst, some instances empty) from the
    config-4 command stream. Returns (recs, cmd_off, op, key, val)."""
    u = stream(seed, 40, 0, n_inst)
    if ragged:
        cnt = (u % np.uint64(2 * cmds_per_inst + 1)).astype(np.int64)
    else:
        cnt = np.full(n_inst, cmds_per_inst, np.int64)
    off = np.zeros(n_inst + 1, np.uint64)
    np.cumsum(cnt, out=off[1:])
    m = int(off[-1])
    op, key, val = commands(m, 1 << 20, 0.5, "uniform", seed=seed)
    recs = np.zeros(n_inst, R.LOG_REC)
    recs["ballot"] = np.where((u >> np.uint64(40)) % np.uint64(64) == 0, 32, 16)
    recs["status"] = R.COMMITTED
    recs["inst_no"] = np.arange(first_inst, first_inst + n_inst, dtype=np.int64).astype(np.int32)
    return recs, off, op, key, val
