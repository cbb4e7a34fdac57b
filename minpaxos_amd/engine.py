"""Python handle over the C ABI (numpy in, numpy out; device pointers for the *_dev paths).

Names and argument meaning follow the reference handlers they replace:
  accept_tally        <- bareminpaxos / paxos  handleAcceptReply
  prepare_select      <- paxos.handlePrepareReply          (CLASSIC, per instance)
  prepare_select_min  <- bareminpaxos.handlePrepareReply   (MIN, per group)
  apply               <- executeCommands -> state.Command.Execute (+ state.Conflict)
  conflict_batch      <- state.ConflictBatch
  committed_prefix    <- updateCommittedUpTo
  group_step          <- handleAcceptReply + executeCommands for many replicas at once
  decode_peer_stream  <- genericsmr.replicaListener framing + AcceptReply.Unmarshal
  encode_replies      <- the ProposeReplyTS fan-out (ReplyProposeTS per executed command)
  replay_durable      <- getDataFromStableStore (bareminpaxos.go:122-161)
  encode_log          <- Instance.Marshal (bcastAccept's CatchUpLog) / recordInstanceMetadata +
                         recordCommands (the durable log)
Errors come back as MpxError carrying the reference-level reason (e.g. E_NIL_INSTANCE where the
Go handler would dereference a nil *Instance).
"""
import ctypes as C

import numpy as np

from . import _lib
from . import records as R


class MpxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{R.ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


def _ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(C.c_void_p)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def device_count():
    lib = _lib.load()
    c = C.c_int(0)
    lib.mpx_device_count(C.byref(c))
    return c.value


def step_one_launch_fits(n_replicas, ipg, kv_per_group):
    """True when a fast group-step variant takes the batch shape, which MPX_FLAG_STEP_ONE_LAUNCH
    requires (the variant choice of step.hip fast_variant / mpx.h)"""
    recs = max(n_replicas - 1, 1) * ipg
    K = kv_per_group or 512
    return ((ipg <= 256 and recs <= 1024 and K <= 1024) or (ipg <= 256 and recs <= 2048 and K <= 256)
            or (ipg <= 512 and recs <= 2048 and K <= 512))


class Engine:
    def __init__(self, device=0, n_replicas=5, mode=R.MODE_MIN, kv_capacity=0, kv_per_group=0,
                 max_groups=0, apply_path=R.APPLY_AUTO, apply_fast_min=0, apply_hot_min=0,
                 apply_chunk=0, step_one_launch=False):
        """apply_* are the handle's mpx_apply settings (mpx_config): the pipeline choice
        (R.APPLY_AUTO / _SMALL / _SORTED / _PARTITIONED), AUTO's partitioned threshold, the hot
        key sample threshold (R.APPLY_NO_HOT: none) and the chunk size; 0 = default.
        step_one_launch: MPX_FLAG_STEP_ONE_LAUNCH (one kernel per group step; every group must
        fit the fast kernel, see mpx.h)"""
        self.lib = _lib.load()
        if isinstance(mode, str):
            mode = {"min": R.MODE_MIN, "classic": R.MODE_CLASSIC}[mode.lower()]
        self.n_replicas = n_replicas
        self.mode = mode
        self.kv_per_group = kv_per_group or 512
        self.step_one_launch = bool(step_one_launch)
        flags = R.FLAG_STEP_ONE_LAUNCH if step_one_launch else 0
        cfg = _lib.MpxConfig(n_replicas, mode, kv_capacity, kv_per_group, flags, max_groups,
                             apply_chunk, apply_path, apply_fast_min, apply_hot_min, 0)
        h = C.c_void_p()
        rc = self.lib.mpx_open(device, C.byref(cfg), C.byref(h))
        if rc != 0:
            raise MpxError(rc, f"mpx_open(device={device})")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.mpx_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.mpx_last_error(self.h)
            raise MpxError(rc, f"{what}: {msg.decode() if msg else ''}")

    @property
    def stream(self):
        return self.lib.mpx_stream(self.h)

    def synchronize(self):
        self._check(self.lib.mpx_synchronize(self.h), "mpx_synchronize")

    # ---- A1 / A2 ----------------------------------------------------------------------------
    def accept_tally(self, recs, st, inst_base=0, committed_upto=-1, peer_commits=None,
                     want_decided=True):
        recs = _c(recs, R.ACCEPT_REPLY)
        st = np.array(st, dtype=R.INST_STATE, copy=True)
        pc = np.zeros(self.n_replicas, np.int32) if peer_commits is None else \
            np.array(peer_commits, dtype=np.int32, copy=True)
        cu = C.c_int32(committed_upto)
        dec = np.zeros(len(st), np.uint8) if want_decided else None
        rc = self.lib.mpx_accept_tally(self.h, _ptr(recs), len(recs), _ptr(st), len(st), inst_base,
                                       C.byref(cu), _ptr(pc), _ptr(dec))
        self._check(rc, "mpx_accept_tally")
        return st, cu.value, pc, dec

    def accept_tally_dev(self, d_recs, n, d_st_in, d_st_out, n_inst, inst_base, d_scalars,
                         d_decided=None, stream=None):
        rc = self.lib.mpx_accept_tally_dev(self.h, d_recs, n, d_st_in, d_st_out, n_inst,
                                           inst_base, d_scalars, d_decided, stream)
        self._check(rc, "mpx_accept_tally_dev")

    def committed_prefix(self, st, inst_base, committed_upto):
        st = _c(st, R.INST_STATE)
        cu = C.c_int32(committed_upto)
        self._check(self.lib.mpx_committed_prefix(self.h, _ptr(st), len(st), inst_base,
                                                  C.byref(cu)), "mpx_committed_prefix")
        return cu.value

    # ---- A4 ---------------------------------------------------------------------------------
    def prepare_select(self, recs, st, inst_base=0, default_ballot=-1, want_prepared=True):
        recs = _c(recs, R.PREPARE_REPLY)
        st = np.array(st, dtype=R.PREP_STATE, copy=True)
        db = C.c_int32(default_ballot)
        prep = np.zeros(len(st), np.uint8) if want_prepared else None
        rc = self.lib.mpx_prepare_select(self.h, _ptr(recs), len(recs), _ptr(st), len(st),
                                         inst_base, C.byref(db), _ptr(prep))
        self._check(rc, "mpx_prepare_select")
        return st, db.value, prep

    def prepare_select_dev(self, d_recs, n, d_st_in, d_st_out, n_inst, inst_base,
                           d_default_ballot, d_prepared=None, stream=None):
        rc = self.lib.mpx_prepare_select_dev(self.h, d_recs, n, d_st_in, d_st_out, n_inst,
                                             inst_base, d_default_ballot, d_prepared, stream)
        self._check(rc, "mpx_prepare_select_dev")

    # ---- A3 ---------------------------------------------------------------------------------
    def prepare_select_min(self, recs, grp_rec_off, gst, peer_commits=None, want_effects=True):
        recs = _c(recs, R.PREPARE_REPLY_MIN)
        off = _c(grp_rec_off, np.uint64)
        gst = np.array(gst, dtype=R.GROUP_PREP_STATE, copy=True)
        g = len(gst)
        pc = np.zeros(g * self.n_replicas, np.int32) if peer_commits is None else \
            np.array(peer_commits, dtype=np.int32, copy=True).reshape(-1)
        eff = np.zeros(len(recs), R.PREPARE_EFFECT) if want_effects else None
        rc = self.lib.mpx_prepare_select_min(self.h, _ptr(recs), len(recs), _ptr(off), _ptr(gst),
                                             g, _ptr(pc), _ptr(eff))
        self._check(rc, "mpx_prepare_select_min")
        return gst, pc, eff

    def prepare_select_min_dev(self, d_recs, n, d_off, d_gst, n_groups, d_peer, d_eff=None,
                               stream=None):
        rc = self.lib.mpx_prepare_select_min_dev(self.h, d_recs, n, d_off, d_gst, n_groups,
                                                 d_peer, d_eff, stream)
        self._check(rc, "mpx_prepare_select_min_dev")

    # ---- A5 / A6 ----------------------------------------------------------------------------
    def apply_buffers(self, max_m):
        """mpx_apply_buffers: numpy views of the engine's pinned op / key / val / ret / conf
        arrays (valid until they grow or the engine closes) for mpx_apply_staged"""
        io = _lib.MpxApplyIo()
        self._check(self.lib.mpx_apply_buffers(self.h, max_m, C.byref(io)), "mpx_apply_buffers")

        def view(ptr, ct, dt):
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(io.cap,)).view(dt)
        return {"op": view(io.op, C.c_uint8, np.uint8), "key": view(io.key, C.c_int64, np.int64),
                "val": view(io.val, C.c_int64, np.int64), "ret": view(io.ret, C.c_int64, np.int64),
                "conf": view(io.conf, C.c_uint8, np.uint8), "cap": int(io.cap)}

    def apply_staged(self, m):
        """mpx_apply_staged: apply the first m commands of the apply_buffers arrays"""
        self._check(self.lib.mpx_apply_staged(self.h, m), "mpx_apply_staged")

    def apply(self, op, key, val, want_conf=True):
        op = _c(op, np.uint8)
        key = _c(key, np.int64)
        val = _c(val, np.int64)
        m = len(op)
        ret = np.zeros(m, np.int64)
        conf = np.zeros(m, np.uint8) if want_conf else None
        rc = self.lib.mpx_apply(self.h, _ptr(op), _ptr(key), _ptr(val), m, _ptr(ret), _ptr(conf))
        self._check(rc, "mpx_apply")
        return ret, conf

    def debug_kv_set_epoch(self, epoch):
        """TEST-ONLY: the KV table's call epoch, its slots untouched (mpx_debug_kv_set_epoch)"""
        self._check(self.lib.mpx_debug_kv_set_epoch(self.h, epoch), "mpx_debug_kv_set_epoch")

    def debug_kv_set_small_tag(self, tag):
        """TEST-ONLY: the tag of the last replica-batch call (mpx_debug_kv_set_small_tag)"""
        self._check(self.lib.mpx_debug_kv_set_small_tag(self.h, tag), "mpx_debug_kv_set_small_tag")

    def debug_kv_state(self):
        """TEST-ONLY: the KV table's per-slot state words (uint32, cap + 1 of them)"""
        n = C.c_size_t(0)
        self._check(self.lib.mpx_debug_kv_state(self.h, None, 0, C.byref(n)), "mpx_debug_kv_state")
        out = np.zeros(n.value, np.uint32)
        self._check(self.lib.mpx_debug_kv_state(self.h, _ptr(out), len(out), C.byref(n)),
                    "mpx_debug_kv_state")
        return out

    def apply_reserve(self, max_cmds):
        self._check(self.lib.mpx_apply_reserve(self.h, max_cmds), "mpx_apply_reserve")

    def apply_dev(self, d_op, d_key, d_val, m, d_ret, d_conf=None, stream=None):
        self._check(self.lib.mpx_apply_dev(self.h, d_op, d_key, d_val, m, d_ret, d_conf, stream),
                    "mpx_apply_dev")

    def kv_size(self):
        n = C.c_size_t(0)
        self._check(self.lib.mpx_kv_size(self.h, C.byref(n)), "mpx_kv_size")
        return n.value

    def kv_export(self):
        """Present (key, value) pairs sorted by key."""
        n = self.kv_size()
        keys = np.zeros(max(n, 1), np.int64)
        vals = np.zeros(max(n, 1), np.int64)
        got = C.c_size_t(0)
        self._check(self.lib.mpx_kv_export(self.h, _ptr(keys), _ptr(vals), n, C.byref(got)),
                    "mpx_kv_export")
        k = min(n, got.value)
        order = np.argsort(keys[:k], kind="stable")
        return keys[:k][order], vals[:k][order]

    def kv_import(self, keys, vals):
        keys = _c(keys, np.int64)
        vals = _c(vals, np.int64)
        self._check(self.lib.mpx_kv_import(self.h, _ptr(keys), _ptr(vals), len(keys)),
                    "mpx_kv_import")

    def kv_clear(self):
        self._check(self.lib.mpx_kv_clear(self.h), "mpx_kv_clear")

    def conflict_batch(self, op, key, inst_off):
        op = _c(op, np.uint8)
        key = _c(key, np.int64)
        off = _c(inst_off, np.uint64)
        n_inst = len(off) - 1
        out = np.zeros(max(n_inst - 1, 1), np.uint8)
        self._check(self.lib.mpx_conflict_batch(self.h, _ptr(op), _ptr(key), _ptr(off), n_inst,
                                                _ptr(out)), "mpx_conflict_batch")
        return out[:max(n_inst - 1, 0)]

    def conflict_batch_dev(self, d_op, d_key, d_inst_off, n_inst, d_out, stream=None):
        self._check(self.lib.mpx_conflict_batch_dev(self.h, d_op, d_key, d_inst_off, n_inst,
                                                    d_out, stream), "mpx_conflict_batch_dev")

    # ---- fused group step -------------------------------------------------------------------
    def group_step(self, b, kv_cnt=None, kv_key=None, kv_val=None, ret=None, want_conf=True,
                   want_decided=True):
        """b: dict from synth.group_batch (or the same fields). Returns a dict of outputs."""
        G, ipg, N = int(b["n_groups"]), int(b["ipg"]), self.n_replicas
        K = self.kv_per_group
        recs = _c(b["recs"], R.ACCEPT_REPLY)
        off = _c(b["grp_rec_off"], np.uint64)
        st = np.array(b["st_in"], dtype=R.INST_STATE, copy=True)
        ci = _c(b["committed_in"], np.int32)
        ei = _c(b["executed_in"], np.int32)
        pi = _c(b["peer_in"], np.int32)
        op, key, val = _c(b["op"], np.uint8), _c(b["key"], np.int64), _c(b["val"], np.int64)
        coff = _c(b["cmd_off"], np.uint32)
        has = _c(b["has_cmds"], np.uint8) if b.get("has_cmds") is not None else None
        m = len(op)
        ret = np.zeros(m, np.int64) if ret is None else np.array(ret, np.int64, copy=True)
        conf = np.zeros(m, np.uint8) if want_conf else None
        kc = np.zeros(G, np.uint32) if kv_cnt is None else np.array(kv_cnt, np.uint32, copy=True)
        kk = np.zeros(G * K, np.int64) if kv_key is None else np.array(kv_key, np.int64, copy=True)
        kv = np.zeros(G * K, np.int64) if kv_val is None else np.array(kv_val, np.int64, copy=True)
        co = np.zeros(G, np.int32)
        eo = np.zeros(G, np.int32)
        po = np.zeros(G * N, np.int32)
        dec = np.zeros(G * ipg, np.uint8) if want_decided else None
        nd = np.zeros(G, np.uint32)
        gb = _lib.MpxGroupBatch(G, ipg, *[C.cast(_ptr(x), C.c_void_p) if x is not None else None
                                          for x in (recs, off, st, st, ci, co, ei, eo, pi, po, op,
                                                    key, val, coff, has, ret, conf, kc, kk, kv,
                                                    kc, kk, kv, dec, nd)])
        self._check(self.lib.mpx_group_step(self.h, C.byref(gb)), "mpx_group_step")
        return dict(st_out=st, committed_out=co, executed_out=eo, peer_out=po, ret=ret,
                    conf_prev=conf, kv_cnt=kc, kv_key=kk, kv_val=kv, decided=dec, n_decided=nd)

    def group_step_dev(self, gb, stream=None):
        self._check(self.lib.mpx_group_step_dev(self.h, C.byref(gb), stream), "mpx_group_step_dev")

    def group_step_totals_dev(self, gb, d_totals, stream=None):
        """mpx_group_step_totals_dev: the group step with its totals from the same kernels"""
        self._check(self.lib.mpx_group_step_totals_dev(self.h, C.byref(gb), d_totals, stream),
                    "mpx_group_step_totals_dev")

    def step_totals_dev(self, gb, d_totals, stream=None):
        """d_totals[0..2] = decided instances, executed instances, executed commands"""
        self._check(self.lib.mpx_step_totals_dev(self.h, C.byref(gb), d_totals, stream),
                    "mpx_step_totals_dev")

    # ---- peer stream framing ------------------------------------------
    def decode_peer_stream(self, buf, ar_cap=None, other_cap=None):
        """Frame one peer connection's bytes. Returns (accept_replies, other_frames, result):
        AcceptReplies in arrival order (mpx_accept_reply), the other fixed-size frames as
        (offset, code), and the mpx_decode_result (consumed, counts, stop reason / code)."""
        buf = np.frombuffer(buf, np.uint8) if isinstance(buf, (bytes, bytearray)) else \
            _c(buf, np.uint8)
        n = len(buf)
        ar_cap = n // 14 + 1 if ar_cap is None else ar_cap
        other_cap = n + 1 if other_cap is None else other_cap
        ar = np.zeros(max(ar_cap, 1), R.ACCEPT_REPLY)
        oth = np.zeros(max(other_cap, 1), R.PEER_FRAME)
        res = np.zeros(1, R.DECODE_RESULT)
        self._check(self.lib.mpx_decode_peer_stream(self.h, _ptr(buf), n, _ptr(ar), ar_cap,
                                                    _ptr(oth), other_cap, _ptr(res)),
                    "mpx_decode_peer_stream")
        r = res[0]
        return (ar[:min(int(r["n_accept_replies"]), ar_cap)],
                oth[:min(int(r["n_other"]), other_cap)], r)

    def decode_stream(self, buf, caps=None):
        """Frame one peer connection's bytes with the engine's protocol (MIN / CLASSIC),
        variable-length messages included. Returns (accept_replies, prepare_replies,
        var_frames, other_frames, mpx_stream_result)."""
        buf = np.frombuffer(buf, np.uint8) if isinstance(buf, (bytes, bytearray)) else \
            _c(buf, np.uint8)
        n = len(buf)
        ca, cp, cv, co = caps or (n // 10 + 1, n // 10 + 1, n // 13 + 1, n + 1)
        ar = np.zeros(max(ca, 1), R.ACCEPT_REPLY)
        pr = np.zeros(max(cp, 1), R.PREPARE_REPLY_MIN if self.mode == R.MODE_MIN
                      else R.PREPARE_REPLY)
        var = np.zeros(max(cv, 1), R.VAR_FRAME)
        oth = np.zeros(max(co, 1), R.PEER_FRAME)
        res = np.zeros(1, R.STREAM_RESULT)
        out = _lib.MpxDecodeOut(_ptr(ar), ca, _ptr(pr), cp, _ptr(var), cv, _ptr(oth), co)
        self._check(self.lib.mpx_decode_stream(self.h, _ptr(buf), n, C.byref(out), _ptr(res)),
                    "mpx_decode_stream")
        r = res[0]
        return (ar[:min(int(r["n_accept_replies"]), ca)], pr[:min(int(r["n_prepare_replies"]), cp)],
                var[:min(int(r["n_var"]), cv)], oth[:min(int(r["n_other"]), co)], r)

    def decode_stream_reserve(self, max_len):
        self._check(self.lib.mpx_decode_stream_reserve(self.h, max_len),
                    "mpx_decode_stream_reserve")

    def decode_stream_dev(self, d_buf, n, start, out, d_res, stream=None):
        """out: _lib.MpxDecodeOut of device pointers; d_res: device mpx_stream_result (in/out)"""
        self._check(self.lib.mpx_decode_stream_dev(self.h, d_buf, n, start, C.byref(out), d_res,
                                                   stream), "mpx_decode_stream_dev")

    def decode_reserve(self, max_len):
        self._check(self.lib.mpx_decode_reserve(self.h, max_len), "mpx_decode_reserve")

    def decode_peer_stream_dev(self, d_buf, n, d_ar, ar_cap, d_other, other_cap, d_res,
                               stream=None):
        self._check(self.lib.mpx_decode_peer_stream_dev(self.h, d_buf, n, d_ar, ar_cap, d_other,
                                                        other_cap, d_res, stream),
                    "mpx_decode_peer_stream_dev")

    # ---- client reply fan-out -----------------------------------------
    def encode_replies(self, recs, n_clients, ok=1, leader=0):
        """recs: REPLY_REC in execution order. Returns (bytes uint8[25 n], client_off u64[C+1]):
        client c's connection receives out[client_off[c]:client_off[c+1]]."""
        recs = _c(recs, R.REPLY_REC)
        n = len(recs)
        out = np.zeros(max(n * R.PROPOSE_REPLY_BYTES, 1), np.uint8)
        off = np.zeros(n_clients + 1, np.uint64)
        self._check(self.lib.mpx_encode_replies(self.h, _ptr(recs), n, n_clients, ok, leader,
                                                _ptr(out), _ptr(off)), "mpx_encode_replies")
        return out[:n * R.PROPOSE_REPLY_BYTES], off

    def encode_replies_reserve(self, max_n):
        self._check(self.lib.mpx_encode_replies_reserve(self.h, max_n),
                    "mpx_encode_replies_reserve")

    def encode_replies_dev(self, d_recs, n, n_clients, ok, leader, d_out, d_off, stream=None):
        self._check(self.lib.mpx_encode_replies_dev(self.h, d_recs, n, n_clients, ok, leader,
                                                    d_out, d_off, stream),
                    "mpx_encode_replies_dev")

    # ---- instance-log encoding ------------------------------------
    def encode_log(self, fmt, recs, cmd_off, op, key, val):
        """Returns (bytes, rec_off u64[n+1]) of the run in format fmt (R.LOG_CATCHUP /
        R.LOG_DURABLE); record i is bytes[rec_off[i]:rec_off[i+1]]."""
        recs = _c(recs, R.LOG_REC)
        off = _c(cmd_off, np.uint64)
        op, key, val = _c(op, np.uint8), _c(key, np.int64), _c(val, np.int64)
        n, m = len(recs), len(op)
        cap = self.lib.mpx_encode_log_bound(n, m)
        out = np.zeros(max(cap, 1), np.uint8)
        ro = np.zeros(n + 1, np.uint64)
        self._check(self.lib.mpx_encode_log(self.h, fmt, _ptr(recs), n, _ptr(off), _ptr(op),
                                            _ptr(key), _ptr(val), m, _ptr(out), cap, _ptr(ro)),
                    "mpx_encode_log")
        return out[:int(ro[-1])], ro

    def encode_log_reserve(self, max_n, max_m):
        self._check(self.lib.mpx_encode_log_reserve(self.h, max_n, max_m),
                    "mpx_encode_log_reserve")

    def encode_log_dev(self, fmt, d_recs, n, d_cmd_off, d_op, d_key, d_val, m, d_out, d_rec_off,
                       stream=None):
        self._check(self.lib.mpx_encode_log_dev(self.h, fmt, d_recs, n, d_cmd_off, d_op, d_key,
                                                d_val, m, d_out, d_rec_off, stream),
                    "mpx_encode_log_dev")

    # ---- durable-log replay (read side) ---------------------------------
    def replay_durable(self, log, inst_cap, default_ballot=0, committed_up_to=-1, rec_base=0,
                       last_rec=None):
        """getDataFromStableStore (bareminpaxos.go:122-161) over a durable log of 29-byte
        records. Returns (recs, op, key, val, last_rec, default_ballot, committed_up_to):
        last_rec[i] is the file index of the last record naming instance i (-1: none). A store
        replayed in chunks passes each chunk's first file index as rec_base and the previous
        chunk's last_rec."""
        log = _c(log, np.uint8)
        n = len(log) // R.DURABLE_REC_BYTES
        recs = np.zeros(n, R.LOG_REC)
        op = np.zeros(n, np.uint8)
        key = np.zeros(n, np.int64)
        val = np.zeros(n, np.int64)
        last = np.full(inst_cap, -1, np.int32) if last_rec is None else \
            np.array(last_rec, np.int32, copy=True)
        sc = np.array([default_ballot, committed_up_to], np.int32)
        self._check(self.lib.mpx_replay_durable(self.h, _ptr(log), len(log), inst_cap, rec_base,
                                                _ptr(recs),
                                                _ptr(op), _ptr(key), _ptr(val), _ptr(last),
                                                _ptr(sc)),
                    "mpx_replay_durable")
        return recs, op, key, val, last, int(sc[0]), int(sc[1])

    def replay_durable_reserve(self, max_len, inst_cap):
        """scratch for the binned slot maximum of replay_durable_dev calls up to max_len bytes
        over inst_cap slots (without it the device form takes one atomic per record)"""
        self._check(self.lib.mpx_replay_durable_reserve(self.h, max_len, inst_cap),
                    "mpx_replay_durable_reserve")

    def replay_durable_dev(self, d_log, nbytes, inst_cap, d_recs, d_op, d_key, d_val, d_last,
                           d_scalars, stream=None, rec_base=0):
        self._check(self.lib.mpx_replay_durable_dev(self.h, d_log, nbytes, inst_cap, rec_base,
                                                    d_recs, d_op,
                                                    d_key, d_val, d_last, d_scalars, stream),
                    "mpx_replay_durable_dev")

    # ---- multi-GPU ----------------------------------------------------------------------------
    @staticmethod
    def comm_unique_id():
        lib = _lib.load()
        buf = (C.c_ubyte * 128)()
        rc = lib.mpx_comm_unique_id(C.cast(buf, C.c_void_p))
        if rc != 0:
            raise MpxError(rc, "mpx_comm_unique_id")
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        buf = (C.c_ubyte * 128).from_buffer_copy(uid)
        self._check(self.lib.mpx_comm_init(self.h, nranks, rank, C.cast(buf, C.c_void_p)),
                    "mpx_comm_init")

    def watermarks_allreduce(self, committed, executed):
        c = np.array(committed, np.int32, copy=True)
        e = np.array(executed, np.int32, copy=True)
        self._check(self.lib.mpx_watermarks_allreduce(self.h, _ptr(c), _ptr(e), len(c)),
                    "mpx_watermarks_allreduce")
        return c, e

    def watermarks_allreduce_dev(self, d_wm, n_groups, stream=None):
        self._check(self.lib.mpx_watermarks_allreduce_dev(self.h, d_wm, n_groups, stream),
                    "mpx_watermarks_allreduce_dev")

    def step_allreduce_dev(self, d_wm, n_groups, d_totals, n_totals, stream=None):
        """max of the watermark vector and sum of the step totals over ranks, one RCCL group"""
        self._check(self.lib.mpx_step_allreduce_dev(self.h, d_wm, n_groups, d_totals, n_totals,
                                                    stream), "mpx_step_allreduce_dev")

    def step_allreduce_oop_dev(self, d_wm_send, d_wm_recv, n_groups, d_totals, n_totals,
                               stream=None):
        """the step exchange out of place: max over ranks of d_wm_send (foreign groups -1 for
        good) into d_wm_recv, sum of d_totals in place (mpx_step_allreduce_oop_dev)"""
        self._check(self.lib.mpx_step_allreduce_oop_dev(self.h, d_wm_send, d_wm_recv, n_groups,
                                                        d_totals, n_totals, stream),
                    "mpx_step_allreduce_oop_dev")

    # ---- device memory / streams / events of the engine's HIP runtime -----------------------
    def dev_alloc(self, nbytes):
        p = C.c_void_p()
        self._check(self.lib.mpx_dev_alloc(self.h, nbytes, C.byref(p)), "mpx_dev_alloc")
        return p.value

    def dev_free(self, ptr):
        self._check(self.lib.mpx_dev_free(self.h, ptr), "mpx_dev_free")

    def memcpy(self, dst, src, nbytes, kind, stream=None):
        self._check(self.lib.mpx_memcpy_async(self.h, dst, src, nbytes, kind, stream),
                    "mpx_memcpy_async")

    def memset(self, ptr, byte_value, nbytes, stream=None):
        self._check(self.lib.mpx_memset_async(self.h, ptr, byte_value, nbytes, stream),
                    "mpx_memset_async")

    def stream_create(self):
        s = C.c_void_p()
        self._check(self.lib.mpx_stream_create(self.h, C.byref(s)), "mpx_stream_create")
        return s.value

    def stream_destroy(self, s):
        self._check(self.lib.mpx_stream_destroy(self.h, s), "mpx_stream_destroy")

    def stream_synchronize(self, s=None):
        self._check(self.lib.mpx_stream_synchronize(self.h, s), "mpx_stream_synchronize")

    def event_create(self, timing=True):
        ev = C.c_void_p()
        self._check(self.lib.mpx_event_create(self.h, 1 if timing else 0, C.byref(ev)),
                    "mpx_event_create")
        return ev.value

    def group_step_events(self, ev0=None, ev1=None):
        """record ev0 / ev1 around the fast kernel of every later group step (None: off)"""
        self._check(self.lib.mpx_group_step_events(self.h, ev0, ev1), "mpx_group_step_events")

    def event_destroy(self, ev):
        self._check(self.lib.mpx_event_destroy(self.h, ev), "mpx_event_destroy")

    def event_record(self, ev, stream=None):
        self._check(self.lib.mpx_event_record(self.h, ev, stream), "mpx_event_record")

    def stream_wait_event(self, stream, ev):
        self._check(self.lib.mpx_stream_wait_event(self.h, stream, ev), "mpx_stream_wait_event")

    def graph_begin(self, stream=None):
        """capture every call issued on `stream` (and streams joined to it) into a graph"""
        self._check(self.lib.mpx_graph_begin(self.h, stream), "mpx_graph_begin")

    def graph_end(self, stream=None):
        x = C.c_void_p()
        self._check(self.lib.mpx_graph_end(self.h, stream, C.byref(x)), "mpx_graph_end")
        return x.value

    def graph_launch(self, graph, stream=None):
        self._check(self.lib.mpx_graph_launch(self.h, graph, stream), "mpx_graph_launch")

    def graph_destroy(self, graph):
        self._check(self.lib.mpx_graph_destroy(self.h, graph), "mpx_graph_destroy")

    def event_elapsed_ms(self, ev0, ev1):
        ms = C.c_float(0.0)
        self._check(self.lib.mpx_event_elapsed_ms(self.h, ev0, ev1, C.byref(ms)),
                    "mpx_event_elapsed_ms")
        return ms.value
