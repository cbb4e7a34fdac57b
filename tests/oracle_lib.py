"""ctypes binding of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Mirrors minpaxos_amd.engine.Engine's numpy-level API so a parity test reads
    got = engine.accept_tally(...); want = oracle.accept_tally(...); assert equal
"""
import ctypes as C
import os
import subprocess

import numpy as np

from minpaxos_amd import records as R
from minpaxos_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# MPX_ORACLE_SO selects another build of the same oracle (the ASan/UBSan one, test_sanitize.py)
ORACLE_SO = os.environ.get("MPX_ORACLE_SO") or os.path.join(ORACLE_DIR, "liboracle.so")

_p = C.c_void_p
_sz = C.c_size_t
_i32 = C.c_int32


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        build()
    lib = C.CDLL(ORACLE_SO)
    sig = {
        "orc_accept_tally": (C.c_int, [C.c_int, C.c_int, _p, _sz, _p, _sz, _i32, _p, _p, _p]),
        "orc_committed_prefix": (C.c_int, [_p, _sz, _i32, _p]),
        "orc_prepare_classic": (C.c_int, [C.c_int, _p, _sz, _p, _sz, _i32, _p, _p]),
        "orc_prepare_min": (C.c_int, [C.c_int, _p, _sz, _p, _p, _sz, _p, _p]),
        "orc_kv_new": (_p, []),
        "orc_kv_free": (None, [_p]),
        "orc_kv_size": (_sz, [_p]),
        "orc_kv_export": (_sz, [_p, _p, _p, _sz]),
        "orc_kv_import": (None, [_p, _p, _p, _sz]),
        "orc_apply": (C.c_int, [_p, _p, _p, _p, _sz, _p, _p]),
        "orc_conflict_batch": (C.c_int, [_p, _p, _p, _sz, _p]),
        "orc_group_step": (C.c_int, [C.c_int, C.c_int, C.POINTER(L.MpxGroupBatch), C.c_uint32]),
        "orc_bench_accept": (C.c_int64, [C.c_int, C.c_int, _p, _sz, _p, _sz, _i32, _p, _p]),
        "orc_bench_apply": (C.c_int64, [_p, _p, _sz, _p, _p, _p, _sz, _p]),
        "orc_decode_peer_stream": (C.c_int, [_p, _sz, _p, _sz, _p, _sz, _p]),
        "orc_encode_replies": (C.c_int, [_p, _sz, C.c_uint32, C.c_uint8, _i32, _p, _p]),
        "orc_encode_log": (C.c_int, [C.c_int, _p, _sz, _p, _p, _p, _p, _p, _sz, _p]),
        "orc_decode_stream": (C.c_int, [C.c_int, _p, _sz, C.POINTER(L.MpxDecodeOut), _p]),
        "orc_replay_durable": (C.c_int, [_p, _sz, _i32, _i32, _p, _p, _p, _p, _p, _p]),
        "orc_bench_group_step": (C.c_int64, [C.c_int, C.c_int, C.POINTER(L.MpxGroupBatch),
                                             C.c_uint32, C.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OracleError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{R.ERROR_NAMES.get(code, code)}: {what}")
        self.code = code


def _check(rc, what):
    if rc != 0:
        raise OracleError(rc, what)


class Oracle:
    def __init__(self, n_replicas=5, mode=R.MODE_MIN, kv_per_group=512):
        self.lib = load()
        if isinstance(mode, str):
            mode = {"min": R.MODE_MIN, "classic": R.MODE_CLASSIC}[mode.lower()]
        self.n_replicas, self.mode, self.kv_per_group = n_replicas, mode, kv_per_group
        self.kv = self.lib.orc_kv_new()

    def __del__(self):
        try:
            if self.kv:
                self.lib.orc_kv_free(self.kv)
                self.kv = None
        except Exception:
            pass

    def accept_tally(self, recs, st, inst_base=0, committed_upto=-1, peer_commits=None,
                     want_decided=True):
        recs = np.ascontiguousarray(recs, R.ACCEPT_REPLY)
        st = np.array(st, R.INST_STATE, copy=True)
        pc = np.zeros(self.n_replicas, np.int32) if peer_commits is None else \
            np.array(peer_commits, np.int32, copy=True)
        cu = C.c_int32(committed_upto)
        dec = np.zeros(len(st), np.uint8) if want_decided else None
        _check(self.lib.orc_accept_tally(self.n_replicas, self.mode, _ptr(recs), len(recs),
                                         _ptr(st), len(st), inst_base, C.byref(cu), _ptr(pc),
                                         _ptr(dec)), "orc_accept_tally")
        return st, cu.value, pc, dec

    def committed_prefix(self, st, inst_base, committed_upto):
        st = np.ascontiguousarray(st, R.INST_STATE)
        cu = C.c_int32(committed_upto)
        _check(self.lib.orc_committed_prefix(_ptr(st), len(st), inst_base, C.byref(cu)), "prefix")
        return cu.value

    def prepare_select(self, recs, st, inst_base=0, default_ballot=-1, want_prepared=True):
        recs = np.ascontiguousarray(recs, R.PREPARE_REPLY)
        st = np.array(st, R.PREP_STATE, copy=True)
        db = C.c_int32(default_ballot)
        prep = np.zeros(len(st), np.uint8) if want_prepared else None
        _check(self.lib.orc_prepare_classic(self.n_replicas, _ptr(recs), len(recs), _ptr(st),
                                            len(st), inst_base, C.byref(db), _ptr(prep)),
               "orc_prepare_classic")
        return st, db.value, prep

    def prepare_select_min(self, recs, grp_rec_off, gst, peer_commits=None, want_effects=True):
        recs = np.ascontiguousarray(recs, R.PREPARE_REPLY_MIN)
        off = np.ascontiguousarray(grp_rec_off, np.uint64)
        gst = np.array(gst, R.GROUP_PREP_STATE, copy=True)
        pc = np.zeros(len(gst) * self.n_replicas, np.int32) if peer_commits is None else \
            np.array(peer_commits, np.int32, copy=True).reshape(-1)
        eff = np.zeros(len(recs), R.PREPARE_EFFECT) if want_effects else None
        _check(self.lib.orc_prepare_min(self.n_replicas, _ptr(recs), len(recs), _ptr(off),
                                        _ptr(gst), len(gst), _ptr(pc), _ptr(eff)),
               "orc_prepare_min")
        return gst, pc, eff

    def apply(self, op, key, val, want_conf=True):
        op = np.ascontiguousarray(op, np.uint8)
        key = np.ascontiguousarray(key, np.int64)
        val = np.ascontiguousarray(val, np.int64)
        ret = np.zeros(len(op), np.int64)
        conf = np.zeros(len(op), np.uint8) if want_conf else None
        _check(self.lib.orc_apply(self.kv, _ptr(op), _ptr(key), _ptr(val), len(op), _ptr(ret),
                                  _ptr(conf)), "orc_apply")
        return ret, conf

    def kv_export(self):
        n = self.lib.orc_kv_size(self.kv)
        k = np.zeros(max(n, 1), np.int64)
        v = np.zeros(max(n, 1), np.int64)
        self.lib.orc_kv_export(self.kv, _ptr(k), _ptr(v), n)
        return k[:n], v[:n]

    def kv_import(self, keys, vals):
        keys = np.ascontiguousarray(keys, np.int64)
        vals = np.ascontiguousarray(vals, np.int64)
        self.lib.orc_kv_import(self.kv, _ptr(keys), _ptr(vals), len(keys))

    def conflict_batch(self, op, key, inst_off):
        op = np.ascontiguousarray(op, np.uint8)
        key = np.ascontiguousarray(key, np.int64)
        off = np.ascontiguousarray(inst_off, np.uint64)
        n_inst = len(off) - 1
        out = np.zeros(max(n_inst - 1, 1), np.uint8)
        _check(self.lib.orc_conflict_batch(_ptr(op), _ptr(key), _ptr(off), n_inst, _ptr(out)),
               "orc_conflict_batch")
        return out[:max(n_inst - 1, 0)]

    def decode_peer_stream(self, buf, ar_cap=None, other_cap=None):
        buf = np.frombuffer(buf, np.uint8) if isinstance(buf, (bytes, bytearray)) else \
            np.ascontiguousarray(buf, np.uint8)
        n = len(buf)
        ar_cap = n // 14 + 1 if ar_cap is None else ar_cap
        other_cap = n + 1 if other_cap is None else other_cap
        ar = np.zeros(max(ar_cap, 1), R.ACCEPT_REPLY)
        oth = np.zeros(max(other_cap, 1), R.PEER_FRAME)
        res = np.zeros(1, R.DECODE_RESULT)
        _check(self.lib.orc_decode_peer_stream(_ptr(buf), n, _ptr(ar), ar_cap, _ptr(oth),
                                               other_cap, _ptr(res)), "orc_decode_peer_stream")
        r = res[0]
        return (ar[:min(int(r["n_accept_replies"]), ar_cap)],
                oth[:min(int(r["n_other"]), other_cap)], r)

    def encode_replies(self, recs, n_clients, ok=1, leader=0):
        recs = np.ascontiguousarray(recs, R.REPLY_REC)
        n = len(recs)
        out = np.zeros(max(n * R.PROPOSE_REPLY_BYTES, 1), np.uint8)
        off = np.zeros(n_clients + 1, np.uint64)
        _check(self.lib.orc_encode_replies(_ptr(recs), n, n_clients, ok, leader, _ptr(out),
                                           _ptr(off)), "orc_encode_replies")
        return out[:n * R.PROPOSE_REPLY_BYTES], off

    def encode_log(self, fmt, recs, cmd_off, op, key, val):
        recs = np.ascontiguousarray(recs, R.LOG_REC)
        off = np.ascontiguousarray(cmd_off, np.uint64)
        op = np.ascontiguousarray(op, np.uint8)
        key = np.ascontiguousarray(key, np.int64)
        val = np.ascontiguousarray(val, np.int64)
        n, m = len(recs), len(op)
        cap = n * 18 + 17 * m
        out = np.zeros(max(cap, 1), np.uint8)
        ro = np.zeros(n + 1, np.uint64)
        _check(self.lib.orc_encode_log(fmt, _ptr(recs), n, _ptr(off), _ptr(op), _ptr(key),
                                       _ptr(val), _ptr(out), cap, _ptr(ro)), "orc_encode_log")
        return out[:int(ro[-1])], ro

    def decode_stream(self, buf, protocol=None):
        """mpx_decode_stream restated (replicaListener + every Unmarshal): returns
        (accept_replies, prepare_replies, var_frames, other_frames, result)"""
        proto = self.mode if protocol is None else protocol
        buf = np.ascontiguousarray(np.frombuffer(buf, np.uint8) if isinstance(buf, bytes) else buf,
                                   np.uint8)
        n = len(buf)
        ar = np.zeros(n // 10 + 1, R.ACCEPT_REPLY)
        pdt = R.PREPARE_REPLY_MIN if proto == R.MODE_MIN else R.PREPARE_REPLY
        pr = np.zeros(n // 10 + 1, pdt)
        var = np.zeros(n // 13 + 1, R.VAR_FRAME)
        oth = np.zeros(n + 1, R.PEER_FRAME)
        res = np.zeros(1, R.STREAM_RESULT)
        out = L.MpxDecodeOut(_ptr(ar), len(ar), _ptr(pr), len(pr), _ptr(var), len(var),
                             _ptr(oth), len(oth))
        _check(self.lib.orc_decode_stream(proto, _ptr(buf), n, C.byref(out), _ptr(res)),
               "orc_decode_stream")
        r = res[0]
        return (ar[:int(r["n_accept_replies"])], pr[:int(r["n_prepare_replies"])],
                var[:int(r["n_var"])], oth[:int(r["n_other"])], r)

    def replay_durable(self, log, inst_cap, default_ballot=0, committed_up_to=-1, rec_base=0,
                       last_rec=None):
        """getDataFromStableStore (bareminpaxos.go:122-161): returns (recs, op, key, val,
        last_rec, default_ballot, committed_up_to); last_rec in/out (default: all -1)."""
        log = np.ascontiguousarray(log, np.uint8)
        n = len(log) // R.DURABLE_REC_BYTES
        recs = np.zeros(n, R.LOG_REC)
        op = np.zeros(n, np.uint8)
        key = np.zeros(n, np.int64)
        val = np.zeros(n, np.int64)
        last = np.full(inst_cap, -1, np.int32) if last_rec is None else \
            np.array(last_rec, np.int32, copy=True)
        sc = np.array([default_ballot, committed_up_to], np.int32)
        _check(self.lib.orc_replay_durable(_ptr(log), len(log), inst_cap, rec_base, _ptr(recs),
                                           _ptr(op),
                                           _ptr(key), _ptr(val), _ptr(last), _ptr(sc)),
               "orc_replay_durable")
        return recs, op, key, val, last, int(sc[0]), int(sc[1])

    def group_step(self, b, kv_cnt=None, kv_key=None, kv_val=None, ret=None, want_conf=True,
                   want_decided=True):
        G, ipg, N, K = int(b["n_groups"]), int(b["ipg"]), self.n_replicas, self.kv_per_group
        recs = np.ascontiguousarray(b["recs"], R.ACCEPT_REPLY)
        off = np.ascontiguousarray(b["grp_rec_off"], np.uint64)
        st = np.array(b["st_in"], R.INST_STATE, copy=True)
        ci = np.ascontiguousarray(b["committed_in"], np.int32)
        ei = np.ascontiguousarray(b["executed_in"], np.int32)
        pi = np.ascontiguousarray(b["peer_in"], np.int32)
        op = np.ascontiguousarray(b["op"], np.uint8)
        key = np.ascontiguousarray(b["key"], np.int64)
        val = np.ascontiguousarray(b["val"], np.int64)
        coff = np.ascontiguousarray(b["cmd_off"], np.uint32)
        has = np.ascontiguousarray(b["has_cmds"], np.uint8) if b.get("has_cmds") is not None else None
        m = len(op)
        ret = np.zeros(m, np.int64) if ret is None else np.array(ret, np.int64, copy=True)
        conf = np.zeros(m, np.uint8) if want_conf else None
        kci = np.zeros(G, np.uint32) if kv_cnt is None else np.array(kv_cnt, np.uint32, copy=True)
        kki = np.zeros(G * K, np.int64) if kv_key is None else np.array(kv_key, np.int64, copy=True)
        kvi = np.zeros(G * K, np.int64) if kv_val is None else np.array(kv_val, np.int64, copy=True)
        kco, kko, kvo = kci.copy(), kki.copy(), kvi.copy()
        sto = st.copy()
        co = np.zeros(G, np.int32)
        eo = np.zeros(G, np.int32)
        po = np.zeros(G * N, np.int32)
        dec = np.zeros(G * ipg, np.uint8) if want_decided else None
        nd = np.zeros(G, np.uint32)
        gb = L.MpxGroupBatch(G, ipg, *[_ptr(x) for x in (recs, off, st, sto, ci, co, ei, eo, pi,
                                                          po, op, key, val, coff, has, ret, conf,
                                                          kci, kki, kvi, kco, kko, kvo, dec, nd)])
        _check(self.lib.orc_group_step(N, self.mode, C.byref(gb), K), "orc_group_step")
        return dict(st_out=sto, committed_out=co, executed_out=eo, peer_out=po, ret=ret,
                    conf_prev=conf, kv_cnt=kco, kv_key=kko, kv_val=kvo, decided=dec, n_decided=nd)


def group_batch_struct(arrs):
    """MpxGroupBatch of numpy arrays (for the baseline timing entry point)."""
    return L.MpxGroupBatch(*arrs[:2], *[_ptr(x) for x in arrs[2:]])
