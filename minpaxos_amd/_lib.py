"""ctypes binding of libmpx.so (the C ABI declared in include/mpx.h).

The library is built in-tree (`make -C minpaxos_amd`, or __graft_entry__.build()). There is no
fallback: if the shared object is missing or fails to load, every entry point raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MPX_LIB selects a diagnostic build of the same engine (e.g. libmpx_stamp.so)
LIB_PATH = os.environ.get("MPX_LIB") or os.path.join(_HERE, "libmpx.so")

_p = C.c_void_p
_i32 = C.c_int32
_sz = C.c_size_t


class MpxConfig(C.Structure):
    _fields_ = [("n_replicas", C.c_int32), ("mode", C.c_int32), ("kv_capacity", C.c_uint64),
                ("kv_per_group", C.c_uint32), ("flags", C.c_uint32), ("max_groups", C.c_uint64),
                ("apply_chunk", C.c_uint64), ("apply_path", C.c_uint32),
                ("apply_fast_min", C.c_uint32), ("apply_hot_min", C.c_uint32),
                ("reserved", C.c_uint32)]


class MpxGroupBatch(C.Structure):
    _fields_ = [("n_groups", C.c_uint32), ("ipg", C.c_uint32)] + [
        (name, _p) for name in (
            "recs", "grp_rec_off", "st_in", "st_out", "committed_in", "committed_out",
            "executed_in", "executed_out", "peer_in", "peer_out", "op", "key", "val", "cmd_off",
            "has_cmds", "ret", "conf_prev", "kv_cnt_in", "kv_key_in", "kv_val_in", "kv_cnt_out",
            "kv_key_out", "kv_val_out", "decided", "n_decided")]


class MpxDecodeOut(C.Structure):
    _fields_ = [("ar", _p), ("ar_cap", _sz), ("prep", _p), ("prep_cap", _sz), ("var", _p),
                ("var_cap", _sz), ("other", _p), ("other_cap", _sz)]


class MpxApplyIo(C.Structure):
    _fields_ = [("op", _p), ("key", _p), ("val", _p), ("ret", _p), ("conf", _p),
                ("cap", C.c_uint64)]


# name -> (restype, argtypes); every symbol of include/mpx.h
SIGNATURES = {
    "mpx_abi_version": (C.c_int, []),
    "mpx_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "mpx_open": (C.c_int, [C.c_int, C.POINTER(MpxConfig), C.POINTER(_p)]),
    "mpx_close": (C.c_int, [_p]),
    "mpx_last_error": (C.c_char_p, [_p]),
    "mpx_stream": (_p, [_p]),
    "mpx_synchronize": (C.c_int, [_p]),
    "mpx_accept_tally": (C.c_int, [_p, _p, _sz, _p, _sz, _i32, _p, _p, _p]),
    "mpx_accept_tally_dev": (C.c_int, [_p, _p, _sz, _p, _p, _sz, _i32, _p, _p, _p]),
    "mpx_prepare_select": (C.c_int, [_p, _p, _sz, _p, _sz, _i32, _p, _p]),
    "mpx_prepare_select_dev": (C.c_int, [_p, _p, _sz, _p, _p, _sz, _i32, _p, _p, _p]),
    "mpx_prepare_select_min": (C.c_int, [_p, _p, _sz, _p, _p, _sz, _p, _p]),
    "mpx_prepare_select_min_dev": (C.c_int, [_p, _p, _sz, _p, _p, _sz, _p, _p, _p]),
    "mpx_apply": (C.c_int, [_p, _p, _p, _p, _sz, _p, _p]),
    "mpx_apply_reserve": (C.c_int, [_p, _sz]),
    "mpx_apply_dev": (C.c_int, [_p, _p, _p, _p, _sz, _p, _p, _p]),
    "mpx_kv_size": (C.c_int, [_p, C.POINTER(_sz)]),
    "mpx_kv_export": (C.c_int, [_p, _p, _p, _sz, C.POINTER(_sz)]),
    "mpx_kv_import": (C.c_int, [_p, _p, _p, _sz]),
    "mpx_kv_clear": (C.c_int, [_p]),
    "mpx_conflict_batch": (C.c_int, [_p, _p, _p, _p, _sz, _p]),
    "mpx_conflict_batch_dev": (C.c_int, [_p, _p, _p, _p, _sz, _p, _p]),
    "mpx_committed_prefix": (C.c_int, [_p, _p, _sz, _i32, _p]),
    "mpx_group_step": (C.c_int, [_p, C.POINTER(MpxGroupBatch)]),
    "mpx_group_step_dev": (C.c_int, [_p, C.POINTER(MpxGroupBatch), _p]),
    "mpx_comm_unique_id": (C.c_int, [_p]),
    "mpx_comm_init": (C.c_int, [_p, C.c_int, C.c_int, _p]),
    "mpx_watermarks_allreduce": (C.c_int, [_p, _p, _p, _sz]),
    "mpx_watermarks_allreduce_dev": (C.c_int, [_p, _p, _sz, _p]),
    "mpx_decode_peer_stream": (C.c_int, [_p, _p, _sz, _p, _sz, _p, _sz, _p]),
    "mpx_decode_reserve": (C.c_int, [_p, _sz]),
    "mpx_decode_peer_stream_dev": (C.c_int, [_p, _p, _sz, _p, _sz, _p, _sz, _p, _p]),
    "mpx_decode_stream": (C.c_int, [_p, _p, _sz, C.POINTER(MpxDecodeOut), _p]),
    "mpx_decode_stream_reserve": (C.c_int, [_p, _sz]),
    "mpx_decode_stream_dev": (C.c_int, [_p, _p, _sz, _sz, C.POINTER(MpxDecodeOut), _p, _p]),
    "mpx_encode_replies": (C.c_int, [_p, _p, _sz, C.c_uint32, C.c_uint8, _i32, _p, _p]),
    "mpx_encode_replies_reserve": (C.c_int, [_p, _sz]),
    "mpx_encode_replies_dev": (C.c_int, [_p, _p, _sz, C.c_uint32, C.c_uint8, _i32, _p, _p, _p]),
    "mpx_encode_log_bound": (_sz, [_sz, _sz]),
    "mpx_encode_log": (C.c_int, [_p, C.c_int, _p, _sz, _p, _p, _p, _p, _sz, _p, _sz, _p]),
    "mpx_encode_log_reserve": (C.c_int, [_p, _sz, _sz]),
    "mpx_encode_log_dev": (C.c_int, [_p, C.c_int, _p, _sz, _p, _p, _p, _p, _sz, _p, _p, _p]),
    "mpx_replay_durable": (C.c_int, [_p, _p, _sz, _i32, _i32, _p, _p, _p, _p, _p, _p]),
    "mpx_replay_durable_dev": (C.c_int, [_p, _p, _sz, _i32, _i32, _p, _p, _p, _p, _p, _p, _p]),
    "mpx_replay_durable_reserve": (C.c_int, [_p, _sz, _i32]),
    "mpx_step_totals_dev": (C.c_int, [_p, C.POINTER(MpxGroupBatch), _p, _p]),
    "mpx_group_step_totals_dev": (C.c_int, [_p, C.POINTER(MpxGroupBatch), _p, _p]),
    "mpx_step_allreduce_dev": (C.c_int, [_p, _p, _sz, _p, _sz, _p]),
    "mpx_step_allreduce_oop_dev": (C.c_int, [_p, _p, _p, _sz, _p, _sz, _p]),
    "mpx_dev_alloc": (C.c_int, [_p, _sz, C.POINTER(_p)]),
    "mpx_dev_free": (C.c_int, [_p, _p]),
    "mpx_memcpy_async": (C.c_int, [_p, _p, _p, _sz, C.c_int, _p]),
    "mpx_memset_async": (C.c_int, [_p, _p, C.c_int, _sz, _p]),
    "mpx_stream_create": (C.c_int, [_p, C.POINTER(_p)]),
    "mpx_stream_destroy": (C.c_int, [_p, _p]),
    "mpx_stream_synchronize": (C.c_int, [_p, _p]),
    "mpx_event_create": (C.c_int, [_p, C.c_int, C.POINTER(_p)]),
    "mpx_group_step_events": (C.c_int, [_p, _p, _p]),
    "mpx_event_destroy": (C.c_int, [_p, _p]),
    "mpx_event_record": (C.c_int, [_p, _p, _p]),
    "mpx_apply_buffers": (C.c_int, [_p, _sz, C.POINTER(MpxApplyIo)]),
    "mpx_apply_staged": (C.c_int, [_p, _sz]),
    "mpx_graph_begin": (C.c_int, [_p, _p]),
    "mpx_graph_end": (C.c_int, [_p, _p, C.POINTER(C.c_void_p)]),
    "mpx_graph_launch": (C.c_int, [_p, _p, _p]),
    "mpx_graph_destroy": (C.c_int, [_p, _p]),
    "mpx_stream_wait_event": (C.c_int, [_p, _p, _p]),
    "mpx_event_elapsed_ms": (C.c_int, [_p, _p, _p, C.POINTER(C.c_float)]),
    "mpx_runtime_info": (C.c_int, [C.c_char_p, _sz]),
    "mpx_debug_kv_set_epoch": (C.c_int, [_p, C.c_uint32]),
    "mpx_debug_kv_set_small_tag": (C.c_int, [_p, C.c_uint32]),
    "mpx_debug_kv_state": (C.c_int, [_p, _p, _sz, C.POINTER(_sz)]),
}

_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def load():
    """Load libmpx.so (once). Raises NativeLibraryMissing if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} is not built; run `make -C minpaxos_amd` (hipcc, gfx950)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        # an A/B run against an older build (MPX_LIB) may lack the newer entry points
        fn = getattr(lib, name) if not os.environ.get("MPX_LIB") else getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def runtime_info():
    """The HIP / RCCL runtimes libmpx.so is bound to in this process (dict)."""
    import json
    lib = load()
    buf = C.create_string_buffer(1024)
    lib.mpx_runtime_info(buf, len(buf))
    return json.loads(buf.value.decode())
