"""numpy mirrors of the packed records in include/mpx.h.

Each dtype is byte-identical to its C struct, so arrays can be handed to the C ABI
(ctypes) or viewed as int32 words for device tensors.
"""
import numpy as np

# minpaxosproto.InstanceStatus  src/minpaxosproto/minpaxosproto.go:8-15
PREPARING, PREPARED, ACCEPTED, COMMITTED = 0, 1, 2, 3
STATUS_NIL = -1  # instanceSpace[i] == nil

# state.Operation  src/state/state.go:10-19
OP_NONE, OP_PUT, OP_GET, OP_DELETE, OP_RLOCK, OP_WLOCK = 0, 1, 2, 3, 4, 5

MODE_MIN, MODE_CLASSIC = 0, 1
MAX_REPLICAS = 16

# mpx_prep_state.flags
PF_HAS_PROPOSALS, PF_REQUEUED, PF_PREPARED_NOW = 1, 2, 4
# mpx_prepare_effect.flags
EF_COUNTED, EF_SELECTED, EF_CATCHUP, EF_TRIGGER = 1, 2, 4, 8

# error codes
OK = 0
E_INVAL, E_NOMEM, E_HIP, E_RCCL, E_NIL_INSTANCE, E_BAD_ID, E_KV_FULL, E_NODEV, E_UNSUPPORTED = (
    -1, -2, -3, -4, -5, -6, -7, -8, -9)
ERROR_NAMES = {
    0: "OK", -1: "E_INVAL", -2: "E_NOMEM", -3: "E_HIP", -4: "E_RCCL", -5: "E_NIL_INSTANCE",
    -6: "E_BAD_ID", -7: "E_KV_FULL", -8: "E_NODEV", -9: "E_UNSUPPORTED",
}

# mpx_accept_reply  <- minpaxosproto.AcceptReply{Instance,OK,Ballot,Id}
ACCEPT_REPLY = np.dtype([("instance", "<i4"), ("ballot", "<i4"), ("id", "<i4"), ("ok", "u1"),
                         ("pad", "u1", (3,))])
# mpx_inst_state  <- Instance.Status + LeaderBookkeeping
INST_STATE = np.dtype([("status", "<i4"), ("accept_oks", "<i4"), ("nacks", "<i4"),
                       ("max_recv_ballot", "<i4")])
# mpx_prepare_reply  <- paxosproto.PrepareReply{Instance,OK,Ballot,Command}
PREPARE_REPLY = np.dtype([("instance", "<i4"), ("ballot", "<i4"), ("ok", "<u4"),
                          ("value_id", "<u4")])
# mpx_prep_state  <- paxos Instance{cmds,ballot,status,lb}
PREP_STATE = np.dtype([("ballot", "<i4"), ("status", "<i4"), ("prepare_oks", "<i4"),
                       ("nacks", "<i4"), ("max_recv_ballot", "<i4"), ("value_id", "<u4"),
                       ("flags", "<u4"), ("pad", "<u4")])
# mpx_prepare_reply_min  <- minpaxosproto.PrepareReply
PREPARE_REPLY_MIN = np.dtype([("id", "<i4"), ("instance", "<i4"), ("ballot", "<i4"),
                              ("last_committed", "<i4"), ("ok", "<u4"), ("value_id", "<u4")])
# mpx_group_prep_state  <- bareminpaxos PrepareBookkeeping + replica scalars
GROUP_PREP_STATE = np.dtype([("default_ballot", "<i4"), ("prepare_oks", "<i4"), ("nacks", "<i4"),
                             ("max_recv_ballot", "<i4"), ("highest_instance", "<i4"),
                             ("value_id", "<u4"), ("committed_upto", "<i4"),
                             ("triggered", "<u4")])
# mpx_prepare_effect
PREPARE_EFFECT = np.dtype([("flags", "<u4"), ("catchup_from", "<i4")])

# peer-stream frame codes (include/mpx.h MPX_PEER_*; genericsmrproto.go:7-18 and the RPC
# registration order of bareminpaxos.NewReplica, bareminpaxos.go:108-113)
PEER_BEACON, PEER_BEACON_REPLY, PEER_PREPARE, PEER_ACCEPT, PEER_COMMIT = 6, 7, 8, 9, 10
PEER_COMMIT_SHORT, PEER_PREPARE_REPLY, PEER_ACCEPT_REPLY = 11, 12, 13
# body bytes after the code byte (None = variable length; unknown codes have none)
PEER_BODY = {PEER_BEACON: 8, PEER_BEACON_REPLY: 8, PEER_PREPARE: 12, PEER_COMMIT_SHORT: 16,
             PEER_ACCEPT_REPLY: 13, PEER_ACCEPT: None, PEER_COMMIT: None, PEER_PREPARE_REPLY: None}
# CLASSIC framing (paxosproto, registration order paxos.go:93-98): Prepare 13, AcceptReply 9
PEER_BODY_CLASSIC = {**PEER_BODY, PEER_PREPARE: 13, PEER_ACCEPT_REPLY: 9}
DECODE_END, DECODE_PARTIAL, DECODE_VARIABLE, DECODE_MALFORMED, DECODE_LONG = 0, 1, 2, 3, 4
DECODE_WINDOW = 64
DECODE_MAX_BYTES = 0x7FFFFFFF
# mpx_var_frame / mpx_stream_result (mpx_decode_stream)
VAR_FRAME = np.dtype([("offset", "<u4"), ("length", "<u4"), ("n_cmds", "<u4"),
                      ("cmds_off", "<u4"), ("n_log", "<u4"), ("log_off", "<u4"), ("code", "u1"),
                      ("pad", "u1", (7,))])
STREAM_RESULT = np.dtype([("consumed", "<u8"), ("next", "<u8"), ("n_accept_replies", "<u8"),
                          ("n_prepare_replies", "<u8"), ("n_var", "<u8"), ("n_other", "<u8"),
                          ("stop_reason", "<i4"), ("stop_code", "<i4")])
# mpx_peer_frame / mpx_decode_result
PEER_FRAME = np.dtype([("offset", "<u4"), ("code", "u1"), ("pad", "u1", (3,))])
DECODE_RESULT = np.dtype([("consumed", "<u8"), ("n_accept_replies", "<u8"), ("n_other", "<u8"),
                          ("stop_reason", "<i4"), ("stop_code", "<i4")])

# mpx_reply_rec: one client reply (genericsmrproto.ProposeReplyTS fields + connection index)
REPLY_REC = np.dtype([("value", "<i8"), ("timestamp", "<i8"), ("command_id", "<i4"),
                      ("client", "<u4")])
PROPOSE_REPLY_BYTES = 25

# mpx_log_rec / log formats (instance-log encoding)
LOG_CATCHUP, LOG_DURABLE = 0, 1
# mpx_replay_durable: getDataFromStableStore reads 12 metadata bytes + one 17-byte Command
DURABLE_REC_BYTES = 29
LOG_REC = np.dtype([("ballot", "<i4"), ("status", "<i4"), ("inst_no", "<i4"), ("pad", "<u4")])

assert LOG_REC.itemsize == 16
assert REPLY_REC.itemsize == 24
assert PEER_FRAME.itemsize == 8 and DECODE_RESULT.itemsize == 32
assert VAR_FRAME.itemsize == 32 and STREAM_RESULT.itemsize == 56
assert ACCEPT_REPLY.itemsize == 16 and INST_STATE.itemsize == 16
assert PREPARE_REPLY.itemsize == 16 and PREP_STATE.itemsize == 32
assert PREPARE_REPLY_MIN.itemsize == 24 and GROUP_PREP_STATE.itemsize == 32
assert PREPARE_EFFECT.itemsize == 8

# mpx_config.apply_path / apply_hot_min (include/mpx.h)
APPLY_AUTO, APPLY_SORTED, APPLY_PARTITIONED, APPLY_SMALL = 0, 1, 2, 3
APPLY_NO_HOT = 0xFFFFFFFF
FLAG_STEP_ONE_LAUNCH = 1  # mpx_config.flags: one kernel per group step (mpx.h)
APPLY_SMALL_MAX = 16384
