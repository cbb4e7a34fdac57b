/*
 * mpx.h — C ABI of the MI355X batched-consensus engine (minpaxos_amd).
 *
 * The engine replaces, for batches of records, the per-message hot path of the
 * MinPaxos replica (arobertlin/MinPaxos, Go):
 *
 *   mpx_accept_tally      <- bareminpaxos.(*Replica).handleAcceptReply
 *                              src/bareminpaxos/bareminpaxos.go:1014-1064   (MPX_MODE_MIN)
 *                            paxos.(*Replica).handleAcceptReply
 *                              src/paxos/paxos.go:631-673 (+ updateCommittedUpTo :259-264)
 *                                                                          (MPX_MODE_CLASSIC)
 *   mpx_prepare_select    <- paxos.(*Replica).handlePrepareReply  src/paxos/paxos.go:577-629
 *   mpx_prepare_select_min<- bareminpaxos.(*Replica).handlePrepareReply
 *                              src/bareminpaxos/bareminpaxos.go:912-966 (+ PrepareBookkeeping :75-82)
 *   mpx_apply             <- (*state.Command).Execute  src/state/state.go:77-103, driven in log
 *                            order by executeCommands  src/bareminpaxos/bareminpaxos.go:1066-1098
 *                            (conf_prev output: state.Conflict  src/state/state.go:53-60)
 *   mpx_conflict_batch    <- state.ConflictBatch  src/state/state.go:62-71
 *   mpx_group_step        <- handleAcceptReply + executeCommands for many independent replicas
 *                            (Paxos groups) at once: one tally and one apply per group
 *   mpx_watermarks_allreduce <- (no reference equivalent; the one cross-shard step: an RCCL
 *                            all-reduce of per-group committedUpTo / executed watermarks)
 *   mpx_decode_peer_stream <- genericsmr.(*Replica).replicaListener
 *                              src/genericsmr/genericsmr.go:402-446 with the fixed-size
 *                            Unmarshal()s it dispatches to (minpaxosprotomarsh.go:259-270,
 *                            :568-580, :737-749; Beacon/BeaconReply): frames a peer byte stream
 *                            and decodes its AcceptReplies into mpx_accept_reply records
 *   mpx_encode_replies    <- the ProposeReplyTS fan-out of handleAcceptReply
 *                              src/bareminpaxos/bareminpaxos.go:1030-1042 and executeCommands
 *                            :1076-1084 through ReplyProposeTS (genericsmr.go:529-535): the byte
 *                            run each client connection receives for a batch of replies
 *   mpx_encode_log        <- minpaxosproto.(*Instance).Marshal (minpaxosprotomarsh.go:100-124) for
 *                            the CatchUpLog of bcastAccept (bareminpaxos.go:488-513), and
 *                            recordInstanceMetadata + recordCommands (bareminpaxos.go:164-188)
 *   mpx_replay_durable    <- getDataFromStableStore (bareminpaxos.go:122-161): the durable log
 *                            read back into records, watermarks and the instance slots
 *
 * Contract (every entry point):
 *   - plain C, no exceptions cross the boundary, never aborts; return 0 (MPX_OK) or a negative
 *     MPX_E_* code; mpx_last_error() explains the last failure of a handle.
 *   - records are processed with SEQUENTIAL semantics in array order: the results equal those of
 *     calling the reference handler once per record, in array order. Records must be grouped by
 *     instance (all replies for one instance contiguous) and the groups must appear in ASCENDING
 *     instance order (what the Go shim's stable sort of a drained batch produces); any other
 *     order is rejected with MPX_E_INVAL. Within a group, slot order = arrival order. MIN
 *     watermarks are "last assignment wins" in array order, which under ascending order is the
 *     highest instance that makes an assignment.
 *   - host-pointer entry points are synchronous: results are in the caller's buffers on return.
 *     *_dev entry points take device pointers and a hipStream_t (passed as void*, NULL = the
 *     engine's stream) and are asynchronous; they never allocate or synchronise, so they can be
 *     captured into a hipGraph.
 *   - a handle is not re-entrant; use one handle per replica event loop / per GPU.
 *   - the tally (mpx_accept_tally_dev), CLASSIC prepare (mpx_prepare_select_dev), apply
 *     (mpx_apply_dev), group-step and durable-log replay (mpx_replay_durable_dev) kernels keep
 *     control words or scratch in the handle between calls (tickets, maxima, the replica-batch
 *     list tags, the replay's binned-maximum scratch), each reset by the call's last workgroup:
 *     all *_dev calls on one handle must be issued in ONE stream order (one stream, or streams
 *     ordered by events) — two such calls in flight at once corrupt every later call.
 *   - a captured graph keeps the scratch pointers of the calls it captured: growing a handle's
 *     scratch afterwards (a larger mpx_apply_reserve / mpx_replay_durable_reserve, or a host-
 *     pointer mpx_apply / mpx_replay_durable call that needs more) frees the old buffers and
 *     invalidates such graphs; reserve the largest size before capturing.
 *   - where the reference would panic (nil instance, peer id outside peerCommits), the engine
 *     returns MPX_E_NIL_INSTANCE / MPX_E_BAD_ID and the outputs are unspecified.
 */
#ifndef MPX_H_
#define MPX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPX_ABI_VERSION 8  /* 4: + mpx_group_step_totals_dev; 5: + mpx_graph_*, mpx_apply_buffers / _staged;
                              6: + mpx_replay_durable_reserve; 7: + mpx_group_step_events;
                              8: + MPX_FLAG_STEP_ONE_LAUNCH */

/* ---- error codes ---------------------------------------------------------------------- */
#define MPX_OK 0
#define MPX_E_INVAL (-1)        /* bad argument / size / layout                            */
#define MPX_E_NOMEM (-2)        /* host or device allocation failed                        */
#define MPX_E_HIP (-3)          /* HIP runtime error                                       */
#define MPX_E_RCCL (-4)         /* RCCL error                                              */
#define MPX_E_NIL_INSTANCE (-5) /* record names an instance outside the window or nil:
                                   the reference dereferences a nil *Instance (panic)     */
#define MPX_E_BAD_ID (-6)       /* reply Id outside [0,N): reference indexes peerCommits   */
#define MPX_E_KV_FULL (-7)      /* KV table capacity exceeded                              */
#define MPX_E_NODEV (-8)        /* no GPU / HIP device unavailable                         */
#define MPX_E_UNSUPPORTED (-9)  /* feature not built in / input beyond supported limits    */

/* ---- enums (values mirror the reference) ---------------------------------------------- */
/* minpaxosproto.InstanceStatus  src/minpaxosproto/minpaxosproto.go:8-15
 * paxos.InstanceStatus          src/paxos/paxos.go:50-55                                   */
#define MPX_PREPARING 0
#define MPX_PREPARED 1
#define MPX_ACCEPTED 2
#define MPX_COMMITTED 3
#define MPX_STATUS_NIL (-1) /* instanceSpace[i] == nil                                      */

/* state.Operation  src/state/state.go:10-19 */
#define MPX_OP_NONE 0
#define MPX_OP_PUT 1
#define MPX_OP_GET 2
#define MPX_OP_DELETE 3
#define MPX_OP_RLOCK 4
#define MPX_OP_WLOCK 5

#define MPX_MODE_MIN 0     /* bareminpaxos semantics (the live protocol)                   */
#define MPX_MODE_CLASSIC 1 /* paxos semantics (classic per-instance Multi-Paxos)           */

#define MPX_MAX_REPLICAS 16 /* ballots are (round<<4)|replicaId: bareminpaxos.go:383-385   */

/* ---- packed records (no pointers: cgo-legal as unsafe.Pointer(&slice[0])) -------------- */

/* minpaxosproto.AcceptReply{Instance,OK,Ballot,Id}  src/minpaxosproto/minpaxosproto.go:75-80
 * (CLASSIC: paxosproto.AcceptReply{Instance,OK,Ballot} src/paxosproto/paxosproto.go:37-41;
 * id unused). ok follows the reference test `OK == TRUE` (TRUE = 1).                        */
typedef struct mpx_accept_reply {
    int32_t instance;
    int32_t ballot;
    int32_t id;
    uint8_t ok;
    uint8_t pad[3];
} mpx_accept_reply; /* 16 B */

/* Instance.Status + LeaderBookkeeping{MaxRecvBallot,AcceptOKs,Nacks}
 * src/minpaxosproto/minpaxosproto.go:17-29 ; src/paxos/paxos.go:57-70                      */
typedef struct mpx_inst_state {
    int32_t status;
    int32_t accept_oks;
    int32_t nacks;
    int32_t max_recv_ballot;
} mpx_inst_state; /* 16 B */

/* paxosproto.PrepareReply{Instance,OK,Ballot,Command}  src/paxosproto/paxosproto.go:23-28.
 * Command is an opaque handle the host resolves (an empty command is just another handle). */
typedef struct mpx_prepare_reply {
    int32_t instance;
    int32_t ballot;
    uint32_t ok;
    uint32_t value_id;
} mpx_prepare_reply; /* 16 B */

/* per-instance CLASSIC prepare state: paxos Instance{cmds,ballot,status,lb}
 * src/paxos/paxos.go:57-70 ; value_id = handle of inst.cmds                                */
#define MPX_PF_HAS_PROPOSALS 1u /* lb.clientProposals != nil                                */
#define MPX_PF_REQUEUED 2u      /* proposals were pushed back on ProposeChan in this call    */
#define MPX_PF_PREPARED_NOW 4u  /* instance became PREPARED in this call (host bcastAccept)  */
typedef struct mpx_prep_state {
    int32_t ballot; /* inst.ballot                                                          */
    int32_t status;
    int32_t prepare_oks;
    int32_t nacks;
    int32_t max_recv_ballot;
    uint32_t value_id;
    uint32_t flags;
    uint32_t pad;
} mpx_prep_state; /* 32 B */

/* minpaxosproto.PrepareReply{Id,Instance,OK,Ballot,LastCommitted,Command,CatchUpLog}
 * src/minpaxosproto/minpaxosproto.go:56-64 (Command -> value_id; CatchUpLog stays host-side) */
typedef struct mpx_prepare_reply_min {
    int32_t id;
    int32_t instance;
    int32_t ballot;
    int32_t last_committed;
    uint32_t ok;
    uint32_t value_id;
} mpx_prepare_reply_min; /* 24 B */

/* bareminpaxos PrepareBookkeeping src/bareminpaxos/bareminpaxos.go:75-82, plus the replica
 * scalars it reads/writes (defaultBallot, committedUpTo). peerCommits lives in a separate
 * [groups][N] int32 array.                                                                */
typedef struct mpx_group_prep_state {
    int32_t default_ballot;   /* r.defaultBallot (read only)                                */
    int32_t prepare_oks;
    int32_t nacks;
    int32_t max_recv_ballot;
    int32_t highest_instance; /* highestInstanceNumber                                      */
    uint32_t value_id;        /* handle of prepareBookkeeping.cmds                          */
    int32_t committed_upto;   /* r.committedUpTo                                            */
    uint32_t triggered;       /* number of times the accept trigger (:945) fired            */
} mpx_group_prep_state; /* 32 B */

/* per-record effect of mpx_prepare_select_min: what the host must do for that reply        */
#define MPX_EF_COUNTED 1u  /* ballot == defaultBallot: counted (:921-923)                   */
#define MPX_EF_SELECTED 2u /* became the max (instance, ballot): cmds = reply.Command (:925) */
#define MPX_EF_CATCHUP 4u  /* copy CatchUpLog[0 .. last_committed-catchup_from] into
                              instanceSpace[catchup_from ..] (:934-940)                     */
#define MPX_EF_TRIGGER 8u  /* install Instance{defaultBallot,ACCEPTED,cmds} at highest and
                              bcastAccept (:945-958)                                        */
typedef struct mpx_prepare_effect {
    uint32_t flags;
    int32_t catchup_from;
} mpx_prepare_effect; /* 8 B */

/* ---- engine ----------------------------------------------------------------------------- */
typedef struct mpx_config {
    int32_t n_replicas;     /* N, 1..16                                                     */
    int32_t mode;           /* MPX_MODE_MIN / MPX_MODE_CLASSIC                              */
    uint64_t kv_capacity;   /* key capacity of the engine's KV table (mpx_apply); 0 = 1<<20.
                               The table has the next power of two >= 2 x kv_capacity slots
                               (at least 1024), cut by key hash into buckets of 256 slots;
                               a key whose bucket is full fails the call with MPX_E_KV_FULL
                               (at the default load of <= 1/2 a practical impossibility
                               for non-adversarial keys)                                  */
    uint32_t kv_per_group;  /* max live keys per group table (mpx_group_step), <= 1024;
                               0 = 512. Also picks the fused step's fast-path variant (256:
                               the config-5 kernel); a group whose call touches more than
                               2048 distinct keys fails with MPX_E_KV_FULL                  */
    uint32_t flags;         /* MPX_FLAG_* (0: none)                                         */
    uint64_t max_groups;    /* groups per mpx_group_step_dev call (work list); 0 = 1<<20    */
    /* mpx_apply tuning, fixed for the handle's life (0 = default everywhere). Every setting
     * gives identical results; they move time and scratch only.                            */
    uint64_t apply_chunk;   /* commands per pipeline chunk (bounds the scratch of one call:
                               34 B / command partitioned, 48 B sorted); 0 = 1<<26          */
    uint32_t apply_path;    /* MPX_APPLY_AUTO: by call size (the replica-batch kernels up to
                               MPX_APPLY_SMALL_MAX commands, the partitioned pipeline past
                               it - the sort-based one only between MPX_APPLY_SMALL_MAX and
                               a raised apply_fast_min); calls past MPX_APPLY_SMALL_MAX
                               commands on tables past 2^30 slots are unsupported (the
                               partitioned pipeline stops there, the sort-based one's result
                               codes at 2^29 slots: the call fails); or
                               force one of MPX_APPLY_SMALL / _SORTED / _PARTITIONED (SMALL
                               and PARTITIONED where the call / table allow, else AUTO's
                               pick)                                                        */
    uint32_t apply_fast_min;  /* AUTO: calls of at least this many commands (and more than
                                 MPX_APPLY_SMALL_MAX) run partitioned; 0 = 16384            */
    uint32_t apply_hot_min;   /* partitioned: samples (of 64K) that make a key hot and keep
                                 its commands in place; 0 = 5; MPX_APPLY_NO_HOT = none      */
    uint32_t reserved;        /* 0                                                          */
} mpx_config; /* 56 B */

/* mpx_config.flags */
#define MPX_FLAG_STEP_ONE_LAUNCH 1u /* every mpx_group_step[_totals]_dev is ONE kernel: the
                               per-group fast kernel, which also reduces the step totals (its
                               last workgroup), with no work-list kernel behind it. The shape
                               must fit a fast variant (R = max(N-1,1) x ipg replies: ipg <= 256
                               with R <= 1024 and kv_per_group <= 1024, or R <= 2048 and
                               kv_per_group <= 256; ipg <= 512 with R <= 2048 and kv_per_group
                               <= 512; else the call returns MPX_E_INVAL) and so must every
                               group: at most R replies, 1024 commands (2048 at ipg > 256), distinct keys
                               within the variant's LDS table - a group past them fails the step
                               (MPX_E_INVAL at the next synchronising call, its outputs not
                               written). For callers that bound their batches; the default
                               two-launch step takes any group.                              */
#define MPX_FLAG_KNOWN 1u

#define MPX_APPLY_AUTO 0
#define MPX_APPLY_SORTED 1
#define MPX_APPLY_PARTITIONED 2
#define MPX_APPLY_SMALL 3
#define MPX_APPLY_NO_HOT 0xFFFFFFFFu
#define MPX_APPLY_SMALL_MAX 16384

typedef struct mpx_engine mpx_engine;

int mpx_abi_version(void);
int mpx_device_count(int* count);
int mpx_open(int device, const mpx_config* cfg, mpx_engine** out);
int mpx_close(mpx_engine* eng);
const char* mpx_last_error(mpx_engine* eng);
/* the engine's HIP stream (hipStream_t), for callers that queue their own work on it      */
void* mpx_stream(mpx_engine* eng);
int mpx_synchronize(mpx_engine* eng);

/* ---- A1/A2: accept tally (host pointers, synchronous) ----------------------------------
 * st[i] is the state of instance inst_base+i, updated in place. committed_upto and
 * peer_commits[N] are in/out (r.committedUpTo, r.prepareBookkeeping.peerCommits).
 * decided_out (optional, n_inst bytes) = 1 for instances decided in this call, else 0.   */
int mpx_accept_tally(mpx_engine* eng, const mpx_accept_reply* recs, size_t n,
                     mpx_inst_state* st, size_t n_inst, int32_t inst_base,
                     int32_t* committed_upto, int32_t* peer_commits, uint8_t* decided_out);

/* device-pointer variant. st_in/st_out may alias; st_out[i] is written for every instance
 * that has at least one record (other entries untouched). d_scalars: int32 in/out
 * [0] = committedUpTo, [1..N] = peerCommits. d_decided (optional): as decided_out.        */
int mpx_accept_tally_dev(mpx_engine* eng, const mpx_accept_reply* d_recs, size_t n,
                         const mpx_inst_state* d_st_in, mpx_inst_state* d_st_out,
                         size_t n_inst, int32_t inst_base, int32_t* d_scalars,
                         uint8_t* d_decided, void* stream);

/* ---- A4: CLASSIC prepare selection (max-ballot value selection) ------------------------
 * default_ballot in/out (r.defaultBallot raised to inst.ballot of newly prepared instances)
 * prepared_out (optional): 1 where the instance became PREPARED in this call.              */
int mpx_prepare_select(mpx_engine* eng, const mpx_prepare_reply* recs, size_t n,
                       mpx_prep_state* st, size_t n_inst, int32_t inst_base,
                       int32_t* default_ballot, uint8_t* prepared_out);
int mpx_prepare_select_dev(mpx_engine* eng, const mpx_prepare_reply* d_recs, size_t n,
                           const mpx_prep_state* d_st_in, mpx_prep_state* d_st_out,
                           size_t n_inst, int32_t inst_base, int32_t* d_default_ballot,
                           uint8_t* d_prepared, void* stream);

/* ---- A3: MIN prepare selection, one PrepareBookkeeping per group ------------------------
 * replies of group g are recs[grp_rec_off[g] .. grp_rec_off[g+1]) in arrival order.
 * peer_commits: [n_groups][N] in/out. eff (optional): one effect per record.              */
int mpx_prepare_select_min(mpx_engine* eng, const mpx_prepare_reply_min* recs, size_t n,
                           const uint64_t* grp_rec_off, mpx_group_prep_state* gst,
                           size_t n_groups, int32_t* peer_commits, mpx_prepare_effect* eff);
int mpx_prepare_select_min_dev(mpx_engine* eng, const mpx_prepare_reply_min* d_recs,
                               size_t n, const uint64_t* d_grp_rec_off,
                               mpx_group_prep_state* d_gst, size_t n_groups,
                               int32_t* d_peer_commits, mpx_prepare_effect* d_eff,
                               void* stream);

/* ---- A5/A6: batched KV apply on the engine's State ---------------------------------------
 * Executes the m commands in array (log) order against the engine's persistent table:
 * ret[i] = Execute's return value; conf_prev[i] (optional) = state.Conflict(previous command
 * on the same key in this call, command i), 0 if there is none. Only keys PUT at some point
 * occupy the table: GETs (and other ops) of absent keys return NIL and leave it unchanged.   */
int mpx_apply(mpx_engine* eng, const uint8_t* op, const int64_t* key, const int64_t* val,
              size_t m, int64_t* ret, uint8_t* conf_prev);
/* allocate the KV table and the apply workspace for calls of up to max_cmds commands, so
 * that mpx_apply_dev (which never allocates) can run; idempotent, grows only               */
int mpx_apply_reserve(mpx_engine* eng, size_t max_cmds);
int mpx_apply_dev(mpx_engine* eng, const uint8_t* d_op, const int64_t* d_key,
                  const int64_t* d_val, size_t m, int64_t* d_ret, uint8_t* d_conf_prev,
                  void* stream);
/* ---- replica-batch apply without copies (the cgo shim's form, ABI 5) -------------------
 * mpx_apply_buffers: the engine's pinned, GPU-mapped command and result arrays for calls of up
 * to max_m (<= MPX_APPLY_SMALL_MAX) commands; the caller writes a drained executeCommands batch
 * straight into io->op / key / val and calls mpx_apply_staged(eng, m): the results of
 * mpx_apply(eng, io->op, io->key, io->val, m, io->ret, io->conf) land in io->ret / io->conf,
 * read and written by the kernels across the link, with no copy on either side. The arrays stay
 * valid until the next mpx_apply_buffers that grows them or mpx_close; needs apply_path AUTO or
 * SMALL. Synchronous, like mpx_apply.                                                       */
typedef struct mpx_apply_io {
    uint8_t* op;
    int64_t* key;
    int64_t* val;
    int64_t* ret;
    uint8_t* conf;
    uint64_t cap;  /* commands the arrays hold                                               */
} mpx_apply_io;
int mpx_apply_buffers(mpx_engine* eng, size_t max_m, mpx_apply_io* io);
int mpx_apply_staged(mpx_engine* eng, size_t m);
/* table access: number of present keys; export (any order) / import / clear               */
int mpx_kv_size(mpx_engine* eng, size_t* n);
int mpx_kv_export(mpx_engine* eng, int64_t* keys, int64_t* vals, size_t cap, size_t* n);
int mpx_kv_import(mpx_engine* eng, const int64_t* keys, const int64_t* vals, size_t n);
int mpx_kv_clear(mpx_engine* eng);

/* state.ConflictBatch over consecutive instances: out[i] = ConflictBatch(inst i, inst i+1),
 * instance i = commands [inst_off[i], inst_off[i+1]). out has n_inst-1 entries.            */
int mpx_conflict_batch(mpx_engine* eng, const uint8_t* op, const int64_t* key,
                       const uint64_t* inst_off, size_t n_inst, uint8_t* out);
/* device form; d_inst_off is trusted (n_inst+1 non-decreasing offsets starting at 0)       */
int mpx_conflict_batch_dev(mpx_engine* eng, const uint8_t* d_op, const int64_t* d_key,
                           const uint64_t* d_inst_off, size_t n_inst, uint8_t* d_out,
                           void* stream);

/* ---- A7: CLASSIC commit watermark (updateCommittedUpTo over a status window) ------------ */
int mpx_committed_prefix(mpx_engine* eng, const mpx_inst_state* st, size_t n_inst,
                         int32_t inst_base, int32_t* committed_upto);

/* ---- fused per-group step (sharded engine, config 5) -------------------------------------
 * G independent groups (replicas), each with ipg instance slots (instances 0..ipg-1 in its
 * own instance space). Group g's accept replies: recs[grp_rec_off[g]..grp_rec_off[g+1]),
 * grouped by instance, instance numbers group-local. Instance (g,i) owns commands
 * [cmd_off[g*ipg+i], cmd_off[g*ipg+i+1]); has_cmds (optional) = 0 marks Cmds == nil.
 * Per group: tally (cfg mode), then executeCommands from executed[g]+1 while
 * i <= committed[g] and Cmds != nil, against the group's KV table.
 * KV tables: kv_cnt[g] live entries in kv_key/kv_val[g*kv_per_group ..].                    */
typedef struct mpx_group_batch {
    uint32_t n_groups;
    uint32_t ipg;
    const mpx_accept_reply* recs;
    const uint64_t* grp_rec_off;   /* n_groups+1                                            */
    const mpx_inst_state* st_in;   /* n_groups*ipg                                          */
    mpx_inst_state* st_out;        /* may alias st_in                                       */
    const int32_t* committed_in;   /* n_groups                                              */
    int32_t* committed_out;
    const int32_t* executed_in;    /* n_groups (last executed instance, -1 = none)          */
    int32_t* executed_out;
    const int32_t* peer_in;        /* n_groups*N                                            */
    int32_t* peer_out;
    const uint8_t* op;             /* commands, global arrays                               */
    const int64_t* key;
    const int64_t* val;
    const uint32_t* cmd_off;       /* n_groups*ipg+1                                        */
    const uint8_t* has_cmds;       /* optional, n_groups*ipg                                */
    int64_t* ret;                  /* written for executed commands                         */
    uint8_t* conf_prev;            /* optional                                              */
    const uint32_t* kv_cnt_in;     /* n_groups                                              */
    const int64_t* kv_key_in;      /* n_groups*kv_per_group                                 */
    const int64_t* kv_val_in;
    uint32_t* kv_cnt_out;          /* may alias the inputs                                  */
    int64_t* kv_key_out;
    int64_t* kv_val_out;
    uint8_t* decided;              /* optional, n_groups*ipg                                */
    uint32_t* n_decided;           /* optional, n_groups: instances decided in this call
                                      (status became COMMITTED at a quorum crossing)        */
} mpx_group_batch;

/* host pointers (synchronous) / device pointers (asynchronous on stream). One handle runs
 * its group steps (and step totals) one at a time in stream order: they share the handle's
 * work-list and accumulator words.                                                         */
int mpx_group_step(mpx_engine* eng, const mpx_group_batch* b);
int mpx_group_step_dev(mpx_engine* eng, const mpx_group_batch* b, void* stream);

/* per-step totals of a group batch after mpx_group_step_dev (device pointers; b->n_decided
 * required): d_totals[0] = instances decided, d_totals[1] = instances executed
 * (executeCommands iterations), d_totals[2] = commands executed (Execute calls). Written, not
 * accumulated; reduce them over ranks with mpx_step_allreduce_dev.                         */
#define MPX_STEP_TOTALS 3
int mpx_step_totals_dev(mpx_engine* eng, const mpx_group_batch* b, int64_t* d_totals,
                        void* stream);
/* mpx_group_step_dev and mpx_step_totals_dev in one (b->n_decided required): the second
 * kernel of the step (the work-list kernel) also reduces the groups' outputs to d_totals[0..2]
 * (same values), so a step is two kernel launches instead of three.                       */
int mpx_group_step_totals_dev(mpx_engine* eng, const mpx_group_batch* b, int64_t* d_totals,
                              void* stream);
/* timing hook (ABI 7): every later group step of the handle records ev_fast_start right before
 * and ev_fast_end right after the launch of its first kernel (the per-group fast kernel, or the
 * work-list fill), on the call's stream, so the pair brackets that kernel alone (the work-list
 * kernel that follows is outside). Both NULL turns it off. Events from mpx_event_create;
 * they must stay alive while registered - mpx_event_destroy of either one unregisters the
 * pair (the hook is then off, as after NULL, NULL).                                           */
int mpx_group_step_events(mpx_engine* eng, void* ev_fast_start, void* ev_fast_end);

/* ---- multi-GPU: the one collective (RCCL over xGMI) -------------------------------------
 * Each rank owns a block of groups; non-owned entries must hold -1. After the call every
 * rank holds max over ranks (= the owner's value) for every group. 128-byte unique id is
 * produced by rank 0 and broadcast by the caller (e.g. through torch.distributed).         */
int mpx_comm_unique_id(void* out128);
int mpx_comm_init(mpx_engine* eng, int nranks, int rank, const void* unique_id128);
int mpx_watermarks_allreduce(mpx_engine* eng, int32_t* committed, int32_t* executed,
                             size_t n_groups);
/* device pointers: committed/executed are one contiguous int32 buffer of 2*n_groups       */
int mpx_watermarks_allreduce_dev(mpx_engine* eng, int32_t* d_watermarks, size_t n_groups,
                                 void* stream);
/* the whole per-step exchange as one RCCL group: max over ranks of the 2*n_groups watermark
 * vector and sum over ranks of n_totals int64 counters (e.g. the mpx_step_totals_dev ones)  */
int mpx_step_allreduce_dev(mpx_engine* eng, int32_t* d_watermarks, size_t n_groups,
                           int64_t* d_totals, size_t n_totals, void* stream);
/* the same exchange out of place: d_wm_send keeps -1 on the groups other ranks own for good
 * (set once; the group step writes only the rank's own range), so a step needs no refill of
 * the foreign ranges; the max over ranks lands in d_wm_recv (2*n_groups). d_totals is reduced
 * in place.                                                                                 */
int mpx_step_allreduce_oop_dev(mpx_engine* eng, const int32_t* d_wm_send, int32_t* d_wm_recv,
                               size_t n_groups, int64_t* d_totals, size_t n_totals, void* stream);

/* ---- peer stream framing + AcceptReply decode ----------------------
 * A peer connection carries frames [code u8][body]. Codes (genericsmrproto.go:7-18 and the
 * registration order of bareminpaxos.NewReplica, bareminpaxos.go:108-113):                 */
#define MPX_PEER_BEACON 6        /* 8-byte timestamp                                         */
#define MPX_PEER_BEACON_REPLY 7  /* 8-byte timestamp                                         */
#define MPX_PEER_PREPARE 8       /* 12-byte body                                             */
#define MPX_PEER_ACCEPT 9        /* variable length (Command + CatchUpLog slices)            */
#define MPX_PEER_COMMIT 10       /* variable length (Command slice)                          */
#define MPX_PEER_COMMIT_SHORT 11 /* 16-byte body                                             */
#define MPX_PEER_PREPARE_REPLY 12/* variable length                                          */
#define MPX_PEER_ACCEPT_REPLY 13 /* 13-byte body {Instance i32, OK u8, Ballot i32, Id i32}   */
/* every other code is a 1-byte frame (replicaListener logs "unknown message type" and reads
 * the next byte as a new code, genericsmr.go:440-442)                                       */

/* a fixed-size frame other than AcceptReply: where it starts (its code byte) and its code  */
typedef struct mpx_peer_frame {
    uint32_t offset;
    uint8_t code;
    uint8_t pad[3];
} mpx_peer_frame; /* 8 B */

#define MPX_DECODE_END 0      /* the buffer ends exactly at a frame boundary                 */
#define MPX_DECODE_PARTIAL 1  /* stopped at a frame whose body runs past the buffer: keep the
                                 tail [consumed, len) and call again when more bytes arrive   */
#define MPX_DECODE_VARIABLE 2 /* stopped at a variable-length frame (Accept / Commit /
                                 PrepareReply) at `consumed`: the host unmarshals it and
                                 calls again after it                                        */
#define MPX_DECODE_MAX_BYTES 0x7FFFFFFFu /* per call                                        */

typedef struct mpx_decode_result {
    uint64_t consumed;         /* bytes framed (start of the stop frame, or len)            */
    uint64_t n_accept_replies; /* AcceptReply frames in [0, consumed)                       */
    uint64_t n_other;          /* other fixed-size frames in [0, consumed)                  */
    int32_t stop_reason;       /* MPX_DECODE_*                                              */
    int32_t stop_code;         /* code byte at `consumed`, -1 at MPX_DECODE_END             */
} mpx_decode_result; /* 32 B */

/* Frames buf[0..len) in stream order. AcceptReplies go to ar[0..min(n, ar_cap)) in arrival
 * order, other fixed-size frames to other[0..min(n, other_cap)); the counts in *res are
 * always complete, so a caller whose capacity was short sees n > cap and can call again.
 * AcceptReply is framed as the 13 bytes its Marshal writes (minpaxosprotomarsh.go:545-566);
 * the reference's io.ReadAtLeast(wire, bs, 9) (:571) can return a short body on a partial
 * TCP read and desynchronise the stream, which the engine does not reproduce.              */
int mpx_decode_peer_stream(mpx_engine* eng, const uint8_t* buf, size_t len,
                           mpx_accept_reply* ar, size_t ar_cap, mpx_peer_frame* other,
                           size_t other_cap, mpx_decode_result* res);
/* scratch for mpx_decode_peer_stream_dev on buffers of up to max_len bytes (grows only)    */
int mpx_decode_reserve(mpx_engine* eng, size_t max_len);
int mpx_decode_peer_stream_dev(mpx_engine* eng, const uint8_t* d_buf, size_t len,
                               mpx_accept_reply* d_ar, size_t ar_cap, mpx_peer_frame* d_other,
                               size_t other_cap, mpx_decode_result* d_res, void* stream);

/* ---- full peer-stream decode: fixed AND variable-length frames, MIN or CLASSIC wire ------
 * mpx_decode_stream frames one connection's bytes with the framing of the engine's protocol
 * (mpx_config.mode): bareminpaxos registers minpaxosproto messages (bareminpaxos.go:108-113),
 * paxos registers paxosproto messages (paxos.go:93-98), both as codes 8..13 in the order
 * Prepare, Accept, Commit, CommitShort, PrepareReply, AcceptReply. Body lengths:
 *                   MIN (minpaxosprotomarsh.go)            CLASSIC (paxosprotomarsh.go)
 *   6/7 Beacon      8                                        8
 *   8  Prepare      12 (:259-270)                            13 (:76-87)
 *   9  Accept       16 + V(n) + 17n + V(m) + m Instances     12 + V(n) + 17n (:244-270)
 *                   (:470-507)
 *   10 Commit       12 + V(n) + 17n (:648-672)               12 + V(n) + 17n (:403-430)
 *   11 CommitShort  16 (:737-749)                            16 (:492-503)
 *   12 PrepareReply 17 + V(n) + 17n + V(m) + m Instances     9 + V(n) + 17n (:152-176)
 *                   (:352-387)
 *   13 AcceptReply  13 (:568-580)                            9 (:324-338)
 * V(x) is a Go binary.PutVarint (zig-zag, 1..10 bytes); an Instance is 8 + V(k) + 17k bytes
 * (:126-153); 17 bytes is one state.Command (statemarsh.go:21-37). Every other code is a 1-byte
 * frame (genericsmr.go:440-442).
 * Outputs, each in stream order:
 *   AcceptReply  -> mpx_accept_reply (CLASSIC: id = -1, the wire carries no Id)
 *   PrepareReply -> mpx_prepare_reply_min (MIN) / mpx_prepare_reply (CLASSIC) with value_id =
 *                   the index of the frame's mpx_var_frame (its Command slice), AND an
 *                   mpx_var_frame
 *   Accept / Commit -> mpx_var_frame (the host unmarshals them from the byte ranges)
 *   other fixed-size frames -> mpx_peer_frame                                               */
typedef struct mpx_var_frame {
    uint32_t offset;      /* the frame's code byte                                          */
    uint32_t length;      /* code byte included                                            */
    uint32_t n_cmds;      /* len(Command)                                                   */
    uint32_t cmds_off;    /* first 17-byte Command                                          */
    uint32_t n_log;       /* len(CatchUpLog) (MIN Accept / PrepareReply), else 0              */
    uint32_t log_off;     /* first Instance of the CatchUpLog (end of Command if n_log == 0)  */
    uint8_t code;
    uint8_t pad[7];
} mpx_var_frame; /* 32 B */

typedef struct mpx_decode_out {
    mpx_accept_reply* ar;     size_t ar_cap;
    void* prep;               size_t prep_cap; /* mpx_prepare_reply_min[] (MIN) or
                                                  mpx_prepare_reply[] (CLASSIC)              */
    mpx_var_frame* var;       size_t var_cap;
    mpx_peer_frame* other;    size_t other_cap;
} mpx_decode_out;

#define MPX_DECODE_MALFORMED 3 /* a varint overflows 64 bits (Unmarshal returns an error and
                                  replicaListener stops, genericsmr.go:433-437) or a slice
                                  length is negative (make panics)                          */
#define MPX_DECODE_LONG 4      /* _dev only: the frame at `consumed` ends more than
                                  MPX_DECODE_WINDOW bytes past the 128-byte chunk it starts
                                  in; it IS decoded (counted, records written) and the chain
                                  resumes at `next`: call again with start = next            */
#define MPX_DECODE_WINDOW 64

typedef struct mpx_stream_result {
    uint64_t consumed;          /* stop position (len at MPX_DECODE_END)                     */
    uint64_t next;              /* MPX_DECODE_LONG: where the next frame starts              */
    uint64_t n_accept_replies;  /* totals over the stream so far (in/out for the _dev form)  */
    uint64_t n_prepare_replies;
    uint64_t n_var;
    uint64_t n_other;
    int32_t stop_reason;        /* MPX_DECODE_END / PARTIAL / MALFORMED (/ LONG, _dev)       */
    int32_t stop_code;          /* code byte at `consumed`, -1 at MPX_DECODE_END             */
} mpx_stream_result; /* 56 B */

/* host pointers, synchronous: the whole buffer (long frames included); res out            */
int mpx_decode_stream(mpx_engine* eng, const uint8_t* buf, size_t len,
                      const mpx_decode_out* out, mpx_stream_result* res);
/* scratch for _dev calls on buffers of up to max_len bytes (grows only)                    */
int mpx_decode_stream_reserve(mpx_engine* eng, size_t max_len);
/* device form: frames d_buf[start, len) (start = 0, or a previous call's res.next) and
 * appends records at the indices the counts in *d_res (in/out: zero it for a new stream)
 * give; one call stops at the first frame that is a terminal (END / PARTIAL / MALFORMED) or
 * LONG. `out` is a host struct of device pointers.                                         */
int mpx_decode_stream_dev(mpx_engine* eng, const uint8_t* d_buf, size_t len, size_t start,
                          const mpx_decode_out* out, mpx_stream_result* d_res, void* stream);

/* ---- client reply fan-out -----------------------------------------
 * One reply per executed (or decided) command, in execution order: the proposing client's
 * connection index, and the ProposeReplyTS fields the leader fills from
 * inst.Lb.ClientProposals[j] (CommandId, Timestamp) and Execute's return (Value; state.NIL = 0
 * for replies sent at decide time). genericsmrproto.ProposeReplyTS  genericsmrproto.go:31-37 */
typedef struct mpx_reply_rec {
    int64_t value;
    int64_t timestamp;
    int32_t command_id;
    uint32_t client; /* 0 .. n_clients-1                                                     */
} mpx_reply_rec; /* 24 B */

#define MPX_PROPOSE_REPLY_BYTES 25 /* gsmrprotomarsh.go:702-732: OK, CommandId, Value,
                                      Timestamp, Leader (little endian)                      */

/* out (25*n bytes) receives, client by client, each client's replies in execution order,
 * encoded exactly as ProposeReplyTS.Marshal writes them with OK = ok and Leader = leader;
 * client c's run is out[client_off[c] .. client_off[c+1]) (client_off: n_clients+1 entries).
 * A record whose client >= n_clients makes the call fail with MPX_E_INVAL.                  */
int mpx_encode_replies(mpx_engine* eng, const mpx_reply_rec* recs, size_t n, uint32_t n_clients,
                       uint8_t ok, int32_t leader, uint8_t* out, uint64_t* client_off);
int mpx_encode_replies_reserve(mpx_engine* eng, size_t max_n);
int mpx_encode_replies_dev(mpx_engine* eng, const mpx_reply_rec* d_recs, size_t n,
                           uint32_t n_clients, uint8_t ok, int32_t leader, uint8_t* d_out,
                           uint64_t* d_client_off, void* stream);

/* ---- instance-log encoding ----------------------------------
 * A run of log records (instance metadata + commands [cmd_off[i], cmd_off[i+1]) of the SoA
 * command arrays op/key/val, the layout mpx_apply takes) encoded back to back in one of the
 * reference's two byte formats; rec_off[i] is where record i starts, rec_off[n] the total.
 *   MPX_LOG_CATCHUP  Instance.Marshal: Ballot i32, Status i32, PutVarint(len(Cmds)), Cmds (17 B
 *                    each: Op, K, V). bcastAccept sends peer q the records peerCommits[q]+1 ..
 *                    lastCommitted: the suffix out[rec_off[from] .. rec_off[n]).
 *   MPX_LOG_DURABLE  recordInstanceMetadata (Ballot u32, Status u32, instNo u32) +
 *                    recordCommands (17 B per command; an empty or nil slice writes nothing). */
#define MPX_LOG_CATCHUP 0
#define MPX_LOG_DURABLE 1
typedef struct mpx_log_rec {
    int32_t ballot;
    int32_t status;
    int32_t inst_no; /* instNo (MPX_LOG_DURABLE; unused by MPX_LOG_CATCHUP)                  */
    uint32_t pad;
} mpx_log_rec; /* 16 B */

/* bytes out must hold for n records with m commands in total                              */
size_t mpx_encode_log_bound(size_t n, size_t m);
/* cmd_off: n+1 non-decreasing offsets with cmd_off[n] <= m. The output is never larger than
 * mpx_encode_log_bound(n, m); if rec_off[n] > out_cap the call fails with MPX_E_INVAL and only
 * rec_off is written.                                                                      */
int mpx_encode_log(mpx_engine* eng, int format, const mpx_log_rec* recs, size_t n,
                   const uint64_t* cmd_off, const uint8_t* op, const int64_t* key,
                   const int64_t* val, size_t m, uint8_t* out, size_t out_cap,
                   uint64_t* rec_off);
int mpx_encode_log_reserve(mpx_engine* eng, size_t max_n, size_t max_m);
/* d_out must hold mpx_encode_log_bound(n, m) bytes; cmd_off is trusted (not validated)     */
int mpx_encode_log_dev(mpx_engine* eng, int format, const mpx_log_rec* d_recs, size_t n,
                       const uint64_t* d_cmd_off, const uint8_t* d_op, const int64_t* d_key,
                       const int64_t* d_val, size_t m, uint8_t* d_out, uint64_t* d_rec_off,
                       void* stream);

/* ---- durable-log replay (read side) ----------------------------------
 * bareminpaxos.(*Replica).getDataFromStableStore  src/bareminpaxos/bareminpaxos.go:122-161:
 * the stable store as back-to-back MPX_DURABLE_REC_BYTES records (metadata Ballot, Status,
 * instNo as LE u32, then exactly ONE state.Command: Op u8, K i64, V i64). Per record, as the
 * sequential loop leaves it:
 *   recs[i] / op[i] / key[i] / val[i]  the decoded record (recs[i].pad = 0)
 *   scalars[0] (in/out) defaultBallot  = max(defaultBallot, every ballot)          (:145-147)
 *   scalars[1] (in/out) committedUpTo  = max(committedUpTo, instNo of COMMITTED)    (:149-151)
 *   last_rec[instNo]  = index of the LAST record naming instNo (-1: none)            (:153-157)
 * len must be a whole number of records (a trailing partial record, which the reference decodes
 * as a zero-padded garbage instance, is rejected with MPX_E_INVAL) and len / 29 < 2^31.
 * instNo outside [0, inst_cap) is where the reference's instanceSpace index panics:
 * MPX_E_NIL_INSTANCE, outputs unspecified.                                                   */
#define MPX_DURABLE_REC_BYTES 29
/* rec_base: the file index of this call's first record (0 for a whole file; the running record
 * count when a long store is replayed in chunks): last_rec holds rec_base + i, so a later
 * chunk's records win over an earlier chunk's. rec_base + len / 29 must stay below 2^31.
 * last_rec[inst_cap] is in/out: the caller initialises it to -1 before the first chunk.      */
int mpx_replay_durable(mpx_engine* eng, const uint8_t* log, size_t len, int32_t inst_cap,
                       int32_t rec_base, mpx_log_rec* recs, uint8_t* op, int64_t* key,
                       int64_t* val, int32_t* last_rec, int32_t* scalars);
/* device form: d_log 16-byte aligned; d_last_rec[inst_cap] and d_scalars[2] in/out.
 * The slot maxima are binned in LDS (no device atomic per record) when the engine holds the
 * scratch for the call: mpx_replay_durable_reserve(max_len, inst_cap) once beforehand (the dev
 * entry never allocates; instance spaces up to 2^25 slots); without it the call takes one
 * device-scope atomicMax per record. Same results either way.                              */
int mpx_replay_durable_reserve(mpx_engine* eng, size_t max_len, int32_t inst_cap);
int mpx_replay_durable_dev(mpx_engine* eng, const uint8_t* d_log, size_t len, int32_t inst_cap,
                           int32_t rec_base, mpx_log_rec* d_recs, uint8_t* d_op,
                           int64_t* d_key, int64_t* d_val, int32_t* d_last_rec,
                           int32_t* d_scalars, void* stream);

/* ---- device memory, streams and events of the engine's HIP runtime -----------------------
 * For hosts with no HIP binding of their own (a cgo shim, the Python bench and tests): every
 * buffer the *_dev entry points take can come from here, so caller and engine share one HIP
 * runtime and one device. Asynchronous calls take a stream (NULL = the engine's).           */
#define MPX_COPY_H2D 1
#define MPX_COPY_D2H 2
#define MPX_COPY_D2D 3
int mpx_dev_alloc(mpx_engine* eng, size_t bytes, void** d_out);
int mpx_dev_free(mpx_engine* eng, void* d);
int mpx_memcpy_async(mpx_engine* eng, void* dst, const void* src, size_t bytes, int kind,
                     void* stream);
int mpx_memset_async(mpx_engine* eng, void* d, int byte_value, size_t bytes, void* stream);
int mpx_stream_create(mpx_engine* eng, void** stream_out);
int mpx_stream_destroy(mpx_engine* eng, void* stream);
int mpx_stream_synchronize(mpx_engine* eng, void* stream);
int mpx_event_create(mpx_engine* eng, int timing, void** event_out);
int mpx_event_destroy(mpx_engine* eng, void* event);
int mpx_event_record(mpx_engine* eng, void* event, void* stream);
int mpx_stream_wait_event(mpx_engine* eng, void* stream, void* event);
/* milliseconds between two recorded (and completed) timing events                          */
int mpx_event_elapsed_ms(mpx_engine* eng, void* ev_start, void* ev_end, float* ms);

/* ---- hipGraph capture of *_dev sequences (ABI 5) -----------------------------------------
 * mpx_graph_begin puts `stream` into capture (relaxed mode): every *_dev call, copy, memset,
 * event record and stream wait issued on it - and on other streams that join it through an
 * event it records - until mpx_graph_end is recorded into a graph, not run. Every stream that
 * joined must be joined back (an event recorded on it, waited on by `stream`) before the end.
 * mpx_graph_end ends the capture and instantiates the graph (*exec_out); mpx_graph_launch
 * replays it on a stream as one submission; mpx_graph_destroy frees it. Captured calls keep
 * the argument values (pointers, sizes) they were issued with. Used by bench.py to replay the
 * whole per-step sequence of the sharded engine (group step, step totals, the RCCL group on a
 * second stream) with one host call per step group.                                         */
int mpx_graph_begin(mpx_engine* eng, void* stream);
int mpx_graph_end(mpx_engine* eng, void* stream, void** exec_out);
int mpx_graph_launch(mpx_engine* eng, void* exec, void* stream);
int mpx_graph_destroy(mpx_engine* eng, void* exec);

/* the HIP and RCCL runtimes this library is bound to, as one JSON object (NUL-terminated,
 * truncated to cap): {"hip_runtime": v, "hip_driver": v, "rccl": v, "hip_path": "...",
 * "rccl_path": "..."}. Returns the full length (excluding the NUL) or a negative error.    */
int mpx_runtime_info(char* buf, size_t cap);

/* ---- diagnostics: TEST-ONLY entry points (the product path never calls them) -----------
 * mpx_debug_kv_set_epoch: set the KV table's call epoch (1 <= epoch < 2^30) without touching
 * its slots, so a test can drive calls across the epoch wrap on a table whose slots carry
 * older tags. mpx_debug_kv_state: copy the table's per-slot state words (bit 0 present, bit 1
 * last command of the tagged call was a PUT, bits 2.. the tag); *n = slots (cap + 1).
 * mpx_debug_kv_set_small_tag: set the tag of the last replica-batch call (0 <= tag < 2^18 - 1;
 * the next call uses tag + 1, and the call with tag 2^18 - 1 clears the per-slot list heads and
 * restarts the tags at 1), so a test can drive calls across the tag wrap.                                                       */
int mpx_debug_kv_set_epoch(mpx_engine* eng, uint32_t epoch);
int mpx_debug_kv_set_small_tag(mpx_engine* eng, uint32_t tag);
int mpx_debug_kv_state(mpx_engine* eng, uint32_t* state, size_t cap, size_t* n);

#ifdef __cplusplus
}
#endif
#endif /* MPX_H_ */
