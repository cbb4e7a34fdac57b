// kernels.hpp — launchers exported by the .hip translation units to the C-ABI layer.
// Every launcher only enqueues on `stream` (no allocation, no synchronisation), so callers can
// capture sequences of them into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mpx.h"

namespace mpx {

// error bits raised by kernels into the engine's device error word
constexpr uint32_t kErrNil = 1u;     // record names a nil / out-of-window instance
constexpr uint32_t kErrBadId = 2u;   // reply id outside [0, N)
constexpr uint32_t kErrOrder = 4u;   // records not in ascending instance order
constexpr uint32_t kErrKvFull = 8u;  // KV capacity exceeded
constexpr uint32_t kErrInval = 16u;  // other malformed input (offsets, sizes)
// (with kErrInval) a one-launch step's fold timed out: its packed totals slots were left as they
// were and must be zeroed by the host before the next one-launch step
constexpr uint32_t kErrSlots = 32u;

// reduction scratch: kRedWords u64 per engine
constexpr int kRedWords = 64;
// the tile kernels (tile.hpp) run a persistent grid of at most kTileGrid workgroups; their
// control words (kTileCtlWords u32, engine-owned, zeroed at mpx_open) carry the call's
// device-scope maxima and the last-workgroup ticket, and are back to zero after every call
constexpr int kTileGrid = 2048;
constexpr int kTileCtlWords = 64;
// workgroups of a persistent launch of `kernel` (block threads) over `tiles` units: two rounds
// of the number resident at once on the device (occupancy x CUs, cached per kernel), at most
// kTileGrid
uint32_t resident_grid(const void* kernel, int block, uint64_t tiles);

hipError_t launch_accept_tally(int mode, const mpx_accept_reply* recs, uint64_t n,
                               const mpx_inst_state* st_in, mpx_inst_state* st_out,
                               uint64_t n_inst, int32_t base, int32_t nrep, int32_t* scalars,
                               uint8_t* decided, unsigned long long* red, uint32_t* ctl,
                               uint32_t* err, hipStream_t stream);

hipError_t launch_committed_prefix(const mpx_inst_state* st, uint64_t n_inst, int32_t base,
                                   int32_t* scalars, unsigned long long* red, hipStream_t stream);

hipError_t launch_prepare_classic(const mpx_prepare_reply* recs, uint64_t n,
                                  const mpx_prep_state* st_in, mpx_prep_state* st_out,
                                  uint64_t n_inst, int32_t base, int32_t nrep,
                                  int32_t* default_ballot, uint8_t* prepared, uint32_t* ctl,
                                  uint32_t* err, hipStream_t stream);

hipError_t launch_prepare_min(const mpx_prepare_reply_min* recs, uint64_t n,
                              const uint64_t* grp_rec_off, mpx_group_prep_state* gst,
                              uint64_t n_groups, int32_t nrep, int32_t* peer_commits,
                              mpx_prepare_effect* eff, uint32_t* err, hipStream_t stream);

hipError_t launch_conflict_batch(const uint8_t* op, const int64_t* key, const uint64_t* inst_off,
                                 uint64_t n_inst, uint8_t* out, hipStream_t stream);

// fused per-group step: tally + executeCommands against per-group compact KV tables.
// worklist: n_groups u32 + wcount (device) for groups the fast kernel hands on.
// totals (optional, device): the step's d_totals[0..2] computed inside the same two kernels
// (per-group partials into kTotSlots accumulators of the control words, added by the kernel
// that finishes the group, folded by the general kernel), so a step needs no k_step_totals
// launch.
// ev_fast0 / ev_fast1 (optional): recorded on `stream` right before and after the fast kernel's
// launch (mpx_group_step_events), so a timer can bracket that kernel alone.
hipError_t launch_group_step(int mode, int32_t nrep, uint32_t kv_per_group,
                             const mpx_group_batch* b, uint32_t* worklist, uint32_t* wcount,
                             int64_t* totals, uint32_t* err, hipStream_t stream,
                             hipEvent_t ev_fast0, hipEvent_t ev_fast1,
                             unsigned long long* pslots = nullptr);
// one-launch steps (pslots: the engine's zeroed packed-totals slots, one u64 per 64 groups): the
// fast kernel alone, which folds the totals in its last workgroup; the shape must fit a fast
// variant (step_one_launch_fits) and a group that does not fit it fails the step
bool step_one_launch_fits(int32_t nrep, uint32_t ipg, uint32_t kv_per_group);
// d_totals[0..2] = decided instances, executed instances, executed commands of the batch
// step control words (engine-owned, zeroed once): [0] work-list count, [1] its ticket, [4..9]
// the totals' 64-bit accumulators, [10] their ticket, [16..) the fused totals' partials
// (kTotSlots x 3 u64, by group % kTotSlots). Every kernel that consumes a count or a partial
// resets it in its last workgroup, so a step launches no memset.
constexpr int kTotSlots = 64;
constexpr int kStepCtlWords = 16 + kTotSlots * 3 * 2;
hipError_t launch_step_totals(const mpx_group_batch* b, int64_t* totals, uint32_t* ctl,
                              hipStream_t stream);

// ---- global KV table apply (mpx_apply) ----------------------------------------------------
struct KvTable {
    int64_t* keys;       // [cap]
    int64_t* vals;       // [cap]
    uint32_t* state;     // [cap] bit 0 present, bit 1 last command of epoch (>> 2) was a PUT
    uint64_t cap;        // power of two, >= 1024
    uint32_t lgnb;       // log2(cap / 256): buckets of 256 slots (kvtab.hpp)
    unsigned long long* n_present;  // device counter
    uint32_t* epoch;     // device: [0] call epoch of mpx_apply (1 .. kKvEpochMax-1), [1] k_epoch_next's
                         // completion counter (0 between calls)
    uint32_t* probe;     // device, kSmallScratchWords: the replica-batch apply's per-command
                         // slot, state word and list link, and its control words (zeroed once)
    uint32_t* lhead;     // device, [cap + 1]: per slot, the head of the replica-batch call's
                         // command list, tagged with the call (zeroed once and at each tag wrap)
};
// probe scratch: 3 x MPX_APPLY_SMALL_MAX per-command words, then the control words:
// [kSmallCtl] LONG commands of the call, [kSmallCtl + 1] the tag of the last call (device-side,
// so a captured graph's replays take fresh tags), [kSmallCtl + 2] the walk kernel's ticket
constexpr uint32_t kSmallCtl = 3 * MPX_APPLY_SMALL_MAX;
// then the call's commands as the probe kernel read them (key, val: 2 words each; op: bytes), so
// the later kernels read device memory, not the host form's pinned staging across the link
constexpr uint32_t kSmallKeyOff = kSmallCtl + 64;
constexpr uint32_t kSmallValOff = kSmallKeyOff + 2 * MPX_APPLY_SMALL_MAX;
constexpr uint32_t kSmallOpOff = kSmallValOff + 2 * MPX_APPLY_SMALL_MAX;
constexpr uint32_t kSmallScratchWords = kSmallOpOff + MPX_APPLY_SMALL_MAX / 4;
constexpr uint32_t kSmallTagMax = 1u << 18;  // 18 tag bits above the 14 position bits

constexpr uint32_t kKvEpochMax = 1u << 30;  // = kvtab.hpp kEpochMax (state bits 2..31)

struct ApplyWork {      // scratch sized for m commands (see apply_work_bytes)
    void* base;
    uint64_t bytes;
};
// the handle's apply settings (mpx_config.apply_*)
struct ApplyOpts {
    uint64_t chunk;     // commands per chunk, 0 = kApplyChunkDefault
    uint32_t path;      // MPX_APPLY_AUTO / _SMALL / _SORTED / _PARTITIONED
    uint32_t fast_min;  // AUTO: partitioned from this many commands, 0 = kFastMinDefault
    uint32_t hot_min;   // partitioned: hot-key sample threshold, 0 = 5, MPX_APPLY_NO_HOT = none
};
// commands per apply chunk (0 = default): bounds the pipeline's scratch (34 B per command on the
// partitioned path, 48 B on the sort-based one)
constexpr uint64_t kApplyChunkDefault = 1ull << 26;
uint64_t apply_chunk_commands(uint64_t chunk, uint64_t m);
uint64_t apply_work_bytes(const KvTable& t, const ApplyOpts& o, uint64_t m);
// a new call epoch for the table (both apply pipelines); zeroes *n_miss when given
hipError_t launch_epoch_next(KvTable& t, uint32_t* n_miss, hipStream_t stream);
// scratch for any call of at most max_m commands (mpx_apply_reserve)
uint64_t apply_reserve_bytes(const KvTable& t, const ApplyOpts& o, uint64_t max_m);
// the partitioned pipeline (apply_fast.hip): tables of at most 1024 bins of 16 buckets
bool apply_fast_ok(const KvTable& t);
// the call runs the replica-batch kernels (apply_small.hip): no pipeline scratch
bool apply_is_one_launch(const ApplyOpts& o, uint64_t m);
uint64_t apply_fast_work_bytes(const KvTable& t, uint64_t c);
hipError_t launch_apply_fast(KvTable& t, const uint8_t* op, const int64_t* key, const int64_t* val,
                             uint64_t m, int64_t* ret, uint8_t* conf, uint64_t C, ApplyWork& w,
                             uint32_t hot_min, uint32_t* err, hipStream_t stream);
// replica-batch apply of at most MPX_APPLY_SMALL_MAX commands (apply_small.hip, three launches).
// err may be a host-mapped word (the host-pointer form): the kernels raise into it with plain
// stores (every bit they raise is kErrKvFull), never atomics. done (optional, host-mapped): the
// last workgroup stores seq there once every result of the call is visible to the host, so the
// host form can poll it instead of waiting on the stream
hipError_t launch_apply_small(KvTable& t, const uint8_t* op, const int64_t* key, const int64_t* val,
                              uint64_t m, int64_t* ret, uint8_t* conf, uint32_t* err,
                              hipStream_t stream, uint32_t* done = nullptr, uint32_t seq = 0,
                              bool host_io = false);
hipError_t launch_apply(KvTable& t, const uint8_t* op, const int64_t* key, const int64_t* val,
                        uint64_t m, int64_t* ret, uint8_t* conf, const ApplyOpts& o, ApplyWork& w,
                        uint32_t* err, hipStream_t stream);
hipError_t launch_kv_clear(KvTable& t, hipStream_t stream);
hipError_t launch_kv_import(KvTable& t, const int64_t* keys, const int64_t* vals, uint64_t n,
                            uint32_t* err, hipStream_t stream);
hipError_t launch_kv_export(KvTable& t, int64_t* keys, int64_t* vals, uint64_t cap,
                            unsigned long long* counter, hipStream_t stream);

// ---- peer stream framing (mpx_decode_peer_stream) ---------------------------------------
uint64_t decode_work_bytes(uint64_t len);
hipError_t launch_decode_peer_stream(const uint8_t* buf, uint64_t len, mpx_accept_reply* ar_out,
                                     uint64_t ar_cap, mpx_peer_frame* oth_out, uint64_t oth_cap,
                                     mpx_decode_result* res, void* work, uint64_t work_bytes,
                                     hipStream_t stream);

// ---- full peer-stream decode (mpx_decode_stream) -----------------------------------------
struct StreamOuts {
    mpx_accept_reply* ar;
    uint64_t ar_cap;
    void* prep;
    uint64_t prep_cap;
    mpx_var_frame* var;
    uint64_t var_cap;
    mpx_peer_frame* oth;
    uint64_t oth_cap;
};
uint64_t stream_work_bytes(uint64_t len);
// frames buf[start, len) with the proto's framing; legacy = stop at variable-length messages
hipError_t launch_decode_stream(int proto, int legacy, const uint8_t* buf, uint64_t len,
                                uint64_t start, const StreamOuts& outs, mpx_stream_result* res,
                                void* work, uint64_t work_bytes, hipStream_t stream);

// ---- client reply fan-out (mpx_encode_replies) -------------------------------------------
uint64_t fanout_work_bytes(uint64_t n);
hipError_t launch_encode_replies(const mpx_reply_rec* recs, uint64_t n, uint32_t n_clients,
                                 uint8_t ok, int32_t leader, uint8_t* out, uint64_t* client_off,
                                 void* work, uint64_t work_bytes, uint32_t* err,
                                 hipStream_t stream);

// ---- instance-log encoding (mpx_encode_log) ----------------------------------------------
uint64_t logenc_work_bytes(uint64_t n, uint64_t m);
uint64_t logenc_max_bytes(uint64_t n, uint64_t m);
hipError_t launch_encode_log(int format, const mpx_log_rec* recs, uint64_t n,
                             const uint64_t* cmd_off, const uint8_t* op, const int64_t* key,
                             const int64_t* val, uint64_t m, uint8_t* out, uint64_t* rec_off,
                             void* work, uint64_t work_bytes, hipStream_t stream);


// ---- durable-log replay (mpx_replay_durable) ---------------------------------------------
hipError_t launch_replay_durable(const uint8_t* log, uint64_t n, int32_t inst_cap,
                                 int32_t rec_base, mpx_log_rec* recs, uint8_t* op, int64_t* key, int64_t* val,
                                 int32_t* last_rec, int32_t* scalars, uint32_t* err,
                                 void* work, uint64_t work_bytes, hipStream_t stream);
// scratch of the binned slot maximum for n records over inst_cap slots (0: the call takes the
// per-record atomic form, which needs none)
uint64_t replay_work_bytes(uint64_t n, int32_t inst_cap);

}  // namespace mpx
