// engine.cpp — the C ABI (include/mpx.h) over the gfx950 kernels.
//
// Host-pointer entry points stage through engine-owned device buffers on the engine's HIP
// stream and return when results are back in caller memory. *_dev entry points enqueue on the
// caller's stream with device pointers, never allocate and never synchronise.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "kernels.hpp"

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

// pinned, GPU-mapped staging of a replica-batch apply: [error word | completion flag] (a cache
// line each), then op (cap rounded to 16), key, val, ret (cap each) and conf
struct PinIo {
    uint8_t* p = nullptr;
    size_t cap = 0;  // commands
};
constexpr size_t kPinHdr = 128;
struct PinView {
    volatile uint32_t* err;
    volatile uint32_t* done;
    uint8_t* op;
    int64_t* key;
    int64_t* val;
    int64_t* ret;
    uint8_t* conf;
};
PinView pin_view_at(uint8_t* base, size_t cap) {
    const size_t a16 = (cap + 15) & ~(size_t)15;
    PinView v;
    v.err = (volatile uint32_t*)base;
    v.done = (volatile uint32_t*)(base + 64);
    v.op = base + kPinHdr;
    v.key = (int64_t*)(v.op + a16);
    v.val = v.key + cap;
    v.ret = v.val + cap;
    v.conf = (uint8_t*)(v.ret + cap);
    return v;
}
PinView pin_view(const PinIo& p) { return pin_view_at(p.p, p.cap); }
size_t pin_bytes(size_t cap) { return kPinHdr + ((cap + 15) & ~(size_t)15) + cap * 25; }

}  // namespace

struct mpx_engine {
    int device = 0;
    mpx_config cfg{};
    hipStream_t stream = nullptr;
    std::string err;
    uint32_t* d_err = nullptr;
    unsigned long long* d_red = nullptr;
    uint32_t* d_tctl = nullptr;  // tile kernels' control words (kTileCtlWords, zero between calls)
    // host-API staging
    DevBuf b[12];
    // global KV table (mpx_apply)
    mpx::KvTable kv{};
    bool kv_ready = false;
    DevBuf apply_work;
    // peer stream decode: staging (bytes, AcceptReplies, other frames, result) + scratch
    DevBuf dec[4];
    DevBuf decode_work;
    // full stream decode: staging (bytes, AcceptReplies, PrepareReplies, var frames, other,
    // result) + scratch
    DevBuf sd[6];
    DevBuf stream_work;
    // client reply fan-out: staging (records, bytes, offsets) + scratch
    DevBuf fan[3];
    DevBuf fan_work;
    // instance-log encoding: staging (records, offsets, op, key, val, out, rec_off) + scratch
    DevBuf lg[7];
    DevBuf log_work;
    // durable-log replay staging: log bytes, records, op, key, val, last_rec, scalars
    DevBuf rp[7];
    DevBuf replay_work;  // the binned slot maximum (mpx_replay_durable_reserve)
    mpx::ApplyOpts apply{};  // mpx_config.apply_* (fixed for the handle's life)
    // replica-sized mpx_apply calls: pinned, GPU-mapped staging the one-launch kernel reads the
    // commands from and writes the results to (no DMA copies on the call's path)
    PinIo pin_io;       // mpx_apply's (copies in and out)
    PinIo pin_staged;   // mpx_apply_buffers / mpx_apply_staged's (the caller fills it)
    uint32_t small_seq = 0;  // the host form's completion flag value of the last call
    // group-step work list (groups the fast kernel hands to the general kernel) + its count
    DevBuf worklist;
    uint32_t* d_wcount = nullptr;
    hipEvent_t ev_fast0 = nullptr, ev_fast1 = nullptr;  // mpx_group_step_events
    bool slots_dirty = false;  // a one-launch fold timed out: zero the packed slots first
    // RCCL
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
};

namespace {

int fail(mpx_engine* e, int code, const std::string& what) {
    if (e) e->err = what;
    return code;
}

int hip_fail(mpx_engine* e, const char* what, hipError_t r) {
    return fail(e, MPX_E_HIP, std::string(what) + ": " + hipGetErrorString(r));
}

#define HIPCHK(e, x)                                        \
    do {                                                    \
        hipError_t _r = (x);                                \
        if (_r != hipSuccess) return hip_fail((e), #x, _r); \
    } while (0)

int grow(mpx_engine* e, DevBuf& b, size_t bytes) {
    if (bytes <= b.cap) return MPX_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    size_t c = std::max(bytes, (size_t)256);
    if (hipMalloc(&b.p, c) != hipSuccess) {
        (void)hipGetLastError();
        return fail(e, MPX_E_NOMEM, "device allocation of " + std::to_string(c) + " bytes failed");
    }
    b.cap = c;
    return MPX_OK;
}

#define GROW(e, buf, bytes)                       \
    do {                                          \
        int _c = grow((e), (buf), (bytes));       \
        if (_c) return _c;                        \
    } while (0)

hipStream_t pick(mpx_engine* e, void* s) { return s ? (hipStream_t)s : e->stream; }

int check_errword(mpx_engine* e, uint32_t w) {
    if (!w) return MPX_OK;
    // a one-launch step's fold gave up on its slots: zero them before the next step (stream
    // order), so no straggler's late add carries into a later step's totals
    if (w & mpx::kErrSlots) e->slots_dirty = true;
    if (w & mpx::kErrNil)
        return fail(e, MPX_E_NIL_INSTANCE, "record names a nil or out-of-window instance");
    if (w & mpx::kErrBadId) return fail(e, MPX_E_BAD_ID, "reply id outside [0, N)");
    if (w & mpx::kErrOrder)
        return fail(e, MPX_E_INVAL, "records are not grouped in ascending instance order");
    if (w & mpx::kErrKvFull) return fail(e, MPX_E_KV_FULL, "KV table capacity exceeded");
    return fail(e, MPX_E_INVAL, "malformed input (offsets / sizes)");
}

// synchronise the engine stream, read and clear the device error word
int finish(mpx_engine* e) {
    uint32_t w = 0;
    HIPCHK(e, hipMemcpyAsync(&w, e->d_err, sizeof(w), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (w) HIPCHK(e, hipMemsetAsync(e->d_err, 0, sizeof(uint32_t), e->stream));
    return check_errword(e, w);
}

int begin(mpx_engine* e) {
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipMemsetAsync(e->d_err, 0, sizeof(uint32_t), e->stream));
    return MPX_OK;
}

int h2d(mpx_engine* e, void* d, const void* h, size_t bytes) {
    if (!bytes) return MPX_OK;
    HIPCHK(e, hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, e->stream));
    return MPX_OK;
}
int d2h(mpx_engine* e, void* h, const void* d, size_t bytes) {
    if (!bytes) return MPX_OK;
    HIPCHK(e, hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, e->stream));
    return MPX_OK;
}
#define CK(x)                  \
    do {                       \
        int _c = (x);          \
        if (_c) return _c;     \
    } while (0)

void free_kv(mpx::KvTable& t) {
    if (t.keys) (void)hipFree(t.keys);
    if (t.vals) (void)hipFree(t.vals);
    if (t.state) (void)hipFree(t.state);
    if (t.n_present) (void)hipFree(t.n_present);
    if (t.epoch) (void)hipFree(t.epoch);
    if (t.probe) (void)hipFree(t.probe);
    if (t.lhead) (void)hipFree(t.lhead);
    t = mpx::KvTable{};
}

int ensure_kv(mpx_engine* e) {
    if (e->kv_ready) return MPX_OK;
    uint64_t want = e->cfg.kv_capacity ? e->cfg.kv_capacity : (1ull << 20);
    uint64_t cap = 1024;
    while (cap < 2 * want) cap <<= 1;
    mpx::KvTable t{};
    t.cap = cap;
    t.lgnb = 0;
    while ((1ull << (t.lgnb + 8)) < cap) ++t.lgnb;
    // cap hash slots + one side slot for the key INT64_MIN (the empty-slot sentinel)
    if (hipMalloc(&t.keys, (cap + 1) * 8) != hipSuccess ||
        hipMalloc(&t.vals, (cap + 1) * 8) != hipSuccess ||
        hipMalloc(&t.state, (cap + 1) * 4) != hipSuccess ||
        hipMalloc(&t.n_present, sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&t.epoch, 2 * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t.probe, mpx::kSmallScratchWords * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t.lhead, (cap + 1) * 4) != hipSuccess) {
        (void)hipGetLastError();
        free_kv(t);
        return fail(e, MPX_E_NOMEM, "KV table allocation failed");
    }
    hipError_t r0 = hipMemsetAsync(t.epoch, 0, 2 * sizeof(uint32_t), e->stream);
    if (r0 == hipSuccess)
        r0 = hipMemsetAsync(t.probe, 0, mpx::kSmallScratchWords * sizeof(uint32_t), e->stream);
    if (r0 == hipSuccess) r0 = hipMemsetAsync(t.lhead, 0, (cap + 1) * 4, e->stream);
    const hipError_t r1 = r0 == hipSuccess ? mpx::launch_kv_clear(t, e->stream) : r0;
    if (r1 != hipSuccess) {
        (void)hipGetLastError();
        free_kv(t);
        return hip_fail(e, "KV table initialisation", r1);
    }
    e->kv = t;
    e->kv_ready = true;
    return MPX_OK;
}

int pin_grow(mpx_engine* e, PinIo& p, size_t m) {
    if (p.cap >= m && p.p) return MPX_OK;
    if (p.p) (void)hipHostFree(p.p);
    p.p = nullptr;
    p.cap = 0;
    const size_t cap = m < 1024 ? 1024 : m;
    void* hp = nullptr;
    if (hipHostMalloc(&hp, pin_bytes(cap), hipHostMallocDefault) != hipSuccess || !hp) {
        (void)hipGetLastError();
        return fail(e, MPX_E_NOMEM, "pinned staging for the replica-batch apply");
    }
    p.p = (uint8_t*)hp;
    p.cap = cap;
    return MPX_OK;
}

// the replica-batch kernels on m commands in pinned staging p, results back in it; returns once
// the stream is done (MPX_SMALL_POLL builds: once the kernels' completion flag is set - the last
// workgroup stores it after every result is visible to the host - the stream queried now and
// then, so a failed launch or a faulted kernel ends the wait with its error)
int run_pinned(mpx_engine* e, const PinIo& p, size_t m, bool want_conf) {
    const PinView v = pin_view(p);
    *v.err = 0u;
    void* dp = nullptr;
    HIPCHK(e, hipHostGetDevicePointer(&dp, p.p, 0));
    const PinView d = pin_view_at((uint8_t*)dp, p.cap);
    uint32_t seq = ++e->small_seq;
    if (!seq) seq = e->small_seq = 1;  // 0 never marks a finished call
// MPX_SMALL_POLL=1 (A/B builds): the kernels store a completion flag into the pinned staging
// after a system-scope release of every result and the host polls it instead of waiting on the
// stream; same-box A/B (profiles/r04/replica): 40.6-45.0 vs 32.0-37.9 us per 5000-command host
// call, 30.6-32.7 vs 22.9-23.0 us staged - the per-thread system fences cost more than the
// stream wait's wake-up, so the default waits on the stream
#ifndef MPX_SMALL_POLL
#define MPX_SMALL_POLL 0
#endif
    HIPCHK(e, mpx::launch_apply_small(e->kv, d.op, d.key, d.val, m, d.ret,
                                      want_conf ? d.conf : nullptr, (uint32_t*)d.err, e->stream,
                                      MPX_SMALL_POLL ? (uint32_t*)d.done : nullptr, seq,
                                      /*host_io=*/true));
    if (!MPX_SMALL_POLL) {
        HIPCHK(e, hipStreamSynchronize(e->stream));
        return check_errword(e, *v.err);
    }
    for (uint64_t it = 1; *v.done != seq; ++it) {
        if ((it & 1023) == 0) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) {
                if (*v.done == seq) break;
                return fail(e, MPX_E_HIP, "mpx_apply: the call ended without its completion flag");
            }
            if (q != hipErrorNotReady) return hip_fail(e, "mpx_apply", q);
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
    return check_errword(e, *v.err);
}

}  // namespace

extern "C" {

int mpx_abi_version(void) { return MPX_ABI_VERSION; }

int mpx_device_count(int* count) {
    if (!count) return MPX_E_INVAL;
    int c = 0;
    hipError_t r = hipGetDeviceCount(&c);
    if (r != hipSuccess) {
        (void)hipGetLastError();
        *count = 0;
        return MPX_OK;
    }
    *count = c;
    return MPX_OK;
}

int mpx_open(int device, const mpx_config* cfg, mpx_engine** out) {
    if (!cfg || !out) return MPX_E_INVAL;
    *out = nullptr;
    if (cfg->n_replicas < 1 || cfg->n_replicas > MPX_MAX_REPLICAS) return MPX_E_INVAL;
    if (cfg->mode != MPX_MODE_MIN && cfg->mode != MPX_MODE_CLASSIC) return MPX_E_INVAL;
    if (cfg->apply_path > MPX_APPLY_SMALL || (cfg->flags & ~MPX_FLAG_KNOWN) || cfg->reserved)
        return MPX_E_INVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || device < 0 || device >= c) {
        (void)hipGetLastError();
        return MPX_E_NODEV;
    }
    mpx_engine* e = new (std::nothrow) mpx_engine();
    if (!e) return MPX_E_NOMEM;
    e->device = device;
    e->cfg = *cfg;
    if (!e->cfg.kv_per_group) e->cfg.kv_per_group = 512;
    e->apply = mpx::ApplyOpts{cfg->apply_chunk, cfg->apply_path, cfg->apply_fast_min,
                              cfg->apply_hot_min};
    if (!e->cfg.max_groups) e->cfg.max_groups = 1ull << 20;
    if (e->cfg.kv_per_group > 1024) {
        delete e;
        return MPX_E_UNSUPPORTED;
    }
    e->worklist.cap = e->cfg.max_groups * sizeof(uint32_t);
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&e->d_err, sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&e->d_red, mpx::kRedWords * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&e->d_tctl, mpx::kTileCtlWords * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(e->d_tctl, 0, mpx::kTileCtlWords * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(e->d_red, 0, mpx::kRedWords * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&e->d_wcount, mpx::kStepCtlWords * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(e->d_wcount, 0, mpx::kStepCtlWords * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&e->worklist.p, e->worklist.cap) != hipSuccess ||
        // (one-launch steps keep their packed totals slots there, zero between steps)
        hipMemset(e->worklist.p, 0, e->worklist.cap) != hipSuccess ||
        hipMemset(e->d_err, 0, sizeof(uint32_t)) != hipSuccess) {
        (void)hipGetLastError();
        mpx_close(e);
        return MPX_E_HIP;
    }
    *out = e;
    return MPX_OK;
}

int mpx_close(mpx_engine* e) {
    if (!e) return MPX_E_INVAL;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->comm) ncclCommDestroy(e->comm);
    for (auto& x : e->b)
        if (x.p) (void)hipFree(x.p);
    if (e->apply_work.p) (void)hipFree(e->apply_work.p);
    if (e->pin_io.p) (void)hipHostFree(e->pin_io.p);
    if (e->pin_staged.p) (void)hipHostFree(e->pin_staged.p);
    for (auto& x : e->dec)
        if (x.p) (void)hipFree(x.p);
    if (e->decode_work.p) (void)hipFree(e->decode_work.p);
    for (auto& x : e->sd)
        if (x.p) (void)hipFree(x.p);
    if (e->stream_work.p) (void)hipFree(e->stream_work.p);
    for (auto& x : e->fan)
        if (x.p) (void)hipFree(x.p);
    if (e->fan_work.p) (void)hipFree(e->fan_work.p);
    for (auto& x : e->lg)
        if (x.p) (void)hipFree(x.p);
    if (e->log_work.p) (void)hipFree(e->log_work.p);
    for (auto& x : e->rp)
        if (x.p) (void)hipFree(x.p);
    if (e->replay_work.p) (void)hipFree(e->replay_work.p);
    if (e->worklist.p) (void)hipFree(e->worklist.p);
    if (e->d_wcount) (void)hipFree(e->d_wcount);
    if (e->kv_ready) free_kv(e->kv);
    if (e->d_err) (void)hipFree(e->d_err);
    if (e->d_red) (void)hipFree(e->d_red);
    if (e->d_tctl) (void)hipFree(e->d_tctl);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return MPX_OK;
}

const char* mpx_last_error(mpx_engine* e) { return e ? e->err.c_str() : "null engine"; }

void* mpx_stream(mpx_engine* e) { return e ? (void*)e->stream : nullptr; }

int mpx_synchronize(mpx_engine* e) {
    if (!e) return MPX_E_INVAL;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipDeviceSynchronize());
    return finish(e);
}

// ---- A1 / A2 --------------------------------------------------------------------------------
int mpx_accept_tally(mpx_engine* e, const mpx_accept_reply* recs, size_t n, mpx_inst_state* st,
                     size_t n_inst, int32_t inst_base, int32_t* committed_upto,
                     int32_t* peer_commits, uint8_t* decided_out) {
    if (!e) return MPX_E_INVAL;
    if ((n && !recs) || (n_inst && !st) || !committed_upto || !peer_commits)
        return fail(e, MPX_E_INVAL, "null argument");
    if (n >= 0xFFFFFFFFull) return fail(e, MPX_E_UNSUPPORTED, "more than 2^32-2 records");
    const int N = e->cfg.n_replicas;
    CK(begin(e));
    GROW(e, e->b[0], n * sizeof(mpx_accept_reply));
    GROW(e, e->b[1], n_inst * sizeof(mpx_inst_state));
    GROW(e, e->b[2], n_inst);
    GROW(e, e->b[3], (1 + N) * sizeof(int32_t));
    int32_t sc[1 + MPX_MAX_REPLICAS];
    sc[0] = *committed_upto;
    memcpy(sc + 1, peer_commits, N * sizeof(int32_t));
    CK(h2d(e, e->b[0].p, recs, n * sizeof(mpx_accept_reply)));
    CK(h2d(e, e->b[1].p, st, n_inst * sizeof(mpx_inst_state)));
    CK(h2d(e, e->b[3].p, sc, (1 + N) * sizeof(int32_t)));
    uint8_t* d_dec = decided_out ? (uint8_t*)e->b[2].p : nullptr;
    HIPCHK(e, mpx::launch_accept_tally(e->cfg.mode, (const mpx_accept_reply*)e->b[0].p, n,
                                       (const mpx_inst_state*)e->b[1].p,
                                       (mpx_inst_state*)e->b[1].p, n_inst, inst_base, N,
                                       (int32_t*)e->b[3].p, d_dec, e->d_red, e->d_tctl,
                                       e->d_err, e->stream));
    CK(d2h(e, st, e->b[1].p, n_inst * sizeof(mpx_inst_state)));
    CK(d2h(e, sc, e->b[3].p, (1 + N) * sizeof(int32_t)));
    if (decided_out) CK(d2h(e, decided_out, d_dec, n_inst));
    CK(finish(e));
    *committed_upto = sc[0];
    memcpy(peer_commits, sc + 1, N * sizeof(int32_t));
    return MPX_OK;
}

int mpx_accept_tally_dev(mpx_engine* e, const mpx_accept_reply* d_recs, size_t n,
                         const mpx_inst_state* d_st_in, mpx_inst_state* d_st_out, size_t n_inst,
                         int32_t inst_base, int32_t* d_scalars, uint8_t* d_decided,
                         void* stream) {
    if (!e) return MPX_E_INVAL;
    if ((n && !d_recs) || (n_inst && (!d_st_in || !d_st_out)) || !d_scalars)
        return fail(e, MPX_E_INVAL, "null argument");
    if (n >= 0xFFFFFFFFull) return fail(e, MPX_E_UNSUPPORTED, "more than 2^32-2 records");
    HIPCHK(e, mpx::launch_accept_tally(e->cfg.mode, d_recs, n, d_st_in, d_st_out, n_inst,
                                       inst_base, e->cfg.n_replicas, d_scalars, d_decided,
                                       e->d_red, e->d_tctl, e->d_err, pick(e, stream)));
    return MPX_OK;
}

int mpx_committed_prefix(mpx_engine* e, const mpx_inst_state* st, size_t n_inst,
                         int32_t inst_base, int32_t* committed_upto) {
    if (!e) return MPX_E_INVAL;
    if ((n_inst && !st) || !committed_upto) return fail(e, MPX_E_INVAL, "null argument");
    CK(begin(e));
    GROW(e, e->b[1], n_inst * sizeof(mpx_inst_state));
    GROW(e, e->b[3], sizeof(int32_t));
    CK(h2d(e, e->b[1].p, st, n_inst * sizeof(mpx_inst_state)));
    CK(h2d(e, e->b[3].p, committed_upto, sizeof(int32_t)));
    HIPCHK(e, mpx::launch_committed_prefix((const mpx_inst_state*)e->b[1].p, n_inst, inst_base,
                                           (int32_t*)e->b[3].p, e->d_red, e->stream));
    CK(d2h(e, committed_upto, e->b[3].p, sizeof(int32_t)));
    return finish(e);
}

// ---- A4 ---------------------------------------------------------------------------------------
int mpx_prepare_select(mpx_engine* e, const mpx_prepare_reply* recs, size_t n, mpx_prep_state* st,
                       size_t n_inst, int32_t inst_base, int32_t* default_ballot,
                       uint8_t* prepared_out) {
    if (!e) return MPX_E_INVAL;
    if ((n && !recs) || (n_inst && !st) || !default_ballot)
        return fail(e, MPX_E_INVAL, "null argument");
    CK(begin(e));
    GROW(e, e->b[0], n * sizeof(mpx_prepare_reply));
    GROW(e, e->b[1], n_inst * sizeof(mpx_prep_state));
    GROW(e, e->b[2], n_inst);
    GROW(e, e->b[3], sizeof(int32_t));
    CK(h2d(e, e->b[0].p, recs, n * sizeof(mpx_prepare_reply)));
    CK(h2d(e, e->b[1].p, st, n_inst * sizeof(mpx_prep_state)));
    CK(h2d(e, e->b[3].p, default_ballot, sizeof(int32_t)));
    uint8_t* d_prep = prepared_out ? (uint8_t*)e->b[2].p : nullptr;
    HIPCHK(e, mpx::launch_prepare_classic((const mpx_prepare_reply*)e->b[0].p, n,
                                          (const mpx_prep_state*)e->b[1].p,
                                          (mpx_prep_state*)e->b[1].p, n_inst, inst_base,
                                          e->cfg.n_replicas, (int32_t*)e->b[3].p, d_prep,
                                          e->d_tctl, e->d_err, e->stream));
    CK(d2h(e, st, e->b[1].p, n_inst * sizeof(mpx_prep_state)));
    CK(d2h(e, default_ballot, e->b[3].p, sizeof(int32_t)));
    if (prepared_out) CK(d2h(e, prepared_out, d_prep, n_inst));
    return finish(e);
}

int mpx_prepare_select_dev(mpx_engine* e, const mpx_prepare_reply* d_recs, size_t n,
                           const mpx_prep_state* d_st_in, mpx_prep_state* d_st_out, size_t n_inst,
                           int32_t inst_base, int32_t* d_default_ballot, uint8_t* d_prepared,
                           void* stream) {
    if (!e) return MPX_E_INVAL;
    if ((n && !d_recs) || (n_inst && (!d_st_in || !d_st_out)) || !d_default_ballot)
        return fail(e, MPX_E_INVAL, "null argument");
    HIPCHK(e, mpx::launch_prepare_classic(d_recs, n, d_st_in, d_st_out, n_inst, inst_base,
                                          e->cfg.n_replicas, d_default_ballot, d_prepared,
                                          e->d_tctl, e->d_err, pick(e, stream)));
    return MPX_OK;
}

// ---- A3 ---------------------------------------------------------------------------------------
int mpx_prepare_select_min(mpx_engine* e, const mpx_prepare_reply_min* recs, size_t n,
                           const uint64_t* grp_rec_off, mpx_group_prep_state* gst,
                           size_t n_groups, int32_t* peer_commits, mpx_prepare_effect* eff) {
    if (!e) return MPX_E_INVAL;
    if ((n && !recs) || !grp_rec_off || (n_groups && (!gst || !peer_commits)))
        return fail(e, MPX_E_INVAL, "null argument");
    if (grp_rec_off[0] != 0 || grp_rec_off[n_groups] != n)
        return fail(e, MPX_E_INVAL, "grp_rec_off must start at 0 and end at n");
    for (size_t g = 0; g < n_groups; ++g)
        if (grp_rec_off[g + 1] < grp_rec_off[g])
            return fail(e, MPX_E_INVAL, "grp_rec_off must be non-decreasing");
    const int N = e->cfg.n_replicas;
    CK(begin(e));
    GROW(e, e->b[0], n * sizeof(mpx_prepare_reply_min));
    GROW(e, e->b[4], (n_groups + 1) * sizeof(uint64_t));
    GROW(e, e->b[1], n_groups * sizeof(mpx_group_prep_state));
    GROW(e, e->b[5], n_groups * N * sizeof(int32_t));
    GROW(e, e->b[6], n * sizeof(mpx_prepare_effect));
    CK(h2d(e, e->b[0].p, recs, n * sizeof(mpx_prepare_reply_min)));
    CK(h2d(e, e->b[4].p, grp_rec_off, (n_groups + 1) * sizeof(uint64_t)));
    CK(h2d(e, e->b[1].p, gst, n_groups * sizeof(mpx_group_prep_state)));
    CK(h2d(e, e->b[5].p, peer_commits, n_groups * N * sizeof(int32_t)));
    mpx_prepare_effect* d_eff = eff ? (mpx_prepare_effect*)e->b[6].p : nullptr;
    HIPCHK(e, mpx::launch_prepare_min((const mpx_prepare_reply_min*)e->b[0].p, n,
                                      (const uint64_t*)e->b[4].p, (mpx_group_prep_state*)e->b[1].p,
                                      n_groups, N, (int32_t*)e->b[5].p, d_eff, e->d_err,
                                      e->stream));
    CK(d2h(e, gst, e->b[1].p, n_groups * sizeof(mpx_group_prep_state)));
    CK(d2h(e, peer_commits, e->b[5].p, n_groups * N * sizeof(int32_t)));
    if (eff) CK(d2h(e, eff, d_eff, n * sizeof(mpx_prepare_effect)));
    return finish(e);
}

int mpx_prepare_select_min_dev(mpx_engine* e, const mpx_prepare_reply_min* d_recs, size_t n,
                               const uint64_t* d_grp_rec_off, mpx_group_prep_state* d_gst,
                               size_t n_groups, int32_t* d_peer_commits,
                               mpx_prepare_effect* d_eff, void* stream) {
    if (!e) return MPX_E_INVAL;
    if ((n && !d_recs) || !d_grp_rec_off || (n_groups && (!d_gst || !d_peer_commits)))
        return fail(e, MPX_E_INVAL, "null argument");
    HIPCHK(e, mpx::launch_prepare_min(d_recs, n, d_grp_rec_off, d_gst, n_groups,
                                      e->cfg.n_replicas, d_peer_commits, d_eff, e->d_err,
                                      pick(e, stream)));
    return MPX_OK;
}

// ---- A5 / A6 ----------------------------------------------------------------------------------
int mpx_apply(mpx_engine* e, const uint8_t* op, const int64_t* key, const int64_t* val, size_t m,
              int64_t* ret, uint8_t* conf_prev) {
    if (!e) return MPX_E_INVAL;
    if (m && (!op || !key || !val || !ret)) return fail(e, MPX_E_INVAL, "null argument");
    if (m >= (1ull << 31)) return fail(e, MPX_E_UNSUPPORTED, "more than 2^31-1 commands per call");
    if (mpx::apply_is_one_launch(e->apply, m)) {
        // one drained executeCommands batch: the commands go into pinned host memory the kernels
        // read over the link, the results and the call's error word come back the same way (no
        // DMA, no memset, no copy of the error word: the host clears and reads it in place); a
        // CPU copy on each side (mpx_apply_staged: none)
        HIPCHK(e, hipSetDevice(e->device));
        CK(ensure_kv(e));
        CK(pin_grow(e, e->pin_io, m));
        const PinView v = pin_view(e->pin_io);
        std::memcpy(v.op, op, m);
        std::memcpy(v.key, key, m * 8);
        std::memcpy(v.val, val, m * 8);
        const int rc = run_pinned(e, e->pin_io, m, conf_prev != nullptr);
        std::memcpy(ret, v.ret, m * 8);
        if (conf_prev) std::memcpy(conf_prev, v.conf, m);
        return rc;
    }
    CK(begin(e));
    CK(ensure_kv(e));
    GROW(e, e->b[7], m);
    GROW(e, e->b[8], m * 8);
    GROW(e, e->b[9], m * 8);
    GROW(e, e->b[10], m * 8);
    GROW(e, e->b[11], m);
    GROW(e, e->apply_work, mpx::apply_work_bytes(e->kv, e->apply, m));
    CK(h2d(e, e->b[7].p, op, m));
    CK(h2d(e, e->b[8].p, key, m * 8));
    CK(h2d(e, e->b[9].p, val, m * 8));
    mpx::ApplyWork w{e->apply_work.p, e->apply_work.cap};
    uint8_t* d_conf = conf_prev ? (uint8_t*)e->b[11].p : nullptr;
    HIPCHK(e, mpx::launch_apply(e->kv, (const uint8_t*)e->b[7].p, (const int64_t*)e->b[8].p,
                                (const int64_t*)e->b[9].p, m, (int64_t*)e->b[10].p, d_conf,
                                e->apply, w, e->d_err, e->stream));
    CK(d2h(e, ret, e->b[10].p, m * 8));
    if (conf_prev) CK(d2h(e, conf_prev, d_conf, m));
    return finish(e);
}

int mpx_apply_buffers(mpx_engine* e, size_t max_m, mpx_apply_io* io) {
    if (!e) return MPX_E_INVAL;
    if (!io) return fail(e, MPX_E_INVAL, "null io");
    if (!max_m || max_m > MPX_APPLY_SMALL_MAX)
        return fail(e, MPX_E_INVAL, "max_m must lie in [1, MPX_APPLY_SMALL_MAX]");
    if (!mpx::apply_is_one_launch(e->apply, max_m))
        return fail(e, MPX_E_INVAL, "the staged apply needs apply_path AUTO or SMALL");
    HIPCHK(e, hipSetDevice(e->device));
    CK(ensure_kv(e));
    if (e->pin_staged.cap < max_m) {
        HIPCHK(e, hipStreamSynchronize(e->stream));  // (no call may still use the old buffers)
        CK(pin_grow(e, e->pin_staged, max_m));
    }
    const PinView v = pin_view(e->pin_staged);
    io->op = v.op;
    io->key = v.key;
    io->val = v.val;
    io->ret = v.ret;
    io->conf = v.conf;
    io->cap = e->pin_staged.cap;
    return MPX_OK;
}

int mpx_apply_staged(mpx_engine* e, size_t m) {
    if (!e) return MPX_E_INVAL;
    if (!m) return MPX_OK;
    if (!e->pin_staged.p || m > e->pin_staged.cap)
        return fail(e, MPX_E_INVAL, "m exceeds the buffers of mpx_apply_buffers");
    HIPCHK(e, hipSetDevice(e->device));
    return run_pinned(e, e->pin_staged, m, true);
}

int mpx_apply_reserve(mpx_engine* e, size_t max_cmds) {
    if (!e) return MPX_E_INVAL;
    if (max_cmds >= (1ull << 31)) return fail(e, MPX_E_UNSUPPORTED, "more than 2^31-1 commands");
    CK(begin(e));
    CK(ensure_kv(e));
    GROW(e, e->apply_work, mpx::apply_reserve_bytes(e->kv, e->apply, max_cmds));
    return finish(e);
}

int mpx_apply_dev(mpx_engine* e, const uint8_t* d_op, const int64_t* d_key, const int64_t* d_val,
                  size_t m, int64_t* d_ret, uint8_t* d_conf_prev, void* stream) {
    if (!e) return MPX_E_INVAL;
    if (m && (!d_op || !d_key || !d_val || !d_ret)) return fail(e, MPX_E_INVAL, "null argument");
    if (m >= (1ull << 31)) return fail(e, MPX_E_UNSUPPORTED, "more than 2^31-1 commands per call");
    if (!e->kv_ready || e->apply_work.cap < mpx::apply_work_bytes(e->kv, e->apply, m))
        return fail(e, MPX_E_INVAL,
                    "mpx_apply_dev: call mpx_apply_reserve(m) first (the dev entry point never "
                    "allocates)");
    mpx::ApplyWork w{e->apply_work.p, e->apply_work.cap};
    HIPCHK(e, mpx::launch_apply(e->kv, d_op, d_key, d_val, m, d_ret, d_conf_prev,
                                e->apply, w, e->d_err, pick(e, stream)));
    return MPX_OK;
}

int mpx_kv_size(mpx_engine* e, size_t* n) {
    if (!e) return MPX_E_INVAL;
    if (!n) return fail(e, MPX_E_INVAL, "null or invalid argument");
    CK(begin(e));
    CK(ensure_kv(e));
    unsigned long long c = 0;
    CK(d2h(e, &c, e->kv.n_present, sizeof(c)));
    CK(finish(e));
    *n = (size_t)c;
    return MPX_OK;
}

int mpx_kv_export(mpx_engine* e, int64_t* keys, int64_t* vals, size_t cap, size_t* n) {
    if (!e) return MPX_E_INVAL;
    if (!n || (cap && (!keys || !vals))) return fail(e, MPX_E_INVAL, "null or invalid argument");
    CK(begin(e));
    CK(ensure_kv(e));
    unsigned long long c = 0;
    CK(d2h(e, &c, e->kv.n_present, sizeof(c)));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const size_t want = (size_t)c;
    GROW(e, e->b[8], std::max<size_t>(want, 1) * 8);
    GROW(e, e->b[9], std::max<size_t>(want, 1) * 8);
    HIPCHK(e, mpx::launch_kv_export(e->kv, (int64_t*)e->b[8].p, (int64_t*)e->b[9].p, want,
                                    (unsigned long long*)e->d_red, e->stream));
    const size_t k = std::min(cap, want);
    CK(d2h(e, keys, e->b[8].p, k * 8));
    CK(d2h(e, vals, e->b[9].p, k * 8));
    CK(finish(e));
    *n = want;
    return MPX_OK;
}

int mpx_kv_import(mpx_engine* e, const int64_t* keys, const int64_t* vals, size_t n) {
    if (!e) return MPX_E_INVAL;
    if ((n && (!keys || !vals))) return fail(e, MPX_E_INVAL, "null or invalid argument");
    CK(begin(e));
    CK(ensure_kv(e));
    GROW(e, e->b[8], n * 8);
    GROW(e, e->b[9], n * 8);
    CK(h2d(e, e->b[8].p, keys, n * 8));
    CK(h2d(e, e->b[9].p, vals, n * 8));
    HIPCHK(e, mpx::launch_kv_import(e->kv, (const int64_t*)e->b[8].p, (const int64_t*)e->b[9].p, n,
                                    e->d_err, e->stream));
    return finish(e);
}

int mpx_kv_clear(mpx_engine* e) {
    if (!e) return MPX_E_INVAL;
    CK(begin(e));
    CK(ensure_kv(e));
    HIPCHK(e, mpx::launch_kv_clear(e->kv, e->stream));
    return finish(e);
}

int mpx_conflict_batch(mpx_engine* e, const uint8_t* op, const int64_t* key,
                       const uint64_t* inst_off, size_t n_inst, uint8_t* out) {
    if (!e) return MPX_E_INVAL;
    if (n_inst < 2) return MPX_OK;
    if (!op || !key || !inst_off || !out) return fail(e, MPX_E_INVAL, "null argument");
    const uint64_t m = inst_off[n_inst];
    if (inst_off[0] != 0) return fail(e, MPX_E_INVAL, "inst_off[0] must be 0");
    for (size_t i = 0; i < n_inst; ++i)
        if (inst_off[i + 1] < inst_off[i]) return fail(e, MPX_E_INVAL, "inst_off not sorted");
    CK(begin(e));
    GROW(e, e->b[7], m);
    GROW(e, e->b[8], m * 8);
    GROW(e, e->b[4], (n_inst + 1) * 8);
    GROW(e, e->b[11], n_inst);
    CK(h2d(e, e->b[7].p, op, m));
    CK(h2d(e, e->b[8].p, key, m * 8));
    CK(h2d(e, e->b[4].p, inst_off, (n_inst + 1) * 8));
    HIPCHK(e, mpx::launch_conflict_batch((const uint8_t*)e->b[7].p, (const int64_t*)e->b[8].p,
                                         (const uint64_t*)e->b[4].p, n_inst,
                                         (uint8_t*)e->b[11].p, e->stream));
    CK(d2h(e, out, e->b[11].p, n_inst - 1));
    return finish(e);
}

int mpx_conflict_batch_dev(mpx_engine* e, const uint8_t* d_op, const int64_t* d_key,
                           const uint64_t* d_inst_off, size_t n_inst, uint8_t* d_out,
                           void* stream) {
    if (!e) return MPX_E_INVAL;
    if (n_inst < 2) return MPX_OK;
    if (!d_op || !d_key || !d_inst_off || !d_out) return fail(e, MPX_E_INVAL, "null argument");
    HIPCHK(e, mpx::launch_conflict_batch(d_op, d_key, d_inst_off, n_inst, d_out, pick(e, stream)));
    return MPX_OK;
}

// ---- fused group step -------------------------------------------------------------------------
namespace {
bool one_launch(const mpx_engine* e) { return (e->cfg.flags & MPX_FLAG_STEP_ONE_LAUNCH) != 0; }
// one-launch steps: the packed totals slots (one u64 per 64 groups) live in the work list's
// memory, which such a handle never uses as a list
unsigned long long* pslots(const mpx_engine* e) {
    return one_launch(e) ? reinterpret_cast<unsigned long long*>(e->worklist.p) : nullptr;
}
// the device-pointer group step; d_totals (optional) gets the step totals from the same kernels
int group_step_dev(mpx_engine* e, const mpx_group_batch* b, int64_t* d_totals, void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!b) return fail(e, MPX_E_INVAL, "null or invalid argument");
    if (b->n_groups && (!b->recs || !b->grp_rec_off || !b->st_in || !b->st_out ||
                        !b->committed_in || !b->committed_out || !b->executed_in ||
                        !b->executed_out || !b->peer_in || !b->peer_out || !b->op || !b->key ||
                        !b->val || !b->cmd_off || !b->ret || !b->kv_cnt_in || !b->kv_key_in ||
                        !b->kv_val_in || !b->kv_cnt_out || !b->kv_key_out || !b->kv_val_out))
        return fail(e, MPX_E_INVAL, "null field in mpx_group_batch");
    if (b->ipg == 0 && b->n_groups) return fail(e, MPX_E_INVAL, "ipg must be > 0");
    if (b->ipg > 8192) return fail(e, MPX_E_UNSUPPORTED, "more than 8192 instances per group");
    if ((uint64_t)b->n_groups * sizeof(uint32_t) > e->worklist.cap)
        return fail(e, MPX_E_INVAL, "n_groups exceeds mpx_config.max_groups");
    if (one_launch(e) && !mpx::step_one_launch_fits(e->cfg.n_replicas, b->ipg, e->cfg.kv_per_group))
        return fail(e, MPX_E_INVAL, "MPX_FLAG_STEP_ONE_LAUNCH: the batch shape fits no fast variant");
    if (one_launch(e) && e->slots_dirty) {
        HIPCHK(e, hipMemsetAsync(e->worklist.p, 0, e->worklist.cap, pick(e, stream)));
        e->slots_dirty = false;
    }
    HIPCHK(e, mpx::launch_group_step(e->cfg.mode, e->cfg.n_replicas, e->cfg.kv_per_group, b,
                                     (uint32_t*)e->worklist.p, e->d_wcount, d_totals, e->d_err,
                                     pick(e, stream), e->ev_fast0, e->ev_fast1, pslots(e)));
    return MPX_OK;
}
}  // namespace

int mpx_group_step_dev(mpx_engine* e, const mpx_group_batch* b, void* stream) {
    return group_step_dev(e, b, nullptr, stream);
}

int mpx_group_step_totals_dev(mpx_engine* e, const mpx_group_batch* b, int64_t* d_totals,
                              void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!d_totals) return fail(e, MPX_E_INVAL, "null d_totals");
    if (b && b->n_groups && !b->n_decided)
        return fail(e, MPX_E_INVAL, "mpx_group_step_totals_dev needs n_decided");
    return group_step_dev(e, b, d_totals, stream);
}

int mpx_group_step_events(mpx_engine* e, void* ev_fast_start, void* ev_fast_end) {
    if (!e) return MPX_E_INVAL;
    if (!ev_fast_start != !ev_fast_end) return fail(e, MPX_E_INVAL, "give both events or neither");
    e->ev_fast0 = (hipEvent_t)ev_fast_start;
    e->ev_fast1 = (hipEvent_t)ev_fast_end;
    return MPX_OK;
}

int mpx_step_totals_dev(mpx_engine* e, const mpx_group_batch* b, int64_t* d_totals,
                        void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!b || !d_totals) return fail(e, MPX_E_INVAL, "null argument");
    if (b->n_groups && (!b->n_decided || !b->executed_in || !b->executed_out || !b->cmd_off))
        return fail(e, MPX_E_INVAL, "mpx_step_totals_dev needs n_decided, executed_in/out, cmd_off");
    HIPCHK(e, mpx::launch_step_totals(b, d_totals, e->d_wcount, pick(e, stream)));
    return MPX_OK;
}

int mpx_group_step(mpx_engine* e, const mpx_group_batch* hb) {
    if (!e) return MPX_E_INVAL;
    if (!hb) return fail(e, MPX_E_INVAL, "null or invalid argument");
    const uint64_t G = hb->n_groups, ipg = hb->ipg, ni = G * ipg;
    const int N = e->cfg.n_replicas;
    const uint64_t K = e->cfg.kv_per_group;
    if (!G) return MPX_OK;
    if (!hb->grp_rec_off || !hb->cmd_off) return fail(e, MPX_E_INVAL, "null offsets");
    const uint64_t nr = hb->grp_rec_off[G];
    const uint64_t m = hb->cmd_off[ni];
    if (hb->grp_rec_off[0] != 0) return fail(e, MPX_E_INVAL, "grp_rec_off[0] must be 0");
    for (uint64_t g = 0; g < G; ++g)
        if (hb->grp_rec_off[g + 1] < hb->grp_rec_off[g])
            return fail(e, MPX_E_INVAL, "grp_rec_off not sorted");
    for (uint64_t i = 0; i < ni; ++i)
        if (hb->cmd_off[i + 1] < hb->cmd_off[i]) return fail(e, MPX_E_INVAL, "cmd_off not sorted");
    CK(begin(e));
    // one device arena for the whole batch
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t o_recs = take(nr * 16), o_roff = take((G + 1) * 8), o_st = take(ni * 16),
                 o_ci = take(G * 4), o_co = take(G * 4), o_ei = take(G * 4), o_eo = take(G * 4),
                 o_pi = take(G * N * 4), o_po = take(G * N * 4), o_op = take(m), o_key = take(m * 8),
                 o_val = take(m * 8), o_coff = take((ni + 1) * 4), o_has = take(ni),
                 o_ret = take(m * 8), o_conf = take(m), o_kc = take(G * 4), o_kk = take(G * K * 8),
                 o_kvv = take(G * K * 8), o_dec = take(ni), o_nd = take(G * 4);
    GROW(e, e->b[0], off);
    char* d = (char*)e->b[0].p;
    mpx_group_batch db{};
    db.n_groups = (uint32_t)G;
    db.ipg = (uint32_t)ipg;
    db.recs = (const mpx_accept_reply*)(d + o_recs);
    db.grp_rec_off = (const uint64_t*)(d + o_roff);
    db.st_in = (const mpx_inst_state*)(d + o_st);
    db.st_out = (mpx_inst_state*)(d + o_st);
    db.committed_in = (const int32_t*)(d + o_ci);
    db.committed_out = (int32_t*)(d + o_co);
    db.executed_in = (const int32_t*)(d + o_ei);
    db.executed_out = (int32_t*)(d + o_eo);
    db.peer_in = (const int32_t*)(d + o_pi);
    db.peer_out = (int32_t*)(d + o_po);
    db.op = (const uint8_t*)(d + o_op);
    db.key = (const int64_t*)(d + o_key);
    db.val = (const int64_t*)(d + o_val);
    db.cmd_off = (const uint32_t*)(d + o_coff);
    db.has_cmds = hb->has_cmds ? (const uint8_t*)(d + o_has) : nullptr;
    db.ret = (int64_t*)(d + o_ret);
    db.conf_prev = hb->conf_prev ? (uint8_t*)(d + o_conf) : nullptr;
    db.kv_cnt_in = (const uint32_t*)(d + o_kc);
    db.kv_key_in = (const int64_t*)(d + o_kk);
    db.kv_val_in = (const int64_t*)(d + o_kvv);
    db.kv_cnt_out = (uint32_t*)(d + o_kc);
    db.kv_key_out = (int64_t*)(d + o_kk);
    db.kv_val_out = (int64_t*)(d + o_kvv);
    db.decided = hb->decided ? (uint8_t*)(d + o_dec) : nullptr;
    db.n_decided = hb->n_decided ? (uint32_t*)(d + o_nd) : nullptr;
    CK(h2d(e, d + o_recs, hb->recs, nr * 16));
    CK(h2d(e, d + o_roff, hb->grp_rec_off, (G + 1) * 8));
    CK(h2d(e, d + o_st, hb->st_in, ni * 16));
    CK(h2d(e, d + o_ci, hb->committed_in, G * 4));
    CK(h2d(e, d + o_ei, hb->executed_in, G * 4));
    CK(h2d(e, d + o_pi, hb->peer_in, G * N * 4));
    CK(h2d(e, d + o_op, hb->op, m));
    CK(h2d(e, d + o_key, hb->key, m * 8));
    CK(h2d(e, d + o_val, hb->val, m * 8));
    CK(h2d(e, d + o_coff, hb->cmd_off, (ni + 1) * 4));
    if (hb->has_cmds) CK(h2d(e, d + o_has, hb->has_cmds, ni));
    CK(h2d(e, d + o_ret, hb->ret, m * 8));  // unexecuted commands keep the caller's values
    if (hb->conf_prev) CK(h2d(e, d + o_conf, hb->conf_prev, m));
    CK(h2d(e, d + o_kc, hb->kv_cnt_in, G * 4));
    CK(h2d(e, d + o_kk, hb->kv_key_in, G * K * 8));
    CK(h2d(e, d + o_kvv, hb->kv_val_in, G * K * 8));
    if (ipg > 8192) return fail(e, MPX_E_UNSUPPORTED, "more than 8192 instances per group");
    if (G * sizeof(uint32_t) > e->worklist.cap) {
        GROW(e, e->worklist, G * sizeof(uint32_t));
        HIPCHK(e, hipMemsetAsync(e->worklist.p, 0, e->worklist.cap, e->stream));  // (slots)
    }
    if (one_launch(e) && !mpx::step_one_launch_fits(N, (uint32_t)ipg, (uint32_t)K))
        return fail(e, MPX_E_INVAL, "MPX_FLAG_STEP_ONE_LAUNCH: the batch shape fits no fast variant");
    if (one_launch(e) && e->slots_dirty) {
        HIPCHK(e, hipMemsetAsync(e->worklist.p, 0, e->worklist.cap, e->stream));
        e->slots_dirty = false;
    }
    HIPCHK(e, mpx::launch_group_step(e->cfg.mode, N, (uint32_t)K, &db, (uint32_t*)e->worklist.p,
                                     e->d_wcount, nullptr, e->d_err, e->stream, nullptr, nullptr,
                                     pslots(e)));
    CK(d2h(e, hb->st_out, d + o_st, ni * 16));
    CK(d2h(e, hb->committed_out, d + o_co, G * 4));
    CK(d2h(e, hb->executed_out, d + o_eo, G * 4));
    CK(d2h(e, hb->peer_out, d + o_po, G * N * 4));
    CK(d2h(e, hb->ret, d + o_ret, m * 8));
    if (hb->conf_prev) CK(d2h(e, hb->conf_prev, d + o_conf, m));
    CK(d2h(e, hb->kv_cnt_out, d + o_kc, G * 4));
    CK(d2h(e, hb->kv_key_out, d + o_kk, G * K * 8));
    CK(d2h(e, hb->kv_val_out, d + o_kvv, G * K * 8));
    if (hb->decided) CK(d2h(e, hb->decided, d + o_dec, ni));
    if (hb->n_decided) CK(d2h(e, hb->n_decided, d + o_nd, G * 4));
    return finish(e);
}

// ---- RCCL -------------------------------------------------------------------------------------
int mpx_comm_unique_id(void* out128) {
    if (!out128) return MPX_E_INVAL;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return MPX_E_RCCL;
    memcpy(out128, &id, sizeof(id));
    return MPX_OK;
}

int mpx_comm_init(mpx_engine* e, int nranks, int rank, const void* unique_id128) {
    if (!e) return MPX_E_INVAL;
    if (!unique_id128 || nranks < 1 || rank < 0 || rank >= nranks) return fail(e, MPX_E_INVAL, "null or invalid argument");
    HIPCHK(e, hipSetDevice(e->device));
    if (e->comm) {
        ncclCommDestroy(e->comm);
        e->comm = nullptr;
    }
    ncclUniqueId id;
    memcpy(&id, unique_id128, sizeof(id));
    ncclResult_t r = ncclCommInitRank(&e->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        e->comm = nullptr;
        return fail(e, MPX_E_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    e->nranks = nranks;
    e->rank = rank;
    return MPX_OK;
}

int mpx_watermarks_allreduce_dev(mpx_engine* e, int32_t* d_wm, size_t n_groups, void* stream) {
    if (!e) return MPX_E_INVAL;
    if (n_groups && !d_wm) return fail(e, MPX_E_INVAL, "null d_watermarks");
    if (!e->comm) return fail(e, MPX_E_INVAL, "mpx_comm_init has not been called");
    ncclResult_t r = ncclAllReduce(d_wm, d_wm, 2 * n_groups, ncclInt32, ncclMax, e->comm,
                                   pick(e, stream));
    if (r != ncclSuccess) return fail(e, MPX_E_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    return MPX_OK;
}

int mpx_step_allreduce_dev(mpx_engine* e, int32_t* d_wm, size_t n_groups, int64_t* d_totals,
                           size_t n_totals, void* stream) {
    if (!e) return MPX_E_INVAL;
    if ((n_groups && !d_wm) || (n_totals && !d_totals)) return fail(e, MPX_E_INVAL, "null argument");
    if (!e->comm) return fail(e, MPX_E_INVAL, "mpx_comm_init has not been called");
    const hipStream_t s = pick(e, stream);
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess && n_groups)
        r = ncclAllReduce(d_wm, d_wm, 2 * n_groups, ncclInt32, ncclMax, e->comm, s);
    if (r == ncclSuccess && n_totals)
        r = ncclAllReduce(d_totals, d_totals, n_totals, ncclInt64, ncclSum, e->comm, s);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess)
        return fail(e, MPX_E_RCCL, std::string("step all-reduce: ") + ncclGetErrorString(r));
    return MPX_OK;
}

int mpx_step_allreduce_oop_dev(mpx_engine* e, const int32_t* d_wm_send, int32_t* d_wm_recv,
                               size_t n_groups, int64_t* d_totals, size_t n_totals, void* stream) {
    if (!e) return MPX_E_INVAL;
    if ((n_groups && (!d_wm_send || !d_wm_recv)) || (n_totals && !d_totals))
        return fail(e, MPX_E_INVAL, "null argument");
    if (n_groups && d_wm_send == d_wm_recv)
        return fail(e, MPX_E_INVAL, "d_wm_send and d_wm_recv must differ (mpx_step_allreduce_dev "
                                    "is the in-place form)");
    if (!e->comm) return fail(e, MPX_E_INVAL, "mpx_comm_init has not been called");
    const hipStream_t s = pick(e, stream);
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess && n_groups)
        r = ncclAllReduce(d_wm_send, d_wm_recv, 2 * n_groups, ncclInt32, ncclMax, e->comm, s);
    if (r == ncclSuccess && n_totals)
        r = ncclAllReduce(d_totals, d_totals, n_totals, ncclInt64, ncclSum, e->comm, s);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess)
        return fail(e, MPX_E_RCCL, std::string("step all-reduce: ") + ncclGetErrorString(r));
    return MPX_OK;
}

int mpx_watermarks_allreduce(mpx_engine* e, int32_t* committed, int32_t* executed,
                             size_t n_groups) {
    if (!e) return MPX_E_INVAL;
    if ((n_groups && (!committed || !executed))) return fail(e, MPX_E_INVAL, "null or invalid argument");
    CK(begin(e));
    GROW(e, e->b[5], 2 * n_groups * 4);
    int32_t* d = (int32_t*)e->b[5].p;
    CK(h2d(e, d, committed, n_groups * 4));
    CK(h2d(e, d + n_groups, executed, n_groups * 4));
    CK(mpx_watermarks_allreduce_dev(e, d, n_groups, e->stream));
    CK(d2h(e, committed, d, n_groups * 4));
    CK(d2h(e, executed, d + n_groups, n_groups * 4));
    return finish(e);
}

// ---- §8(f) rank 1: peer stream framing + AcceptReply decode --------------------------------
int mpx_decode_reserve(mpx_engine* e, size_t max_len) {
    if (!e) return MPX_E_INVAL;
    if (max_len > MPX_DECODE_MAX_BYTES)
        return fail(e, MPX_E_UNSUPPORTED, "decode buffers are limited to 2^31-1 bytes per call");
    CK(begin(e));
    GROW(e, e->decode_work, mpx::decode_work_bytes(max_len));
    return finish(e);
}

int mpx_decode_peer_stream_dev(mpx_engine* e, const uint8_t* d_buf, size_t len,
                               mpx_accept_reply* d_ar, size_t ar_cap, mpx_peer_frame* d_other,
                               size_t other_cap, mpx_decode_result* d_res, void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!d_res || (len && !d_buf) || (ar_cap && !d_ar) || (other_cap && !d_other))
        return fail(e, MPX_E_INVAL, "null or invalid argument");
    if (len > MPX_DECODE_MAX_BYTES)
        return fail(e, MPX_E_UNSUPPORTED, "decode buffers are limited to 2^31-1 bytes per call");
    if (e->decode_work.cap < mpx::decode_work_bytes(len))
        return fail(e, MPX_E_INVAL,
                    "mpx_decode_peer_stream_dev: call mpx_decode_reserve(len) first (the dev "
                    "entry point never allocates)");
    HIPCHK(e, mpx::launch_decode_peer_stream(d_buf, len, d_ar, ar_cap, d_other, other_cap, d_res,
                                             e->decode_work.p, e->decode_work.cap,
                                             pick(e, stream)));
    return MPX_OK;
}

int mpx_decode_peer_stream(mpx_engine* e, const uint8_t* buf, size_t len, mpx_accept_reply* ar,
                           size_t ar_cap, mpx_peer_frame* other, size_t other_cap,
                           mpx_decode_result* res) {
    if (!e) return MPX_E_INVAL;
    if (!res || (len && !buf) || (ar_cap && !ar) || (other_cap && !other))
        return fail(e, MPX_E_INVAL, "null or invalid argument");
    if (len > MPX_DECODE_MAX_BYTES)
        return fail(e, MPX_E_UNSUPPORTED, "decode buffers are limited to 2^31-1 bytes per call");
    CK(begin(e));
    GROW(e, e->dec[0], len);
    GROW(e, e->dec[1], ar_cap * sizeof(mpx_accept_reply));
    GROW(e, e->dec[2], other_cap * sizeof(mpx_peer_frame));
    GROW(e, e->dec[3], sizeof(mpx_decode_result));
    GROW(e, e->decode_work, mpx::decode_work_bytes(len));
    CK(h2d(e, e->dec[0].p, buf, len));
    CK(mpx_decode_peer_stream_dev(e, (const uint8_t*)e->dec[0].p, len,
                                  (mpx_accept_reply*)e->dec[1].p, ar_cap,
                                  (mpx_peer_frame*)e->dec[2].p, other_cap,
                                  (mpx_decode_result*)e->dec[3].p, e->stream));
    CK(d2h(e, res, e->dec[3].p, sizeof(mpx_decode_result)));
    CK(finish(e));
    CK(d2h(e, ar, e->dec[1].p, std::min<uint64_t>(res->n_accept_replies, ar_cap) *
                                   sizeof(mpx_accept_reply)));
    CK(d2h(e, other, e->dec[2].p, std::min<uint64_t>(res->n_other, other_cap) *
                                      sizeof(mpx_peer_frame)));
    return finish(e);
}

// ---- §8(f) rank 1, full: fixed and variable-length frames -------------------------------------
namespace {
size_t prep_rec_bytes(const mpx_engine* e) {
    return e->cfg.mode == MPX_MODE_MIN ? sizeof(mpx_prepare_reply_min) : sizeof(mpx_prepare_reply);
}
}  // namespace

int mpx_decode_stream_reserve(mpx_engine* e, size_t max_len) {
    if (!e) return MPX_E_INVAL;
    if (max_len > MPX_DECODE_MAX_BYTES)
        return fail(e, MPX_E_UNSUPPORTED, "decode buffers are limited to 2^31-1 bytes per call");
    CK(begin(e));
    GROW(e, e->stream_work, mpx::stream_work_bytes(max_len));
    return finish(e);
}

int mpx_decode_stream_dev(mpx_engine* e, const uint8_t* d_buf, size_t len, size_t start,
                          const mpx_decode_out* out, mpx_stream_result* d_res, void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!out || !d_res || (len && !d_buf) || (out->ar_cap && !out->ar) ||
        (out->prep_cap && !out->prep) || (out->var_cap && !out->var) ||
        (out->other_cap && !out->other))
        return fail(e, MPX_E_INVAL, "null or invalid argument");
    if (len > MPX_DECODE_MAX_BYTES)
        return fail(e, MPX_E_UNSUPPORTED, "decode buffers are limited to 2^31-1 bytes per call");
    if (start > len) return fail(e, MPX_E_INVAL, "start is past the end of the buffer");
    if ((uintptr_t)d_buf % 16)
        return fail(e, MPX_E_INVAL, "d_buf must be 16-byte aligned (tiles load 16 B vectors)");
    if (e->stream_work.cap < mpx::stream_work_bytes(len))
        return fail(e, MPX_E_INVAL,
                    "mpx_decode_stream_dev: call mpx_decode_stream_reserve(len) first (the dev "
                    "entry point never allocates)");
    const mpx::StreamOuts o{out->ar, out->ar_cap, out->prep, out->prep_cap, out->var,
                            out->var_cap, out->other, out->other_cap};
    HIPCHK(e, mpx::launch_decode_stream(e->cfg.mode, 0, d_buf, len, start, o, d_res,
                                        e->stream_work.p, e->stream_work.cap, pick(e, stream)));
    return MPX_OK;
}

int mpx_decode_stream(mpx_engine* e, const uint8_t* buf, size_t len, const mpx_decode_out* out,
                      mpx_stream_result* res) {
    if (!e) return MPX_E_INVAL;
    if (!out || !res || (len && !buf) || (out->ar_cap && !out->ar) ||
        (out->prep_cap && !out->prep) || (out->var_cap && !out->var) ||
        (out->other_cap && !out->other))
        return fail(e, MPX_E_INVAL, "null or invalid argument");
    if (len > MPX_DECODE_MAX_BYTES)
        return fail(e, MPX_E_UNSUPPORTED, "decode buffers are limited to 2^31-1 bytes per call");
    const size_t pb = prep_rec_bytes(e);
    CK(begin(e));
    GROW(e, e->sd[0], len);
    GROW(e, e->sd[1], out->ar_cap * sizeof(mpx_accept_reply));
    GROW(e, e->sd[2], out->prep_cap * pb);
    GROW(e, e->sd[3], out->var_cap * sizeof(mpx_var_frame));
    GROW(e, e->sd[4], out->other_cap * sizeof(mpx_peer_frame));
    GROW(e, e->sd[5], sizeof(mpx_stream_result));
    GROW(e, e->stream_work, mpx::stream_work_bytes(len));
    CK(h2d(e, e->sd[0].p, buf, len));
    const mpx_decode_out d{(mpx_accept_reply*)e->sd[1].p, out->ar_cap, e->sd[2].p, out->prep_cap,
                           (mpx_var_frame*)e->sd[3].p, out->var_cap,
                           (mpx_peer_frame*)e->sd[4].p, out->other_cap};
    mpx_stream_result r;
    memset(&r, 0, sizeof(r));
    CK(h2d(e, e->sd[5].p, &r, sizeof(r)));
    // one call per frame longer than the in-map window (MPX_DECODE_LONG); after one, windows
    // of the buffer (a PARTIAL stop at a window's end just continues) keep each call short
    size_t start = 0, window = len;
    for (;;) {
        const size_t end = std::min(len, start + window);
        CK(mpx_decode_stream_dev(e, (const uint8_t*)e->sd[0].p, end, start, &d,
                                 (mpx_stream_result*)e->sd[5].p, e->stream));
        CK(d2h(e, &r, e->sd[5].p, sizeof(r)));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        if (r.stop_reason == MPX_DECODE_LONG && r.next <= len) {
            start = r.next;
            window = 1u << 18;
        } else if ((r.stop_reason == MPX_DECODE_PARTIAL || r.stop_reason == MPX_DECODE_END) &&
                   end < len) {
            // the window ended inside the buffer: a frame that runs past it (PARTIAL) or one
            // that ends exactly at it (END) - both continue from there
            start = r.consumed;
            window = std::min<size_t>(window * 2, len);
        } else {
            break;
        }
    }
    *res = r;
    CK(d2h(e, out->ar, e->sd[1].p, std::min<uint64_t>(r.n_accept_replies, out->ar_cap) *
                                      sizeof(mpx_accept_reply)));
    CK(d2h(e, out->prep, e->sd[2].p, std::min<uint64_t>(r.n_prepare_replies, out->prep_cap) * pb));
    CK(d2h(e, out->var, e->sd[3].p, std::min<uint64_t>(r.n_var, out->var_cap) *
                                       sizeof(mpx_var_frame)));
    CK(d2h(e, out->other, e->sd[4].p, std::min<uint64_t>(r.n_other, out->other_cap) *
                                         sizeof(mpx_peer_frame)));
    return finish(e);
}

// ---- §8(f) rank 2: client reply fan-out -----------------------------------------------------
int mpx_encode_replies_reserve(mpx_engine* e, size_t max_n) {
    if (!e) return MPX_E_INVAL;
    if (max_n >= (1ull << 32)) return fail(e, MPX_E_UNSUPPORTED, "at most 2^32-1 replies per call");
    CK(begin(e));
    GROW(e, e->fan_work, mpx::fanout_work_bytes(max_n));
    return finish(e);
}

int mpx_encode_replies_dev(mpx_engine* e, const mpx_reply_rec* d_recs, size_t n,
                           uint32_t n_clients, uint8_t ok, int32_t leader, uint8_t* d_out,
                           uint64_t* d_client_off, void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!n_clients || !d_client_off || (n && (!d_recs || !d_out))) return fail(e, MPX_E_INVAL, "null or invalid argument");
    if (n >= (1ull << 32)) return fail(e, MPX_E_UNSUPPORTED, "at most 2^32-1 replies per call");
    if (e->fan_work.cap < mpx::fanout_work_bytes(n))
        return fail(e, MPX_E_INVAL,
                    "mpx_encode_replies_dev: call mpx_encode_replies_reserve(n) first (the dev "
                    "entry point never allocates)");
    HIPCHK(e, mpx::launch_encode_replies(d_recs, n, n_clients, ok, leader, d_out, d_client_off,
                                         e->fan_work.p, e->fan_work.cap, e->d_err,
                                         pick(e, stream)));
    return MPX_OK;
}

int mpx_encode_replies(mpx_engine* e, const mpx_reply_rec* recs, size_t n, uint32_t n_clients,
                       uint8_t ok, int32_t leader, uint8_t* out, uint64_t* client_off) {
    if (!e) return MPX_E_INVAL;
    if (!n_clients || !client_off || (n && (!recs || !out))) return fail(e, MPX_E_INVAL, "null or invalid argument");
    if (n >= (1ull << 32)) return fail(e, MPX_E_UNSUPPORTED, "at most 2^32-1 replies per call");
    CK(begin(e));
    GROW(e, e->fan[0], n * sizeof(mpx_reply_rec));
    GROW(e, e->fan[1], n * MPX_PROPOSE_REPLY_BYTES);
    GROW(e, e->fan[2], ((size_t)n_clients + 1) * sizeof(uint64_t));
    GROW(e, e->fan_work, mpx::fanout_work_bytes(n));
    CK(h2d(e, e->fan[0].p, recs, n * sizeof(mpx_reply_rec)));
    CK(mpx_encode_replies_dev(e, (const mpx_reply_rec*)e->fan[0].p, n, n_clients, ok, leader,
                              (uint8_t*)e->fan[1].p, (uint64_t*)e->fan[2].p, e->stream));
    CK(d2h(e, out, e->fan[1].p, n * MPX_PROPOSE_REPLY_BYTES));
    CK(d2h(e, client_off, e->fan[2].p, ((size_t)n_clients + 1) * sizeof(uint64_t)));
    int rc = finish(e);
    if (rc == MPX_E_INVAL) return fail(e, MPX_E_INVAL, "a reply names a client >= n_clients");
    return rc;
}

// ---- §8(f) ranks 3/4: instance-log encoding -------------------------------------------------
size_t mpx_encode_log_bound(size_t n, size_t m) { return (size_t)mpx::logenc_max_bytes(n, m); }

int mpx_encode_log_reserve(mpx_engine* e, size_t max_n, size_t max_m) {
    if (!e) return MPX_E_INVAL;
    CK(begin(e));
    GROW(e, e->log_work, mpx::logenc_work_bytes(max_n, max_m));
    return finish(e);
}

int mpx_encode_log_dev(mpx_engine* e, int format, const mpx_log_rec* d_recs, size_t n,
                       const uint64_t* d_cmd_off, const uint8_t* d_op, const int64_t* d_key,
                       const int64_t* d_val, size_t m, uint8_t* d_out, uint64_t* d_rec_off,
                       void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!d_rec_off || (n && (!d_recs || !d_cmd_off || !d_out)) || (m && (!d_op || !d_key || !d_val)))
        return fail(e, MPX_E_INVAL, "null or invalid argument");
    if (format != MPX_LOG_CATCHUP && format != MPX_LOG_DURABLE)
        return fail(e, MPX_E_INVAL, "unknown log format");
    if (e->log_work.cap < mpx::logenc_work_bytes(n, m))
        return fail(e, MPX_E_INVAL,
                    "mpx_encode_log_dev: call mpx_encode_log_reserve(n, m) first (the dev entry "
                    "point never allocates)");
    HIPCHK(e, mpx::launch_encode_log(format, d_recs, n, d_cmd_off, d_op, d_key, d_val, m, d_out,
                                     d_rec_off, e->log_work.p, e->log_work.cap, pick(e, stream)));
    return MPX_OK;
}

int mpx_encode_log(mpx_engine* e, int format, const mpx_log_rec* recs, size_t n,
                   const uint64_t* cmd_off, const uint8_t* op, const int64_t* key,
                   const int64_t* val, size_t m, uint8_t* out, size_t out_cap,
                   uint64_t* rec_off) {
    if (!e) return MPX_E_INVAL;
    if (!rec_off || (n && (!recs || !cmd_off)) || (m && (!op || !key || !val)) || (out_cap && !out))
        return fail(e, MPX_E_INVAL, "null or invalid argument");
    if (format != MPX_LOG_CATCHUP && format != MPX_LOG_DURABLE)
        return fail(e, MPX_E_INVAL, "unknown log format");
    for (size_t i = 0; i < n; ++i)  // the device kernels trust the offsets
        if (cmd_off[i] > cmd_off[i + 1] || cmd_off[i + 1] > m)
            return fail(e, MPX_E_INVAL, "cmd_off must be non-decreasing and <= m");
    const size_t bound = mpx::logenc_max_bytes(n, m);
    CK(begin(e));
    GROW(e, e->lg[0], n * sizeof(mpx_log_rec));
    GROW(e, e->lg[1], (n + 1) * 8);
    GROW(e, e->lg[2], m);
    GROW(e, e->lg[3], m * 8);
    GROW(e, e->lg[4], m * 8);
    GROW(e, e->lg[5], bound);
    GROW(e, e->lg[6], (n + 1) * 8);
    GROW(e, e->log_work, mpx::logenc_work_bytes(n, m));
    CK(h2d(e, e->lg[0].p, recs, n * sizeof(mpx_log_rec)));
    if (n) CK(h2d(e, e->lg[1].p, cmd_off, (n + 1) * 8));
    CK(h2d(e, e->lg[2].p, op, m));
    CK(h2d(e, e->lg[3].p, key, m * 8));
    CK(h2d(e, e->lg[4].p, val, m * 8));
    CK(mpx_encode_log_dev(e, format, (const mpx_log_rec*)e->lg[0].p, n,
                          (const uint64_t*)e->lg[1].p, (const uint8_t*)e->lg[2].p,
                          (const int64_t*)e->lg[3].p, (const int64_t*)e->lg[4].p, m,
                          (uint8_t*)e->lg[5].p, (uint64_t*)e->lg[6].p, e->stream));
    CK(d2h(e, rec_off, e->lg[6].p, (n + 1) * 8));
    CK(finish(e));
    if (rec_off[n] > out_cap) return fail(e, MPX_E_INVAL, "out_cap is smaller than the encoding");
    CK(d2h(e, out, e->lg[5].p, rec_off[n]));
    return finish(e);
}

// ---- §8(f) rank 3, read side: durable-log replay --------------------------------------------
namespace {
// shared argument checks of both forms; *n_out = number of records
int replay_args(mpx_engine* e, size_t len, int32_t inst_cap, int32_t rec_base, size_t* n_out) {
    if (inst_cap < 0) return fail(e, MPX_E_INVAL, "inst_cap must be >= 0");
    if (rec_base < 0) return fail(e, MPX_E_INVAL, "rec_base must be >= 0");
    if (len % MPX_DURABLE_REC_BYTES)
        return fail(e, MPX_E_INVAL, "durable log ends in a partial record");
    const size_t n = len / MPX_DURABLE_REC_BYTES;
    if ((uint64_t)rec_base + n > (uint64_t)INT32_MAX)
        return fail(e, MPX_E_UNSUPPORTED, "rec_base + records must stay below 2^31");
    // every record indexes instanceSpace[instNo]: with no instance space, the first one panics
    if (n && inst_cap == 0)
        return fail(e, MPX_E_NIL_INSTANCE, "a durable record's instNo is outside [0, inst_cap)");
    *n_out = n;
    return MPX_OK;
}
}  // namespace

int mpx_replay_durable_dev(mpx_engine* e, const uint8_t* d_log, size_t len, int32_t inst_cap,
                           int32_t rec_base, mpx_log_rec* d_recs, uint8_t* d_op, int64_t* d_key,
                           int64_t* d_val, int32_t* d_last_rec, int32_t* d_scalars, void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!d_scalars) return fail(e, MPX_E_INVAL, "null d_scalars");
    size_t n = 0;
    CK(replay_args(e, len, inst_cap, rec_base, &n));
    if (n && (!d_log || !d_recs || !d_op || !d_key || !d_val || !d_last_rec))
        return fail(e, MPX_E_INVAL, "null device buffer");
    if ((uintptr_t)d_log % 16)
        return fail(e, MPX_E_INVAL, "d_log must be 16-byte aligned (the tiles load 16 B vectors)");
    HIPCHK(e, mpx::launch_replay_durable(d_log, n, inst_cap, rec_base, d_recs, d_op, d_key, d_val,
                                         d_last_rec, d_scalars, e->d_err, e->replay_work.p,
                                         e->replay_work.cap, pick(e, stream)));
    return MPX_OK;
}

int mpx_replay_durable_reserve(mpx_engine* e, size_t max_len, int32_t inst_cap) {
    if (!e) return MPX_E_INVAL;
    if (inst_cap < 0) return fail(e, MPX_E_INVAL, "inst_cap must be >= 0");
    const size_t n = max_len / MPX_DURABLE_REC_BYTES;
    CK(begin(e));
    GROW(e, e->replay_work, mpx::replay_work_bytes(n, inst_cap));
    return finish(e);
}

int mpx_replay_durable(mpx_engine* e, const uint8_t* log, size_t len, int32_t inst_cap,
                       int32_t rec_base, mpx_log_rec* recs, uint8_t* op, int64_t* key, int64_t* val,
                       int32_t* last_rec, int32_t* scalars) {
    if (!e) return MPX_E_INVAL;
    if (!scalars || (inst_cap > 0 && !last_rec)) return fail(e, MPX_E_INVAL, "null argument");
    size_t n = 0;
    CK(replay_args(e, len, inst_cap, rec_base, &n));
    if (n && (!log || !recs || !op || !key || !val)) return fail(e, MPX_E_INVAL, "null argument");
    CK(begin(e));
    GROW(e, e->rp[0], len);
    GROW(e, e->rp[1], n * sizeof(mpx_log_rec));
    GROW(e, e->rp[2], n);
    GROW(e, e->rp[3], n * 8);
    GROW(e, e->rp[4], n * 8);
    GROW(e, e->rp[5], (size_t)inst_cap * 4);
    GROW(e, e->rp[6], 2 * sizeof(int32_t));
    GROW(e, e->replay_work, mpx::replay_work_bytes(n, inst_cap));
    CK(h2d(e, e->rp[0].p, log, len));
    CK(h2d(e, e->rp[5].p, last_rec, (size_t)inst_cap * 4));
    CK(h2d(e, e->rp[6].p, scalars, 2 * sizeof(int32_t)));
    if (n)
        CK(mpx_replay_durable_dev(e, (const uint8_t*)e->rp[0].p, len, inst_cap, rec_base,
                                  (mpx_log_rec*)e->rp[1].p, (uint8_t*)e->rp[2].p,
                                  (int64_t*)e->rp[3].p, (int64_t*)e->rp[4].p,
                                  (int32_t*)e->rp[5].p, (int32_t*)e->rp[6].p, e->stream));
    CK(d2h(e, recs, e->rp[1].p, n * sizeof(mpx_log_rec)));
    CK(d2h(e, op, e->rp[2].p, n));
    CK(d2h(e, key, e->rp[3].p, n * 8));
    CK(d2h(e, val, e->rp[4].p, n * 8));
    CK(d2h(e, last_rec, e->rp[5].p, (size_t)inst_cap * 4));
    CK(d2h(e, scalars, e->rp[6].p, 2 * sizeof(int32_t)));
    int rc = finish(e);
    if (rc == MPX_E_NIL_INSTANCE)
        return fail(e, rc, "a durable record's instNo is outside [0, inst_cap)");
    return rc;
}

// ---- diagnostics (test-only; never called on the product path) -----------------------------
int mpx_debug_kv_set_epoch(mpx_engine* e, uint32_t epoch) {
    if (!e) return MPX_E_INVAL;
    if (epoch < 1 || epoch >= mpx::kKvEpochMax)
        return fail(e, MPX_E_INVAL, "epoch must lie in [1, 2^30)");
    CK(begin(e));
    CK(ensure_kv(e));
    HIPCHK(e, hipMemcpyAsync(e->kv.epoch, &epoch, sizeof epoch, hipMemcpyHostToDevice, e->stream));
    return finish(e);
}

int mpx_debug_kv_set_small_tag(mpx_engine* e, uint32_t tag) {
    if (!e) return MPX_E_INVAL;
    if (tag >= mpx::kSmallTagMax - 1) return fail(e, MPX_E_INVAL, "tag must lie in [0, 2^18 - 1)");
    CK(begin(e));
    CK(ensure_kv(e));
    // the heads carry the tags of earlier calls: a tag moved backwards would let a later call
    // follow one of them, so every head is cleared with the move (as at the wrap)
    HIPCHK(e, hipMemsetAsync(e->kv.lhead, 0, (e->kv.cap + 1) * 4, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->kv.probe + mpx::kSmallCtl + 1, &tag, sizeof tag,
                             hipMemcpyHostToDevice, e->stream));
    return finish(e);
}

int mpx_debug_kv_state(mpx_engine* e, uint32_t* state, size_t cap, size_t* n) {
    if (!e) return MPX_E_INVAL;
    if (!n || (cap && !state)) return fail(e, MPX_E_INVAL, "null or invalid argument");
    CK(begin(e));
    CK(ensure_kv(e));
    *n = (size_t)e->kv.cap + 1;
    CK(d2h(e, state, e->kv.state, std::min<size_t>(cap, *n) * sizeof(uint32_t)));
    return finish(e);
}

// ---- device memory, streams, events (the engine's HIP runtime) --------------------------------
int mpx_dev_alloc(mpx_engine* e, size_t bytes, void** out) {
    if (!e) return MPX_E_INVAL;
    if (!out) return fail(e, MPX_E_INVAL, "null or invalid argument");
    *out = nullptr;
    HIPCHK(e, hipSetDevice(e->device));
    if (hipMalloc(out, bytes ? bytes : 1) != hipSuccess) {
        (void)hipGetLastError();
        *out = nullptr;
        return fail(e, MPX_E_NOMEM, "device allocation of " + std::to_string(bytes) + " bytes failed");
    }
    return MPX_OK;
}

int mpx_dev_free(mpx_engine* e, void* d) {
    if (!e) return MPX_E_INVAL;
    if (!d) return MPX_OK;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipFree(d));
    return MPX_OK;
}

int mpx_memcpy_async(mpx_engine* e, void* dst, const void* src, size_t bytes, int kind,
                     void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!bytes) return MPX_OK;
    if (!dst || !src) return fail(e, MPX_E_INVAL, "null copy pointer");
    hipMemcpyKind k;
    switch (kind) {
        case MPX_COPY_H2D: k = hipMemcpyHostToDevice; break;
        case MPX_COPY_D2H: k = hipMemcpyDeviceToHost; break;
        case MPX_COPY_D2D: k = hipMemcpyDeviceToDevice; break;
        default: return fail(e, MPX_E_INVAL, "unknown copy kind");
    }
    HIPCHK(e, hipMemcpyAsync(dst, src, bytes, k, pick(e, stream)));
    return MPX_OK;
}

int mpx_memset_async(mpx_engine* e, void* d, int byte_value, size_t bytes, void* stream) {
    if (!e) return MPX_E_INVAL;
    if (!bytes) return MPX_OK;
    if (!d) return fail(e, MPX_E_INVAL, "null memset pointer");
    HIPCHK(e, hipMemsetAsync(d, byte_value, bytes, pick(e, stream)));
    return MPX_OK;
}

int mpx_stream_create(mpx_engine* e, void** out) {
    if (!e) return MPX_E_INVAL;
    if (!out) return fail(e, MPX_E_INVAL, "null or invalid argument");
    HIPCHK(e, hipSetDevice(e->device));
    hipStream_t s = nullptr;
    HIPCHK(e, hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *out = (void*)s;
    return MPX_OK;
}

int mpx_stream_destroy(mpx_engine* e, void* s) {
    if (!e) return MPX_E_INVAL;
    if (!s || s == (void*)e->stream) return fail(e, MPX_E_INVAL, "not a stream of mpx_stream_create");
    HIPCHK(e, hipStreamDestroy((hipStream_t)s));
    return MPX_OK;
}

int mpx_stream_synchronize(mpx_engine* e, void* s) {
    if (!e) return MPX_E_INVAL;
    HIPCHK(e, hipStreamSynchronize(pick(e, s)));
    return MPX_OK;
}

int mpx_event_create(mpx_engine* e, int timing, void** out) {
    if (!e) return MPX_E_INVAL;
    if (!out) return fail(e, MPX_E_INVAL, "null or invalid argument");
    HIPCHK(e, hipSetDevice(e->device));
    hipEvent_t ev = nullptr;
    HIPCHK(e, hipEventCreateWithFlags(&ev, timing ? hipEventDefault : hipEventDisableTiming));
    *out = (void*)ev;
    return MPX_OK;
}

int mpx_event_destroy(mpx_engine* e, void* ev) {
    if (!e) return MPX_E_INVAL;
    if (!ev) return fail(e, MPX_E_INVAL, "null or invalid argument");
    // a destroyed event never stays registered as the group step's timing hook: the pair is
    // unregistered together (the hook records both or neither)
    if ((hipEvent_t)ev == e->ev_fast0 || (hipEvent_t)ev == e->ev_fast1)
        e->ev_fast0 = e->ev_fast1 = nullptr;
    HIPCHK(e, hipEventDestroy((hipEvent_t)ev));
    return MPX_OK;
}

int mpx_event_record(mpx_engine* e, void* ev, void* s) {
    if (!e) return MPX_E_INVAL;
    if (!ev) return fail(e, MPX_E_INVAL, "null or invalid argument");
    HIPCHK(e, hipEventRecord((hipEvent_t)ev, pick(e, s)));
    return MPX_OK;
}

int mpx_stream_wait_event(mpx_engine* e, void* s, void* ev) {
    if (!e) return MPX_E_INVAL;
    if (!ev) return fail(e, MPX_E_INVAL, "null or invalid argument");
    HIPCHK(e, hipStreamWaitEvent(pick(e, s), (hipEvent_t)ev, 0));
    return MPX_OK;
}

int mpx_event_elapsed_ms(mpx_engine* e, void* ev0, void* ev1, float* ms) {
    if (!e) return MPX_E_INVAL;
    if (!ev0 || !ev1 || !ms) return fail(e, MPX_E_INVAL, "null or invalid argument");
    HIPCHK(e, hipEventElapsedTime(ms, (hipEvent_t)ev0, (hipEvent_t)ev1));
    return MPX_OK;
}

// ---- hipGraph capture ----------------------------------------------------------------------------
int mpx_graph_begin(mpx_engine* e, void* s) {
    if (!e) return MPX_E_INVAL;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamBeginCapture(pick(e, s), hipStreamCaptureModeRelaxed));
    return MPX_OK;
}

int mpx_graph_end(mpx_engine* e, void* s, void** exec_out) {
    if (!e) return MPX_E_INVAL;
    if (!exec_out) return fail(e, MPX_E_INVAL, "null exec_out");
    *exec_out = nullptr;
    hipGraph_t g = nullptr;
    HIPCHK(e, hipStreamEndCapture(pick(e, s), &g));
    hipGraphExec_t x = nullptr;
    const hipError_t r = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (r != hipSuccess) return hip_fail(e, "hipGraphInstantiate", r);
    *exec_out = (void*)x;
    return MPX_OK;
}

int mpx_graph_launch(mpx_engine* e, void* exec, void* s) {
    if (!e) return MPX_E_INVAL;
    if (!exec) return fail(e, MPX_E_INVAL, "null graph");
    HIPCHK(e, hipGraphLaunch((hipGraphExec_t)exec, pick(e, s)));
    return MPX_OK;
}

int mpx_graph_destroy(mpx_engine* e, void* exec) {
    if (!e) return MPX_E_INVAL;
    if (!exec) return fail(e, MPX_E_INVAL, "null graph");
    HIPCHK(e, hipGraphExecDestroy((hipGraphExec_t)exec));
    return MPX_OK;
}

int mpx_runtime_info(char* buf, size_t cap) {
    int rt = 0, drv = 0, nv = 0;
    (void)hipRuntimeGetVersion(&rt);
    (void)hipDriverGetVersion(&drv);
    (void)ncclGetVersion(&nv);
    (void)hipGetLastError();
    auto path_of = [](const void* sym) {
        Dl_info info{};
        return (sym && dladdr(sym, &info) && info.dli_fname) ? std::string(info.dli_fname)
                                                              : std::string("?");
    };
    const std::string s = "{\"hip_runtime\": " + std::to_string(rt) +
                          ", \"hip_driver\": " + std::to_string(drv) +
                          ", \"rccl\": " + std::to_string(nv) + ", \"hip_path\": \"" +
                          path_of((const void*)&hipRuntimeGetVersion) + "\", \"rccl_path\": \"" +
                          path_of((const void*)&ncclAllReduce) + "\"}";
    if (buf && cap) {
        const size_t k = std::min(cap - 1, s.size());
        memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (int)s.size();
}

}  // extern "C"
