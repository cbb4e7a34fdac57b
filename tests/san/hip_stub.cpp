// tests/san/hip_stub.cpp — TEST INFRASTRUCTURE ONLY: a host-memory stand-in for the HIP / RCCL
// runtime calls engine.cpp makes, so the C ABI's host side can be built and run on a CPU.
// "Device" memory is host memory, copies are memcpy, every call completes before it returns
// (so stream and event order hold trivially) and events carry a host timestamp.
//
// Two builds (never shipped, never loaded by the product path):
//   * default (tests/test_sanitize.py): kernel launchers enqueue nothing; engine.cpp's argument
//     validation, staging and error paths run under ASan + UBSan.
//   * -DMPX_STUB_ORACLE=1 (tests/test_dist.py, libmpx_stub.so): the group-step launchers run the
//     CPU oracle (oracle/oracle.cpp, linked into the stub) and the RCCL calls really reduce across
//     PROCESSES — every rank maps one /dev/shm segment named after the unique id, deposits its
//     buffer in its slot, waits at a barrier, and reads the reduction of all slots. That is what
//     lets bench.py's multi-rank step (engine.cpp's nranks > 1 path: comm init, the fused
//     max + sum group, double-buffered watermark vectors) run end to end without a GPU.
// MPX_STUB_DEVICES (default 1) sets the device count the stub reports.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../minpaxos_amd/csrc/kernels.hpp"

namespace {
double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

// ---- cross-process communicator: one shared segment per unique id ---------------------------
constexpr size_t kSlotBytes = 64ull << 20;  // per rank (sparse: only touched pages use memory)
constexpr int kMaxRanks = 16;
struct ShmHeader {
    std::atomic<uint32_t> arrived;
    std::atomic<uint32_t> generation;
    std::atomic<uint32_t> joined;
    uint32_t nranks;
};
struct StubComm {
    ShmHeader* hdr = nullptr;
    char* slots = nullptr;
    size_t map_bytes = 0;
    int nranks = 1, rank = 0;
    char name[64] = {0};
};

// sense-reversing barrier over the segment; false after 120 s (a peer died)
bool barrier(StubComm* c) {
    if (c->nranks == 1) return true;
    const uint32_t gen = c->hdr->generation.load(std::memory_order_acquire);
    if (c->hdr->arrived.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)c->nranks - 1) {
        c->hdr->arrived.store(0, std::memory_order_relaxed);
        c->hdr->generation.fetch_add(1, std::memory_order_acq_rel);
        return true;
    }
    const double t0 = now_s();
    while (c->hdr->generation.load(std::memory_order_acquire) == gen) {
        sched_yield();
        if (now_s() - t0 > 120.0) return false;
    }
    return true;
}

template <typename T>
void reduce_into(T* d, const char* slots, int nranks, size_t n, ncclRedOp_t op) {
    for (size_t i = 0; i < n; ++i) {
        T acc = reinterpret_cast<const T*>(slots)[i];
        for (int r = 1; r < nranks; ++r) {
            const T v = reinterpret_cast<const T*>(slots + (size_t)r * kSlotBytes)[i];
            switch (op) {
                case ncclMax: acc = v > acc ? v : acc; break;
                case ncclMin: acc = v < acc ? v : acc; break;
                default: acc = (T)(acc + v); break;
            }
        }
        d[i] = acc;
    }
}

size_t el_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 4;
    }
}

int stub_devices() {
    const char* s = getenv("MPX_STUB_DEVICES");
    const int n = s ? atoi(s) : 1;
    return n > 0 ? n : 1;
}
}  // namespace

extern "C" {
hipError_t hipSetDevice(int d) { return d >= 0 && d < stub_devices() ? hipSuccess : hipErrorInvalidDevice; }
hipError_t hipGetDeviceCount(int* c) { *c = stub_devices(); return hipSuccess; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
    *s = reinterpret_cast<hipStream_t>(malloc(8));
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) { free(s); return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamQuery(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned int) { return hipSuccess; }
hipError_t hipDeviceSynchronize(void) { return hipSuccess; }
hipError_t hipMalloc(void** p, size_t n) { *p = calloc(1, n ? n : 1); return *p ? hipSuccess : hipErrorOutOfMemory; }
hipError_t hipFree(void* p) { free(p); return hipSuccess; }
hipError_t hipHostMalloc(void** p, size_t n, unsigned int) {
    *p = calloc(1, n ? n : 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipHostFree(void* p) { free(p); return hipSuccess; }
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int) { *d = h; return hipSuccess; }
hipError_t hipMemset(void* p, int v, size_t n) { memset(p, v, n); return hipSuccess; }
hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) { memset(p, v, n); return hipSuccess; }
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
    memmove(d, s, n);
    return hipSuccess;
}
hipError_t hipGetLastError(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "stub"; }
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
    *e = reinterpret_cast<hipEvent_t>(calloc(1, sizeof(double)));
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) { free(e); return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t e, hipStream_t) {
    *reinterpret_cast<double*>(e) = now_s();  // the work before it has completed (synchronous)
    return hipSuccess;
}
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
    *ms = (float)((*reinterpret_cast<double*>(b) - *reinterpret_cast<double*>(a)) * 1e3);
    return hipSuccess;
}
// graph capture: the stub runs every call at once, so it has nothing to record
hipError_t hipStreamBeginCapture(hipStream_t, hipStreamCaptureMode) { return hipErrorNotSupported; }
hipError_t hipStreamEndCapture(hipStream_t, hipGraph_t*) { return hipErrorNotSupported; }
hipError_t hipGraphInstantiate(hipGraphExec_t*, hipGraph_t, hipGraphNode_t*, char*, size_t) {
    return hipErrorNotSupported;
}
hipError_t hipGraphDestroy(hipGraph_t) { return hipErrorNotSupported; }
hipError_t hipGraphLaunch(hipGraphExec_t, hipStream_t) { return hipErrorNotSupported; }
hipError_t hipGraphExecDestroy(hipGraphExec_t) { return hipErrorNotSupported; }
hipError_t hipRuntimeGetVersion(int* v) { *v = 1; return hipSuccess; }
hipError_t hipDriverGetVersion(int* v) { *v = 1; return hipSuccess; }

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    memset(id, 0, sizeof(*id));
    int fd = open("/dev/urandom", O_RDONLY);
    if (fd < 0 || read(fd, id->internal, 16) != 16) {
        if (fd >= 0) close(fd);
        return ncclSystemError;
    }
    close(fd);
    return ncclSuccess;
}
ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
    if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    StubComm* c = new StubComm();
    c->nranks = nranks;
    c->rank = rank;
    char* p = c->name + snprintf(c->name, sizeof c->name, "/mpxstub_");
    for (int i = 0; i < 16; ++i) p += sprintf(p, "%02x", (unsigned char)id.internal[i]);
    c->map_bytes = 4096 + (size_t)nranks * kSlotBytes;
    int fd = shm_open(c->name, O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)c->map_bytes) != 0) {
        if (fd >= 0) close(fd);
        delete c;
        return ncclSystemError;
    }
    void* m = mmap(nullptr, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        delete c;
        return ncclSystemError;
    }
    c->hdr = reinterpret_cast<ShmHeader*>(m);  // a fresh segment is zero-filled
    c->slots = reinterpret_cast<char*>(m) + 4096;
    c->hdr->joined.fetch_add(1);
    if (!barrier(c)) {
        munmap(m, c->map_bytes);
        delete c;
        return ncclSystemError;
    }
    if (rank == 0) shm_unlink(c->name);  // every rank has it mapped: nothing left in /dev/shm
    *out = reinterpret_cast<ncclComm_t>(c);
    return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t h) {
    StubComm* c = reinterpret_cast<StubComm*>(h);
    if (c) {
        munmap(c->hdr, c->map_bytes);
        delete c;
    }
    return ncclSuccess;
}
ncclResult_t ncclAllReduce(const void* s, void* d, size_t n, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t h, hipStream_t) {
    StubComm* c = reinterpret_cast<StubComm*>(h);
    const size_t bytes = n * el_size(t);
    if (!c || bytes > kSlotBytes) return ncclInvalidArgument;
    memcpy(c->slots + (size_t)c->rank * kSlotBytes, s, bytes);
    if (!barrier(c)) return ncclSystemError;  // every rank has deposited its buffer
    switch (t) {
        case ncclInt64: reduce_into((int64_t*)d, c->slots, c->nranks, n, op); break;
        case ncclUint64: reduce_into((uint64_t*)d, c->slots, c->nranks, n, op); break;
        case ncclUint32: reduce_into((uint32_t*)d, c->slots, c->nranks, n, op); break;
        default: reduce_into((int32_t*)d, c->slots, c->nranks, n, op); break;
    }
    if (!barrier(c)) return ncclSystemError;  // every rank has read the slots
    return ncclSuccess;
}
// the calls inside a group complete one by one, in the same order on every rank
ncclResult_t ncclGroupStart(void) { return ncclSuccess; }
ncclResult_t ncclGroupEnd(void) { return ncclSuccess; }
const char* ncclGetErrorString(ncclResult_t) { return "stub"; }
ncclResult_t ncclGetVersion(int* v) { *v = 1; return ncclSuccess; }
}

#if MPX_STUB_ORACLE
extern "C" int orc_group_step(int N, int mode, const mpx_group_batch* b, uint32_t kv_per_group);
#endif

namespace mpx {
hipError_t launch_accept_tally(int, const mpx_accept_reply*, uint64_t, const mpx_inst_state*,
                               mpx_inst_state*, uint64_t, int32_t, int32_t, int32_t*, uint8_t*,
                               unsigned long long*, uint32_t*, uint32_t*, hipStream_t) { return hipSuccess; }
hipError_t launch_committed_prefix(const mpx_inst_state*, uint64_t, int32_t, int32_t*,
                                   unsigned long long*, hipStream_t) { return hipSuccess; }
hipError_t launch_prepare_classic(const mpx_prepare_reply*, uint64_t, const mpx_prep_state*,
                                  mpx_prep_state*, uint64_t, int32_t, int32_t, int32_t*, uint8_t*,
                                  uint32_t*, uint32_t*, hipStream_t) { return hipSuccess; }
hipError_t launch_prepare_min(const mpx_prepare_reply_min*, uint64_t, const uint64_t*,
                              mpx_group_prep_state*, uint64_t, int32_t, int32_t*,
                              mpx_prepare_effect*, uint32_t*, hipStream_t) { return hipSuccess; }
hipError_t launch_conflict_batch(const uint8_t*, const int64_t*, const uint64_t*, uint64_t,
                                 uint8_t*, hipStream_t) { return hipSuccess; }
#if MPX_STUB_ORACLE
bool step_one_launch_fits(int32_t, uint32_t, uint32_t) { return true; }
// the group step through the oracle; its error codes become the kernels' error-word bits
hipError_t launch_step_totals(const mpx_group_batch* b, int64_t* totals, uint32_t*, hipStream_t);
hipError_t launch_group_step(int mode, int32_t nrep, uint32_t kv_per_group, const mpx_group_batch* b,
                             uint32_t*, uint32_t* ctl, int64_t* totals, uint32_t* err,
                             hipStream_t s, hipEvent_t ev0, hipEvent_t ev1, unsigned long long*) {
    if (ev0) hipEventRecord(ev0, s);
    // the fused form needs the per-group decided counts the oracle writes to n_decided
    std::vector<uint32_t> nd;
    mpx_group_batch bb = *b;
    if (totals && !bb.n_decided) {
        nd.resize(b->n_groups);
        bb.n_decided = nd.data();
    }
    const int rc = orc_group_step(nrep, mode, &bb, kv_per_group);
    if (rc == MPX_E_NIL_INSTANCE) *err |= kErrNil;
    else if (rc == MPX_E_BAD_ID) *err |= kErrBadId;
    else if (rc == MPX_E_KV_FULL) *err |= kErrKvFull;
    else if (rc) *err |= kErrInval;
    if (ev1) hipEventRecord(ev1, s);
    return totals ? launch_step_totals(&bb, totals, ctl, s) : hipSuccess;
}
// k_step_totals (step.hip) over host memory
hipError_t launch_step_totals(const mpx_group_batch* b, int64_t* totals, uint32_t*, hipStream_t) {
    int64_t d = 0, xi = 0, xc = 0;
    for (uint32_t g = 0; g < b->n_groups; ++g) {
        d += b->n_decided[g];
        const int64_t ei = b->executed_in[g], eo = b->executed_out[g];
        const int64_t lo = ei + 1 < 0 ? 0 : ei + 1;
        if (eo >= lo && eo < (int64_t)b->ipg) {
            const uint64_t gi0 = (uint64_t)g * b->ipg;
            xi += eo - lo + 1;
            xc += b->cmd_off[gi0 + eo + 1] - b->cmd_off[gi0 + lo];
        }
    }
    totals[0] = d;
    totals[1] = xi;
    totals[2] = xc;
    return hipSuccess;
}
#else
bool step_one_launch_fits(int32_t, uint32_t, uint32_t) { return true; }
hipError_t launch_group_step(int, int32_t, uint32_t, const mpx_group_batch*, uint32_t*, uint32_t*,
                             int64_t*, uint32_t*, hipStream_t, hipEvent_t, hipEvent_t,
                             unsigned long long*) { return hipSuccess; }
hipError_t launch_step_totals(const mpx_group_batch*, int64_t*, uint32_t*, hipStream_t) { return hipSuccess; }
#endif
uint64_t apply_chunk_commands(uint64_t c, uint64_t m) { return c ? c : m; }
// the engine's pinned-staging branch for replica-sized calls (same rule as apply.hip)
bool apply_is_one_launch(const ApplyOpts& o, uint64_t m) {
    return m && m <= MPX_APPLY_SMALL_MAX && (o.path == MPX_APPLY_AUTO || o.path == MPX_APPLY_SMALL);
}
uint64_t apply_work_bytes(const KvTable&, const ApplyOpts&, uint64_t m) { return 48 * m + 256; }
uint64_t apply_reserve_bytes(const KvTable&, const ApplyOpts&, uint64_t m) { return 48 * m + 256; }
hipError_t launch_apply(KvTable&, const uint8_t*, const int64_t*, const int64_t*, uint64_t,
                        int64_t*, uint8_t*, const ApplyOpts&, ApplyWork&, uint32_t*, hipStream_t) { return hipSuccess; }
// the replica-batch form: nothing to compute on the stub, but the call completes (its flag)
hipError_t launch_apply_small(KvTable&, const uint8_t*, const int64_t*, const int64_t*, uint64_t,
                              int64_t*, uint8_t*, uint32_t*, hipStream_t, uint32_t* done,
                              uint32_t seq, bool) {
    if (done) *done = seq;
    return hipSuccess;
}
hipError_t launch_kv_clear(KvTable&, hipStream_t) { return hipSuccess; }
hipError_t launch_kv_import(KvTable&, const int64_t*, const int64_t*, uint64_t, uint32_t*,
                            hipStream_t) { return hipSuccess; }
hipError_t launch_kv_export(KvTable&, int64_t*, int64_t*, uint64_t, unsigned long long*,
                            hipStream_t) { return hipSuccess; }
uint64_t decode_work_bytes(uint64_t len) { return len / 8 + 256; }
hipError_t launch_decode_peer_stream(const uint8_t*, uint64_t, mpx_accept_reply*, uint64_t,
                                     mpx_peer_frame*, uint64_t, mpx_decode_result*, void*,
                                     uint64_t, hipStream_t) { return hipSuccess; }
uint64_t stream_work_bytes(uint64_t len) { return len + 256; }
hipError_t launch_decode_stream(int, int, const uint8_t*, uint64_t, uint64_t, const StreamOuts&,
                                mpx_stream_result*, void*, uint64_t, hipStream_t) { return hipSuccess; }
uint64_t fanout_work_bytes(uint64_t n) { return 8 * n + 256; }
hipError_t launch_encode_replies(const mpx_reply_rec*, uint64_t, uint32_t, uint8_t, int32_t,
                                 uint8_t*, uint64_t*, void*, uint64_t, uint32_t*, hipStream_t) { return hipSuccess; }
uint64_t logenc_work_bytes(uint64_t n, uint64_t) { return 8 * n + 256; }
uint64_t logenc_max_bytes(uint64_t n, uint64_t m) { return 18 * n + 17 * m; }
hipError_t launch_encode_log(int, const mpx_log_rec*, uint64_t, const uint64_t*, const uint8_t*,
                             const int64_t*, const int64_t*, uint64_t, uint8_t*, uint64_t*, void*,
                             uint64_t, hipStream_t) { return hipSuccess; }
hipError_t launch_replay_durable(const uint8_t*, uint64_t, int32_t, int32_t, mpx_log_rec*,
                                 uint8_t*, int64_t*, int64_t*, int32_t*, int32_t*, uint32_t*,
                                 void*, uint64_t, hipStream_t) { return hipSuccess; }
uint64_t replay_work_bytes(uint64_t n, int32_t) { return 16 * n + 256; }
}  // namespace mpx
