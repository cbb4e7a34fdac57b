// tests/san/hip_stub.cpp — TEST INFRASTRUCTURE ONLY: a host-memory stand-in for the HIP / RCCL
// runtime calls engine.cpp makes, plus no-op kernel launchers, so the C ABI's host-side code
// (argument validation, staging, the decode loop, error reporting) can be built and run under
// AddressSanitizer + UBSan on a CPU. "Device" memory is host memory; copies are
// memcpy; launchers enqueue nothing.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>

#include "../../minpaxos_amd/csrc/kernels.hpp"

extern "C" {
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipGetDeviceCount(int* c) { *c = 1; return hipSuccess; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
    *s = reinterpret_cast<hipStream_t>(malloc(8));
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) { free(s); return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned int) { return hipSuccess; }
hipError_t hipDeviceSynchronize(void) { return hipSuccess; }
hipError_t hipMalloc(void** p, size_t n) { *p = calloc(1, n ? n : 1); return *p ? hipSuccess : hipErrorOutOfMemory; }
hipError_t hipFree(void* p) { free(p); return hipSuccess; }
hipError_t hipMemset(void* p, int v, size_t n) { memset(p, v, n); return hipSuccess; }
hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) { memset(p, v, n); return hipSuccess; }
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
    memmove(d, s, n);
    return hipSuccess;
}
hipError_t hipGetLastError(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "stub"; }
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
    *e = reinterpret_cast<hipEvent_t>(malloc(8));
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) { free(e); return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) { *ms = 0.f; return hipSuccess; }
hipError_t hipRuntimeGetVersion(int* v) { *v = 1; return hipSuccess; }
hipError_t hipDriverGetVersion(int* v) { *v = 1; return hipSuccess; }
ncclResult_t ncclGetUniqueId(ncclUniqueId* id) { memset(id, 7, sizeof(*id)); return ncclSuccess; }
ncclResult_t ncclCommInitRank(ncclComm_t* c, int, ncclUniqueId, int) {
    *c = reinterpret_cast<ncclComm_t>(malloc(8));
    return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t c) { free(c); return ncclSuccess; }
ncclResult_t ncclAllReduce(const void* s, void* d, size_t n, ncclDataType_t t, ncclRedOp_t,
                           ncclComm_t, hipStream_t) {
    const size_t el = t == ncclInt64 ? 8 : 4;
    memmove(d, s, n * el);  // one rank: the reduction is the identity
    return ncclSuccess;
}
ncclResult_t ncclGroupStart(void) { return ncclSuccess; }
ncclResult_t ncclGroupEnd(void) { return ncclSuccess; }
const char* ncclGetErrorString(ncclResult_t) { return "stub"; }
ncclResult_t ncclGetVersion(int* v) { *v = 1; return ncclSuccess; }
}

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
hipError_t launch_group_step(int, int32_t, uint32_t, const mpx_group_batch*, uint32_t*, uint32_t*,
                             uint32_t*, hipStream_t) { return hipSuccess; }
hipError_t launch_step_totals(const mpx_group_batch*, int64_t*, uint32_t*, hipStream_t) { return hipSuccess; }
uint64_t apply_chunk_commands(uint64_t c, uint64_t m) { return c ? c : m; }
uint64_t apply_work_bytes(const KvTable&, uint64_t, uint64_t m) { return 48 * m + 256; }
uint64_t apply_reserve_bytes(const KvTable&, uint64_t, uint64_t m) { return 48 * m + 256; }
hipError_t launch_apply(KvTable&, const uint8_t*, const int64_t*, const int64_t*, uint64_t,
                        int64_t*, uint8_t*, uint64_t, ApplyWork&, uint32_t*, hipStream_t) { return hipSuccess; }
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
                                 hipStream_t) { return hipSuccess; }
}  // namespace mpx
