// fanout.hip — client reply fan-out.
//
// Reference: the leader answers every command of a decided instance with a
// genericsmrproto.ProposeReplyTS{OK, CommandId, Value, Timestamp, Leader}
// (genericsmrproto.go:31-37) written to the proposing client's connection:
//   at decide time  bareminpaxos.go:1030-1042 (Value = state.NIL, unless -dreply)
//   at apply time   bareminpaxos.go:1076-1084 (Value = Execute's return, with -dreply)
// through genericsmr.(*Replica).ReplyProposeTS (genericsmr.go:529-535), whose Marshal
// (gsmrprotomarsh.go:702-732) writes 25 bytes: OK u8, CommandId i32, Value i64, Timestamp i64,
// Leader i32, little endian, no frame code.
// The engine takes a batch of replies in execution order and produces, for every client
// connection, the exact byte run its bufio.Writer would receive: the replies are stably
// partitioned by client (rocPRIM radix sort of the client id with the reply index as payload;
// per-client order = execution order; carrying the 24-byte records through the sort instead
// measured slower, rocPRIM leaves onesweep for values that wide), then each block gathers 256
// replies, assembles their 25-byte encodings in LDS and stores the 6400-byte run with 16-byte
// vector stores.
// client_off[c] = byte offset of client c's run; client_off[n_clients] = 25 n.
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "common.hpp"
#include "kernels.hpp"

namespace mpx {

namespace {
constexpr int kFanBlock = 256;
constexpr int kRecBytes = 25;

unsigned bits_for_clients(uint32_t c) {  // bits to represent every client id < c
    unsigned b = 1;
    while ((1ull << b) < c) ++b;
    return b;
}
}  // namespace

struct ClientOf {
    __host__ __device__ uint32_t operator()(const mpx_reply_rec& r) const { return r.client; }
};
using ClientKeys = rocprim::transform_iterator<const mpx_reply_rec*, ClientOf, uint32_t>;

template <bool kAligned>
__global__ __launch_bounds__(kFanBlock) void k_fan_encode(
    const mpx_reply_rec* __restrict__ recs, const uint32_t* __restrict__ skeys,
    const uint32_t* __restrict__ perm, uint64_t n, uint32_t n_clients, uint8_t ok, int32_t leader,
    uint8_t* __restrict__ out, uint64_t* __restrict__ client_off, uint32_t* err) {
    __shared__ __attribute__((aligned(16))) uint8_t S[kFanBlock * kRecBytes];
    const uint64_t q0 = (uint64_t)blockIdx.x * kFanBlock;
    const uint64_t q = q0 + threadIdx.x;
    const uint32_t cnt = (uint32_t)(n - q0 < (uint64_t)kFanBlock ? n - q0 : kFanBlock);
    if (q < n) {
        const mpx_reply_rec r = recs[perm[q]];
        uint8_t* b = S + threadIdx.x * kRecBytes;
        b[0] = ok;
        const uint32_t cid = (uint32_t)r.command_id;
        const uint64_t v = (uint64_t)r.value, ts = (uint64_t)r.timestamp;
        const uint32_t ld = (uint32_t)leader;
#pragma unroll
        for (int k = 0; k < 4; ++k) b[1 + k] = (uint8_t)(cid >> (8 * k));
#pragma unroll
        for (int k = 0; k < 8; ++k) b[5 + k] = (uint8_t)(v >> (8 * k));
#pragma unroll
        for (int k = 0; k < 8; ++k) b[13 + k] = (uint8_t)(ts >> (8 * k));
#pragma unroll
        for (int k = 0; k < 4; ++k) b[21 + k] = (uint8_t)(ld >> (8 * k));
        // client run boundaries: every client id in (previous key, this key] starts here. A
        // client id >= n_clients (sorted on its low bits only) fails the call; it is clamped so
        // no offset outside client_off is ever written.
        if (r.client >= n_clients) raise_err(err, kErrInval);
        const int64_t c = skeys[q] < n_clients ? (int64_t)skeys[q] : (int64_t)n_clients - 1;
        const int64_t prev = q == 0 ? -1
                                    : (skeys[q - 1] < n_clients ? (int64_t)skeys[q - 1]
                                                                : (int64_t)n_clients - 1);
        for (int64_t x = prev + 1; x <= c; ++x) client_off[x] = q * kRecBytes;
        if (q + 1 == n)
            for (uint64_t x = (uint64_t)c + 1; x <= n_clients; ++x) client_off[x] = n * kRecBytes;
    }
    __syncthreads();
    const uint32_t bytes = cnt * kRecBytes;
    uint8_t* dst = out + q0 * kRecBytes;
    if (kAligned) {  // q0 * 25 is a multiple of 16: full 16-byte vectors, then the tail
        const uint32_t nv = bytes / 16;
        for (uint32_t i = threadIdx.x; i < nv; i += kFanBlock)
            st_stream(reinterpret_cast<uint4*>(dst) + i, reinterpret_cast<const uint4*>(S)[i]);
        for (uint32_t i = nv * 16 + threadIdx.x; i < bytes; i += kFanBlock) dst[i] = S[i];
    } else {
        for (uint32_t i = threadIdx.x; i < bytes; i += kFanBlock) dst[i] = S[i];
    }
}

__global__ void k_fan_empty(uint64_t* client_off, uint32_t n_clients) {
    for (uint32_t x = threadIdx.x; x <= n_clients; x += blockDim.x) client_off[x] = 0;
}

uint64_t fanout_work_bytes(uint64_t n) {
    size_t tmp = 0;
    const uint64_t m = n ? n : 1;
    (void)rocprim::radix_sort_pairs(nullptr, tmp, ClientKeys(nullptr, ClientOf()),
                                    (uint32_t*)nullptr, rocprim::counting_iterator<uint32_t>(0),
                                    (uint32_t*)nullptr, (size_t)m, 0u, 32u);
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    return 2 * al(m * 4) + al(tmp);
}

hipError_t launch_encode_replies(const mpx_reply_rec* recs, uint64_t n, uint32_t n_clients,
                                 uint8_t ok, int32_t leader, uint8_t* out, uint64_t* client_off,
                                 void* work, uint64_t work_bytes, uint32_t* err,
                                 hipStream_t stream) {
    if (!n_clients || n >= (1ull << 32)) return hipErrorInvalidValue;
    if (work_bytes < fanout_work_bytes(n)) return hipErrorInvalidValue;
    if (n == 0) {
        k_fan_empty<<<1, 256, 0, stream>>>(client_off, n_clients);
        return hipGetLastError();
    }
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    char* w = (char*)work;
    uint32_t* skeys = (uint32_t*)w;
    uint32_t* perm = (uint32_t*)(w + al(n * 4));
    void* tmp = w + 2 * al(n * 4);
    size_t tmp_bytes = work_bytes - 2 * al(n * 4);
    // keys read straight from the records (no separate key pass)
    hipError_t r = rocprim::radix_sort_pairs(tmp, tmp_bytes, ClientKeys(recs, ClientOf()), skeys,
                                             rocprim::counting_iterator<uint32_t>(0), perm,
                                             (size_t)n, 0u, bits_for_clients(n_clients), stream);
    if (r != hipSuccess) return r;
    const unsigned blocks = (unsigned)((n + kFanBlock - 1) / kFanBlock);
    if (((uintptr_t)out & 15) == 0)
        k_fan_encode<true><<<blocks, kFanBlock, 0, stream>>>(recs, skeys, perm, n, n_clients, ok,
                                                             leader, out, client_off, err);
    else
        k_fan_encode<false><<<blocks, kFanBlock, 0, stream>>>(recs, skeys, perm, n, n_clients, ok,
                                                              leader, out, client_off, err);
    return hipGetLastError();
}

}  // namespace mpx
