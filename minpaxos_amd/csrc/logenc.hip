// logenc.hip — instance-log encoding: catch-up logs and the durable log.
//
// Two byte formats of a run of log records (instance metadata + its commands):
//   MPX_LOG_CATCHUP  minpaxosproto.(*Instance).Marshal  src/minpaxosproto/minpaxosprotomarsh.go:100-124:
//                    Ballot i32, Status i32, binary.PutVarint(len(Cmds)) (zigzag varint), then
//                    state.(*Command).Marshal per command (statemarsh.go:8-19: Op u8, K i64,
//                    V i64). bcastAccept (bareminpaxos.go:488-513) sends every peer q the
//                    instances peerCommits[q]+1 .. lastCommitted, i.e. a SUFFIX of one run: the
//                    engine encodes the run once and rec_off[] gives every suffix's start.
//   MPX_LOG_DURABLE  recordInstanceMetadata (bareminpaxos.go:164-174: Ballot u32, Status u32,
//                    instNo u32) followed by recordCommands (:177-188: Command.Marshal each; a
//                    nil slice writes nothing), one record per stable-store append.
// Pipeline: k_log_sizes (bytes per record) -> rocPRIM inclusive scan (record offsets) ->
// k_log_emit, output-parallel: each 4 KB block finds its first record by binary search over the
// offsets, stages the offsets of the records it overlaps in LDS, and every thread produces 16
// consecutive output bytes and stores them as one vector (coalesced, no partial lines except at
// the run's two ends).
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "common.hpp"
#include "kernels.hpp"

namespace mpx {

namespace {
constexpr int kLogBlock = 256;
constexpr int kLogBlockBytes = kLogBlock * 16;
// the fewest bytes a record can take (catch-up: 8 + a 1-byte varint; durable: 12)
constexpr int kLogMinRec = 9;
constexpr int kLogMaxRecs = kLogBlockBytes / kLogMinRec + 2;

__device__ __forceinline__ uint64_t zigzag(int64_t x) {  // binary.PutVarint's mapping
    return x < 0 ? ~((uint64_t)x << 1) : (uint64_t)x << 1;
}
__device__ __forceinline__ uint32_t uvarint_len(uint64_t u) {
    uint32_t l = 1;
    while (u >= 0x80) {
        u >>= 7;
        ++l;
    }
    return l;
}
__device__ __forceinline__ uint32_t uvarint_byte(uint64_t u, uint32_t k) {
    u >>= 7 * k;
    return (uint32_t)(u & 0x7F) | (u >= 0x80 ? 0x80u : 0u);
}
__device__ __forceinline__ uint32_t hdr_bytes(int format, uint64_t ncmd) {
    return format == MPX_LOG_CATCHUP ? 8u + uvarint_len(zigzag((int64_t)ncmd)) : 12u;
}
}  // namespace

__global__ __launch_bounds__(256) void k_log_sizes(int format, const uint64_t* __restrict__ cmd_off,
                                                   uint64_t n, uint64_t* __restrict__ sizes) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t nc = cmd_off[i + 1] - cmd_off[i];
        sizes[i] = hdr_bytes(format, nc) + 17 * nc;
    }
}

__global__ void k_log_zero(uint64_t* rec_off) { rec_off[0] = 0; }

// blk_first[b] = the record holding output byte b * kLogBlockBytes (a block start falls inside
// exactly one record), so no emit block has to binary-search the offsets in global memory
__global__ __launch_bounds__(256) void k_log_block_first(const uint64_t* __restrict__ rec_off,
                                                         uint64_t n, uint32_t n_blocks,
                                                         uint64_t* __restrict__ blk_first) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t s = rec_off[i], e = rec_off[i + 1];
        for (uint64_t b = (s + kLogBlockBytes - 1) / kLogBlockBytes;
             b * kLogBlockBytes < e && b < n_blocks; ++b)
            blk_first[b] = i;
    }
}

// rec_off: n+1 record offsets (rec_off[n] = total bytes)
__global__ __launch_bounds__(kLogBlock) void k_log_emit(
    int format, const mpx_log_rec* __restrict__ recs, const uint64_t* __restrict__ cmd_off,
    const uint8_t* __restrict__ op, const int64_t* __restrict__ key,
    const int64_t* __restrict__ val, uint64_t n, const uint64_t* __restrict__ rec_off,
    const uint64_t* __restrict__ blk_first, uint8_t* __restrict__ out) {
    __shared__ uint64_t off[kLogMaxRecs + 1];
    const uint64_t total = rec_off[n];
    const uint64_t b0 = (uint64_t)blockIdx.x * kLogBlockBytes;
    if (b0 >= total) return;  // uniform per block
    const uint64_t first = blk_first[blockIdx.x];
    const uint64_t b1 = b0 + kLogBlockBytes < total ? b0 + kLogBlockBytes : total;
    // offsets of the records overlapping [b0, b1), plus the end of the last one
    const uint64_t maxr = n - first < (uint64_t)kLogMaxRecs ? n - first : (uint64_t)kLogMaxRecs;
    for (uint64_t k = threadIdx.x; k <= maxr; k += kLogBlock) off[k] = rec_off[first + k];
    __syncthreads();
    // at most kLogMaxRecs - 1 records start inside one block, so off[0..maxr] covers every
    // record that overlaps it
    const uint32_t nr = (uint32_t)maxr;
    const uint64_t o0 = b0 + (uint64_t)threadIdx.x * 16;
    if (o0 >= b1) return;
    // the record holding o0
    uint32_t lo = 0, hi = nr;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (off[mid] <= o0) lo = mid;
        else hi = mid;
    }
    // walk the 16 bytes with a cursor: the record's header fields and the current command are
    // loaded once, not per byte
    uint32_t r = lo;
    uint64_t rs = 0, re = off[r], ri = 0, c0 = 0;
    uint32_t hb = 0, w_ballot = 0, w_status = 0, w_third = 0;
    uint64_t zz = 0;
    uint64_t cur_x = ~0ull, k_key = 0, k_val = 0;
    uint32_t k_op = 0;
    bool first_rec = true;
    uint32_t bytes[4] = {0, 0, 0, 0};
    const uint32_t cnt = (uint32_t)(b1 - o0 < 16 ? b1 - o0 : 16);
    for (uint32_t k = 0; k < cnt; ++k) {
        const uint64_t o = o0 + k;
        while (first_rec || o >= re) {  // (next) record
            if (!first_rec) ++r;
            first_rec = false;
            rs = off[r];
            re = off[r + 1];
            ri = first + r;
            c0 = cmd_off[ri];
            const uint64_t nc = cmd_off[ri + 1] - c0;
            hb = (uint32_t)(re - rs - 17 * nc);
            const mpx_log_rec m = recs[ri];
            w_ballot = (uint32_t)m.ballot;
            w_status = (uint32_t)m.status;
            w_third = (uint32_t)m.inst_no;
            zz = zigzag((int64_t)nc);
            cur_x = ~0ull;
        }
        const uint32_t rel = (uint32_t)(o - rs);
        uint32_t v;
        if (rel < hb) {
            if (rel < 4) v = (w_ballot >> (8 * rel)) & 0xFF;
            else if (rel < 8) v = (w_status >> (8 * (rel - 4))) & 0xFF;
            else if (format == MPX_LOG_DURABLE) v = (w_third >> (8 * (rel - 8))) & 0xFF;
            else v = uvarint_byte(zz, rel - 8);
        } else {
            const uint64_t x = rel - hb;
            if (cur_x == ~0ull || x >= cur_x + 17) {  // a new command: load it once
                cur_x = x - x % 17;
                const uint64_t j = c0 + x / 17;
                k_op = op[j];
                k_key = (uint64_t)key[j];
                k_val = (uint64_t)val[j];
            }
            const uint32_t f = (uint32_t)(x - cur_x);
            if (f == 0) v = k_op;
            else if (f < 9) v = (uint32_t)(k_key >> (8 * (f - 1))) & 0xFF;
            else v = (uint32_t)(k_val >> (8 * (f - 9))) & 0xFF;
        }
        bytes[k >> 2] |= v << (8 * (k & 3));
    }
    if (cnt == 16 && (((uintptr_t)(out + o0)) & 15) == 0) {
        *reinterpret_cast<uint4*>(out + o0) = make_uint4(bytes[0], bytes[1], bytes[2], bytes[3]);
    } else {
        for (uint32_t k = 0; k < cnt; ++k) out[o0 + k] = (uint8_t)(bytes[k >> 2] >> (8 * (k & 3)));
    }
}

uint64_t logenc_max_bytes(uint64_t n, uint64_t m) { return n * (8 + 10) + 17 * m; }

namespace {
// emit blocks: the output of n records with m commands is at most n * 18 + 17 m bytes
uint64_t blocks_for(uint64_t n, uint64_t m) {
    return (logenc_max_bytes(n, m) + kLogBlockBytes - 1) / kLogBlockBytes;
}
}  // namespace

uint64_t logenc_work_bytes(uint64_t n, uint64_t m) {
    size_t tmp = 0;
    (void)rocprim::inclusive_scan(nullptr, tmp, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                  (size_t)(n ? n : 1), rocprim::plus<uint64_t>());
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    return al((n ? n : 1) * 8) + al(tmp) + al(blocks_for(n, m) * 8);
}

hipError_t launch_encode_log(int format, const mpx_log_rec* recs, uint64_t n,
                             const uint64_t* cmd_off, const uint8_t* op, const int64_t* key,
                             const int64_t* val, uint64_t m, uint8_t* out, uint64_t* rec_off,
                             void* work, uint64_t work_bytes, hipStream_t stream) {
    if (format != MPX_LOG_CATCHUP && format != MPX_LOG_DURABLE) return hipErrorInvalidValue;
    if (work_bytes < logenc_work_bytes(n, m)) return hipErrorInvalidValue;
    k_log_zero<<<1, 1, 0, stream>>>(rec_off);
    if (n == 0) return hipGetLastError();
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t blocks = blocks_for(n, m);
    uint64_t* sizes = (uint64_t*)work;
    uint64_t* blk_first = (uint64_t*)((char*)work + al(n * 8));
    void* tmp = (char*)blk_first + al(blocks * 8);
    size_t tmp_bytes = work_bytes - al(n * 8) - al(blocks * 8);
    const uint64_t g = (n + 255) / 256;
    const unsigned gg = (unsigned)(g > 8192 ? 8192 : g);
    k_log_sizes<<<gg, 256, 0, stream>>>(format, cmd_off, n, sizes);
    hipError_t r = rocprim::inclusive_scan(tmp, tmp_bytes, sizes, rec_off + 1, (size_t)n,
                                           rocprim::plus<uint64_t>(), stream);
    if (r != hipSuccess) return r;
    k_log_block_first<<<gg, 256, 0, stream>>>(rec_off, n, (uint32_t)blocks, blk_first);
    // grid from the largest possible output (the exact size is only known on the device)
    k_log_emit<<<(unsigned)blocks, kLogBlock, 0, stream>>>(format, recs, cmd_off, op, key, val, n,
                                                          rec_off, blk_first, out);
    return hipGetLastError();
}

}  // namespace mpx
