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
// Pipeline: a scan of the record sizes (scan.hpp, computed from cmd_off as it reads them; its
// last pass also writes, per 8 KB output block, the record holding the block's first byte) ->
// k_log_emit:
// per block, the overlapping records' headers and commands are written into an LDS image of the
// block (one thread per header, one per command, so the command loads are coalesced) and the
// image goes out as 16-byte vector stores (no partial lines except at the run's two ends).
#include <cstring>

#include "common.hpp"
#include "kernels.hpp"
#include "scan.hpp"

namespace mpx {

namespace {
constexpr int kLogBlock = 256;
// output window of one emit block: kLogWindowVec 16-byte vectors per thread (8 KB: 4 KB
// windows measured 14% slower, 16 KB ones 13% slower at 3 workgroups per CU)
#ifndef MPX_LOG_WINDOW_VEC
#define MPX_LOG_WINDOW_VEC 2
#endif
constexpr int kLogWindowVec = MPX_LOG_WINDOW_VEC;
constexpr int kLogBlockBytes = kLogBlock * 16 * kLogWindowVec;
// the fewest bytes a record can take (catch-up: 8 + a 1-byte varint; durable: 12)
constexpr int kLogMinRec = 9;
constexpr int kLogMaxRecs = kLogBlockBytes / kLogMinRec + 2;
// commands overlapping one window: at most a whole 17 bytes each, plus a partial one per end
constexpr int kLogMaxCmds = kLogBlockBytes / 17 + 3;

__host__ __device__ __forceinline__ uint64_t zigzag(int64_t x) {  // binary.PutVarint's mapping
    return x < 0 ? ~((uint64_t)x << 1) : (uint64_t)x << 1;
}
__host__ __device__ __forceinline__ uint32_t uvarint_len(uint64_t u) {
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
__host__ __device__ __forceinline__ uint32_t hdr_bytes(int format, uint64_t ncmd) {
    return format == MPX_LOG_CATCHUP ? 8u + uvarint_len(zigzag((int64_t)ncmd)) : 12u;
}
}  // namespace

// bytes of record i, read by the offsets scan straight from cmd_off (no sizes array: one pass
// and one launch less than a sizes kernel + a scan of its output)
struct RecBytes {
    int format;
    const uint64_t* cmd_off;
    __device__ __forceinline__ uint64_t operator()(uint64_t i) const {
        const uint64_t nc = cmd_off[i + 1] - cmd_off[i];
        return hdr_bytes(format, nc) + 17 * nc;
    }
};
// the scan's output: rec_off[i + 1] = end of record i, and blk_first[b] = the record holding
// output byte b * kLogBlockBytes (a block start falls inside exactly one record), so no emit
// block has to binary-search the offsets in global memory
struct RecOffOut {
    uint64_t* rec_off;
    uint64_t* blk_first;
    uint32_t n_blocks;
    __device__ __forceinline__ void operator()(uint64_t i, uint64_t s, uint64_t bytes) const {
        const uint64_t e = s + bytes;
        rec_off[i + 1] = e;
        for (uint64_t b = (s + kLogBlockBytes - 1) / kLogBlockBytes;
             b * kLogBlockBytes < e && b < n_blocks; ++b)
            blk_first[b] = i;
    }
};

__global__ void k_log_zero(uint64_t* rec_off) { rec_off[0] = 0; }

// OR the n bytes of w (little-endian dwords, bytes past n zero) into the zeroed LDS window W at
// byte offset s (may be negative: the part before the window is dropped, as is anything past
// it): one ds_or_b32 per touched dword, so two writers of one dword (a record boundary inside
// it) meet in the OR
template <int ND>
__device__ __forceinline__ void or_bytes(uint32_t* W, int64_t s, const uint32_t (&w)[ND],
                                         uint32_t n) {
    const int64_t d0 = s >> 2;  // floor
    const uint32_t sh = (uint32_t)(s & 3) * 8u;
    const uint32_t nout = (uint32_t)(((s & 3) + n + 3) >> 2);
#pragma unroll
    for (int i = 0; i <= ND; ++i) {
        if ((uint32_t)i >= nout) break;
        const int64_t d = d0 + i;
        if (d < 0 || d >= kLogBlockBytes / 4) continue;
        const uint64_t pair = ((uint64_t)(i < ND ? w[i] : 0u) << 32) | (i ? w[i - 1] : 0u);
        const uint32_t v = (uint32_t)(pair >> (32 - sh));
        if (v) atomicOr(&W[d], v);
    }
}

// rec_off: n+1 record offsets (rec_off[n] = total bytes). One block per 8 KB output window:
// the records overlapping it are first .. first+nr-1 (blk_first of this block and the next).
// The window is an LDS image, zeroed, into which every header (a thread per record) and every
// command overlapping the window (a thread per command: op/key/val loads coalesced across
// threads; the command -> record map built by the record threads, so no search) is ORed as
// dwords (17 bytes = 5 dwords shifted into at most 6), then stored as 16-byte vectors.
__global__ __launch_bounds__(kLogBlock) void k_log_emit(
    int format, const mpx_log_rec* __restrict__ recs, const uint64_t* __restrict__ cmd_off,
    const uint8_t* __restrict__ op, const int64_t* __restrict__ key,
    const int64_t* __restrict__ val, uint64_t n, const uint64_t* __restrict__ rec_off,
    const uint64_t* __restrict__ blk_first, uint32_t n_blocks, uint8_t* __restrict__ out) {
    __shared__ uint64_t off[kLogMaxRecs + 1];
    __shared__ uint64_t coff[kLogMaxRecs + 1];
    __shared__ uint16_t cmap[kLogMaxCmds];  // command - j_lo -> record index in the window
    __shared__ __attribute__((aligned(16))) uint32_t W[kLogBlockBytes / 4];
    const uint64_t total = rec_off[n];
    const uint64_t b0 = (uint64_t)blockIdx.x * kLogBlockBytes;
    if (b0 >= total) return;  // uniform per block
    const uint64_t first = blk_first[blockIdx.x];
    const uint64_t b1 = b0 + kLogBlockBytes < total ? b0 + kLogBlockBytes : total;
    const uint64_t nr = (b1 < total && blockIdx.x + 1 < n_blocks)
                            ? blk_first[blockIdx.x + 1] - first + 1
                            : n - first;
    for (uint64_t k = threadIdx.x; k <= nr; k += kLogBlock) {
        off[k] = rec_off[first + k];
        coff[k] = cmd_off[first + k];
    }
#pragma unroll
    for (int i = 0; i < kLogWindowVec; ++i)
        reinterpret_cast<uint4*>(W)[threadIdx.x + i * kLogBlock] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    // commands overlapping [b0, b1): [j_lo, j_hi) (all commands of the records strictly
    // inside, the tail of the first record, the head of the last)
    uint64_t j_lo, j_hi;
    {
        const uint64_t hb0 = off[1] - off[0] - 17 * (coff[1] - coff[0]);
        const uint64_t cs0 = off[0] + hb0;  // first record's commands start here
        j_lo = coff[0] + (b0 > cs0 ? (b0 - cs0) / 17 : 0);
        const uint64_t L = nr - 1;
        const uint64_t hbl = off[L + 1] - off[L] - 17 * (coff[L + 1] - coff[L]);
        const uint64_t csl = off[L] + hbl;
        const uint64_t c = b1 > csl ? (b1 - csl + 16) / 17 : 0;
        j_hi = coff[L] + c < coff[L + 1] ? coff[L] + c : coff[L + 1];
    }
    // headers, and the command -> record map
    for (uint64_t k = threadIdx.x; k < nr; k += kLogBlock) {
        const uint64_t rs = off[k], c0 = coff[k], c1 = coff[k + 1], nc = c1 - c0;
        for (uint64_t j = c0 > j_lo ? c0 : j_lo; j < c1 && j < j_hi; ++j)
            cmap[j - j_lo] = (uint16_t)k;
        const uint32_t hb = (uint32_t)(off[k + 1] - rs - 17 * nc);
        if (rs + hb <= b0 || rs >= b1) continue;
        const mpx_log_rec m = recs[first + k];
        uint32_t h[5] = {(uint32_t)m.ballot, (uint32_t)m.status, 0u, 0u, 0u};
        if (format == MPX_LOG_DURABLE) {
            h[2] = (uint32_t)m.inst_no;
        } else {
            const uint64_t zz = zigzag((int64_t)nc);
            for (uint32_t q = 0; q + 8 < hb; ++q) h[2 + (q >> 2)] |= uvarint_byte(zz, q) << (8 * (q & 3));
        }
        or_bytes(W, (int64_t)(rs - b0), h, hb);
    }
    __syncthreads();
    for (uint64_t j = j_lo + threadIdx.x; j < j_hi; j += kLogBlock) {
        const uint32_t lo = cmap[j - j_lo];
        const uint64_t nc = coff[lo + 1] - coff[lo];
        const uint64_t cs = off[lo + 1] - 17 * nc;  // commands of record lo start here
        const uint64_t pos = cs + 17 * (j - coff[lo]);
        const uint32_t o8 = op[j];
        const uint64_t k8 = (uint64_t)key[j], v8 = (uint64_t)val[j];
        const uint32_t kl = (uint32_t)k8, kh = (uint32_t)(k8 >> 32);
        const uint32_t vl = (uint32_t)v8, vh = (uint32_t)(v8 >> 32);
        const uint32_t c[5] = {o8 | (kl << 8), (kl >> 24) | (kh << 8), (kh >> 24) | (vl << 8),
                               (vl >> 24) | (vh << 8), vh >> 24};
        or_bytes(W, (int64_t)pos - (int64_t)b0, c, 17);
    }
    __syncthreads();
    const uint32_t bytes = (uint32_t)(b1 - b0);
    const uint8_t* S = reinterpret_cast<const uint8_t*>(W);
    uint8_t* dst = out + b0;
    if (((uintptr_t)dst & 15) == 0) {
        const uint32_t nv = bytes / 16;
        for (uint32_t i = threadIdx.x; i < nv; i += kLogBlock)
            st_stream(reinterpret_cast<uint4*>(dst) + i, reinterpret_cast<const uint4*>(W)[i]);
        for (uint32_t i = nv * 16 + threadIdx.x; i < bytes; i += kLogBlock) dst[i] = S[i];
    } else {
        for (uint32_t i = threadIdx.x; i < bytes; i += kLogBlock) dst[i] = S[i];
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
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    return al(scan_scratch_bytes<uint64_t>(n ? n : 1)) + al(blocks_for(n, m) * 8);
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
    uint64_t* blk_first = (uint64_t*)work;
    uint64_t* tmp = (uint64_t*)((char*)blk_first + al(blocks * 8));
    const hipError_t r = device_scan(RecBytes{format, cmd_off},
                                     RecOffOut{rec_off, blk_first, (uint32_t)blocks}, n,
                                     ScanSum64{}, (uint64_t)0, tmp, stream);
    if (r != hipSuccess) return r;
    // grid from the largest possible output (the exact size is only known on the device)
    k_log_emit<<<(unsigned)blocks, kLogBlock, 0, stream>>>(format, recs, cmd_off, op, key, val, n,
                                                          rec_off, blk_first, (uint32_t)blocks,
                                                          out);
    return hipGetLastError();
}

}  // namespace mpx
