// replay.hip — durable-log replay (the read side of the durable log).
//
// bareminpaxos.(*Replica).getDataFromStableStore  src/bareminpaxos/bareminpaxos.go:122-161 reads
// the stable store as back-to-back 29-byte records: 12 bytes of metadata (Ballot, Status, instNo as
// little-endian u32, :130-140) and exactly one state.Command (:142-143, Command.Unmarshal
// statemarsh.go:21-37: Op u8, K i64, V i64). Per record, in file order:
//   defaultBallot = ballot            if ballot > defaultBallot                     (:145-147)
//   committedUpTo = instNo            if instNo > committedUpTo && COMMITTED        (:149-151)
//   instanceSpace[instNo] = {ballot, status, {0,0,0,nil}, [command]}               (:153-157)
// The two watermarks are running maxima, so they are order-free; the last record naming an
// instance wins its slot, so the slot keeps the HIGHEST record index.
// The slot maximum without a device-scope atomic per record (MPX_REPLAY_ATOMIC=0, default):
//   pass 1 (k_replay_durable) raises a slot with a plain load + store when its record index is
//          higher: racing records of one instance may leave a lower index, never a value below
//          the slot's value at call start (memory holds it when the kernel begins);
//   pass 2 (k_replay_fix) re-reads every record's instNo from the SoA output and lifts a slot
//          that still holds a lower index with atomicMax - only where records of one instance
//          raced, so (almost) no atomics.
// MPX_REPLAY_ATOMIC=1 keeps the single pass with one atomicMax per record (A/B builds).
//
// Layout: 256-record tiles (7424 bytes = 464 x 16 B, so every tile starts
// 16-byte aligned when the log does); the tile is staged into LDS with 16-byte loads and each lane
// cuts its record out of LDS, then writes the SoA outputs coalesced (16-byte mpx_log_rec, op,
// key, val); a grid of 8 workgroups per CU walks the tiles, and each workgroup's max-reductions
// feed one atomicMax per watermark. HBM-bound:
// 29 B in + 33 B out + one 4-byte slot update per record (+ pass 2's 16-byte re-read).
#include "common.hpp"
#include "kernels.hpp"

namespace mpx {

namespace {
constexpr int kReplayBlock = 256;
constexpr int kRecBytes = MPX_DURABLE_REC_BYTES;               // 12 + 17
constexpr int kTileBytes = kReplayBlock * kRecBytes;           // 7424
constexpr int kTileVec = kTileBytes / 16;                      // 464
constexpr uint64_t kReplayGrid = 256 * 8;  // 256 CUs x 8 workgroups
#ifndef MPX_REPLAY_ATOMIC
#define MPX_REPLAY_ATOMIC 1
#endif
static_assert(kTileBytes % 16 == 0, "tile must be a whole number of 16-byte vectors");

__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const int32_t t = __shfl_xor(v, d);
        v = v > t ? v : t;
    }
    return v;
}

__global__ __launch_bounds__(kReplayBlock) void k_replay_durable(
    const uint8_t* __restrict__ log, uint64_t n, int32_t inst_cap, int32_t rec_base,
    mpx_log_rec* __restrict__ recs,
    uint8_t* __restrict__ op, int64_t* __restrict__ key, int64_t* __restrict__ val,
    int32_t* __restrict__ last_rec, int32_t* __restrict__ scalars, uint32_t* __restrict__ err) {
    __shared__ uint4 tile[kTileVec + 1];  // +1: the last lane's 9th dword reads past the tile
    __shared__ int32_t red[2][kReplayBlock / kWave];
    const int t = threadIdx.x;
    int32_t ballot = INT32_MIN, committed = INT32_MIN;
    const uint64_t n_tiles = (n + kReplayBlock - 1) / kReplayBlock;
    for (uint64_t tl = blockIdx.x; tl < n_tiles; tl += gridDim.x) {
        const uint64_t r0 = tl * kReplayBlock;
        const uint64_t nrec = n - r0 < (uint64_t)kReplayBlock ? n - r0 : (uint64_t)kReplayBlock;
        const uint64_t tile_bytes = nrec * kRecBytes;
        const uint8_t* src = log + r0 * kRecBytes;
        // stage: whole 16-byte vectors inside the tile's records, the ragged tail byte by byte
        const uint64_t nvec = tile_bytes / 16;
        __syncthreads();  // the previous tile's readers are done with the LDS image
        for (int v = t; v < kTileVec; v += kReplayBlock) {
            if ((uint64_t)v < nvec) {
                tile[v] = ld_stream(reinterpret_cast<const uint4*>(src) + v);
            } else if ((uint64_t)v * 16 < tile_bytes) {
                uint8_t b[16] = {};
                for (uint64_t k = (uint64_t)v * 16; k < tile_bytes; ++k)
                    b[k - (uint64_t)v * 16] = src[k];
                tile[v] = *reinterpret_cast<const uint4*>(b);
            }
        }
        __syncthreads();
        if ((uint64_t)t < nrec) {
            // the record as 8 realigned dwords from 9 aligned LDS dword reads (not 29 byte reads)
            const int off = t * kRecBytes;
            const uint32_t* wsrc = reinterpret_cast<const uint32_t*>(tile) + (off >> 2);
            const int sh = (off & 3) * 8;
            uint32_t w[9], d[8];
#pragma unroll
            for (int k = 0; k < 9; ++k) w[k] = wsrc[k];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                d[k] = (uint32_t)((((uint64_t)w[k + 1] << 32) | w[k]) >> sh);
            const int32_t b = (int32_t)d[0];
            const int32_t st = (int32_t)d[1];
            const int32_t inst = (int32_t)d[2];
            const uint8_t opb = (uint8_t)d[3];
            const uint64_t kv = ((((uint64_t)d[4] << 32) | d[3]) >> 8) | ((uint64_t)(d[5] & 0xff) << 56);
            const uint64_t vv = ((((uint64_t)d[6] << 32) | d[5]) >> 8) | ((uint64_t)(d[7] & 0xff) << 56);
            const uint64_t i = r0 + t;
            mpx_log_rec r;
            r.ballot = b;
            r.status = st;
            r.inst_no = inst;
            r.pad = 0;
            st_stream(reinterpret_cast<int4*>(recs + i), *reinterpret_cast<const int4*>(&r));
            st_stream(op + i, opb);
            st_stream(key + i, (int64_t)kv);
            st_stream(val + i, (int64_t)vv);
            ballot = b > ballot ? b : ballot;
            if (st == MPX_COMMITTED && inst > committed) committed = inst;
            // instanceSpace[instNo] panics outside the array (Go index check)
            if (inst < 0 || inst >= inst_cap)
                raise_err(err, kErrNil);
            else if (MPX_REPLAY_ATOMIC)
                atomicMax(last_rec + inst, rec_base + (int32_t)i);
            else if (last_rec[inst] < rec_base + (int32_t)i)
                last_rec[inst] = rec_base + (int32_t)i;
        }
    }
    // one atomic per workgroup and watermark, skipped when it cannot raise the running value:
    // per-wave atomics on the two words serialised at L2 (2 x 262k atomics for 2^24 records)
    ballot = wave_max_i32(ballot);
    committed = wave_max_i32(committed);
    if (lane_id() == 0) {
        red[0][t / kWave] = ballot;
        red[1][t / kWave] = committed;
    }
    __syncthreads();
    if (t < 2) {
        int32_t m = INT32_MIN;
        for (int w = 0; w < kReplayBlock / kWave; ++w) m = red[t][w] > m ? red[t][w] : m;
        if (m != INT32_MIN && m > __hip_atomic_load(scalars + t, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT))
            atomicMax(scalars + t, m);
    }
}

// pass 2: a slot below one of its records' indices lost a race in pass 1
__global__ __launch_bounds__(256) void k_replay_fix(const mpx_log_rec* __restrict__ recs,
                                                    uint64_t n, int32_t inst_cap,
                                                    int32_t rec_base,
                                                    int32_t* __restrict__ last_rec) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int32_t inst = reinterpret_cast<const int32_t*>(recs + i)[2];  // inst_no
        if (inst < 0 || inst >= inst_cap) continue;
        const int32_t me = rec_base + (int32_t)i;
        if (last_rec[inst] < me) atomicMax(last_rec + inst, me);
    }
}
}  // namespace

hipError_t launch_replay_durable(const uint8_t* log, uint64_t n, int32_t inst_cap,
                                 int32_t rec_base, mpx_log_rec* recs, uint8_t* op, int64_t* key, int64_t* val,
                                 int32_t* last_rec, int32_t* scalars, uint32_t* err,
                                 hipStream_t stream) {
    if (!n) return hipSuccess;
    // a few workgroups per CU walk the tiles (grid-stride), so the watermark atomics stay few
    const uint64_t tiles = (n + kReplayBlock - 1) / kReplayBlock;
    const uint64_t grid = tiles < kReplayGrid ? tiles : kReplayGrid;
    hipLaunchKernelGGL(k_replay_durable, dim3((unsigned)grid), dim3(kReplayBlock), 0, stream, log,
                       n, inst_cap, rec_base, recs, op, key, val, last_rec, scalars, err);
    if (!MPX_REPLAY_ATOMIC) {
        const uint64_t g = (n + 255) / 256;
        hipLaunchKernelGGL(k_replay_fix, dim3((unsigned)(g < 8192 ? g : 8192)), dim3(256), 0,
                           stream, recs, n, inst_cap, rec_base, last_rec);
    }
    return hipGetLastError();
}

}  // namespace mpx
