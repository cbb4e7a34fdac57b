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
// The slot maximum, binned (the default when the engine holds the call's scratch,
// replay_work_bytes; instance spaces up to kRbMaxCap slots): 2^24 random device-scope atomics
// are request-bound on this chip (0.45 ms of the 0.69 ms call, round 3), so the slots are
// maximised in LDS instead (round 5's form, MPX_REPLAY_SORTCHUNK=0):
//   k_replay_durable  writes pair[i] = (rec_base + i) << 32 | instNo, coalesced (8 B / record)
//   k_rb_count        a workgroup per chunk of kRbChunk pairs: LDS histogram of the bins
//                     (kRbSlots = 32768 instance slots each) into hist[bin][chunk], bin-major
//   scan              scan.hpp over the bins x chunks counts (+1: the total)
//   k_rb_scatter      the chunk's pairs sorted by bin in LDS, then stored as the bins' runs
//                     (order inside a bin is free: a maximum does not depend on it)
//   k_rb_max          a workgroup per bin: the bin's slice of last_rec into LDS, one LDS
//                     atomicMax per pair, the slice written back
// 8 B x 4 of pair traffic per record + the slots read and written once, all coalesced.
// MPX_REPLAY_SORTCHUNK=1 (round 6, the default) drops the count, scan and scatter passes:
//   k_replay_durable  writes the record's instNo (4 B; the record index is its position)
//   k_rb_sort         a workgroup per chunk: the chunk's instNos sorted by bin in LDS and written
//                     back packed (chunk-local record index << 15 | slot in bin, 4 bytes) into
//                     the chunk's own range, with each bin's start in the chunk (run starts,
//                     chunks x (bins + 1)) - no global histogram or scan needed
//   k_rb_max_runs     a workgroup per bin: its run in every chunk (8 lanes per run), one LDS
//                     atomicMax per pair as before
// 4 B written + 4 B read + 4 B written + 4 B read per record.
// Without the scratch (or past kRbMaxCap slots), one atomicMax per record:
// The slot maximum without a device-scope atomic per record (MPX_REPLAY_ATOMIC=0, A/B):
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
#include "scan.hpp"

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
constexpr int kVecPer = (kTileVec + kReplayBlock - 1) / kReplayBlock;  // vectors per thread

__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const int32_t t = __shfl_xor(v, d);
        v = v > t ? v : t;
    }
    return v;
}

constexpr int kRbLg = 15;
constexpr uint32_t kRbSlots = 1u << kRbLg;      // instance slots per bin (128 KB of LDS)
constexpr uint32_t kRbMaxBins = 1024;           // the count / scatter LDS tables (4 KB)
constexpr int64_t kRbMaxCap = (int64_t)kRbSlots * kRbMaxBins;  // 2^25 slots
constexpr int kRbT = 1024;
constexpr int kRbPer = 16;
constexpr uint64_t kRbChunk = kRbPer * kRbT;    // pairs per count / scatter workgroup (128 KB)
constexpr uint64_t kRbNone = ~0ull;             // an instNo outside [0, inst_cap): no slot
#ifndef MPX_REPLAY_SORTCHUNK
#define MPX_REPLAY_SORTCHUNK 1
#endif
static_assert(kRbChunk <= (1u << (32 - kRbLg)), "packed pair: chunk-local index above the slot bits");

// pairs: null = the atomic form
__global__ __launch_bounds__(kReplayBlock) void k_replay_durable(
    const uint8_t* __restrict__ log, uint64_t n, int32_t inst_cap, int32_t rec_base,
    mpx_log_rec* __restrict__ recs,
    uint8_t* __restrict__ op, int64_t* __restrict__ key, int64_t* __restrict__ val,
    int32_t* __restrict__ last_rec, int32_t* __restrict__ scalars, uint32_t* __restrict__ err,
    uint64_t* __restrict__ pairs) {
    __shared__ uint4 tile[kTileVec + 1];  // +1: the last lane's 9th dword reads past the tile
    __shared__ int32_t red[2][kReplayBlock / kWave];
    const int t = threadIdx.x;
    int32_t ballot = INT32_MIN, committed = INT32_MIN;
    const uint64_t n_tiles = (n + kReplayBlock - 1) / kReplayBlock;
    // the tile's 16-byte vectors: whole ones inside its records, the ragged tail byte by byte
    auto load_tile = [&](uint64_t tl, uint4 (&v)[kVecPer]) {
        const uint64_t r0 = tl * kReplayBlock;
        const uint64_t nrec = n - r0 < (uint64_t)kReplayBlock ? n - r0 : (uint64_t)kReplayBlock;
        const uint64_t tile_bytes = nrec * kRecBytes;
        const uint8_t* src = log + r0 * kRecBytes;
        const uint64_t nvec = tile_bytes / 16;
#pragma unroll
        for (int k = 0; k < kVecPer; ++k) {
            const int vi = t + k * kReplayBlock;
            v[k] = make_uint4(0, 0, 0, 0);
            if ((uint64_t)vi < nvec) {
                v[k] = ld_stream(reinterpret_cast<const uint4*>(src) + vi);
            } else if (vi < kTileVec && (uint64_t)vi * 16 < tile_bytes) {
                uint8_t b[16] = {};
                for (uint64_t q = (uint64_t)vi * 16; q < tile_bytes; ++q) b[q - (uint64_t)vi * 16] = src[q];
                v[k] = *reinterpret_cast<const uint4*>(b);
            }
        }
    };
    uint4 cur[kVecPer];
    if (blockIdx.x < n_tiles) load_tile(blockIdx.x, cur);
    for (uint64_t tl = blockIdx.x; tl < n_tiles; tl += gridDim.x) {
        const uint64_t r0 = tl * kReplayBlock;
        const uint64_t nrec = n - r0 < (uint64_t)kReplayBlock ? n - r0 : (uint64_t)kReplayBlock;
        __syncthreads();  // the previous tile's readers are done with the LDS image
#pragma unroll
        for (int k = 0; k < kVecPer; ++k)
            if (t + k * kReplayBlock < kTileVec) tile[t + k * kReplayBlock] = cur[k];
        // the workgroup's next tile: in flight while this one is cut into records
        if (tl + gridDim.x < n_tiles) load_tile(tl + gridDim.x, cur);
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
            const bool bad = inst < 0 || inst >= inst_cap;
            if (pairs && MPX_REPLAY_SORTCHUNK)  // the instNo alone: the record index is its place
                st_stream(reinterpret_cast<uint32_t*>(pairs) + i, bad ? ~0u : (uint32_t)inst);
            else if (pairs)
                st_stream(pairs + i, bad ? kRbNone
                                         : ((uint64_t)(uint32_t)(rec_base + (int32_t)i) << 32) |
                                               (uint32_t)inst);
            if (bad)
                raise_err(err, kErrNil);
            else if (pairs)
                ;
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
// ---- the binned slot maximum --------------------------------------------------------------
__global__ __launch_bounds__(kRbT) void k_rb_count(const uint64_t* __restrict__ pairs, uint64_t n,
                                                  uint32_t bins, uint32_t chunks,
                                                  uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kRbMaxBins];
    for (uint32_t b = threadIdx.x; b < bins; b += kRbT) h[b] = 0;
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * kRbChunk;
    // all of a thread's loads in flight before its first LDS atomic (an early-exit loop waited
    // out each load in turn)
    uint64_t p[kRbPer];
#pragma unroll
    for (int k = 0; k < kRbPer; ++k) {
        const uint64_t i = c0 + (uint64_t)(threadIdx.x + k * kRbT);
        p[k] = i < n ? ld_stream(pairs + i) : kRbNone;
    }
#pragma unroll
    for (int k = 0; k < kRbPer; ++k)
        if (p[k] != kRbNone) atomicAdd(&h[(uint32_t)p[k] >> kRbLg], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < bins; b += kRbT) hist[(uint64_t)b * chunks + blockIdx.x] = h[b];
}

// the chunk's pairs sorted by bin in LDS first (ranks from LDS counters, a block scan of the
// counts), then stored in that order: consecutive lanes write consecutive positions of a bin's
// run (~32 pairs per bin and chunk at 2^24 slots) instead of 64 random 8-byte stores per wave
// instruction (0.30 -> see DESIGN §5)
__global__ __launch_bounds__(kRbT) void k_rb_scatter(const uint64_t* __restrict__ pairs, uint64_t n,
                                                    uint32_t bins, uint32_t chunks,
                                                    const uint32_t* __restrict__ offs,
                                                    uint64_t* __restrict__ binned) {
    __shared__ uint64_t sp[kRbChunk];
    __shared__ uint32_t cnt[kRbMaxBins];  // counts, then the bins' starts in sp
    __shared__ uint32_t gof[kRbMaxBins];  // the bins' first output position for this chunk
    __shared__ uint32_t wtot[kRbT / kWave];
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    for (uint32_t b = t; b < bins; b += kRbT) {
        cnt[b] = 0;
        gof[b] = offs[(uint64_t)b * chunks + blockIdx.x];
    }
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * kRbChunk;
    uint64_t p[kRbPer];
    uint32_t rk[kRbPer];
#pragma unroll
    for (int k = 0; k < kRbPer; ++k) {
        const uint64_t i = c0 + (uint64_t)(t + k * kRbT);
        p[k] = i < n ? ld_stream(pairs + i) : kRbNone;
    }
#pragma unroll
    for (int k = 0; k < kRbPer; ++k)
        rk[k] = p[k] != kRbNone ? atomicAdd(&cnt[(uint32_t)p[k] >> kRbLg], 1u) : 0u;
    __syncthreads();
    // exclusive scan of the counts, one bin per thread (bins <= kRbT)
    const uint32_t c = (uint32_t)t < bins ? cnt[t] : 0u;
    uint32_t x = c;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (l >= d) x += y;
    }
    if (l == kWave - 1) wtot[w] = x;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (int v = 0; v < kRbT / kWave; ++v) {
        before += v < w ? wtot[v] : 0u;
        total += wtot[v];
    }
    if ((uint32_t)t < bins) cnt[t] = before + x - c;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRbPer; ++k)
        if (p[k] != kRbNone) sp[cnt[(uint32_t)p[k] >> kRbLg] + rk[k]] = p[k];
    __syncthreads();
    for (uint32_t i = t; i < total; i += kRbT) {
        const uint64_t q = sp[i];
        const uint32_t b = (uint32_t)q >> kRbLg;
        binned[gof[b] + (i - cnt[b])] = q;
    }
}

__global__ __launch_bounds__(kRbT) void k_rb_max(const uint64_t* __restrict__ binned,
                                                uint32_t chunks, const uint32_t* __restrict__ offs,
                                                int32_t inst_cap, int32_t* __restrict__ last_rec) {
    __shared__ int32_t sl[kRbSlots];
    const uint32_t b = blockIdx.x;
    const uint64_t s0 = (uint64_t)b * kRbSlots;
    const uint32_t ns = (uint64_t)inst_cap - s0 < kRbSlots ? (uint32_t)((uint64_t)inst_cap - s0)
                                                            : kRbSlots;
    // the slice's current values, then the bin's pairs, kB loads in flight per thread at a time
    // (load-use loops waited out each load in turn)
    constexpr int kB = 8;
    static_assert(kRbSlots % (kB * kRbT) == 0, "whole batches of slots");
    for (uint32_t j0 = 0; j0 < ns; j0 += kB * kRbT) {
        int32_t v[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const uint32_t j = j0 + threadIdx.x + k * kRbT;
            v[k] = j < ns ? last_rec[s0 + j] : 0;
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const uint32_t j = j0 + threadIdx.x + k * kRbT;
            if (j < ns) sl[j] = v[k];
        }
    }
    // the bin's run: from its first chunk's offset to the next bin's (the total after the last)
    const uint64_t lo = offs[(uint64_t)b * chunks], hi = offs[(uint64_t)(b + 1) * chunks];
    __syncthreads();
    for (uint64_t i0 = lo; i0 < hi; i0 += (uint64_t)kB * kRbT) {
        uint64_t p[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const uint64_t i = i0 + threadIdx.x + (uint64_t)k * kRbT;
            p[k] = i < hi ? ld_stream(binned + i) : kRbNone;
        }
#pragma unroll
        for (int k = 0; k < kB; ++k)
            if (p[k] != kRbNone) atomicMax(&sl[(uint32_t)p[k] & (kRbSlots - 1)], (int32_t)(p[k] >> 32));
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < ns; j += kRbT) last_rec[s0 + j] = sl[j];
}

// the chunk's instNos sorted by bin in LDS, stored packed over the chunk's own range of `packed`,
// and the bins' starts in the chunk (rs[chunk][b], b <= bins: rs[chunk][bins] = the chunk's total)
#ifndef MPX_RB_SORT_WPE  // k_rb_sort's waves per SIMD bound (8: two workgroups per CU)
#define MPX_RB_SORT_WPE 0
#endif
__global__ __launch_bounds__(kRbT)
#if MPX_RB_SORT_WPE
__attribute__((amdgpu_waves_per_eu(MPX_RB_SORT_WPE)))
#endif
void k_rb_sort(const uint32_t* __restrict__ insts, uint64_t n,
                                                 uint32_t bins, uint32_t* __restrict__ packed,
                                                 uint32_t* __restrict__ rs) {
    __shared__ uint32_t sp[kRbChunk];
    __shared__ uint32_t cnt[kRbMaxBins];  // counts, then the bins' starts in sp
    __shared__ uint32_t wtot[kRbT / kWave];
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    for (uint32_t b = t; b < bins; b += kRbT) cnt[b] = 0;
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * kRbChunk;
    uint32_t p[kRbPer];  // instNo, ~0 = none
    uint32_t rk[kRbPer];
#pragma unroll
    for (int k = 0; k < kRbPer; ++k) {
        const uint64_t i = c0 + (uint64_t)(t + k * kRbT);
        p[k] = i < n ? ld_stream(insts + i) : ~0u;
    }
#pragma unroll
    for (int k = 0; k < kRbPer; ++k)
        rk[k] = p[k] != ~0u ? atomicAdd(&cnt[p[k] >> kRbLg], 1u) : 0u;
    __syncthreads();
    // exclusive scan of the counts, one bin per thread (bins <= kRbT)
    const uint32_t c = (uint32_t)t < bins ? cnt[t] : 0u;
    uint32_t x = c;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (l >= d) x += y;
    }
    if (l == kWave - 1) wtot[w] = x;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (int v = 0; v < kRbT / kWave; ++v) {
        before += v < w ? wtot[v] : 0u;
        total += wtot[v];
    }
    uint32_t* r = rs + (uint64_t)blockIdx.x * (bins + 1);
    if ((uint32_t)t < bins) {
        cnt[t] = before + x - c;
        r[t] = before + x - c;
    }
    if (t == 0) r[bins] = total;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRbPer; ++k)
        if (p[k] != ~0u)
            sp[cnt[p[k] >> kRbLg] + rk[k]] =
                ((uint32_t)(t + k * kRbT) << kRbLg) | (p[k] & (kRbSlots - 1));
    __syncthreads();
    for (uint32_t i = t; i < total; i += kRbT) st_stream(packed + c0 + i, sp[i]);
}

// a workgroup per bin: the slice into LDS, then the bin's run in every chunk, 8 lanes per run
// and four runs per 8 lanes in flight (~32 pairs per run for 2^24 records over 2^24 slots), the
// slice written back
__global__ __launch_bounds__(kRbT) void k_rb_max_runs(const uint32_t* __restrict__ packed,
                                                     const uint32_t* __restrict__ rs,
                                                     uint32_t chunks, uint32_t bins,
                                                     int32_t inst_cap, int32_t rec_base,
                                                     int32_t* __restrict__ last_rec) {
    __shared__ int32_t sl[kRbSlots];
    const uint32_t b = blockIdx.x;
    const uint64_t s0 = (uint64_t)b * kRbSlots;
    const uint32_t ns = (uint64_t)inst_cap - s0 < kRbSlots ? (uint32_t)((uint64_t)inst_cap - s0)
                                                            : kRbSlots;
    constexpr int kB = 8;
    static_assert(kRbSlots % (kB * kRbT) == 0, "whole batches of slots");
    for (uint32_t j0 = 0; j0 < ns; j0 += kB * kRbT) {
        int32_t v[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const uint32_t j = j0 + threadIdx.x + k * kRbT;
            v[k] = j < ns ? last_rec[s0 + j] : 0;
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const uint32_t j = j0 + threadIdx.x + k * kRbT;
            if (j < ns) sl[j] = v[k];
        }
    }
    __syncthreads();
    // the bin's run starts / ends for up to kRbT chunks at a time, into LDS with one load each
    // (a run's bounds loaded just before its pairs had put two round trips on every run)
    __shared__ uint32_t rlo[kRbT], rhi[kRbT];
    constexpr uint32_t kSub = 8, kGroups = kRbT / kSub;
    constexpr int kU = 4, kR = 6;  // runs per group and pairs per lane in flight
    const uint32_t g = threadIdx.x / kSub, sub = threadIdx.x % kSub;
    for (uint32_t cb = 0; cb < chunks; cb += kRbT) {
        const uint32_t nc = chunks - cb < (uint32_t)kRbT ? chunks - cb : (uint32_t)kRbT;
        __syncthreads();  // the previous batch's readers are done
        if (threadIdx.x < nc) {
            const uint32_t* r = rs + (uint64_t)(cb + threadIdx.x) * (bins + 1) + b;
            rlo[threadIdx.x] = r[0];
            rhi[threadIdx.x] = r[1];
        }
        __syncthreads();
        for (uint32_t c0 = g; c0 < nc; c0 += kU * kGroups) {
            uint32_t q[kU][kR];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint32_t c = c0 + u * kGroups;
                const uint32_t lo = c < nc ? rlo[c] : 0u, hi = c < nc ? rhi[c] : 0u;
                const uint32_t* src = packed + (uint64_t)(cb + c) * kRbChunk;
#pragma unroll
                for (int k = 0; k < kR; ++k) {
                    const uint32_t j = lo + sub + k * kSub;
                    q[u][k] = j < hi ? src[j] : ~0u;  // cached: the run's next pieces share its lines
                }
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint32_t c = c0 + u * kGroups;
                const int32_t cbase = (int32_t)((uint32_t)rec_base + (cb + c) * (uint32_t)kRbChunk);
#pragma unroll
                for (int k = 0; k < kR; ++k)
                    if (q[u][k] != ~0u)
                        atomicMax(&sl[q[u][k] & (kRbSlots - 1)],
                                  (int32_t)((uint32_t)cbase + (q[u][k] >> kRbLg)));
                if (c < nc) {  // a run longer than kSub * kR pairs: its tail
                    const uint32_t* src = packed + (uint64_t)(cb + c) * kRbChunk;
                    for (uint32_t j = rlo[c] + sub + kR * kSub; j < rhi[c]; j += kSub) {
                        const uint32_t x = src[j];
                        atomicMax(&sl[x & (kRbSlots - 1)], (int32_t)((uint32_t)cbase + (x >> kRbLg)));
                    }
                }
            }
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < ns; j += kRbT) last_rec[s0 + j] = sl[j];
}

// the scan of hist: bins x chunks counts, then one zero item whose prefix is the total
struct RbHistIn {
    const uint32_t* h;
    uint64_t n;
    __device__ __forceinline__ uint32_t operator()(uint64_t i) const { return i < n ? h[i] : 0u; }
};
struct RbHistOut {
    uint32_t* o;
    __device__ __forceinline__ void operator()(uint64_t i, uint32_t ex, uint32_t) const { o[i] = ex; }
};

struct RbLayout {
    uint64_t pairs, binned, hist, offs, scan, packed, rs, total;
};
RbLayout rb_layout(uint64_t n, int32_t inst_cap) {
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t chunks = (n + kRbChunk - 1) / kRbChunk;
    const uint64_t bins = ((uint64_t)inst_cap + kRbSlots - 1) / kRbSlots;
    const uint64_t h = bins * chunks + 1;
    RbLayout L{};
    uint64_t o = 0;
    L.pairs = o; o += al(n * 8);
    L.binned = o; o += al(n * 8);
    L.hist = o; o += al(h * 4);
    L.offs = o; o += al(h * 4);
    L.scan = o; o += al(scan_scratch_bytes<uint32_t>(h));
    L.packed = o; o += al(n * 4);
    L.rs = o; o += al(chunks * (bins + 1) * 4);
    L.total = o;
    return L;
}
bool rb_eligible(uint64_t n, int32_t inst_cap) {
    return n > 0 && inst_cap > 0 && (int64_t)inst_cap <= kRbMaxCap && n < (1ull << 32);
}
}  // namespace

uint64_t replay_work_bytes(uint64_t n, int32_t inst_cap) {
    return rb_eligible(n, inst_cap) ? rb_layout(n, inst_cap).total : 0;
}

hipError_t launch_replay_durable(const uint8_t* log, uint64_t n, int32_t inst_cap,
                                 int32_t rec_base, mpx_log_rec* recs, uint8_t* op, int64_t* key, int64_t* val,
                                 int32_t* last_rec, int32_t* scalars, uint32_t* err,
                                 void* work, uint64_t work_bytes, hipStream_t stream) {
    if (!n) return hipSuccess;
    const bool binned = rb_eligible(n, inst_cap) && work &&
                        work_bytes >= rb_layout(n, inst_cap).total;
    const RbLayout L = binned ? rb_layout(n, inst_cap) : RbLayout{};
    char* w = (char*)work;
    uint64_t* pairs = binned ? (uint64_t*)(w + L.pairs) : nullptr;
    // a few workgroups per CU walk the tiles (grid-stride), so the watermark atomics stay few
    const uint64_t tiles = (n + kReplayBlock - 1) / kReplayBlock;
    const uint64_t grid = tiles < kReplayGrid ? tiles : kReplayGrid;
    hipLaunchKernelGGL(k_replay_durable, dim3((unsigned)grid), dim3(kReplayBlock), 0, stream, log,
                       n, inst_cap, rec_base, recs, op, key, val, last_rec, scalars, err, pairs);
    if (binned) {
        const uint32_t chunks = (uint32_t)((n + kRbChunk - 1) / kRbChunk);
        const uint32_t bins = (uint32_t)(((uint64_t)inst_cap + kRbSlots - 1) / kRbSlots);
        const uint64_t h = (uint64_t)bins * chunks;
#if MPX_REPLAY_SORTCHUNK
        uint32_t* packed = (uint32_t*)(w + L.packed);
        uint32_t* rs = (uint32_t*)(w + L.rs);
        k_rb_sort<<<chunks, kRbT, 0, stream>>>((const uint32_t*)pairs, n, bins, packed, rs);
        k_rb_max_runs<<<bins, kRbT, 0, stream>>>(packed, rs, chunks, bins, inst_cap, rec_base,
                                                 last_rec);
        return hipGetLastError();
#endif
        uint32_t* hist = (uint32_t*)(w + L.hist);
        uint32_t* offs = (uint32_t*)(w + L.offs);
        k_rb_count<<<chunks, kRbT, 0, stream>>>(pairs, n, bins, chunks, hist);
        const hipError_t r = device_scan(RbHistIn{hist, h}, RbHistOut{offs}, h + 1, ScanSum32{},
                                         0u, (uint32_t*)(w + L.scan), stream);
        if (r != hipSuccess) return r;
        k_rb_scatter<<<chunks, kRbT, 0, stream>>>(pairs, n, bins, chunks, offs,
                                                  (uint64_t*)(w + L.binned));
        k_rb_max<<<bins, kRbT, 0, stream>>>((const uint64_t*)(w + L.binned), chunks, offs,
                                            inst_cap, last_rec);
        return hipGetLastError();
    }
    if (!MPX_REPLAY_ATOMIC) {
        const uint64_t g = (n + 255) / 256;
        hipLaunchKernelGGL(k_replay_fix, dim3((unsigned)(g < 8192 ? g : 8192)), dim3(256), 0,
                           stream, recs, n, inst_cap, rec_base, last_rec);
    }
    return hipGetLastError();
}

}  // namespace mpx
