// scan.hpp — device-wide scans for the engine's pipelines (log encoding offsets, fan-out client
// offsets, the sort-based apply's per-slot last-PUT scan), hand-written for gfx950.
//
// Three plain launches, no decoupled look-back (device-scope look-back loads bypass the XCD L2s
// and queue behind the tiles in flight: DESIGN §9, stream decoder):
//   k_scan_reduce   one workgroup per tile of kScTile items: the tile's total
//   k_scan_totals   one workgroup: exclusive scan of the tile totals, in place
//   k_scan_tiles    one workgroup per tile: the tile's items again (held in registers while the
//                   waves' totals meet), each handed to the caller's `out(i, exclusive prefix,
//                   item)`
// Items come from the caller's `in(i)` (so a scan of computed values needs no array of them).
// A wave takes a contiguous run of 64 x kScRounds items, 64 consecutive ones per round
// (coalesced loads and output stores), a wave-wide inclusive scan per round, a running carry
// between rounds; the waves' totals meet in LDS. `op(a, b)` combines an earlier a with a later
// b: associative, not necessarily commutative (the segmented max-scan is not).
#pragma once
#include "common.hpp"

namespace mpx {

constexpr int kScT = 256;                      // threads of a tile workgroup
constexpr int kScWaves = kScT / kWave;         // 4
constexpr int kScRounds = 16;                  // 64-item rounds per wave
constexpr int kScWaveItems = kWave * kScRounds;  // 1024
constexpr int kScTile = kScWaveItems * kScWaves;  // 4096 items per tile
constexpr int kScTotT = 1024;                  // threads of k_scan_totals

// values up to 8 bytes move between lanes as one 64-bit shuffle
template <typename T>
__device__ __forceinline__ T shfl_up_any(T v, int d) {
    static_assert(sizeof(T) <= 8, "scan items of at most 8 bytes");
    unsigned long long x = 0;
    __builtin_memcpy(&x, &v, sizeof(T));
    x = (unsigned long long)__shfl_up((long long)x, d);
    T r;
    __builtin_memcpy(&r, &x, sizeof(T));
    return r;
}
template <typename T>
__device__ __forceinline__ T shfl_any(T v, int src) {
    unsigned long long x = 0;
    __builtin_memcpy(&x, &v, sizeof(T));
    x = (unsigned long long)__shfl((long long)x, src);
    T r;
    __builtin_memcpy(&r, &x, sizeof(T));
    return r;
}

template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan(T v, Op op) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const T t = shfl_up_any(v, d);
        if (l >= d) v = op(t, v);
    }
    return v;
}

// the wave's run of a tile: items [w0, w0 + kScWaveItems) clipped to n
template <typename T, typename Op, typename In>
__global__ __launch_bounds__(kScT) void k_scan_reduce(In in, uint64_t n, T* __restrict__ tot, Op op,
                                                     T id) {
    __shared__ T ws[kScWaves];
    const int l = lane_id(), w = threadIdx.x / kWave;
    const uint64_t w0 = (uint64_t)blockIdx.x * kScTile + (uint64_t)w * kScWaveItems;
    // every round's item loaded before the first is combined (a loop that loaded round r + 1
    // only after combining round r waited for 16 dependent loads per wave), then combined in
    // index order (op need not be commutative)
    T xs[kScRounds];
#pragma unroll
    for (int r = 0; r < kScRounds; ++r) {
        const uint64_t i = w0 + (uint64_t)r * kWave + l;
        xs[r] = i < n ? in(i) : id;
    }
    T acc = id;
    if constexpr (Op::kCommutes) {  // a sum: each lane folds its rounds, then one wave reduction
#pragma unroll
        for (int r = 0; r < kScRounds; ++r) acc = op(acc, xs[r]);
#pragma unroll
        for (int d = kWave / 2; d >= 1; d >>= 1) acc = op(acc, shfl_any(acc, l ^ d));
    } else {
#pragma unroll
        for (int r = 0; r < kScRounds; ++r)
            acc = op(acc, shfl_any(wave_incl_scan(xs[r], op), kWave - 1));
    }
    if (l == 0) ws[w] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T s = ws[0];
        for (int x = 1; x < kScWaves; ++x) s = op(s, ws[x]);
        tot[blockIdx.x] = s;
    }
}

// exclusive scan of the tile totals in place (one workgroup; kScTotT totals per round)
template <typename T, typename Op>
__global__ __launch_bounds__(kScTotT) void k_scan_totals(T* __restrict__ tot, uint64_t tiles, Op op,
                                                        T id) {
    __shared__ T ws[kScTotT / kWave];
    __shared__ T carry_s;
    const int l = lane_id(), w = threadIdx.x / kWave;
    T carry = id;
    for (uint64_t b = 0; b < tiles; b += kScTotT) {
        const uint64_t i = b + threadIdx.x;
        const T x = i < tiles ? tot[i] : id;
        const T v = wave_incl_scan(x, op);
        if (l == kWave - 1) ws[w] = v;
        __syncthreads();
        T before = carry;
        for (int k = 0; k < w; ++k) before = op(before, ws[k]);
        const T excl_in_wave = shfl_up_any(v, 1);
        const T ex = l ? op(before, excl_in_wave) : before;
        if (i < tiles) tot[i] = ex;
        if (threadIdx.x == kScTotT - 1) carry_s = op(ex, x);
        __syncthreads();
        carry = carry_s;
        __syncthreads();  // ws and carry_s are rewritten by the next round
    }
}

template <typename T, typename Op, typename In, typename Out>
__global__ __launch_bounds__(kScT) void k_scan_tiles(In in, uint64_t n, const T* __restrict__ tot,
                                                    Op op, T id, Out out) {
    __shared__ T ws[kScWaves];
    const int l = lane_id(), w = threadIdx.x / kWave;
    const uint64_t w0 = (uint64_t)blockIdx.x * kScTile + (uint64_t)w * kScWaveItems;
    // the wave's rounds, scanned and kept in registers, then its run total
    T xs[kScRounds], vs[kScRounds];
    T acc = id;
#pragma unroll
    for (int r = 0; r < kScRounds; ++r) {
        const uint64_t i = w0 + (uint64_t)r * kWave + l;
        xs[r] = i < n ? in(i) : id;
        vs[r] = wave_incl_scan(xs[r], op);
        acc = op(acc, shfl_any(vs[r], kWave - 1));
    }
    if (l == 0) ws[w] = acc;
    __syncthreads();
    T carry = tot[blockIdx.x];
    for (int x = 0; x < w; ++x) carry = op(carry, ws[x]);
#pragma unroll
    for (int r = 0; r < kScRounds; ++r) {
        const uint64_t i = w0 + (uint64_t)r * kWave + l;
        const T up = shfl_up_any(vs[r], 1);
        const T ex = l ? op(carry, up) : carry;
        if (i < n) out(i, ex, xs[r]);
        carry = op(carry, shfl_any(vs[r], kWave - 1));
    }
}

// k_scan_tiles for a commutative op (sums): each wave's 1024 items go through LDS so that a lane
// holds 16 CONSECUTIVE items, scans them serially, and one wave scan of the lane totals replaces
// a wave scan per round (16 x 6 shuffle steps, of 64-bit values for the log offsets); the
// prefixes go back through LDS so the loads and the out() stores stay coalesced
template <typename T, typename Op, typename In, typename Out>
__global__ __launch_bounds__(kScT) void k_scan_tiles_c(In in, uint64_t n, const T* __restrict__ tot,
                                                      Op op, T id, Out out) {
    constexpr int kPad = kScWaveItems + kScWaveItems / kScRounds;  // one pad slot per 16 items
    __shared__ T tx[kScWaves][kPad];
    __shared__ T ws[kScWaves];
    const int l = lane_id(), w = threadIdx.x / kWave;
    const uint64_t w0 = (uint64_t)blockIdx.x * kScTile + (uint64_t)w * kScWaveItems;
    auto at = [](int j) { return j + j / kScRounds; };  // item j of the wave's run -> LDS slot
    T xs[kScRounds];
#pragma unroll
    for (int r = 0; r < kScRounds; ++r) {
        const uint64_t i = w0 + (uint64_t)r * kWave + l;
        xs[r] = i < n ? in(i) : id;
        tx[w][at(r * kWave + l)] = xs[r];
    }
    __syncthreads();
    T pre[kScRounds];  // exclusive prefixes of the lane's 16 consecutive items
    T run = id;
#pragma unroll
    for (int j = 0; j < kScRounds; ++j) {
        pre[j] = run;
        run = op(run, tx[w][at(l * kScRounds + j)]);
    }
    const T incl = wave_incl_scan(run, op);
    const T up = shfl_up_any(incl, 1);  // every lane takes part in the shuffle
    const T lane_ex = l ? up : id;
    if (l == kWave - 1) ws[w] = incl;
    __syncthreads();
    T carry = tot[blockIdx.x];
    for (int x = 0; x < w; ++x) carry = op(carry, ws[x]);
    carry = op(carry, lane_ex);
#pragma unroll
    for (int j = 0; j < kScRounds; ++j) tx[w][at(l * kScRounds + j)] = op(carry, pre[j]);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kScRounds; ++r) {
        const uint64_t i = w0 + (uint64_t)r * kWave + l;
        if (i < n) out(i, tx[w][at(r * kWave + l)], xs[r]);
    }
}

// scratch: one T per tile
template <typename T>
__host__ __forceinline__ uint64_t scan_scratch_bytes(uint64_t n) {
    return ((n + kScTile - 1) / kScTile + 1) * sizeof(T);
}

template <typename T, typename Op, typename In, typename Out>
hipError_t device_scan(In in, Out out, uint64_t n, Op op, T id, T* scratch, hipStream_t stream) {
    if (!n) return hipSuccess;
    const uint64_t tiles = (n + kScTile - 1) / kScTile;
    if (tiles >= (1ull << 31)) return hipErrorInvalidValue;
    k_scan_reduce<T, Op, In><<<(unsigned)tiles, kScT, 0, stream>>>(in, n, scratch, op, id);
    k_scan_totals<T, Op><<<1, kScTotT, 0, stream>>>(scratch, tiles, op, id);
    if constexpr (Op::kCommutes)
        k_scan_tiles_c<T, Op, In, Out><<<(unsigned)tiles, kScT, 0, stream>>>(in, n, scratch, op, id,
                                                                             out);
    else
        k_scan_tiles<T, Op, In, Out><<<(unsigned)tiles, kScT, 0, stream>>>(in, n, scratch, op, id,
                                                                           out);
    return hipGetLastError();
}

// an op's kCommutes lets the tile reduction fold in any order (sums); order-sensitive ops (the
// segmented max-scan) combine in index order
struct ScanSum64 {
    static constexpr bool kCommutes = true;
    __device__ __forceinline__ uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
};
struct ScanSum32 {
    static constexpr bool kCommutes = true;
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};

}  // namespace mpx
