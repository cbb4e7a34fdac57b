// radix.hpp — stable LSD radix sort of (key, value) pairs or keys alone, hand-written for gfx950:
// the fan-out's client partition past 1024 connections and the sort-based apply pipeline.
//
// 8-bit digits, one pass per digit of the key bits [b0, b1); per pass three launches:
//   k_rs_count    one workgroup per tile of kRsTile elements: the tile's digit histogram (LDS
//                 atomics) into hist[digit][tile] (digit-major, so one exclusive scan of hist
//                 gives every (digit, tile) run its first output position)
//   scan          scan.hpp over the 256 x tiles counts
//   k_rs_scatter  one workgroup per tile: a wave takes a contiguous 1024-element run, 64
//                 consecutive elements a round; lanes with the same digit in a round find each
//                 other by 8 ballots (one per digit bit), their rank is the wave's running count
//                 of the digit (per-wave LDS counters) plus the lanes below; the waves' counts,
//                 prefixed per digit, place each wave after the earlier ones: stable
// The passes alternate between the output and a scratch buffer so the last one writes the
// output (the input is only read).
#pragma once
#include <type_traits>

#include "common.hpp"
#include "scan.hpp"

namespace mpx {

constexpr int kRsT = 256;
constexpr int kRsWaves = kRsT / kWave;
constexpr int kRsRounds = 16;
constexpr int kRsWaveItems = kWave * kRsRounds;    // 1024
constexpr int kRsTile = kRsWaveItems * kRsWaves;   // 4096
constexpr int kRsDigits = 256;
#ifndef MPX_RS_LDS  // the scatter's tile digit-sorted in LDS before the stores (A/B: 0)
#define MPX_RS_LDS 1
#endif

struct RsNoValue {};

// the pass's digit: key bits [sh, sh + 8) clipped to the sorted range (mask)
template <typename K>
__device__ __forceinline__ uint32_t rs_digit(K k, unsigned sh, uint32_t mask) {
    return (uint32_t)(k >> sh) & mask;
}

template <typename K>
__global__ __launch_bounds__(kRsT) void k_rs_count(const K* __restrict__ keys, uint64_t n,
                                                  unsigned sh, uint32_t mask, uint32_t tiles,
                                                  uint32_t* __restrict__ hist) {
    __shared__ uint32_t c[kRsDigits];
    c[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kRsTile;
#pragma unroll 4
    for (int r = 0; r < kRsTile / kRsT; ++r) {
        const uint64_t i = t0 + (uint64_t)r * kRsT + threadIdx.x;
        if (i < n) atomicAdd(&c[rs_digit(keys[i], sh, mask)], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * tiles + blockIdx.x] = c[threadIdx.x];
}

template <typename K, typename V>
__global__ __launch_bounds__(kRsT) void k_rs_scatter(const K* __restrict__ kin, K* __restrict__ kout,
                                                    const V* __restrict__ vin, V* __restrict__ vout,
                                                    uint64_t n, unsigned sh, uint32_t mask,
                                                    uint32_t tiles,
                                                    const uint32_t* __restrict__ offs) {
    constexpr bool kVals = !__is_same(V, RsNoValue);
    __shared__ uint32_t cnt[kRsWaves][kRsDigits];
    __shared__ uint32_t base[kRsDigits];
#if MPX_RS_LDS
    __shared__ uint32_t tst[kRsDigits];  // the digits' first positions in the sorted tile
    __shared__ uint32_t wtot[kRsWaves];
    __shared__ K sk[kRsTile];
    __shared__ typename std::conditional<kVals, V, char>::type sv[kVals ? kRsTile : 1];
#endif
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    const uint64_t below = lanes_below(l);
#pragma unroll
    for (int x = 0; x < kRsWaves; ++x) cnt[x][t] = 0;
    base[t] = offs[(uint64_t)t * tiles + blockIdx.x];
    __syncthreads();
    const uint64_t w0 = (uint64_t)blockIdx.x * kRsTile + (uint64_t)w * kRsWaveItems;
    K k[kRsRounds];
    V v[kRsRounds];
    uint32_t rk[kRsRounds];
#pragma unroll
    for (int r = 0; r < kRsRounds; ++r) {  // every load in flight before the first rank
        const uint64_t i = w0 + (uint64_t)r * kWave + l;
        k[r] = i < n ? kin[i] : K{};
        if constexpr (kVals) v[r] = i < n ? vin[i] : V{};
    }
#pragma unroll
    for (int r = 0; r < kRsRounds; ++r) {
        const uint64_t i = w0 + (uint64_t)r * kWave + l;
        const bool live = i < n;
        const uint32_t d = rs_digit(k[r], sh, mask);
        uint64_t peers = __ballot(live);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const uint32_t run = live ? cnt[w][d] : 0u;
        rk[r] = run + (uint32_t)popc(peers & below);
        if (live && !(peers >> l >> 1)) cnt[w][d] = run + (uint32_t)popc(peers);  // last lane
    }
    __syncthreads();
    uint32_t tot_d;  // this thread's digit: its count in the tile
    {  // per digit: the earlier waves' counts
        uint32_t p = 0;
#pragma unroll
        for (int x = 0; x < kRsWaves; ++x) {
            const uint32_t c = cnt[x][t];
            cnt[x][t] = p;
            p += c;
        }
        tot_d = p;
    }
#if MPX_RS_LDS
    // the tile digit-sorted in LDS first, then stored in that order: consecutive threads write
    // consecutive positions of a digit's run (a tile holds ~16 elements per digit) instead of
    // each wave instruction landing in up to 64 runs
    {  // the digits' starts in the tile (block exclusive scan of the 256 counts)
        uint32_t x = tot_d;
#pragma unroll
        for (int d2 = 1; d2 < kWave; d2 <<= 1) {
            const uint32_t y = __shfl_up(x, d2);
            if (l >= d2) x += y;
        }
        if (l == kWave - 1) wtot[w] = x;
        __syncthreads();
        uint32_t before = 0;
#pragma unroll
        for (int x2 = 0; x2 < kRsWaves; ++x2) before += x2 < w ? wtot[x2] : 0u;
        tst[t] = before + x - tot_d;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRsRounds; ++r) {
        const uint64_t i = w0 + (uint64_t)r * kWave + l;
        if (i >= n) continue;
        const uint32_t d = rs_digit(k[r], sh, mask);
        const uint32_t pos = tst[d] + cnt[w][d] + rk[r];
        sk[pos] = k[r];
        if constexpr (kVals) sv[pos] = v[r];
    }
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kRsTile;
    const uint32_t tn = (uint32_t)(n - t0 < (uint64_t)kRsTile ? n - t0 : (uint64_t)kRsTile);
    for (uint32_t i = t; i < tn; i += kRsT) {
        const K kk = sk[i];
        const uint32_t d = rs_digit(kk, sh, mask);
        const uint64_t dst = (uint64_t)base[d] + (i - tst[d]);
        kout[dst] = kk;
        if constexpr (kVals) vout[dst] = sv[i];
    }
#else
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRsRounds; ++r) {
        const uint64_t i = w0 + (uint64_t)r * kWave + l;
        if (i >= n) continue;
        const uint32_t d = rs_digit(k[r], sh, mask);
        const uint64_t dst = (uint64_t)base[d] + cnt[w][d] + rk[r];
        kout[dst] = k[r];
        if constexpr (kVals) vout[dst] = v[r];
    }
#endif
}

struct RsHistIn {
    const uint32_t* h;
    __device__ __forceinline__ uint32_t operator()(uint64_t i) const { return h[i]; }
};
struct RsHistOut {
    uint32_t* h;
    __device__ __forceinline__ void operator()(uint64_t i, uint32_t ex, uint32_t) const {
        h[i] = ex;
    }
};

// scratch of a sort of n elements: the ping-pong keys and values, the histogram, its scan's
template <typename K, typename V>
__host__ __forceinline__ uint64_t radix_scratch_bytes(uint64_t n) {
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t tiles = (n + kRsTile - 1) / kRsTile + 1;
    const uint64_t vb = __is_same(V, RsNoValue) ? 0 : al(n * sizeof(V));
    return al(n * sizeof(K)) + vb + al(tiles * kRsDigits * 4) +
           al(scan_scratch_bytes<uint32_t>(tiles * kRsDigits));
}

// sorts (kin, vin) by key bits [b0, b1) into (kout, vout), stably; n < 2^32
template <typename K, typename V>
hipError_t radix_sort(const K* kin, K* kout, const V* vin, V* vout, uint64_t n, unsigned b0,
                      unsigned b1, void* scratch, uint64_t scratch_bytes, hipStream_t stream) {
    if (!n) return hipSuccess;
    if (n >= (1ull << 32) || scratch_bytes < radix_scratch_bytes<K, V>(n))
        return hipErrorInvalidValue;
    constexpr bool kVals = !__is_same(V, RsNoValue);
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    char* s = (char*)scratch;
    K* ktmp = (K*)s;
    s += al(n * sizeof(K));
    V* vtmp = nullptr;
    if constexpr (kVals) {
        vtmp = (V*)s;
        s += al(n * sizeof(V));
    }
    const uint32_t tiles = (uint32_t)((n + kRsTile - 1) / kRsTile);
    uint32_t* hist = (uint32_t*)s;
    s += al(((uint64_t)tiles + 1) * kRsDigits * 4);
    uint32_t* scan_tmp = (uint32_t*)s;
    const unsigned passes = b1 > b0 ? (b1 - b0 + 7) / 8 : 0;
    if (!passes) {  // nothing to sort on: a copy
        hipError_t r = hipMemcpyAsync(kout, kin, n * sizeof(K), hipMemcpyDeviceToDevice, stream);
        if (r == hipSuccess && kVals)
            r = hipMemcpyAsync(vout, vin, n * sizeof(V), hipMemcpyDeviceToDevice, stream);
        return r;
    }
    const K* ks = kin;
    const V* vs = vin;
    for (unsigned p = 0; p < passes; ++p) {
        // the last pass writes the output, the ones before alternate so that holds
        const bool to_out = ((passes - 1 - p) & 1u) == 0;
        K* kd = to_out ? kout : ktmp;
        V* vd = to_out ? vout : vtmp;
        const unsigned sh = b0 + 8 * p;
        const unsigned nb = b1 - sh < 8 ? b1 - sh : 8;
        const uint32_t mask = (1u << nb) - 1u;
        k_rs_count<K><<<tiles, kRsT, 0, stream>>>(ks, n, sh, mask, tiles, hist);
        const hipError_t r = device_scan(RsHistIn{hist}, RsHistOut{hist},
                                         (uint64_t)tiles * kRsDigits, ScanSum32{}, 0u, scan_tmp,
                                         stream);
        if (r != hipSuccess) return r;
        k_rs_scatter<K, V><<<tiles, kRsT, 0, stream>>>(ks, kd, vs, vd, n, sh, mask, tiles, hist);
        ks = kd;
        vs = vd;
    }
    return hipGetLastError();
}

}  // namespace mpx
