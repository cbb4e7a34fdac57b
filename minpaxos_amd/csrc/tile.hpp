// tile.hpp — lane-per-instance processing of one instance log's reply records (configs 2 and 3).
//
// The records of a call (16 B each, instance number first) are grouped by instance in ascending
// order with arbitrary (ragged) fan-in. A 256-thread workgroup walks tiles of kTileRecs records
// (grid-stride, the next tile's records prefetched into registers while the current one is
// processed):
//   1. the tile goes to LDS with coalesced 16-byte loads;
//   2. head flags (first record of an instance) are compacted into the tile's list of OWNED
//      instances: those whose first record lies in the tile. Records at the start of a tile that
//      continue an instance of the previous tile belong to that tile's last instance, which
//      reads them (the "overhang") straight from global memory;
//   3. one lane per owned instance applies the reference handler to the instance's records in
//      arrival order, with the instance state in registers (the caller's `body`).
// A call's record array therefore needs no instance-boundary search and every record is read
// once from HBM (overhangs aside, which are at most the rest of one instance per tile).
#pragma once
#include "common.hpp"

namespace mpx {

#ifndef MPX_TILE_RECS  // A/B builds (make variant_of): other tile shapes
#define MPX_TILE_RECS 1024
#endif
#ifndef MPX_TILE_BLOCK
#define MPX_TILE_BLOCK 256
#endif
constexpr int kTileRecs = MPX_TILE_RECS;
constexpr int kTileBlock = MPX_TILE_BLOCK;
static_assert(kTileRecs % kTileBlock == 0 && kTileRecs < 65536, "tile shape");
constexpr int kTilePer = kTileRecs / kTileBlock;
constexpr int kTileWaves = kTileBlock / kWave;

struct TileLds {
    int4 rec[kTileRecs];                 // the tile's records
    uint16_t hpos[kTileRecs + 1];        // positions of the owned instances' first records
    uint32_t wcnt[kTilePer * kTileWaves];  // heads per (register k, wave), then their offsets
    int4 ovr[kWave];                     // the records after the tile: the overhang's start
    uint32_t nh;                         // owned instances in the tile
    uint64_t oend;                       // end of the last owned instance's overhang
    int64_t onext;                       // instance of the record at oend (kNoNext: none)
};

constexpr int64_t kNoNext = INT64_MAX;  // no record follows the instance in the log

// record q of the tile's last instance's overhang [after, oend): the first kWave from LDS
__device__ __forceinline__ int4 over_rec(const TileLds& S, const int4* __restrict__ recs,
                                         uint64_t after, uint64_t q) {
    return q - after < (uint64_t)kWave ? S.ovr[q - after] : recs[q];
}

__device__ __forceinline__ int4 tile_load(const int4* __restrict__ recs, uint64_t n, uint64_t p) {
    return p < n ? ld_stream(recs + p) : make_int4(0, 0, 0, 0);
}

// Runs body(pos_first, count, tile_end, overhang_end, own, next_inst, first) for every owned
// instance of every tile this workgroup takes. Records of the instance are
// S.rec[pos_first .. pos_first+count) followed, for the tile's last instance, by global records
// [tile_end, overhang_end). next_inst is the instance of the next record in the log after the
// instance's records (kNoNext after the last one) and `first` marks the instance of the log's
// first record: together they tell a lane which instances without records border its own
// (tile_gaps). Every lane of the workgroup calls `body` the same number of times per tile
// (rounds of 256 instances; lanes without an instance in a round get count = 0), so `body` may
// use wave-level ballots. `err` receives kErrOrder when instances are not ascending.
// pre(inst0), called by every thread as soon as a tile is in LDS (inst0 = the instance of its
// first record), lets the caller issue the loads of the per-instance state its lanes will most
// likely own in round 0 (instance inst0 + lane, when the tile's instances are dense) while the
// tile's heads are found: the state load is otherwise a dependent round trip after two barriers.
template <typename Pre, typename Body>
__device__ __forceinline__ void tile_walk(TileLds& S, const int4* __restrict__ recs, uint64_t n,
                                          uint32_t* err, Pre&& pre, Body&& body) {
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    const uint64_t n_tiles = (n + kTileRecs - 1) / kTileRecs;
    const unsigned long long below = (1ull << l) - 1ull;
    uint64_t T = blockIdx.x;
    int4 cur[kTilePer];
#pragma unroll
    for (int k = 0; k < kTilePer; ++k)
        cur[k] = tile_load(recs, n, T * kTileRecs + t + k * kTileBlock);
    uint32_t ebits = 0;
    for (; T < n_tiles; T += gridDim.x) {
        const uint64_t p0 = T * kTileRecs;
        const uint32_t cnt = (uint32_t)((n - p0) < (uint64_t)kTileRecs ? (n - p0) : kTileRecs);
        // neighbours of the tile: the record before it and the one after it
        const int32_t prev_inst = p0 ? recs[p0 - 1].x : 0;
        const uint64_t after = p0 + cnt;
        const int32_t after_inst = after < n ? recs[after].x : 0;
#pragma unroll
        for (int k = 0; k < kTilePer; ++k) S.rec[t + k * kTileBlock] = cur[k];
        // the next tile of this workgroup: issued now, consumed after this tile's barriers
        const uint64_t Tn = T + gridDim.x;
#pragma unroll
        for (int k = 0; k < kTilePer; ++k)
            cur[k] = Tn < n_tiles ? tile_load(recs, n, Tn * kTileRecs + t + k * kTileBlock)
                                  : make_int4(0, 0, 0, 0);
        __syncthreads();
        pre(S.rec[0].x);
        bool head[kTilePer];
#pragma unroll
        for (int k = 0; k < kTilePer; ++k) {
            const uint32_t p = t + k * kTileBlock;
            const bool valid = p < cnt;
            const int32_t inst = S.rec[p].x;
            const int32_t prev = p ? S.rec[p - 1].x : prev_inst;
            const bool first = p0 + p == 0;
            head[k] = valid && (first || inst != prev);
            ebits |= (head[k] && !first && inst < prev) ? kErrOrder : 0u;
            const unsigned long long hm = __ballot(head[k]);
            if (l == 0) S.wcnt[k * kTileWaves + w] = (uint32_t)__popcll(hm);
        }
        __syncthreads();
        uint32_t base[kTilePer];
        {
            // exclusive offsets of (k, w) in record order (p = 256k + 64w + l)
            uint32_t run = 0, tot = 0;
#pragma unroll
            for (int k = 0; k < kTilePer; ++k)
#pragma unroll
                for (int w2 = 0; w2 < kTileWaves; ++w2) {
                    const uint32_t c = S.wcnt[k * kTileWaves + w2];
                    if (w2 == w) base[k] = run;
                    run += c;
                    tot += c;
                }
            if (t == 0) S.nh = tot;
        }
        // the tile's last record continues into the next tile: wave 0 finds where its
        // instance ends, 64 records per step
        if (w == 0) {
            uint64_t oend = after;
            int64_t onext = after < n ? (int64_t)after_inst : kNoNext;
            if (after < n && cnt && after_inst == S.rec[cnt - 1].x) {
                const int32_t inst = after_inst;
                // whole records, so the first 64 of the overhang reach its lane through LDS
                // instead of one dependent global load per record (over_rec)
                for (uint64_t q = after;; q += kWave) {
                    const uint64_t p = q + l;
                    const int4 rr = p < n ? recs[p] : make_int4(0, 0, 0, 0);
                    if (q == after) S.ovr[l] = rr;
                    const int32_t pi = rr.x;
                    const bool stop = p >= n || pi != inst;
                    const unsigned long long m = __ballot(stop);
                    if (m) {
                        const int src = __ffsll((long long)m) - 1;
                        oend = q + (uint64_t)src;
                        onext = oend < n ? (int64_t)__builtin_amdgcn_readlane(pi, src) : kNoNext;
                        break;
                    }
                }
            }
            if (l == 0) {
                S.oend = oend;
                S.onext = onext;
            }
        }
#pragma unroll
        for (int k = 0; k < kTilePer; ++k) {
            const unsigned long long hm = __ballot(head[k]);
            if (head[k]) S.hpos[base[k] + (uint32_t)__popcll(hm & below)] = (uint16_t)(t + k * kTileBlock);
        }
        __syncthreads();
        const uint32_t nh = S.nh;
        const uint64_t oend_t = S.oend;
        const int64_t onext_t = S.onext;
        const uint32_t rounds = (nh + kTileBlock - 1) / kTileBlock;
        for (uint32_t r = 0; r < rounds; ++r) {
            const uint32_t j = (uint32_t)t + r * kTileBlock;
            const bool own = j < nh;
            const bool last = own && j + 1 == nh;
            const uint32_t a = own ? S.hpos[j] : 0u;
            const uint32_t z = own ? (!last ? (uint32_t)S.hpos[j + 1] : cnt) : 0u;
            // end of the overhang (global position), == after if none
            const uint64_t oend = last ? oend_t : after;
            const int64_t nxt = !own ? kNoNext : (!last ? (int64_t)S.rec[z].x : onext_t);
            body(a, z - a, after, oend, own, nxt, own && p0 + a == 0);
        }
        __syncthreads();  // the LDS tile is rewritten next
    }
    if (ebits) raise_err(err, ebits);
}

}  // namespace mpx

namespace mpx {

// The instances without records that border an owned instance (window-relative index idx, next
// instance with records nxt, both from tile_walk): (idx, nxt) clamped to the window [0, n_inst),
// and for the log's first instance also [0, idx). Such instances receive no reply, so a lane
// that writes per-instance outputs for the whole window covers them here: fn(q) runs once for
// every such q, the wave's 64 lanes striding over one range at a time (coalesced). Wave-uniform:
// all lanes must call. Every instance of the window is then either owned by exactly one lane or
// in exactly one such range (records grouped in ascending order; on kErrOrder the outputs are
// unspecified anyway).
template <typename Fn>
__device__ __forceinline__ void tile_gaps(bool own, int64_t idx, int64_t nxt_idx, bool first,
                                          uint64_t n_inst, Fn&& fn) {
    const int l = lane_id();
    const int64_t ni = (int64_t)n_inst;
    for (int pass = 0; pass < 2; ++pass) {
        int64_t lo = 0, hi = 0;
        if (own && pass == 0) {  // after the instance
            lo = idx + 1 < 0 ? 0 : idx + 1;
            hi = nxt_idx < ni ? nxt_idx : ni;
        } else if (own && first) {  // before the log's first instance
            hi = idx < ni ? idx : ni;
        }
        unsigned long long m = __ballot(hi > lo);
        while (m) {
            const int src = __ffsll((long long)m) - 1;
            m &= m - 1;
            const int64_t a = (int64_t)__shfl((long long)lo, src);
            const int64_t b = (int64_t)__shfl((long long)hi, src);
            for (int64_t q = a + l; q < b; q += kWave) fn((uint64_t)q);
        }
    }
}

}  // namespace mpx
