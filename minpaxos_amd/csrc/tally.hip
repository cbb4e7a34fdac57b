// tally.hip — accept tally kernels for one instance log (configs 2 and the single-group API).
#include <mutex>

#include "kernels.hpp"
#include "tally.hpp"
#include "tile.hpp"

namespace mpx {

// Accept tally of one instance log, ONE launch: tile_walk (tile.hpp) hands every lane one
// instance and its replies in arrival order; the lane applies handleAcceptReply to each (state in
// registers).
//   MIN      bareminpaxos.go:1023-1053: OK replies only, no status check
//   CLASSIC  paxos.go:634-673: replies to instances not PREPARED/ACCEPTED are ignored
// The "last assignment wins" scalars of MIN (committedUpTo :1048, peerCommits[id] :1050) come
// from the highest instance that assigns them (instances ascend in array order; all of an
// instance's assignments of one scalar write the same value): per round a wave ballot finds the
// highest lane, one LDS max per wave, one device-scope max per workgroup. CLASSIC's
// updateCommittedUpTo (paxos.go:259-264) is the first instance >= committedUpTo+1 whose final
// status is not COMMITTED: a minimum over the owned instances (final status in registers) and
// the instances without replies (their input status, read in the gap pass). Window-relative
// keys idx+1 (0 = none) keep the maxima unsigned; the minimum is kept as a max of ~idx.
// The workgroup that finishes last (ticket) turns the maxima into the scalars and resets the
// control words, so a call is one kernel and no memset: the decided flags of instances without
// replies are written 0 in the gap pass.
// Control words (engine-owned, zero between calls): [0] ticket, [1..1+N) MIN keys / [1] CLASSIC
// "some instance committed", [2] CLASSIC ~first_bad.
#ifndef MPX_TALLY_WPE
#define MPX_TALLY_WPE 0
#endif
#if MPX_TALLY_WPE
#define MPX_TALLY_ATTR __attribute__((amdgpu_waves_per_eu(MPX_TALLY_WPE, MPX_TALLY_WPE)))
#else
#define MPX_TALLY_ATTR
#endif
template <int MODE>
__global__ MPX_TALLY_ATTR __launch_bounds__(kTileBlock) void k_accept_tile(
    const mpx_accept_reply* __restrict__ recs, uint64_t n, const mpx_inst_state* __restrict__ st_in,
    mpx_inst_state* __restrict__ st_out, uint64_t n_inst, int32_t base, int32_t half, int32_t nrep,
    int32_t* __restrict__ scalars, uint32_t* __restrict__ ctl, uint8_t* __restrict__ decided,
    uint32_t* err) {
    __shared__ TileLds S;
    __shared__ uint32_t red[1 + MPX_MAX_REPLICAS];
    const int t = threadIdx.x, l = lane_id();
    if (t <= MPX_MAX_REPLICAS) red[t] = 0;
    uint32_t ebits = 0;
    // CLASSIC: updateCommittedUpTo scans from committedUpTo+1 (the call's input; the last
    // workgroup writes scalars[0] only after every workgroup has read it)
    const int64_t j0 = MODE == MPX_MODE_CLASSIC ? (int64_t)scalars[0] + 1 - base : 0;
    uint32_t fb_key = 0;  // ~(first non-committed instance >= j0) seen by this lane, 0 = none
    const int4* r4 = reinterpret_cast<const int4*>(recs);
    const int4* s4 = reinterpret_cast<const int4*>(st_in);
    int64_t spec_idx = -1;  // the state loaded ahead for round 0 (tile_walk's pre)
    int4 spec = make_int4(0, 0, 0, 0);
    auto pre = [&](int32_t inst0) {
        spec_idx = (int64_t)inst0 - base + t;
        if (spec_idx >= 0 && (uint64_t)spec_idx < n_inst) spec = ld_stream(s4 + spec_idx);
    };
    tile_walk(S, r4, n, err, pre, [&](uint32_t a, uint32_t cnt, uint64_t after, uint64_t oend,
                                      bool own, int64_t nxt, bool first) {
        const int32_t inst = own ? S.rec[a].x : 0;
        const int64_t idx = (int64_t)inst - base;
        const bool inwin = own && idx >= 0 && (uint64_t)idx < n_inst;
        int4 st = inwin ? (idx == spec_idx ? spec : ld_stream(s4 + idx))
                        : make_int4(MPX_STATUS_NIL, 0, 0, 0);
        spec_idx = -1;  // (later rounds of the tile load their own)
        const bool nil = st.x == MPX_STATUS_NIL;
        ebits |= (own && !inwin) ? kErrNil : 0u;  // outside instanceSpace
        if (MODE == MPX_MODE_CLASSIC) ebits |= (own && nil) ? kErrNil : 0u;  // paxos.go:634
        uint32_t idmask = 0;
        int32_t deci = 0;
        auto step = [&](int4 r, int32_t act) {  // act: 0/1, the record takes part
            const int32_t okj = (r.w & 0xff) == 1 ? act : 0;  // OK == TRUE
            if (MODE == MPX_MODE_MIN) {
                ebits |= (okj && nil) ? kErrNil : 0u;  // inst.Lb of a nil instance (:1024)
                const int32_t oks = st.y + okj;       // AcceptOKs++
                const int32_t c1 = oks >= half ? okj : 0;   // AcceptOKs+1 > N>>1
                const int32_t dj = oks == half ? c1 : 0;    // AcceptOKs == N>>1: COMMITTED
                st.y = oks;
                st.x = dj ? MPX_COMMITTED : st.x;
                deci |= dj;
                const bool badid = r.z < 0 || r.z >= nrep;
                ebits |= (c1 && badid) ? kErrBadId : 0u;
                idmask |= (c1 && !badid) ? (1u << r.z) : 0u;
            } else {
                const int32_t live = (uint32_t)(st.x - MPX_PREPARED) < 2u ? act : 0;
                const int32_t okl = live & okj, nk = live & (okj ^ act);
                const int32_t oks = st.y + okl;
                const int32_t c = oks >= half ? okl : 0;  // acceptOKs+1 > N>>1
                st.y = oks;
                st.x = c ? MPX_COMMITTED : st.x;
                deci |= c;
                st.z += nk;
                const int32_t nb = nk ? r.y : INT32_MIN;
                st.w = st.w > nb ? st.w : nb;
            }
        };
        // the tile part: uniform trip count (wave maximum), predicated body
        uint32_t rmax = cnt;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t x = (uint32_t)__shfl_xor((int)rmax, d);
            rmax = rmax > x ? rmax : x;
        }
        rmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)rmax);
        for (uint32_t j = 0; j < rmax; ++j) {
            const int4 r = S.rec[j < cnt ? a + j : 0];
            step(r, (j < cnt && inwin) ? 1 : 0);
        }
        // the overhang of the tile's last instance (one lane per tile)
        for (uint64_t q = after; inwin && q < oend; ++q) step(over_rec(S, r4, after, q), 1);
        if (inwin) {
            st_stream(reinterpret_cast<int4*>(st_out) + idx, st);
            if (decided) st_stream(decided + idx, (uint8_t)(deci ? 1 : 0));
            if (MODE == MPX_MODE_CLASSIC && idx >= j0 && st.x != MPX_COMMITTED) {
                const uint32_t k = ~(uint32_t)idx;
                fb_key = fb_key > k ? fb_key : k;
            }
        }
        // instances without replies: not decided; CLASSIC also reads their (final = input)
        // status for updateCommittedUpTo, until this lane has a smaller candidate
        tile_gaps(own, idx, nxt == kNoNext ? INT64_MAX : nxt - base, first, n_inst,
                  [&](uint64_t q) {
                      if (decided) decided[q] = 0;
                      if (MODE == MPX_MODE_CLASSIC && (int64_t)q >= j0 && ~(uint32_t)q > fb_key &&
                          st_in[q].status != MPX_COMMITTED)
                          fb_key = ~(uint32_t)q;
                  });
        const uint32_t key = (uint32_t)(idx + 1);
        if (MODE == MPX_MODE_MIN) {
            const unsigned long long dm = __ballot(inwin && deci);
            if (dm) {
                const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)key, 63 - __clzll(dm));
                if (l == 0) atomicMax(&red[0], k);
            }
            for (int i = 0; i < nrep; ++i) {
                const unsigned long long m = __ballot(inwin && ((idmask >> i) & 1u));
                if (m) {
                    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)key, 63 - __clzll(m));
                    if (l == 0) atomicMax(&red[1 + i], k);
                }
            }
        } else {
            if (__ballot(inwin && deci) && l == 0) atomicMax(&red[0], 1u);
        }
    });
    if (MODE == MPX_MODE_CLASSIC) {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t x = (uint32_t)__shfl_xor((int)fb_key, d);
            fb_key = fb_key > x ? fb_key : x;
        }
        if (l == 0 && fb_key) atomicMax(&red[1], fb_key);
    }
    if (ebits) raise_err(err, ebits);
    __syncthreads();
    // this workgroup's maxima into the call's (device scope), then its ticket
    const int nw = MODE == MPX_MODE_MIN ? 1 + nrep : 2;
    if (t < nw && red[t]) atomic_max_done(&ctl[1 + t], red[t]);
    if (!last_workgroup(&ctl[0])) return;
    if (t < nw) red[t] = atomic_take(&ctl[1 + t]);  // read and reset for the next call
    __syncthreads();
    if (t != 0) return;
    if (MODE == MPX_MODE_MIN) {
        for (int w = 0; w <= nrep; ++w)  // committedUpTo = inst; peerCommits[id] = inst - 1
            if (red[w]) scalars[w] = (int32_t)((int64_t)base + red[w] - 1 - (w ? 1 : 0));
    } else if (red[0] && j0 >= 0 && (uint64_t)j0 < n_inst) {
        // some instance committed: committedUpTo = first non-committed - 1 (n_inst if none)
        const uint64_t fb = red[1] ? (uint64_t)~red[1] : n_inst;
        scalars[0] = (int32_t)(base + (int64_t)fb - 1);
    }
}

// mpx_committed_prefix's reduction words: [0] some instance counts as committed, then the
// first non-committed instance (a running minimum)
constexpr int kRedFirstBad = 1 + MPX_MAX_REPLICAS;

__global__ void k_tally_init(unsigned long long* red, uint64_t n_inst) {
    const int t = threadIdx.x;
    if (t < kRedFirstBad) red[t] = 0;
    if (t == kRedFirstBad) red[t] = n_inst;
}

// CLASSIC updateCommittedUpTo (paxos.go:259-264) over a status window (mpx_committed_prefix):
// find the first instance >= committedUpTo+1 that is not COMMITTED (final COMMITTED <=> st
// COMMITTED or decided).
// The first non-committed instance is almost always a few instances past committedUpTo, so one
// block scans the head window [j0, j0 + kHeadWindow) in order and stops at the first hit; the
// grid-wide kernel below then covers the rest of the window only if the head found nothing.
constexpr uint64_t kHeadWindow = 1ull << 16;
__global__ __launch_bounds__(256) void k_classic_first_bad_head(
    const mpx_inst_state* __restrict__ st, const uint8_t* __restrict__ decided, uint64_t n_inst,
    int32_t base, const int32_t* __restrict__ scalars, unsigned long long* __restrict__ red) {
    __shared__ int found;
    if (red[0] == 0) return;
    const int64_t j0 = (int64_t)scalars[0] + 1 - base;
    if (j0 < 0 || (uint64_t)j0 >= n_inst) return;
    const uint64_t end = (uint64_t)j0 + kHeadWindow < n_inst ? (uint64_t)j0 + kHeadWindow : n_inst;
    if (threadIdx.x == 0) found = 0;
    __syncthreads();
    for (uint64_t b = (uint64_t)j0; b < end; b += blockDim.x) {
        const uint64_t j = b + threadIdx.x;
        const bool bad = j < end && !(st[j].status == MPX_COMMITTED || (decided && decided[j]));
        const uint64_t m = ballot(bad);
        if (m && lane_id() == 0) {
            atomicMin(&red[kRedFirstBad], (unsigned long long)(j + lo_bit(m)));
            found = 1;
        }
        __syncthreads();
        if (found) break;  // uniform per block
    }
}

__global__ __launch_bounds__(256) void k_classic_first_bad(
    const mpx_inst_state* __restrict__ st, const uint8_t* __restrict__ decided, uint64_t n_inst,
    int32_t base, const int32_t* __restrict__ scalars, unsigned long long* __restrict__ red) {
    __shared__ unsigned long long fb_s;
    if (red[0] == 0) return;  // no crossing in this call: committedUpTo unchanged
    const int64_t jc = (int64_t)scalars[0] + 1 - base;
    if (jc < 0 || (uint64_t)jc >= n_inst) return;
    const int64_t j0 = jc + (int64_t)kHeadWindow;  // the head kernel covered [jc, j0)
    if ((uint64_t)j0 >= n_inst) return;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)j0 + (uint64_t)blockIdx.x * blockDim.x; b < n_inst; b += stride) {
        // one read of the running minimum per block and round (a per-thread atomic load of one
        // address serialises every thread of the grid on a single L2 channel)
        if (threadIdx.x == 0)
            fb_s = __hip_atomic_load(&red[kRedFirstBad], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const unsigned long long fb = fb_s;
        __syncthreads();
        if (b >= fb) break;  // uniform per block
        const uint64_t j = b + threadIdx.x;
        const bool bad = j < n_inst && !(st[j].status == MPX_COMMITTED || (decided && decided[j]));
        const uint64_t m = ballot(bad);
        if (m && lane_id() == 0)  // the wave's first non-committed instance, one atomic per wave
            atomicMin(&red[kRedFirstBad], (unsigned long long)(j + lo_bit(m)));
    }
}

__global__ void k_prefix_finalize(const unsigned long long* __restrict__ red, int32_t* scalars,
                                  uint64_t n_inst, int32_t base) {
    if (threadIdx.x != 0 || red[0] == 0) return;
    const int64_t j0 = (int64_t)scalars[0] + 1 - base;
    if (j0 < 0 || (uint64_t)j0 >= n_inst) return;
    const uint64_t fb = red[kRedFirstBad];  // first non-committed (n_inst if none)
    scalars[0] = (int32_t)(base + (int64_t)fb - 1);
}

uint32_t resident_grid(const void* kernel, int block, uint64_t tiles) {
    // the kernels are the engine's own, one gfx950 device type: per kernel, the count is cached
    static std::mutex mu;
    static const void* keys[16];
    static uint32_t vals[16];
    static int used = 0;
    uint32_t g = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (int i = 0; i < used; ++i)
            if (keys[i] == kernel) g = vals[i];
        if (!g) {
            int dev = 0, nb = 0, cus = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, block, 0);
            (void)hipGetLastError();
            // two rounds of resident workgroups: the second round's start staggers the
            // workgroups' tile phases (load / walk / store), which measured 2-3 % faster than
            // one round on the config-2 tally (same-box A/B, profiles/r03)
            const uint64_t r = 2 * (uint64_t)(nb > 0 ? nb : 1) * (uint64_t)(cus > 0 ? cus : 256);
            g = (uint32_t)(r < (uint64_t)kTileGrid ? r : kTileGrid);
#ifdef MPX_TILE_GRID  // A/B builds: a fixed grid
            g = MPX_TILE_GRID;
#endif
            if (used < 16) {
                keys[used] = kernel;
                vals[used++] = g;
            }
        }
    }
    return (uint32_t)(tiles < g ? (tiles ? tiles : 1) : g);
}

hipError_t launch_accept_tally(int mode, const mpx_accept_reply* recs, uint64_t n,
                               const mpx_inst_state* st_in, mpx_inst_state* st_out,
                               uint64_t n_inst, int32_t base, int32_t nrep, int32_t* scalars,
                               uint8_t* decided, unsigned long long* red, uint32_t* ctl,
                               uint32_t* err, hipStream_t stream) {
    const int32_t half = nrep >> 1;
    const uint64_t tiles = (n + kTileRecs - 1) / kTileRecs;
    if (n == 0) {
        // no replies: nothing changes but the decided flags (all 0)
        if (decided && n_inst) (void)hipMemsetAsync(decided, 0, n_inst, stream);
        return hipGetLastError();
    }
    if (mode == MPX_MODE_MIN) {
        const uint32_t grid = resident_grid((const void*)k_accept_tile<MPX_MODE_MIN>, kTileBlock, tiles);
        k_accept_tile<MPX_MODE_MIN><<<grid, kTileBlock, 0, stream>>>(
            recs, n, st_in, st_out, n_inst, base, half, nrep, scalars, ctl, decided, err);
    } else {
        const uint32_t grid = resident_grid((const void*)k_accept_tile<MPX_MODE_CLASSIC>, kTileBlock, tiles);
        k_accept_tile<MPX_MODE_CLASSIC><<<grid, kTileBlock, 0, stream>>>(
            recs, n, st_in, st_out, n_inst, base, half, nrep, scalars, ctl, decided, err);
    }
    (void)red;
    return hipGetLastError();
}

// Standalone CLASSIC watermark over a status window (mpx_committed_prefix).
__global__ void k_prefix_mark(unsigned long long* red) { red[0] = 1; }

hipError_t launch_committed_prefix(const mpx_inst_state* st, uint64_t n_inst, int32_t base,
                                   int32_t* scalars, unsigned long long* red, hipStream_t stream) {
    k_tally_init<<<1, 64, 0, stream>>>(red, n_inst);
    k_prefix_mark<<<1, 1, 0, stream>>>(red);
    if (n_inst) {
        uint64_t blocks = (n_inst + 255) / 256;
        if (blocks > 2048) blocks = 2048;
        k_classic_first_bad_head<<<1, 256, 0, stream>>>(st, nullptr, n_inst, base, scalars, red);
        k_classic_first_bad<<<dim3((unsigned)blocks), 256, 0, stream>>>(st, nullptr, n_inst, base,
                                                                         scalars, red);
    }
    k_prefix_finalize<<<1, 64, 0, stream>>>(red, scalars, n_inst, base);
    return hipGetLastError();
}

}  // namespace mpx
