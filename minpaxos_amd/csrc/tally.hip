// tally.hip — accept tally kernels for one instance log (configs 2 and the single-group API).
#include "kernels.hpp"
#include "tally.hpp"
#include "tile.hpp"

namespace mpx {

// Accept tally of one instance log: tile_walk (tile.hpp) hands every lane one instance and its
// replies in arrival order; the lane applies handleAcceptReply to each (state in registers).
//   MIN      bareminpaxos.go:1023-1053: OK replies only, no status check
//   CLASSIC  paxos.go:634-673: replies to instances not PREPARED/ACCEPTED are ignored
// The "last assignment wins" scalars of MIN (committedUpTo :1048, peerCommits[id] :1050) come
// from the highest instance that assigns them (instances ascend in array order; all of an
// instance's assignments of one scalar write the same value): per round a wave ballot finds the
// highest lane, one LDS max per wave, one partial per workgroup, a final one-block reduction.
// Window-relative keys idx+1 (0 = none) keep them unsigned.
constexpr int kRedFirstBad = 1 + MPX_MAX_REPLICAS;

template <int MODE>
__global__ __launch_bounds__(kTileBlock) void k_accept_tile(
    const mpx_accept_reply* __restrict__ recs, uint64_t n, const mpx_inst_state* __restrict__ st_in,
    mpx_inst_state* __restrict__ st_out, uint64_t n_inst, int32_t base, int32_t half, int32_t nrep,
    uint32_t* __restrict__ part, uint8_t* __restrict__ decided, uint32_t* err) {
    __shared__ TileLds S;
    __shared__ uint32_t red[1 + MPX_MAX_REPLICAS];
    const int t = threadIdx.x, l = lane_id();
    if (t <= MPX_MAX_REPLICAS) red[t] = 0;
    uint32_t ebits = 0;
    const int4* r4 = reinterpret_cast<const int4*>(recs);
    tile_walk(S, r4, n, err, [&](uint32_t a, uint32_t cnt, uint64_t after, uint64_t oend, bool own) {
        const int32_t inst = own ? S.rec[a].x : 0;
        const int64_t idx = (int64_t)inst - base;
        const bool inwin = own && idx >= 0 && (uint64_t)idx < n_inst;
        int4 st = inwin ? ld_stream(reinterpret_cast<const int4*>(st_in) + idx)
                        : make_int4(MPX_STATUS_NIL, 0, 0, 0);
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
        for (uint64_t q = after; inwin && q < oend; ++q) step(r4[q], 1);
        if (inwin) {
            st_stream(reinterpret_cast<int4*>(st_out) + idx, st);
            if (decided) st_stream(decided + idx, (uint8_t)(deci ? 1 : 0));
        }
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
    __syncthreads();
    if (t <= nrep) part[(uint64_t)blockIdx.x * kPartStride + t] = red[t];
    if (ebits) raise_err(err, ebits);
}

// reduce the workgroups' partials; MIN: write committedUpTo / peerCommits; CLASSIC: set red[0]
// (some instance committed) and red[kRedFirstBad] for k_classic_first_bad
template <int MODE>
__global__ void k_accept_reduce(const uint32_t* __restrict__ part, uint32_t n_part, int32_t nrep,
                                int32_t base, uint64_t n_inst, int32_t* scalars,
                                unsigned long long* red) {
    const int l = lane_id();  // each wave takes every (blockDim/64)-th scalar
    for (int w = threadIdx.x / kWave; w <= nrep; w += blockDim.x / kWave) {
        uint32_t m = 0;
        for (uint32_t i = l; i < n_part; i += kWave) {
            const uint32_t x = part[(uint64_t)i * kPartStride + w];
            m = m > x ? m : x;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t x = (uint32_t)__shfl_xor((int)m, d);
            m = m > x ? m : x;
        }
        if (l != 0) continue;
        if (MODE == MPX_MODE_MIN) {
            if (m) scalars[w] = (int32_t)((int64_t)base + m - 1 - (w ? 1 : 0));  // peerCommits: inst-1
        } else if (w == 0) {
            red[0] = m;
            red[kRedFirstBad] = n_inst;
        }
    }
}

__global__ void k_tally_init(unsigned long long* red, uint64_t n_inst) {
    const int t = threadIdx.x;
    if (t < kRedFirstBad) red[t] = 0;
    if (t == kRedFirstBad) red[t] = n_inst;
}

// CLASSIC updateCommittedUpTo (paxos.go:259-264) over the final statuses: find the first
// instance >= committedUpTo+1 that is not COMMITTED (final COMMITTED <=> st_in COMMITTED or
// decided in this call).
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

template <int MODE>
__global__ void k_tally_finalize(const unsigned long long* __restrict__ red, int32_t* scalars,
                                 int32_t nrep, uint64_t n_inst, int32_t base) {
    if (threadIdx.x != 0) return;
    if (MODE == MPX_MODE_MIN) {
        if (red[0]) scalars[0] = (int32_t)(uint32_t)(red[0] & 0xffffffffull);
        for (int j = 0; j < nrep; ++j)
            if (red[1 + j]) scalars[1 + j] = (int32_t)(uint32_t)(red[1 + j] & 0xffffffffull);
    } else {
        if (red[0] == 0) return;
        const int64_t j0 = (int64_t)scalars[0] + 1 - base;
        if (j0 < 0 || (uint64_t)j0 >= n_inst) return;
        const uint64_t fb = red[kRedFirstBad];  // first non-committed (n_inst if none)
        scalars[0] = (int32_t)(base + (int64_t)fb - 1);
    }
}

hipError_t launch_accept_tally(int mode, const mpx_accept_reply* recs, uint64_t n,
                               const mpx_inst_state* st_in, mpx_inst_state* st_out,
                               uint64_t n_inst, int32_t base, int32_t nrep, int32_t* scalars,
                               uint8_t* decided, unsigned long long* red, uint32_t* part,
                               uint32_t* err, hipStream_t stream) {
    const int32_t half = nrep >> 1;
    if (decided && n_inst) (void)hipMemsetAsync(decided, 0, n_inst, stream);
    const uint64_t tiles = (n + kTileRecs - 1) / kTileRecs;
    const uint32_t grid = (uint32_t)(tiles < (uint64_t)kTileGrid ? (tiles ? tiles : 1) : kTileGrid);
    const unsigned rblock = (unsigned)(kWave * (1 + nrep) < 256 ? kWave * (1 + nrep) : 256);
    if (mode == MPX_MODE_MIN) {
        k_accept_tile<MPX_MODE_MIN><<<grid, kTileBlock, 0, stream>>>(
            recs, n, st_in, st_out, n_inst, base, half, nrep, part, decided, err);
        k_accept_reduce<MPX_MODE_MIN><<<1, rblock, 0, stream>>>(part, grid, nrep, base, n_inst,
                                                                scalars, red);
    } else {
        k_accept_tile<MPX_MODE_CLASSIC><<<grid, kTileBlock, 0, stream>>>(
            recs, n, st_in, st_out, n_inst, base, half, nrep, part, decided, err);
        k_accept_reduce<MPX_MODE_CLASSIC><<<1, kWave, 0, stream>>>(part, grid, 0, base, n_inst,
                                                                   scalars, red);
        if (n_inst) {
            uint64_t blocks = (n_inst + 255) / 256;
            if (blocks > 2048) blocks = 2048;
            k_classic_first_bad_head<<<1, 256, 0, stream>>>(st_in, decided, n_inst, base,
                                                            scalars, red);
            k_classic_first_bad<<<dim3((unsigned)blocks), 256, 0, stream>>>(st_in, decided, n_inst,
                                                                             base, scalars, red);
        }
        k_tally_finalize<MPX_MODE_CLASSIC><<<1, 64, 0, stream>>>(red, scalars, nrep, n_inst,
                                                                 base);
    }
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
    k_tally_finalize<MPX_MODE_CLASSIC><<<1, 64, 0, stream>>>(red, scalars, 0, n_inst, base);
    return hipGetLastError();
}

}  // namespace mpx
