// prepare.hip — Prepare-phase recovery kernels.
//
// A4 CLASSIC, per instance: paxos.(*Replica).handlePrepareReply  src/paxos/paxos.go:577-629.
//   Per reply in slot order, while status == PREPARING:
//     OK:   prepareOKs++; if ballot > maxRecvBallot {cmds = reply.Command; maxRecvBallot =
//           ballot; requeue proposals}; if prepareOKs+1 > N>>1 {PREPARED; nacks = 0;
//           defaultBallot = max(defaultBallot, inst.ballot); bcastAccept}
//     NACK: nacks++; maxRecvBallot = max(...); if nacks >= N>>1 {requeue proposals}
//   Data-parallel restatement: the replies processed are a prefix of the instance's segment
//   (up to the OK with okrank == rc = max(1, N>>1 - oks)). A reply is "selected" iff it is an
//   OK whose ballot strictly exceeds the exclusive segmented prefix-max of (maxRecvBallot,
//   earlier processed ballots) — the first arrival wins ties. The chosen value is the last
//   selected reply's value (or the instance's own value).
//
// A3 MIN, per group: bareminpaxos.(*Replica).handlePrepareReply
//   src/bareminpaxos/bareminpaxos.go:912-966. Strictly sequential per group (the selection,
//   catch-up and trigger all depend on the running committedUpTo), so one lane owns one group
//   and walks its R replies in arrival order; groups are independent.
#include "common.hpp"
#include "kernels.hpp"
#include "tile.hpp"

namespace mpx {

// CLASSIC prepare of one instance log, ONE launch: tile_walk (tile.hpp) gives every lane one
// instance and its replies in arrival order, and the lane runs paxos.go:580-627 on each with the
// 32-byte state in registers. defaultBallot (:606-608) is a max over the newly prepared
// instances' ballots: per workgroup an LDS max, one device-scope max per workgroup into the
// control words, and the workgroup that finishes last (ticket) raises defaultBallot and resets
// them. Instances without replies get prepared = 0 in the gap pass (no memset).
// Control words: [0] ticket, [1] ballot key (ballot ^ 0x80000000, 0 = none).
__global__ __launch_bounds__(kTileBlock) void k_prepare_tile(
    const mpx_prepare_reply* __restrict__ recs, uint64_t n, const mpx_prep_state* __restrict__ st_in,
    mpx_prep_state* __restrict__ st_out, uint64_t n_inst, int32_t base, int32_t half,
    int32_t* __restrict__ default_ballot, uint32_t* __restrict__ ctl, uint8_t* __restrict__ prepared,
    uint32_t* err) {
    __shared__ TileLds S;
    __shared__ uint32_t red;
    const int t = threadIdx.x, l = lane_id();
    if (t == 0) red = 0;
    uint32_t ebits = 0;
    const int4* r4 = reinterpret_cast<const int4*>(recs);
    const int4* s4 = reinterpret_cast<const int4*>(st_in);
    int4* o4 = reinterpret_cast<int4*>(st_out);
    int64_t spec_idx = -1;  // the state loaded ahead for round 0 (tile_walk's pre)
    int4 specA = make_int4(0, 0, 0, 0), specB = make_int4(0, 0, 0, 0);
    auto pre = [&](int32_t inst0) {
        spec_idx = (int64_t)inst0 - base + t;
        if (spec_idx >= 0 && (uint64_t)spec_idx < n_inst) {
            specA = ld_stream(s4 + 2 * spec_idx);
            specB = ld_stream(s4 + 2 * spec_idx + 1);
        }
    };
    tile_walk(S, r4, n, err, pre, [&](uint32_t a, uint32_t cnt, uint64_t after, uint64_t oend,
                                      bool own, int64_t nxt, bool first) {
        const int32_t inst = own ? S.rec[a].x : 0;
        const int64_t idx = (int64_t)inst - base;
        const bool inwin = own && idx >= 0 && (uint64_t)idx < n_inst;
        const bool hit = idx == spec_idx;
        spec_idx = -1;  // (later rounds of the tile load their own)
        int4 A = inwin ? (hit ? specA : ld_stream(s4 + 2 * idx))
                       : make_int4(0, MPX_STATUS_NIL, 0, 0);  // ballot status oks nacks
        int4 B = inwin ? (hit ? specB : ld_stream(s4 + 2 * idx + 1))
                       : make_int4(0, 0, 0, 0);  // mx value_id flags pad
        const bool live_inst = inwin && A.y != MPX_STATUS_NIL;
        ebits |= (own && !live_inst) ? kErrNil : 0u;
        // per-call event flags describe this call (the head record clears them)
        uint32_t fl = (uint32_t)B.z & ~(MPX_PF_REQUEUED | MPX_PF_PREPARED_NOW);
        int32_t prep = 0;
        auto step = [&](int4 r) {
            if (A.y != MPX_PREPARING) return;                       // :580-584
            const bool ok = (uint32_t)r.z == 1u;                    // OK == TRUE
            const bool higher = r.y > B.x;                          // :589 / :616 (strict)
            const bool hasp = (fl & MPX_PF_HAS_PROPOSALS) != 0;
            if (ok) {
                A.z++;                                              // :587
                if (higher) {
                    B.y = r.w;                                      // :590 cmds = reply.Command
                    B.x = r.y;                                      // :591
                    if (hasp) fl = (fl & ~MPX_PF_HAS_PROPOSALS) | MPX_PF_REQUEUED;  // :592-600
                }
                if (A.z + 1 > half) {                               // :603
                    A.y = MPX_PREPARED;                             // :604
                    A.w = 0;                                        // :605
                    fl |= MPX_PF_PREPARED_NOW;                      // :611 bcastAccept (host)
                    prep = 1;
                }
            } else {
                A.w++;                                              // :615
                if (higher) B.x = r.y;                              // :616-618
                if (A.w >= half && hasp)                            // :619-626
                    fl = (fl & ~MPX_PF_HAS_PROPOSALS) | MPX_PF_REQUEUED;
            }
        };
        uint32_t rmax = cnt;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t x = (uint32_t)__shfl_xor((int)rmax, d);
            rmax = rmax > x ? rmax : x;
        }
        rmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)rmax);
        for (uint32_t j = 0; j < rmax; ++j) {
            const int4 r = S.rec[j < cnt ? a + j : 0];
            if (j < cnt && live_inst) step(r);
        }
        for (uint64_t q = after; live_inst && q < oend; ++q) step(over_rec(S, r4, after, q));
        if (inwin && live_inst) {
            B.z = (int32_t)fl;
            st_stream(o4 + 2 * idx, A);
            st_stream(o4 + 2 * idx + 1, B);
            if (prepared) st_stream(prepared + idx, (uint8_t)(prep ? 1 : 0));
        }
        if (prepared)  // instances without replies (and nil ones between them) stay unprepared
            tile_gaps(own, idx, nxt == kNoNext ? INT64_MAX : nxt - base, first, n_inst,
                      [&](uint64_t q) { prepared[q] = 0; });
        // defaultBallot = max(defaultBallot, inst.ballot) over newly prepared instances
        uint32_t key = (live_inst && prep) ? ((uint32_t)A.x ^ 0x80000000u) : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t x = (uint32_t)__shfl_xor((int)key, d);
            key = key > x ? key : x;
        }
        if (l == 0 && key) atomicMax(&red, key);
    });
    if (ebits) raise_err(err, ebits);
    __syncthreads();
    if (t == 0 && red) atomic_max_done(&ctl[1], red);
    if (!last_workgroup(&ctl[0]) || t != 0) return;
    const uint32_t m = atomic_take(&ctl[1]);
    if (m) {
        const int32_t b = (int32_t)(m ^ 0x80000000u);
        if (b > *default_ballot) *default_ballot = b;
    }
}

hipError_t launch_prepare_classic(const mpx_prepare_reply* recs, uint64_t n,
                                  const mpx_prep_state* st_in, mpx_prep_state* st_out,
                                  uint64_t n_inst, int32_t base, int32_t nrep,
                                  int32_t* default_ballot, uint8_t* prepared, uint32_t* ctl,
                                  uint32_t* err, hipStream_t stream) {
    if (!n) {  // no replies: nothing changes, no instance prepared
        if (prepared && n_inst) (void)hipMemsetAsync(prepared, 0, n_inst, stream);
        return hipGetLastError();
    }
    const uint64_t tiles = (n + kTileRecs - 1) / kTileRecs;
    const uint32_t grid = resident_grid((const void*)k_prepare_tile, kTileBlock, tiles);
    k_prepare_tile<<<grid, kTileBlock, 0, stream>>>(recs, n, st_in, st_out, n_inst, base,
                                                     nrep >> 1, default_ballot, ctl, prepared, err);
    return hipGetLastError();
}

// ---- A3 MIN ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prepare_min(
    const mpx_prepare_reply_min* __restrict__ recs, const uint64_t* __restrict__ off,
    mpx_group_prep_state* __restrict__ gst, uint64_t n_groups, int32_t nrep,
    int32_t* __restrict__ peer, mpx_prepare_effect* __restrict__ eff, uint32_t* err) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    const int32_t half = nrep >> 1;
    mpx_group_prep_state b = gst[g];
    int32_t* pc = peer + g * (uint64_t)nrep;
    const uint64_t r0 = off[g], r1 = off[g + 1];
    if (r1 < r0) {
        raise_err(err, kErrInval);
        return;
    }
    for (uint64_t p = r0; p < r1; ++p) {
        const mpx_prepare_reply_min r = recs[p];
        uint32_t fl = 0;
        int32_t from = -1;
        if (b.default_ballot == r.ballot) {                           // :916-921
            fl |= MPX_EF_COUNTED;
            b.prepare_oks++;                                          // :922
            if (r.id < 0 || r.id >= nrep) {
                raise_err(err, kErrBadId);
            } else {
                pc[r.id] = r.last_committed;                          // :923
            }
            if (r.instance > b.highest_instance ||
                (r.instance == b.highest_instance && r.ballot > b.max_recv_ballot)) {  // :925
                b.value_id = r.value_id;
                b.max_recv_ballot = r.ballot;
                b.highest_instance = r.instance;
                fl |= MPX_EF_SELECTED;
            }
            if (b.committed_upto <= r.last_committed) {               // :934-940
                from = b.committed_upto + 1;
                fl |= MPX_EF_CATCHUP;
                b.committed_upto = r.last_committed;
            }
            if (b.prepare_oks == half && b.highest_instance > b.committed_upto) {  // :945-958
                b.committed_upto = b.highest_instance;
                b.triggered++;
                fl |= MPX_EF_TRIGGER;
            }
        }
        if (eff) {
            mpx_prepare_effect e;
            e.flags = fl;
            e.catchup_from = from;
            eff[p] = e;
        }
    }
    gst[g] = b;
}

hipError_t launch_prepare_min(const mpx_prepare_reply_min* recs, uint64_t n,
                              const uint64_t* grp_rec_off, mpx_group_prep_state* gst,
                              uint64_t n_groups, int32_t nrep, int32_t* peer_commits,
                              mpx_prepare_effect* eff, uint32_t* err, hipStream_t stream) {
    (void)n;
    if (n_groups) {
        const uint64_t blocks = (n_groups + 255) / 256;
        k_prepare_min<<<dim3((unsigned)blocks), 256, 0, stream>>>(recs, grp_rec_off, gst,
                                                                   n_groups, nrep, peer_commits,
                                                                   eff, err);
    }
    return hipGetLastError();
}

}  // namespace mpx
