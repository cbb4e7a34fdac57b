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

namespace mpx {

constexpr uint64_t kPrepTile = 512;
constexpr int kPrepBlock = 256;

__device__ __forceinline__ uint64_t find_head_prep(const mpx_prepare_reply* __restrict__ recs,
                                                   uint64_t pos, uint64_t n) {
    if (pos == 0) return n ? 0 : n;
    const int l = lane_id();
    for (uint64_t q = pos; q < n; q += kWave) {
        const uint64_t p = q + l;
        bool h = false;
        if (p < n) h = recs[p].instance != recs[p - 1].instance;
        const uint64_t m = ballot(h);
        if (m) return q + lo_bit(m);
    }
    return n;
}

struct PrepFinal {
    int4 a, b;
    bool crossed;
};

__device__ __forceinline__ PrepFinal prep_final(int32_t ib, int32_t st, int32_t oks, int32_t nacks,
                                                int32_t mx, uint32_t vid, uint32_t fl,
                                                int32_t tot_ok, int32_t tot_nack, int32_t bmax,
                                                uint32_t lastval, int32_t nsel, int32_t half) {
    PrepFinal f;
    fl &= ~(MPX_PF_REQUEUED | MPX_PF_PREPARED_NOW);
    if (st != MPX_PREPARING) {
        f.crossed = false;
        f.a = make_int4(ib, st, oks, nacks);
        f.b = make_int4(mx, (int)vid, (int)fl, 0);
        return f;
    }
    const int32_t rc = (half - oks) > 1 ? (half - oks) : 1;
    const bool crossed = tot_ok >= rc;
    const bool requeue = (fl & MPX_PF_HAS_PROPOSALS) &&
                         (nsel > 0 || (tot_nack >= 1 && nacks + tot_nack >= half));
    if (requeue) fl = (fl & ~MPX_PF_HAS_PROPOSALS) | MPX_PF_REQUEUED;
    if (crossed) fl |= MPX_PF_PREPARED_NOW;
    f.crossed = crossed;
    f.a = make_int4(ib, crossed ? MPX_PREPARED : st, oks + (crossed ? rc : tot_ok),
                    crossed ? 0 : nacks + tot_nack);
    f.b = make_int4(mx > bmax ? mx : bmax, (int)(nsel > 0 ? lastval : vid), (int)fl, 0);
    return f;
}

__global__ __launch_bounds__(kPrepBlock) void k_prepare_classic(
    const mpx_prepare_reply* __restrict__ recs, uint64_t n, const mpx_prep_state* __restrict__ st_in,
    mpx_prep_state* __restrict__ st_out, uint64_t n_inst, int32_t base, int32_t half,
    int32_t* __restrict__ default_ballot, uint8_t* __restrict__ prepared, uint32_t* err) {
    const uint64_t wave = ((uint64_t)blockIdx.x * kPrepBlock + threadIdx.x) / kWave;
    const uint64_t s0 = wave * kPrepTile;
    if (s0 >= n) return;
    const uint64_t s = find_head_prep(recs, s0, n);
    const uint64_t e = s0 + kPrepTile >= n ? n : find_head_prep(recs, s0 + kPrepTile, n);
    if (s >= e) return;
    const int l = lane_id();
    const uint64_t mine = lanes_upto(l);
    const int4* st4 = reinterpret_cast<const int4*>(st_in);
    int4* so4 = reinterpret_cast<int4*>(st_out);

    bool c_open = false;
    int32_t c_inst = 0, c_ib = 0, c_st = 0, c_oks = 0, c_nacks = 0, c_mx = 0;
    uint32_t c_vid = 0, c_fl = 0, c_lastval = 0;
    int32_t c_okcnt = 0, c_nackcnt = 0, c_bmax = INT32_MIN, c_nsel = 0;
    int32_t maxb = INT32_MIN;  // max inst.ballot of newly prepared instances (wave-local)

    auto flush = [&](int32_t inst, int32_t ib, int32_t st, int32_t oks, int32_t nacks, int32_t mx,
                     uint32_t vid, uint32_t fl, int32_t tot_ok, int32_t tot_nack, int32_t bmax,
                     uint32_t lastval, int32_t nsel) {
        PrepFinal f = prep_final(ib, st, oks, nacks, mx, vid, fl, tot_ok, tot_nack, bmax, lastval,
                                 nsel, half);
        const int64_t idx = (int64_t)inst - base;
        so4[2 * idx] = f.a;
        so4[2 * idx + 1] = f.b;
        if (prepared) prepared[idx] = f.crossed;
        if (f.crossed && ib > maxb) maxb = ib;
    };

    for (uint64_t b = s; b < e; b += kWave) {
        const uint64_t p = b + l;
        const bool valid = p < e;
        int4 r = make_int4(0, 0, 0, 0);
        if (valid) r = reinterpret_cast<const int4*>(recs)[p];
        const int32_t inst = r.x, bal = r.y;
        const bool ok = valid && (uint32_t)r.z == 1u;  // OK == TRUE
        const uint32_t vid = (uint32_t)r.w;
        int32_t prev = __shfl_up(inst, 1);
        if (l == 0) prev = c_inst;
        const bool head = valid && (p == s || inst != prev);
        if (valid && p != s && inst < prev) raise_err(err, kErrOrder);
        const uint64_t H = ballot(head), O = ballot(ok), Vm = ballot(valid);

        if (c_open && (H & 1ull)) {
            if (l == 0)
                flush(c_inst, c_ib, c_st, c_oks, c_nacks, c_mx, c_vid, c_fl, c_okcnt, c_nackcnt,
                      c_bmax, c_lastval, c_nsel);
            c_open = false;
        }
        const uint64_t hb = H & mine;
        const int segstart = hb ? hi_bit(hb) : -1;
        const bool carried = segstart < 0;
        const uint64_t segmask = carried ? mine : (mine & ~lanes_below(segstart));
        const int32_t okrank = popc(O & segmask) + (carried ? c_okcnt : 0);

        int4 sa = make_int4(0, MPX_STATUS_NIL, 0, 0), sb = make_int4(0, 0, 0, 0);
        if (head) {
            const int64_t idx = (int64_t)inst - base;
            if (idx >= 0 && (uint64_t)idx < n_inst) {
                sa = st4[2 * idx];
                sb = st4[2 * idx + 1];
                if (sa.y == MPX_STATUS_NIL) raise_err(err, kErrNil);
            } else {
                raise_err(err, kErrNil);
            }
        }
        const int src = carried ? 0 : segstart;
        int32_t s_ib = __shfl(sa.x, src), s_st = __shfl(sa.y, src), s_oks = __shfl(sa.z, src);
        int32_t s_nacks = __shfl(sa.w, src), s_mx = __shfl(sb.x, src);
        uint32_t s_vid = (uint32_t)__shfl(sb.y, src), s_fl = (uint32_t)__shfl(sb.z, src);
        if (carried) {
            s_ib = c_ib; s_st = c_st; s_oks = c_oks; s_nacks = c_nacks; s_mx = c_mx;
            s_vid = c_vid; s_fl = c_fl;
        }
        const bool act = s_st == MPX_PREPARING;
        const int32_t rc = (half - s_oks) > 1 ? (half - s_oks) : 1;
        const bool proc = valid && act && (okrank - (ok ? 1 : 0)) < rc;
        // processed records form a prefix of each segment: a scan over proc-masked ballots
        // gives both the exclusive prefix-max of every processed record and the final max
        const int32_t pb = proc ? bal : INT32_MIN;
        int32_t incl = seg_max_scan(pb, head);
        int32_t excl = __shfl_up(incl, 1);
        if (head || l == 0) excl = INT32_MIN;
        const int32_t init = carried ? (s_mx > c_bmax ? s_mx : c_bmax) : s_mx;
        excl = excl > init ? excl : init;
        if (carried) incl = incl > c_bmax ? incl : c_bmax;
        const bool sel = ok && proc && bal > excl;
        const uint64_t SEL = ballot(sel);
        const uint64_t NK = ballot(valid && !ok && proc);
        const int32_t tot_nack = popc(NK & segmask) + (carried ? c_nackcnt : 0);
        const uint64_t sm = SEL & segmask;
        const int32_t nsel = popc(sm) + (carried ? c_nsel : 0);
        const int ls = sm ? hi_bit(sm) : l;
        const uint32_t vls = (uint32_t)__shfl((int)vid, ls);
        const uint32_t lastval = sm ? vls : (carried ? c_lastval : s_vid);

        const bool inner_end = valid && l < 63 && ((H >> (l + 1)) & 1ull);
        if (inner_end && s_st != MPX_STATUS_NIL)
            flush(inst, s_ib, s_st, s_oks, s_nacks, s_mx, s_vid, s_fl, okrank, tot_nack, incl,
                  lastval, nsel);
        const int L = hi_bit(Vm);
        c_inst = readlane(inst, L);
        c_ib = readlane(s_ib, L);
        c_st = readlane(s_st, L);
        c_oks = readlane(s_oks, L);
        c_nacks = readlane(s_nacks, L);
        c_mx = readlane(s_mx, L);
        c_vid = readlane(s_vid, L);
        c_fl = readlane(s_fl, L);
        c_okcnt = readlane(okrank, L);
        c_nackcnt = readlane(tot_nack, L);
        c_bmax = readlane(incl, L);
        c_lastval = readlane(lastval, L);
        c_nsel = readlane(nsel, L);
        c_open = c_st != MPX_STATUS_NIL;
    }
    if (c_open && l == 0)
        flush(c_inst, c_ib, c_st, c_oks, c_nacks, c_mx, c_vid, c_fl, c_okcnt, c_nackcnt, c_bmax,
              c_lastval, c_nsel);
    // defaultBallot = max(defaultBallot, inst.ballot) over newly prepared instances
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const int32_t t = __shfl_xor(maxb, d);
        maxb = maxb > t ? maxb : t;
    }
    if (l == 0 && maxb != INT32_MIN) atomicMax(default_ballot, maxb);
}

hipError_t launch_prepare_classic(const mpx_prepare_reply* recs, uint64_t n,
                                  const mpx_prep_state* st_in, mpx_prep_state* st_out,
                                  uint64_t n_inst, int32_t base, int32_t nrep,
                                  int32_t* default_ballot, uint8_t* prepared, uint32_t* err,
                                  hipStream_t stream) {
    if (prepared && n_inst) (void)hipMemsetAsync(prepared, 0, n_inst, stream);
    if (n) {
        const uint64_t waves = (n + kPrepTile - 1) / kPrepTile;
        const uint64_t blocks = (waves * kWave + kPrepBlock - 1) / kPrepBlock;
        k_prepare_classic<<<dim3((unsigned)blocks), kPrepBlock, 0, stream>>>(
            recs, n, st_in, st_out, n_inst, base, nrep >> 1, default_ballot, prepared, err);
    }
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
