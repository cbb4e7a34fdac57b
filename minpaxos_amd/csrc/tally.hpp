// tally.hpp — accept-phase quorum tally as a wave-level device routine (A1 MIN / A2 CLASSIC).
//
// Reference semantics (record at a time, array order):
//   MIN     bareminpaxos.(*Replica).handleAcceptReply  src/bareminpaxos/bareminpaxos.go:1014-1064
//   CLASSIC paxos.(*Replica).handleAcceptReply         src/paxos/paxos.go:631-673
//
// Data-parallel restatement. Records are grouped by instance in ascending order, so one
// instance = one contiguous "segment". A wave takes 64 records per piece:
//   H = ballot(head), O = ballot(ok)                          (the per-instance ack bitvector)
//   okrank(l) = popcount(O & lanes[segstart(l) .. l]) (+ OKs carried from earlier pieces)
// MIN:     AcceptOKs after record l is old+okrank; decided at the record where it == N>>1;
//          peerCommits[id] set by every OK with old+okrank+1 > N>>1.
// CLASSIC: the instance commits at the OK with okrank == rc = max(1, N>>1 - old); records
//          after it are ignored (status COMMITTED), so NACK count / max ballot are taken over
//          the records before the crossing only (segmented max-scan).
// "Last assignment wins" scalars (committedUpTo, peerCommits) become max-reductions over
// 64-bit keys (position+1)<<32 | value.
#pragma once
#include "common.hpp"

namespace mpx {

struct TallyOut {
    uint64_t cu_key;  // MIN: key of the last crossing record (wave-uniform)
    uint64_t pc_key;  // MIN: lane j holds the key of the last peer-commit record from id j
    bool any_dec;     // CLASSIC: some instance committed
};

__device__ __forceinline__ int4 load_rec(const mpx_accept_reply* __restrict__ recs, uint64_t p) {
    return reinterpret_cast<const int4*>(recs)[p];
}

// First position p in [pos, n) such that p == lo or recs[p].instance != recs[p-1].instance.
// Wave-uniform; returns n if there is none.
__device__ __forceinline__ uint64_t find_head(const mpx_accept_reply* __restrict__ recs,
                                              uint64_t pos, uint64_t lo, uint64_t n) {
    if (pos <= lo) return lo < n ? lo : n;
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

__device__ __forceinline__ void mark_bit(uint32_t* bits, int64_t i) {
    atomicOr(&bits[i >> 5], 1u << (i & 31));
}

// final state of one instance from its old state and segment totals
template <int MODE>
__device__ __forceinline__ int4 tally_final(int32_t st, int32_t oks, int32_t nacks, int32_t mx,
                                            int32_t tot_ok, int32_t tot_nack, int32_t tmax,
                                            int32_t half, bool& crossed) {
    if (MODE == MPX_MODE_MIN) {
        // some k in (oks, oks+tot_ok] with k == half  (k+1 > half holds then)
        crossed = (oks < half) && (half <= oks + tot_ok);
        return make_int4(crossed ? MPX_COMMITTED : st, oks + tot_ok, nacks, mx);
    } else {
        const bool act = (st == MPX_PREPARED || st == MPX_ACCEPTED);
        if (!act) {
            crossed = false;
            return make_int4(st, oks, nacks, mx);
        }
        const int32_t rc = (half - oks) > 1 ? (half - oks) : 1;
        crossed = tot_ok >= rc;
        return make_int4(crossed ? MPX_COMMITTED : st, oks + (crossed ? rc : tot_ok),
                         nacks + tot_nack, mx > tmax ? mx : tmax);
    }
}

// Tally records [s, e) (s must be a segment head; e = n or a segment head). Instance state
// index = instance - base, window [0, n_inst). Positions for the last-wins keys are
// pos_off + p. Wave-cooperative: all 64 lanes must call.
template <int MODE>
__device__ __forceinline__ void tally_range(const mpx_accept_reply* __restrict__ recs,
                                            uint64_t s, uint64_t e,
                                            const mpx_inst_state* __restrict__ st_in,
                                            mpx_inst_state* __restrict__ st_out,
                                            uint64_t n_inst, int32_t base, int32_t half,
                                            int32_t nrep, uint8_t* __restrict__ decided,
                                            uint32_t* err, uint64_t pos_off, TallyOut& out,
                                            uint32_t* lds_dec_bits = nullptr,
                                            uint32_t* lds_touch_bits = nullptr) {
    const int l = lane_id();
    const uint64_t mine = lanes_upto(l);
    // open (carried) segment, wave-uniform
    bool c_open = false;
    int32_t c_inst = 0, c_status = 0, c_oks = 0, c_nacks = 0, c_max = 0;
    int32_t c_okcnt = 0, c_nackcnt = 0, c_nmax = INT32_MIN;

    int4 nxt = make_int4(0, 0, 0, 0);
    if (s + l < e) nxt = load_rec(recs, s + l);
    for (uint64_t b = s; b < e; b += kWave) {
        const int4 r = nxt;
        if (b + kWave + l < e) nxt = load_rec(recs, b + kWave + l);
        const uint64_t p = b + l;
        const bool valid = p < e;
        const int32_t inst = r.x, bal = r.y, id = r.z;
        const bool ok = valid && ((r.w & 0xff) == 1);  // OK == TRUE
        int32_t prev = __shfl_up(inst, 1);
        if (l == 0) prev = c_inst;
        const bool head = valid && (p == s || inst != prev);
        if (valid && p != s && inst < prev) raise_err(err, kErrOrder);
        const uint64_t H = ballot(head), O = ballot(ok), Vm = ballot(valid);

        // a segment carried from the previous piece that ended exactly at its last lane
        if (c_open && (H & 1ull)) {
            if (l == 0) {
                bool cr;
                const int4 f = tally_final<MODE>(c_status, c_oks, c_nacks, c_max, c_okcnt,
                                                 c_nackcnt, c_nmax, half, cr);
                reinterpret_cast<int4*>(st_out)[c_inst - base] = f;
                if (decided) decided[c_inst - base] = cr;
                if (lds_dec_bits && cr) mark_bit(lds_dec_bits, c_inst - base);
                if (lds_touch_bits) mark_bit(lds_touch_bits, c_inst - base);
            }
            c_open = false;
        }

        const uint64_t hb = H & mine;
        const int segstart = hb ? hi_bit(hb) : -1;
        const bool carried = segstart < 0;  // only possible while c_open
        const uint64_t segmask = carried ? mine : (mine & ~lanes_below(segstart));
        const int32_t okrank = popc(O & segmask) + (carried ? c_okcnt : 0);

        // old state of my instance: head lanes load, the segment shares it
        int4 sv = make_int4(0, 0, 0, 0);
        if (head) {
            const int64_t idx = (int64_t)inst - base;
            if (idx >= 0 && (uint64_t)idx < n_inst) {
                sv = reinterpret_cast<const int4*>(st_in)[idx];
                // CLASSIC reads inst.status for every reply (paxos.go:634)
                if (MODE == MPX_MODE_CLASSIC && sv.x == MPX_STATUS_NIL) raise_err(err, kErrNil);
            } else {
                raise_err(err, kErrNil);
                sv.x = MPX_STATUS_NIL;
            }
        }
        const int src = carried ? 0 : segstart;
        int32_t s_status = __shfl(sv.x, src), s_oks = __shfl(sv.y, src);
        int32_t s_nacks = __shfl(sv.z, src), s_max = __shfl(sv.w, src);
        if (carried) { s_status = c_status; s_oks = c_oks; s_nacks = c_nacks; s_max = c_max; }
        const bool inwin = s_status != MPX_STATUS_NIL;
        // MIN dereferences the instance only for OK replies (bareminpaxos.go:1023-1024)
        if (MODE == MPX_MODE_MIN && ok && !inwin) raise_err(err, kErrNil);

        bool dec;
        int32_t tot_nack = 0, tmax = INT32_MIN;
        if (MODE == MPX_MODE_MIN) {
            const int32_t k = s_oks + okrank;
            const bool c1 = ok && inwin && (k + 1 > half);
            dec = c1 && (k == half);
            if (c1 && (id < 0 || id >= nrep)) raise_err(err, kErrBadId);
            const uint64_t Dm = ballot(dec);
            if (Dm) {
                const int hl = hi_bit(Dm);
                out.cu_key = ((pos_off + b + hl + 1) << 32) | (uint32_t)readlane(inst, hl);
            }
            const uint64_t Pm = ballot(c1);
            if (Pm) {
                for (int j = 0; j < nrep; ++j) {
                    const uint64_t m = ballot(c1 && id == j);
                    if (m) {
                        const int hl = hi_bit(m);
                        const uint64_t key = ((pos_off + b + hl + 1) << 32) |
                                             (uint32_t)(readlane(inst, hl) - 1);
                        if (l == j) out.pc_key = key;
                    }
                }
            }
        } else {
            const bool act = inwin && (s_status == MPX_PREPARED || s_status == MPX_ACCEPTED);
            const int32_t rc = (half - s_oks) > 1 ? (half - s_oks) : 1;
            const bool proc = valid && act && (okrank - (ok ? 1 : 0)) < rc;
            dec = ok && proc && okrank == rc;
            const bool nk = valid && !ok && proc;
            const uint64_t NK = ballot(nk);
            tot_nack = popc(NK & segmask) + (carried ? c_nackcnt : 0);
            tmax = seg_max_scan(nk ? bal : INT32_MIN, head);
            if (carried) tmax = tmax > c_nmax ? tmax : c_nmax;
            if (ballot(dec)) out.any_dec = true;
        }

        // segments that end inside this piece (followed by a head in the same piece)
        const bool inner_end = valid && l < 63 && ((H >> (l + 1)) & 1ull);
        if (inner_end && inwin) {
            bool cr;
            const int4 f = tally_final<MODE>(s_status, s_oks, s_nacks, s_max, okrank, tot_nack,
                                             tmax, half, cr);
            reinterpret_cast<int4*>(st_out)[inst - base] = f;
            if (decided) decided[inst - base] = cr;
            if (lds_dec_bits && cr) mark_bit(lds_dec_bits, inst - base);
            if (lds_touch_bits) mark_bit(lds_touch_bits, inst - base);
        }
        // the segment holding the last valid lane stays open
        const int L = hi_bit(Vm);
        c_inst = readlane(inst, L);
        c_status = readlane(s_status, L);
        c_oks = readlane(s_oks, L);
        c_nacks = readlane(s_nacks, L);
        c_max = readlane(s_max, L);
        c_okcnt = readlane(okrank, L);
        c_nackcnt = readlane(tot_nack, L);
        c_nmax = readlane(tmax, L);
        c_open = c_status != MPX_STATUS_NIL;
    }
    if (c_open && l == 0) {
        bool cr;
        const int4 f = tally_final<MODE>(c_status, c_oks, c_nacks, c_max, c_okcnt, c_nackcnt,
                                         c_nmax, half, cr);
        reinterpret_cast<int4*>(st_out)[c_inst - base] = f;
        if (decided) decided[c_inst - base] = cr;
        if (lds_dec_bits && cr) mark_bit(lds_dec_bits, c_inst - base);
        if (lds_touch_bits) mark_bit(lds_touch_bits, c_inst - base);
    }
}

}  // namespace mpx
