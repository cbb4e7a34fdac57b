// step.hip — fused per-group step for the sharded engine.
//
// One 256-thread workgroup owns one group (= one replica with its own instance space, leader
// bookkeeping and state.State) and does, back to back:
//   1. handleAcceptReply for the group's replies (tally_range, shared with tally.hip):
//      MIN   bareminpaxos.go:1014-1064, CLASSIC paxos.go:631-673 (+ updateCommittedUpTo
//      paxos.go:259-264 over the group's final statuses)
//   2. executeCommands  bareminpaxos.go:1066-1098 / paxos.go:675-706: instances
//      executed+1 .. committedUpTo while Cmds != nil, each command through Execute
//      (state.go:77-103) against the group's table, plus Conflict with the previous command
//      on the same key (state.go:53-60).
// The group's table lives in LDS as a dictionary (key, value, present) with an LDS hash
// index. Commands are processed in LDS-sized chunks in log order; within a chunk they are
// bucketed by key (counting sort in LDS) and each command finds its predecessor and the last
// PUT before it in its key's bucket. HBM traffic is one pass over replies, instance state,
// commands, outputs and the table.
#include "common.hpp"
#include "kernels.hpp"
#include "tally.hpp"

namespace mpx {

constexpr int kStepBlock = 256;
constexpr int kDCap = 1024;          // dictionary entries (table + distinct keys of the batch)
constexpr int kHCap = 2 * kDCap;     // LDS hash slots
constexpr int kChunk = 1024;         // commands per LDS chunk
constexpr int kPer = kChunk / kStepBlock;
constexpr int kMaxIpgBits = 8192;    // decided bitmap (CLASSIC prefix) covers ipg <= 8192
constexpr uint32_t kLock = 0xFFFFFFFFu;
constexpr uint32_t kDead = 0xFFFFFFFEu;
constexpr uint32_t kNoFirst = 0xFFFFFFFFu;

struct StepLds {
    int64_t dkey[kDCap];
    int64_t dval[kDCap];
    uint32_t dfirst[kDCap];   // first PUT (command index) of keys new to the table
    uint32_t cnt[kDCap];      // per-chunk commands per key
    uint32_t off[kDCap];      // exclusive scan of cnt
    uint32_t hslot[kHCap];    // 0 empty, kid+1, kLock, kDead
    int64_t cval[kChunk];     // chunk values
    uint16_t list[kChunk];    // (local index << 1) | isPut, bucketed by key
    uint8_t dpresent[kDCap];  // key present in the table (has a value)
    uint8_t dseen[kDCap];     // bit0: seen in this call, bit1: last op on it was a PUT
    uint32_t dec_bits[kMaxIpgBits / 32];
    uint32_t wsum[kStepBlock / kWave];
    unsigned long long red[1 + MPX_MAX_REPLICAS];
    uint32_t dn;
    uint32_t n_orig;
    uint32_t scal[4];
};

__device__ __forceinline__ uint32_t lhash(int64_t k) {
    uint64_t x = (uint64_t)k;
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return (uint32_t)x;
}

// find-or-insert into the LDS dictionary; returns kid or -1 (full)
__device__ int dict_insert(StepLds& S, int64_t key, bool is_new_value_unknown, uint32_t* err) {
    uint32_t h = lhash(key) & (kHCap - 1);
    for (int probe = 0; probe < kHCap;) {
        uint32_t cur = __hip_atomic_load(&S.hslot[h], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == 0) {
            const uint32_t old = atomicCAS(&S.hslot[h], 0u, kLock);
            if (old == 0) {
                const uint32_t kid = atomicAdd(&S.dn, 1u);
                if (kid >= (uint32_t)kDCap) {
                    raise_err(err, kErrKvFull);
                    __hip_atomic_store(&S.hslot[h], kDead, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    return -1;
                }
                S.dkey[kid] = key;
                S.dval[kid] = 0;
                S.dpresent[kid] = 0;
                S.dseen[kid] = 0;
                S.dfirst[kid] = kNoFirst;
                S.cnt[kid] = 0;
                __hip_atomic_store(&S.hslot[h], kid + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                return (int)kid;
            }
            cur = old;
        }
        if (cur == kLock) continue;  // being published by another lane: re-read this slot
        if (cur != kDead && S.dkey[cur - 1] == key) return (int)(cur - 1);
        h = (h + 1) & (kHCap - 1);
        ++probe;
    }
    raise_err(err, kErrKvFull);
    return -1;
}

// exclusive scan of S.cnt[0..n) into S.off (n <= kDCap), whole block
__device__ __forceinline__ void block_scan_cnt(StepLds& S, uint32_t n) {
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    constexpr int per = kDCap / kStepBlock;  // 4 contiguous entries per thread
    uint32_t v[per];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        const uint32_t i = t * per + k;
        v[k] = i < n ? S.cnt[i] : 0;
        sum += v[k];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t x = __shfl_up(incl, d);
        if (l >= d) incl += x;
    }
    if (l == kWave - 1) S.wsum[w] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (int k = 0; k < w; ++k) wbase += S.wsum[k];
    uint32_t run = wbase + incl - sum;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        const uint32_t i = t * per + k;
        if (i < (uint32_t)kDCap) S.off[i] = run;
        run += v[k];
    }
    __syncthreads();
}

template <int MODE>
__global__ __launch_bounds__(kStepBlock) void k_group_step(mpx_group_batch b, int32_t nrep,
                                                           uint32_t kvpg, uint32_t* err) {
    __shared__ StepLds S;
    const uint32_t g = blockIdx.x;
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    const int32_t half = nrep >> 1;
    const uint64_t ipg = b.ipg;
    const uint64_t gi0 = (uint64_t)g * ipg;
    const mpx_inst_state* st_in = b.st_in + gi0;
    mpx_inst_state* st_out = b.st_out + gi0;
    const bool use_bits = MODE == MPX_MODE_CLASSIC;

    if (t <= MPX_MAX_REPLICAS) S.red[t] = 0;
    if (use_bits)
        for (int i = t; i < kMaxIpgBits / 32; i += kStepBlock) S.dec_bits[i] = 0;
    for (int i = t; i < kHCap; i += kStepBlock) S.hslot[i] = 0;
    if (t == 0) {
        S.dn = 0;
        S.scal[0] = 0;
    }
    __syncthreads();

    // ---- 1. tally: 4 waves, each on an instance-aligned quarter of the group's replies ----
    const uint64_t r0 = b.grp_rec_off[g], r1 = b.grp_rec_off[g + 1];
    if (r1 > r0) {
        const uint64_t len = r1 - r0;
        const uint64_t n0 = r0 + len * w / (kStepBlock / kWave);
        const uint64_t n1 = r0 + len * (w + 1) / (kStepBlock / kWave);
        const uint64_t s = find_head(b.recs, n0, r0, r1);
        const uint64_t e = (n1 >= r1) ? r1 : find_head(b.recs, n1, r0, r1);
        if (s < e) {
            TallyOut out{0, 0, false};
            tally_range<MODE>(b.recs, s, e, st_in, st_out, ipg, 0, half, nrep,
                              b.decided ? b.decided + gi0 : nullptr, err, 0, out,
                              use_bits ? S.dec_bits : nullptr);
            if (MODE == MPX_MODE_MIN) {
                if (l == 0 && out.cu_key) atomicMax(&S.red[0], (unsigned long long)out.cu_key);
                if (l < nrep && out.pc_key) atomicMax(&S.red[1 + l], (unsigned long long)out.pc_key);
            } else {
                if (l == 0 && out.any_dec) atomicMax(&S.red[0], 1ull);
            }
        }
    }
    // decided flags of instances without replies
    if (b.decided && r1 == r0)
        for (uint64_t i = t; i < ipg; i += kStepBlock) b.decided[gi0 + i] = 0;
    __syncthreads();

    // ---- watermarks ----------------------------------------------------------------------
    const int32_t cu_in = b.committed_in[g];
    int32_t cu = cu_in;
    if (MODE == MPX_MODE_MIN) {
        if (S.red[0]) cu = (int32_t)(uint32_t)(S.red[0] & 0xffffffffull);
        if (t < nrep) {
            const unsigned long long k = S.red[1 + t];
            b.peer_out[(uint64_t)g * nrep + t] =
                k ? (int32_t)(uint32_t)(k & 0xffffffffull) : b.peer_in[(uint64_t)g * nrep + t];
        }
    } else {
        if (t < nrep) b.peer_out[(uint64_t)g * nrep + t] = b.peer_in[(uint64_t)g * nrep + t];
        if (S.red[0]) {
            // updateCommittedUpTo: first instance >= cu_in+1 neither COMMITTED nor decided now
            if (t == 0) S.scal[1] = (uint32_t)ipg;
            __syncthreads();
            const int64_t j0 = (int64_t)cu_in + 1;
            if (j0 >= 0 && (uint64_t)j0 < ipg) {
                for (uint64_t j = (uint64_t)j0 + t; j < ipg; j += kStepBlock) {
                    const bool dec = j < (uint64_t)kMaxIpgBits && ((S.dec_bits[j >> 5] >> (j & 31)) & 1u);
                    const bool c = dec || st_in[j].status == MPX_COMMITTED;
                    if (!c) {
                        atomicMin(&S.scal[1], (uint32_t)j);
                        break;
                    }
                }
            }
            __syncthreads();
            if (j0 >= 0 && (uint64_t)j0 < ipg) cu = (int32_t)S.scal[1] - 1;
        }
    }
    if (t == 0) b.committed_out[g] = cu;

    // ---- 2. executeCommands: instances exec+1 .. cu while Cmds != nil -------------------------
    const int32_t ex_in = b.executed_in[g];
    int64_t lo = (int64_t)ex_in + 1;
    int64_t hi = (int64_t)cu;  // inclusive
    if (hi >= (int64_t)ipg) hi = (int64_t)ipg - 1;
    if (lo < 0) lo = 0;  // (executed_in < -1 is treated as -1)
    if (t == 0) S.scal[2] = (uint32_t)(hi + 1 > lo ? hi + 1 : lo);
    __syncthreads();
    if (hi >= lo) {
        for (int64_t i = lo + t; i <= hi; i += kStepBlock) {
            const bool nil = st_in[i].status == MPX_STATUS_NIL ||
                             (b.has_cmds && !b.has_cmds[gi0 + i]);
            if (nil) {
                atomicMin(&S.scal[2], (uint32_t)i);
                break;
            }
        }
    }
    __syncthreads();
    const int64_t stop = hi >= lo ? (int64_t)S.scal[2] : lo;  // first instance not executed
    if (t == 0) b.executed_out[g] = stop > lo ? (int32_t)(stop - 1) : ex_in;

    // load the group's table into the dictionary
    const uint32_t ncnt = b.kv_cnt_in[g];
    if (ncnt > kvpg) {
        raise_err(err, kErrInval);
        return;
    }
    for (uint32_t e = t; e < ncnt; e += kStepBlock) {
        const int64_t k = b.kv_key_in[(uint64_t)g * kvpg + e];
        const int64_t v = b.kv_val_in[(uint64_t)g * kvpg + e];
        S.dkey[e] = k;
        S.dval[e] = v;
        S.dpresent[e] = 1;
        S.dseen[e] = 0;
        S.dfirst[e] = kNoFirst;
        uint32_t h = lhash(k) & (kHCap - 1);
        while (atomicCAS(&S.hslot[h], 0u, e + 1) != 0u) h = (h + 1) & (kHCap - 1);
    }
    if (t == 0) {
        S.dn = ncnt;
        S.n_orig = ncnt;
    }
    __syncthreads();

    if (stop > lo) {
        const uint64_t c_begin = b.cmd_off[gi0 + lo], c_end = b.cmd_off[gi0 + stop];
        for (uint64_t c0 = c_begin; c0 < c_end; c0 += kChunk) {
            const uint32_t n = (uint32_t)((c_end - c0) < (uint64_t)kChunk ? (c_end - c0) : kChunk);
            for (uint32_t i = t; i < (uint32_t)kDCap; i += kStepBlock) S.cnt[i] = 0;
            __syncthreads();
            uint8_t o[kPer];
            int kid[kPer];
            uint32_t pos[kPer];
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const uint32_t li = t + k * kStepBlock;
                kid[k] = -1;
                o[k] = 0;
                if (li < n) {
                    o[k] = b.op[c0 + li];
                    const int64_t key = b.key[c0 + li];
                    S.cval[li] = b.val[c0 + li];
                    kid[k] = dict_insert(S, key, true, err);
                    if (kid[k] >= 0) pos[k] = atomicAdd(&S.cnt[kid[k]], 1u);
                }
            }
            __syncthreads();
            const uint32_t dn = S.dn < (uint32_t)kDCap ? S.dn : (uint32_t)kDCap;
            block_scan_cnt(S, dn);
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const uint32_t li = t + k * kStepBlock;
                if (li < n && kid[k] >= 0)
                    S.list[S.off[kid[k]] + pos[k]] = (uint16_t)((li << 1) | (o[k] == MPX_OP_PUT ? 1u : 0u));
            }
            __syncthreads();
            // resolve every command against its key's bucket
            uint8_t fl[kPer];  // bit0 last of key in chunk, bit1 last PUT, bit2 first PUT
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const uint32_t li = t + k * kStepBlock;
                fl[k] = 0;
                if (li >= n || kid[k] < 0) continue;
                const int kd = kid[k];
                const bool isput = o[k] == MPX_OP_PUT;
                int prev = -1, prevput = 0, lastput = -1;
                bool later = false, laterput = false;
                const uint32_t a = S.off[kd], z = a + S.cnt[kd];
                for (uint32_t j = a; j < z; ++j) {
                    const uint32_t ent = S.list[j];
                    const int lj = (int)(ent >> 1);
                    const uint32_t pj = ent & 1u;
                    if (lj < (int)li) {
                        if (lj > prev) { prev = lj; prevput = (int)pj; }
                        if (pj && lj > lastput) lastput = lj;
                    } else if (lj > (int)li) {
                        later = true;
                        laterput |= pj != 0;
                    }
                }
                const uint8_t seen = S.dseen[kd];
                bool conf;
                if (prev >= 0) conf = prevput || isput;
                else conf = (seen & 1u) && ((seen & 2u) || isput);
                int64_t r = 0;
                if (isput) r = S.cval[li];
                else if (o[k] == MPX_OP_GET) {
                    if (lastput >= 0) r = S.cval[lastput];
                    else if (S.dpresent[kd]) r = S.dval[kd];
                }
                b.ret[c0 + li] = r;
                if (b.conf_prev) b.conf_prev[c0 + li] = conf ? 1 : 0;
                if (!later) fl[k] |= 1;
                if (isput && !laterput) fl[k] |= 2;
                if (isput && lastput < 0) fl[k] |= 4;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const uint32_t li = t + k * kStepBlock;
                if (li >= n || kid[k] < 0) continue;
                const int kd = kid[k];
                if (fl[k] & 1) S.dseen[kd] = (uint8_t)(1u | (o[k] == MPX_OP_PUT ? 2u : 0u));
                if (fl[k] & 2) {
                    S.dval[kd] = S.cval[li];
                    S.dpresent[kd] = 1;
                }
                if ((fl[k] & 4) && (uint32_t)kd >= S.n_orig && S.dfirst[kd] == kNoFirst)
                    S.dfirst[kd] = (uint32_t)(c0 + li - c_begin);
            }
            __syncthreads();
        }
    }

    // ---- write the table back: original entries in place, new keys in first-PUT order ----
    const uint32_t dn = S.dn < (uint32_t)kDCap ? S.dn : (uint32_t)kDCap;
    const uint32_t norig = S.n_orig;
    for (uint32_t e = t; e < norig; e += kStepBlock) {
        b.kv_key_out[(uint64_t)g * kvpg + e] = S.dkey[e];
        b.kv_val_out[(uint64_t)g * kvpg + e] = S.dval[e];
    }
    if (t == 0) S.scal[3] = 0;
    __syncthreads();
    for (uint32_t e = norig + t; e < dn; e += kStepBlock) {
        if (!S.dpresent[e]) continue;
        const uint32_t f = S.dfirst[e];
        uint32_t rank = 0;
        for (uint32_t x = norig; x < dn; ++x)
            if (S.dpresent[x] && S.dfirst[x] < f) ++rank;
        atomicAdd(&S.scal[3], 1u);
        const uint32_t dst = norig + rank;
        if (dst < kvpg) {
            b.kv_key_out[(uint64_t)g * kvpg + dst] = S.dkey[e];
            b.kv_val_out[(uint64_t)g * kvpg + dst] = S.dval[e];
        }
    }
    __syncthreads();
    if (t == 0) {
        const uint32_t total = norig + S.scal[3];
        if (total > kvpg) raise_err(err, kErrKvFull);
        b.kv_cnt_out[g] = total < kvpg ? total : kvpg;
    }
}

hipError_t launch_group_step(int mode, int32_t nrep, uint32_t kv_per_group,
                             const mpx_group_batch* b, uint32_t* err, hipStream_t stream) {
    if (!b->n_groups) return hipSuccess;
    if (kv_per_group > (uint32_t)kDCap) return hipErrorInvalidValue;
    if (mode == MPX_MODE_CLASSIC && b->ipg > (uint32_t)kMaxIpgBits) return hipErrorInvalidValue;
    if (mode == MPX_MODE_MIN)
        k_group_step<MPX_MODE_MIN><<<b->n_groups, kStepBlock, 0, stream>>>(*b, nrep, kv_per_group, err);
    else
        k_group_step<MPX_MODE_CLASSIC><<<b->n_groups, kStepBlock, 0, stream>>>(*b, nrep, kv_per_group,
                                                                             err);
    return hipGetLastError();
}

}  // namespace mpx
