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
// Two kernels:
//   k_group_fast     groups that fit one LDS image (<= 1024 replies, <= 256 instances,
//                    <= 1024 commands, <= 256 table entries, <= 512 distinct keys). The replies
//                    and instance state are loaded up front (the reply image goes to LDS), the
//                    commands while the tally runs; the group's table becomes an LDS hash table
//                    keyed by the 64-bit key and the commands are resolved by a chunk scan in
//                    log order (see "fast path" below). Nothing is written until the group is
//                    known to fit; a group that does not is appended to a work list instead.
//   k_group_general  the work list: chunked apply of any size, larger instance spaces; its
//                    dictionary and per-key command buckets live in LDS.
#include "common.hpp"
#include "kernels.hpp"
#include "tally.hpp"

namespace mpx {

// Diagnostic build only (-DMPX_STAMPS=1, tools/stamp_step.py): thread 0 of every workgroup adds
// the s_memtime delta of each barrier-delimited phase to a global accumulator.
#ifndef MPX_STAMPS
#define MPX_STAMPS 0
#endif
// MPX_STAMPS=2 (tools/stamp_span.py) keeps instead every fast workgroup's start and end on the
// chip-wide 100 MHz clock (s_memrealtime), stored by thread 0 with a vector store (no shared
// accumulator: 65,536 workgroups' atomics on one word serialise), so the rounds of resident
// workgroups - and the last, partial one - can be told apart
#if MPX_STAMPS
__device__ unsigned long long mpx_stamp_acc[16];
constexpr uint32_t kSpanMax = 1u << 17;
__device__ unsigned long long mpx_wg_span[kSpanMax][2];
#define STAMP_DECL                                                     \
    unsigned long long _st_prev = 0, _st_rt0 = 0;                      \
    if (threadIdx.x == 0) {                                            \
        _st_prev = __builtin_amdgcn_s_memtime();                       \
        _st_rt0 = __builtin_amdgcn_s_memrealtime();                    \
    }
#define STAMP_SPAN()                                                   \
    do {                                                               \
        if (MPX_STAMPS >= 2 && threadIdx.x == 0 && blockIdx.x < kSpanMax) { \
            mpx_wg_span[blockIdx.x][0] = _st_rt0;                      \
            mpx_wg_span[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime(); \
        }                                                              \
    } while (0)
#define STAMP(k)                                                       \
    do {                                                               \
        if (MPX_STAMPS == 1 && threadIdx.x == 0) { /* (2: spans only) */ \
            unsigned long long _n = __builtin_amdgcn_s_memtime();      \
            atomicAdd(&mpx_stamp_acc[k], _n - _st_prev);               \
            _st_prev = _n;                                             \
        }                                                              \
    } while (0)
#else
#define STAMP_DECL
#define STAMP(k)
#define STAMP_SPAN()
#endif
// Diagnostic A/B builds only (make variant DEFS=-DMPX_ABLATE=bits): skip a phase of k_group_fast
// to price it (results are wrong). 1 tally, 2 key lookup, 4 resolve scan, 8 reply ranges,
// 16 table/state outputs, 32 every instance commits (with 1: the apply without the tally).
#ifndef MPX_ABLATE
#define MPX_ABLATE 0
#endif

// the fast kernel's per-chunk slot match: LDS peer masks (0) or ballots over the slot bits (1:
// 4 KB less LDS, 7-8 workgroups per CU instead of 6, but 0.667 -> 0.755 ms per config-5 step
// in a same-box A/B, tools/gpu_step_ab.sh: more resident groups contend for the memory system)
#ifndef MPX_STEP_BALLOT
#define MPX_STEP_BALLOT 0
#endif

constexpr int kStepBlock = 256;
constexpr uint32_t kLock = 0xFFFFFFFFu;
constexpr uint32_t kDead = 0xFFFFFFFEu;
constexpr uint32_t kNoFirst = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t lhash(int64_t k) {
    uint64_t x = (uint64_t)k;
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return (uint32_t)x;
}

// LDS dictionary views shared by both kernels
struct Dict {
    int64_t* dkey;
    int64_t* dval;
    uint32_t* dfirst;
    uint32_t* cnt;
    uint32_t* hslot;
    uint8_t* dpresent;
    uint8_t* dseen;
    uint32_t* dn;
    uint32_t dcap, hcap;
};

// find-or-insert; returns kid, or -1 when the dictionary is full
__device__ int dict_insert(const Dict& D, int64_t key) {
    uint32_t h = lhash(key) & (D.hcap - 1);
    for (uint32_t probe = 0; probe < D.hcap;) {
        uint32_t cur = __hip_atomic_load(&D.hslot[h], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == 0) {
            const uint32_t old = atomicCAS(&D.hslot[h], 0u, kLock);
            if (old == 0) {
                const uint32_t kid = atomicAdd(D.dn, 1u);
                if (kid >= D.dcap) {
                    __hip_atomic_store(&D.hslot[h], kDead, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    return -1;
                }
                D.dkey[kid] = key;
                D.dval[kid] = 0;
                D.dpresent[kid] = 0;
                D.dseen[kid] = 0;
                D.dfirst[kid] = kNoFirst;
                D.cnt[kid] = 0;
                __hip_atomic_store(&D.hslot[h], kid + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                return (int)kid;
            }
            cur = old;
        }
        if (cur == kLock) continue;  // being published by another lane: re-read this slot
        if (cur != kDead && D.dkey[cur - 1] == key) return (int)(cur - 1);
        h = (h + 1) & (D.hcap - 1);
        ++probe;
    }
    return -1;
}

// insert a key known to be absent (table load): no lock needed, keys are unique
__device__ __forceinline__ void dict_put_unique(const Dict& D, uint32_t e, int64_t k, int64_t v) {
    D.dkey[e] = k;
    D.dval[e] = v;
    D.dpresent[e] = 1;
    D.dseen[e] = 0;
    D.dfirst[e] = kNoFirst;
    uint32_t h = lhash(k) & (D.hcap - 1);
    while (atomicCAS(&D.hslot[h], 0u, e + 1) != 0u) h = (h + 1) & (D.hcap - 1);
}

// exclusive scan of cnt[0..n) into off (n <= PER*256), whole block
template <int PER, typename OffT>
__device__ __forceinline__ void block_scan(const uint32_t* cnt, OffT* off, uint32_t n,
                                           uint32_t* wsum) {
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    uint32_t v[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const uint32_t i = t * PER + k;
        v[k] = i < n ? cnt[i] : 0;
        sum += v[k];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t x = __shfl_up(incl, d);
        if (l >= d) incl += x;
    }
    if (l == kWave - 1) wsum[w] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (int k = 0; k < w; ++k) wbase += wsum[k];
    uint32_t run = wbase + incl - sum;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const uint32_t i = t * PER + k;
        if (i < n) off[i] = (OffT)run;
        run += v[k];
    }
    __syncthreads();
}

// resolve one command against its key's bucket; returns flags bit0 last-of-key, bit1 last PUT,
// bit2 first PUT (all within the bucket = this chunk)
template <typename OffT>
__device__ __forceinline__ uint8_t resolve_cmd(const Dict& D, const OffT* off,
                                               const uint16_t* list, const int64_t* cval, int kd,
                                               uint32_t li, uint8_t o, int64_t& r, bool& conf) {
    const bool isput = o == MPX_OP_PUT;
    int prev = -1, prevput = 0, lastput = -1;
    bool later = false, laterput = false;
    const uint32_t a = off[kd], z = a + D.cnt[kd];
    for (uint32_t j = a; j < z; ++j) {
        const uint32_t ent = list[j];
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
    const uint8_t seen = D.dseen[kd];
    if (prev >= 0) conf = prevput || isput;
    else conf = (seen & 1u) && ((seen & 2u) || isput);
    r = 0;
    if (isput) r = cval[li];
    else if (o == MPX_OP_GET) {
        if (lastput >= 0) r = cval[lastput];
        else if (D.dpresent[kd]) r = D.dval[kd];
    }
    uint8_t fl = 0;
    if (!later) fl |= 1;
    if (isput && !laterput) fl |= 2;
    if (isput && lastput < 0) fl |= 4;
    return fl;
}

__device__ __forceinline__ void apply_update(const Dict& D, int kd, uint8_t fl, uint8_t o,
                                             int64_t v, uint32_t first_pos, uint32_t n_orig) {
    if (fl & 1) D.dseen[kd] = (uint8_t)(1u | (o == MPX_OP_PUT ? 2u : 0u));
    if (fl & 2) {
        D.dval[kd] = v;
        D.dpresent[kd] = 1;
    }
    if ((fl & 4) && (uint32_t)kd >= n_orig && D.dfirst[kd] == kNoFirst) D.dfirst[kd] = first_pos;
}

// write the dictionary back as the group's compact table: original entries in place, new
// present keys appended in order of their first PUT. Returns nothing; sets *total (LDS).
__device__ __forceinline__ void table_writeback(const Dict& D, uint32_t norig, uint32_t dn,
                                                int64_t* kk, int64_t* kv, uint32_t kvpg,
                                                uint32_t* total, uint32_t* err) {
    const int t = threadIdx.x;
    for (uint32_t e = t; e < norig; e += kStepBlock) {
        kk[e] = D.dkey[e];
        kv[e] = D.dval[e];
    }
    if (t == 0) *total = norig;
    __syncthreads();
    for (uint32_t e = norig + t; e < dn; e += kStepBlock) {
        if (!D.dpresent[e]) continue;
        const uint32_t f = D.dfirst[e];
        uint32_t rank = 0;
        for (uint32_t x = norig; x < dn; ++x)
            if (D.dpresent[x] && D.dfirst[x] < f) ++rank;
        atomicAdd(total, 1u);
        const uint32_t dst = norig + rank;
        if (dst < kvpg) {
            kk[dst] = D.dkey[e];
            kv[dst] = D.dval[e];
        }
    }
    __syncthreads();
    if (t == 0 && *total > kvpg) raise_err(err, kErrKvFull);
}

// ======================================== fast path ===========================================
// Per workgroup = per group, transpositions of the sequential reference loops, written with
// uniform control flow (loop trip counts are wave maxima, bodies are predicated) because the
// scalar unit, shared by the CU's four SIMDs, is what divergent code saturates:
//   tally    one lane per INSTANCE applies the handler to that instance's replies in arrival
//            order (state in registers); the only cross-instance outputs (committedUpTo,
//            peerCommits: last assignment in array order) are max-reductions over
//            (position+1)<<32 | value keys
//   table    the group's table and the executed commands' keys share one open-addressing LDS
//            table keyed by the 64-bit key itself: one 64-bit compare-and-swap per probe finds
//            the key or claims a free slot for it (no locks, no second lookup)
//   scan     commands in log order, wave w owning commands [256w, 256w+256) as four chunks of
//            64: a command's predecessor and last earlier PUT on its key come from the lower
//            lanes of its chunk (ballot match on the slot), the wave's earlier chunks (a per-wave
//            slot table) and the earlier waves (their tables); the key's last PUT overall is its
//            value after the step
// The group is applied in one chunk, so no per-key state carries between chunks: a key is
// present at the start iff it is one of the table's entries. Nothing reaches global memory
// before the group is known to fit; otherwise it goes to k_group_general via the work list
// (also for the one key the free-slot marker cannot hold, INT64_MIN).
// Capacities of one fast-path variant: T threads = T instance slots, R replies, C commands,
// TB table entries at the start of the step, 2^HB hash slots (table + new keys). The launcher
// picks the smallest variant a batch's shape (N, ipg, kv_per_group) fits; a group that still
// overflows one at run time goes to the general kernel.
template <int T_, int R_, int C_, int TB_, int HB_, int HN_ = (1 << HB_)>
struct FastCfg {
    static constexpr int kFT = T_, kFRecs = R_, kFIpg = T_, kFCmds = C_, kFTab = TB_;
    // kFH key slots (HN_, a power of two by default), slot ids of kFHB bits
    static constexpr int kFHB = HB_, kFH = HN_;
    static constexpr bool kFHPow2 = (HN_ & (HN_ - 1)) == 0;
    static_assert(HN_ <= (1 << HB_) && HN_ >= TB_ && HN_ % 8 == 0, "slot count");
    static constexpr int kFPer = kFCmds / kFT;    // commands per thread
    static constexpr int kFRecPer = kFRecs / kFT; // replies per thread
    static constexpr int kFTabPer = (kFTab + kFT - 1) / kFT;
    static constexpr int kFWaves = kFT / kWave;
    static constexpr int kWaveCmds = kFCmds / kFWaves;  // commands per wave
    // the table's start values in LDS (GETs of keys present at the start read them there);
    // the 1024-key variant reads them from the input table instead: its 8 KB would hold the
    // workgroup at 3 per CU (41.7 KB), without them 4 fit (33.5 KB)
#ifndef MPX_DVAL_LDS_MAX
#define MPX_DVAL_LDS_MAX 512
#endif
    static constexpr bool kFDvalLds = TB_ <= MPX_DVAL_LDS_MAX;
    static_assert(kFCmds % kFT == 0 && kFRecs % kFT == 0, "whole items per thread");
    static_assert(kFCmds / 32 <= kWave, "the new-key bitmap is scanned by one wave");
    static_assert(kWaveCmds < 2047, "kTabLp holds 1 + a wave-relative command index");
    static_assert((kFH * 2) % 16 == 0, "the wave tables are cleared by 16-byte stores");
};
#ifndef MPX_FASTBASE_SLOTS  // A/B builds: FastBase's key slots (512, or 384: 7 workgroups per CU)
#define MPX_FASTBASE_SLOTS 512
#endif
using FastBase = FastCfg<256, 1024, 1024, 256, 9, MPX_FASTBASE_SLOTS>;  // config 5: N <= 5, keys <= 256
using FastRecs = FastCfg<256, 2048, 1024, 256, 9>;   // N <= 9
using FastKeys = FastCfg<256, 1024, 1024, 1024, 10>; // group tables of up to 1024 keys
using FastWide = FastCfg<512, 2048, 2048, 512, 10>;  // 512 instances per group
// 512 instances per group with tables of up to 256 keys: a 512-slot hash halves the per-wave
// slot tables, 3 workgroups per CU instead of 2
using FastWide256 = FastCfg<512, 2048, 2048, 256, 9>;
constexpr uint16_t kNone16 = 0xFFFF;
constexpr uint8_t kIdBad = 31;
constexpr unsigned long long kFreeKey = 0x8000000000000000ull;  // INT64_MIN marks a free slot
constexpr uint32_t kOverflow = 0x80000000u;                      // ebits: group leaves the fast path
// chunk-scan state of a slot: a per-wave table entry (16 bits) and a command's view of its
// predecessors (32 bits) share the two flag bits; the low bits hold 1 + the last PUT (0 = none),
// relative to the wave's first command in a table entry, absolute in a command's view
constexpr uint32_t kTabAny = 0x8000u;  // some earlier command used the slot
constexpr uint32_t kTabPut = 0x4000u;  // ... and the latest of them is a PUT
constexpr uint32_t kTabLp = 0x07FFu;

#define MPX_FAST_CONSTS                                                      \
    constexpr int kFT = Cfg::kFT, kFRecs = Cfg::kFRecs, kFIpg = Cfg::kFIpg;    \
    constexpr int kFCmds = Cfg::kFCmds, kFTab = Cfg::kFTab, kFH = Cfg::kFH;    \
    constexpr int kFPer = Cfg::kFPer, kFRecPer = Cfg::kFRecPer;                \
    constexpr int kFTabPer = Cfg::kFTabPer, kFWaves = Cfg::kFWaves;            \
    constexpr int kWaveCmds = Cfg::kWaveCmds;                                   \
    (void)kFT; (void)kFRecs; (void)kFIpg; (void)kFCmds; (void)kFTab; (void)kFH; \
    (void)kFPer; (void)kFRecPer; (void)kFTabPer; (void)kFWaves; (void)kWaveCmds;

template <class Cfg, int MODE>
struct FastLds {
    static constexpr int kFRecs = Cfg::kFRecs, kFIpg = Cfg::kFIpg, kFCmds = Cfg::kFCmds;
    static constexpr int kFTab = Cfg::kFTab, kFH = Cfg::kFH, kFWaves = Cfg::kFWaves;
    union {
        struct {                 // until the tally: the group's replies (SoA) + reply ranges
            int32_t inst[kFRecs];
            // reply ballots: CLASSIC only (MIN's handleAcceptReply ignores them; without them
            // the N <= 9 variant's MIN workgroup fits 6 per CU instead of 5)
            int32_t bal[MODE == MPX_MODE_CLASSIC ? kFRecs : 1];
            uint8_t idok[kFRecs];    // (id code << 1) | ok, id code kIdBad = outside [0, N)
            uint16_t rstart[kFIpg];
            uint16_t rend[kFIpg];
        } a;
        struct {                 // after the tally: command values and the chunk-scan tables
            int64_t cval[kFCmds];
            // per wave and slot, over the wave's commands seen so far (see kTabAny): whether any
            // command used the slot, whether the last one was a PUT, 1 + the last PUT relative
            // to the wave's first command (0 = none)
            uint16_t tab[kFWaves * kFH];
#if !MPX_STEP_BALLOT
            // per wave, the chunk match: slot -> a lane of the chunk on that slot (the class),
            // class -> mask of the chunk's lanes on the slot
            uint8_t win[kFWaves * kFH];
            unsigned long long pmask[kFWaves * kWave];
#endif
        } b;
    } u;
    unsigned long long hkey[kFH];  // slot -> key; kFreeKey = free
    int64_t dval[Cfg::kFDvalLds ? kFTab : 1];  // table entry values at the start of the step
    uint16_t tabidx[kFH];    // table entry holding the slot's key; kNone16 = new to the table
    uint32_t newbits[kFCmds / 32];  // first PUTs of new keys, as a bitmap over command index
    uint16_t coff[kFIpg + 2];       // instance -> first command (group-relative)
    uint32_t red[1 + MPX_MAX_REPLICAS];  // 1 + instance: last crossing, last peerCommits[id] source
    uint32_t firstnil, firstbad, flags, ndec;
#ifdef MPX_LDS_PAD
    uint8_t lds_pad[MPX_LDS_PAD];  // A/B builds only: lowers occupancy to price it
#endif
};

// wave-uniform maximum of a per-lane value
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t x = __shfl_xor(v, d);
        v = v > x ? v : x;
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// home slot of a key in the fast path's table: Fibonacci hashing of the folded key (the top
// HB bits of a 32-bit multiplicative hash; for a slot count that is not a power of two, the
// hash scaled to [0, kFH) by a multiply-high)
template <int HB>
__device__ __forceinline__ uint32_t fhash(int64_t k) {
    const uint32_t x = (uint32_t)(uint64_t)k ^ (uint32_t)((uint64_t)k >> 32);
    return (x * 0x9E3779B1u) >> (32 - HB);
}
template <class Cfg>
__device__ __forceinline__ uint32_t fhome(int64_t k) {
    if constexpr (Cfg::kFHPow2) {
        return fhash<Cfg::kFHB>(k);
    } else {
        const uint32_t x = (uint32_t)(uint64_t)k ^ (uint32_t)((uint64_t)k >> 32);
        return (uint32_t)(((uint64_t)(x * 0x9E3779B1u) * (uint32_t)Cfg::kFH) >> 32);
    }
}

// slot of key in the group's table, claiming a free slot if the key is absent (*fresh = 1);
// -1 when the table is full. Linear probing; the CAS returns the slot's key, so a probe that
// meets the key (inserted earlier or concurrently by another lane) ends there too.
template <class Cfg, class Lds>
__device__ __forceinline__ int fast_slot(Lds& S, unsigned long long key, uint32_t h,
                                         int& fresh) {
    constexpr int kFH = Cfg::kFH;
    uint32_t i = h;  // (fhome: < kFH)
    for (int probe = 0; probe < kFH; ++probe) {
        const unsigned long long old = atomicCAS(&S.hkey[i], kFreeKey, key);
        if (old == kFreeKey || old == key) {
            fresh = old == kFreeKey;
            return (int)i;
        }
        i = Cfg::kFHPow2 ? (i + 1) & (kFH - 1) : (i + 1 == (uint32_t)kFH ? 0u : i + 1);
    }
    return -1;
}

// One-launch steps (mpx_config.flags MPX_FLAG_STEP_ONE_LAUNCH): no work-list kernel follows.
// A group the fast kernel cannot take fails the step (kErrInval) instead of going on the list,
// and with totals every group adds one packed word - arrival | decided << 7 | executed
// instances << 23 | executed commands << 39 - into slot g % ceil(G / 64) of `pslots` (at most 64
// groups of at most 512 instances and 2048 commands: no field overflows into the next). The grid's last
// workgroup (dispatched last: every other one is resident or done) waits for every slot's
// arrivals, sums and zeroes the slots and writes the totals: one kernel per step. Measured
// (same box, graph replay, --emulate-world 8): 0.1026-0.1037 ms per step against 0.0967-0.0980
// for the two-launch step - the fold's serial tail (the grid's last group, a round trip to the
// slots, the zeroing stores) outlasts the work-list kernel's launch inside a graph (~2 us; the
// fast kernel without any totals: 0.0945-0.0954; polling sleeps 2/16/64 change nothing), so
// the flag is an option, not the default.
constexpr uint32_t kPkGroups = 64;
__device__ __forceinline__ unsigned long long pk_word(uint32_t d, uint32_t xi, uint32_t xc) {
    return 1ull | ((unsigned long long)d << 7) | ((unsigned long long)xi << 23) |
           ((unsigned long long)xc << 39);
}
// slot of group g: interleaved (g % nslots), so the groups running at the same time add into
// different words; slot s then holds (G - 1 - s) / nslots + 1 <= 64 groups
__device__ __forceinline__ uint32_t pk_slots(uint32_t n_groups) {
    return (n_groups + kPkGroups - 1) / kPkGroups;
}
__device__ void fold_packed(unsigned long long* pslots, uint32_t n_groups, int64_t* totals,
                            uint32_t* err) {
    __shared__ unsigned long long fsum[3];
    if (threadIdx.x < 3) fsum[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long d = 0, xi = 0, xc = 0;
    const uint32_t nslots = pk_slots(n_groups);
    // slots a thread loads at once (one round trip for them); 2 keeps the fast kernel's VGPRs
    // (8: 60 -> 90, one workgroup per CU fewer, the step 2-5 % slower)
    constexpr int kBatch = 2;
    for (uint32_t s0 = threadIdx.x; s0 < nslots; s0 += blockDim.x * kBatch) {
        unsigned long long w[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const uint32_t sl = s0 + k * blockDim.x;
            w[k] = sl < nslots ? __hip_atomic_load(pslots + sl, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)
                               : 0ull;
        }
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const uint32_t sl = s0 + k * blockDim.x;
            if (sl >= nslots) continue;
            const uint32_t want = (n_groups - 1u - sl) / nslots + 1u;
            uint32_t spins = 0;
            bool late = false;
            while ((w[k] & 127ull) < want) {  // a group still running (the grid's tail)
                __builtin_amdgcn_s_sleep(2);
                w[k] = __hip_atomic_load(pslots + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (++spins == (1u << 22)) {  // never on a well-formed launch: fail, do not hang
                    // the slot is left as it is (a straggler's add may still land in it): the
                    // host zeroes every slot before the next one-launch step (kErrSlots)
                    raise_err(err, kErrInval | kErrSlots);
                    late = true;
                    break;
                }
            }
            if (!late) __hip_atomic_store(pslots + sl, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            d += (w[k] >> 7) & 0xFFFFull;
            xi += (w[k] >> 23) & 0xFFFFull;
            xc += w[k] >> 39;
        }
    }
    if (d) atomicAdd(&fsum[0], d);
    if (xi) atomicAdd(&fsum[1], xi);
    if (xc) atomicAdd(&fsum[2], xc);
    __syncthreads();
    if (threadIdx.x < 3) totals[threadIdx.x] = (int64_t)fsum[threadIdx.x];
}

// kOne: the one-launch step's instance (pslots / totals used); the two-launch step's instance has
// them compiled out (pointers known null), so its code carries none of the fold's paths - code a
// step never runs still costs the kernel through register allocation and scheduling (a dormant
// timing hook cost 2.5-4 %)
template <int MODE, class Cfg, bool kOne>
__global__ __launch_bounds__(Cfg::kFT) void k_group_fast(mpx_group_batch b, int32_t nrep,
                                                         uint32_t kvpg, uint32_t* worklist,
                                                         uint32_t* wcount,
                                                         unsigned long long* tacc, uint32_t* err,
                                                         unsigned long long* pslots,
                                                         int64_t* totals) {
    if constexpr (!kOne) {
        pslots = nullptr;
        totals = nullptr;
    }
    MPX_FAST_CONSTS
    __shared__ FastLds<Cfg, MODE> S;
    STAMP_DECL
    const uint32_t g = blockIdx.x;
    const int t = threadIdx.x, l = lane_id();
    const int32_t half = nrep >> 1;
    const uint32_t ipg = b.ipg;
    const uint64_t gi0 = (uint64_t)g * ipg;
    const uint64_t r0 = b.grp_rec_off[g], r1 = b.grp_rec_off[g + 1];
    const uint32_t c_lo = b.cmd_off[gi0], c_hi = b.cmd_off[gi0 + ipg];
    const uint32_t kcnt = b.kv_cnt_in[g];
    const int32_t cu_in = b.committed_in[g];
    const int32_t ex_in = b.executed_in[g];
    const uint64_t nrec = r1 - r0;
    const uint32_t ncmd = c_hi - c_lo;
    if (r1 < r0 || c_hi < c_lo || nrec > (uint64_t)kFRecs || ncmd > (uint32_t)kFCmds ||
        kcnt > (uint32_t)kFTab || kcnt > kvpg) {
        if (pslots) {  // one-launch step: no work list behind this kernel
            if (t == 0) {
                raise_err(err, kErrInval);
                if (totals) (void)__hip_atomic_fetch_add(pslots + g % pk_slots(gridDim.x), 1ull, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
            }
            if (totals && g == gridDim.x - 1) fold_packed(pslots, gridDim.x, totals, err);
        } else if (t == 0) {
            worklist[atomicAdd(wcount, 1u)] = g;
        }
        return;
    }
    const int64_t lo = (int64_t)ex_in + 1 < 0 ? 0 : (int64_t)ex_in + 1;  // first instance to run
    uint32_t ebits = 0;                                                  // error bits of this lane

    // ---- phase 0: one round of loads (indices clamped, not guarded: no branch splits the batch)
    int4 rr[kFRecPer];
    if (nrec) {  // uniform: groups without replies read nothing (the array may end here)
        const uint32_t last = (uint32_t)nrec - 1;
#pragma unroll
        for (int k = 0; k < kFRecPer; ++k) {
            const uint32_t p = t + k * kFT;
            rr[k] = ld_stream(reinterpret_cast<const int4*>(b.recs) + r0 + (p < last ? p : last));
        }
    } else {
#pragma unroll
        for (int k = 0; k < kFRecPer; ++k) rr[k] = make_int4(-1, 0, 0, 0);
    }
    const bool own = (uint32_t)t < ipg;  // this lane owns instance t
    const uint32_t ti = own ? (uint32_t)t : ipg - 1;
    int4 st = ld_stream(reinterpret_cast<const int4*>(b.st_in) + gi0 + ti);
    const uint32_t co = b.cmd_off[gi0 + ti];
    const uint8_t hs = b.has_cmds ? b.has_cmds[gi0 + ti] : (uint8_t)1;
    int64_t tk[kFTabPer], tv[kFTabPer];  // this lane's table entries t, t + T, ...
#pragma unroll
    for (int k = 0; k < kFTabPer; ++k) {
        const uint32_t e = (uint32_t)t + k * kFT;
        const uint64_t ei = (uint64_t)g * kvpg + (e < kcnt ? e : (kcnt ? kcnt - 1 : 0));
        tk[k] = b.kv_key_in[ei];
        tv[k] = b.kv_val_in[ei];
    }
    // LDS initialisation (regions outside the reply image)
#pragma unroll
    for (int k = 0; k < (kFH + kFT - 1) / kFT; ++k)
        if (kFH % kFT == 0 || t + k * kFT < kFH) S.hkey[t + k * kFT] = kFreeKey;
    for (int i = t; i < kFH / 2; i += kFT)
        reinterpret_cast<uint32_t*>(S.tabidx)[i] = 0xFFFFFFFFu;  // kNone16 pairs
    if (t < kFCmds / 32) S.newbits[t] = 0u;
    S.u.a.rstart[t] = kNone16;
    S.coff[t] = (uint16_t)(own ? co - c_lo : ncmd);
    if (t <= MPX_MAX_REPLICAS) S.red[t] = 0;
    if (t == 0) {
        S.coff[kFIpg] = (uint16_t)ncmd;
        S.firstnil = ipg;
        S.firstbad = ipg;
        S.flags = 0;
        S.ndec = 0;
    }
#pragma unroll
    for (int k = 0; k < kFRecPer; ++k) {
        const uint32_t p = t + k * kFT;
        const uint32_t idc = (rr[k].z >= 0 && rr[k].z < nrep) ? (uint32_t)rr[k].z : kIdBad;
        S.u.a.inst[p] = rr[k].x;
        if (MODE == MPX_MODE_CLASSIC) S.u.a.bal[p] = rr[k].y;
        S.u.a.idok[p] = (uint8_t)((idc << 1) | ((rr[k].w & 0xff) == 1 ? 1u : 0u));
    }
    // command keys and opcodes: issued now, they arrive during the tally (the replies' registers
    // are free again, so the two batches of loads are never in flight together). Values follow
    // after the tally. Uniform guard: a group without commands reads nothing.
    const uint32_t clast = ncmd ? ncmd - 1 : 0;
    // wave w owns commands [256w, 256w + 256) in four chunks of 64: lane l of chunk k holds
    // command cbase + 64k (the chunk scan below relies on this log order)
    const uint32_t cbase = (uint32_t)(t - l) * kFPer + (uint32_t)l;
    uint8_t o[kFPer];
    int64_t ck[kFPer];
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
        const uint32_t li = cbase + k * kWave;
        const uint64_t ci = c_lo + (li < clast ? li : clast);
        o[k] = ncmd ? ld_stream(b.op + ci) : (uint8_t)0;
        ck[k] = ncmd ? ld_stream(b.key + ci) : 0;
    }
    __syncthreads();  // B1
    STAMP(0);

    // ---- phase 1: reply ranges from head flags; the group's table into the dictionary ----------
#pragma unroll
    for (int k = 0; k < kFRecPer; ++k) {
        const uint32_t p = t + k * kFT;
        const bool valid = p < nrec;
        const int32_t inst = S.u.a.inst[p];
        const int32_t prev = S.u.a.inst[p ? p - 1 : 0];
        const bool inwin = inst >= 0 && (uint32_t)inst < ipg;
        const bool pinwin = prev >= 0 && (uint32_t)prev < ipg;
        const bool head = valid && (p == 0 || inst != prev);
        ebits |= (valid && !inwin) ? kErrNil : 0u;               // outside instanceSpace
        ebits |= (head && p && inst < prev) ? kErrOrder : 0u;
        if (head && inwin) S.u.a.rstart[inst] = (uint16_t)p;
        if (head && p && pinwin) S.u.a.rend[prev] = (uint16_t)p;
        if (valid && p + 1 == nrec && inwin) S.u.a.rend[inst] = (uint16_t)nrec;
    }
    int tslot[kFTabPer];  // slots of this lane's table entries
#pragma unroll
    for (int k = 0; k < kFTabPer; ++k) {
        const uint32_t e = (uint32_t)t + k * kFT;
        tslot[k] = 0;
        if (e < kcnt) {
            int fresh = 0;
            const int sl = (unsigned long long)tk[k] == kFreeKey
                               ? -1
                               : fast_slot<Cfg>(S, (unsigned long long)tk[k], fhome<Cfg>(tk[k]),
                                           fresh);
            ebits |= sl < 0 ? kOverflow : 0u;
            tslot[k] = sl < 0 ? 0 : sl;
            if (fresh) S.tabidx[sl] = (uint16_t)e;  // (a duplicate entry of a malformed table
            if (Cfg::kFDvalLds) S.dval[e] = tv[k];  //  shares the first one's slot)
        }
    }
    __syncthreads();  // B2
    STAMP(1);

    // ---- phase 2: tally, one lane per instance (uniform trip count, predicated body) ----------
    bool dec = false;
#if MPX_ABLATE & 8
    const uint32_t ra = (uint32_t)t * 4;
    const bool touched = true;
    const uint32_t rn = 4;
#else
    const uint32_t ra = own ? S.u.a.rstart[t] : kNone16;
    const bool touched = ra != kNone16;
    const uint32_t rn = touched ? (uint32_t)S.u.a.rend[t] - ra : 0;
#endif
#if MPX_ABLATE & 1
    const uint32_t rmax = 0;
#else
    const uint32_t rmax = wave_max_u32(rn);
#endif
    if (MODE == MPX_MODE_MIN) {
        // bareminpaxos.go:1023-1053: no status check; NACKs and ballots ignored. Replies arrive in
        // ascending instance order (anything else is MPX_E_INVAL), so the LAST assignment in array
        // order of committedUpTo and of peerCommits[id] comes from the HIGHEST instance that makes
        // one: each lane keeps which ids it assigned (a bitmask), a wave ballot per id finds the
        // highest such lane, one LDS atomic per wave and id. Predicates are 0/1 integers (see the
        // resolve scan): no lane-mask arithmetic per reply.
        uint32_t idmask = 0;
        int32_t deci = 0;
        for (uint32_t j = 0; j < rmax; ++j) {
            const uint32_t p = j < rn ? ra + j : 0;
            const uint32_t io0 = S.u.a.idok[p];            // unconditional load, then select
            const uint32_t io = j < rn ? io0 : 0u;
            const int32_t okj = (int32_t)(io & 1u);                      // OK == TRUE
            const uint32_t nilbit = st.x == MPX_STATUS_NIL ? kErrNil : 0u;
            ebits |= okj ? nilbit : 0u;                                  // inst.Lb of a nil instance
            const int32_t oks = st.y + okj;                              // AcceptOKs++
            const int32_t c1 = oks >= half ? okj : 0;                    // AcceptOKs+1 > N>>1
            const int32_t dj = oks == half ? c1 : 0;                     // the crossing: COMMITTED
            st.y = oks;
            st.x = dj ? MPX_COMMITTED : st.x;
            deci |= dj;
            const uint32_t id = io >> 1;                                 // peerCommits[Id] = inst-1
            const uint32_t badbit = id == kIdBad ? kErrBadId : 0u;
            ebits |= c1 ? badbit : 0u;
            idmask |= c1 ? (1u << id) : 0u;  // (kIdBad = 31 lies above every valid id)
        }
        dec = deci != 0;
        const uint32_t wbase = (uint32_t)(t - l) + 1;  // 1 + instance of lane 0
        const unsigned long long dm = __ballot(deci != 0);
        if (l == 0 && dm) atomicMax(&S.red[0], wbase + 63u - (uint32_t)__clzll(dm));
        for (int i = 0; i < nrep; ++i) {
            const unsigned long long m = __ballot((idmask >> i) & 1u);
            if (l == 0 && m) atomicMax(&S.red[1 + i], wbase + 63u - (uint32_t)__clzll(m));
        }
    } else {
        // paxos.go:634-673
        ebits |= (touched && st.x == MPX_STATUS_NIL) ? kErrNil : 0u;
        int32_t deci = 0;
        for (uint32_t j = 0; j < rmax; ++j) {
            const uint32_t p = j < rn ? ra + j : 0;
            const int32_t act = j < rn ? 1 : 0;
            const int32_t io = (int32_t)S.u.a.idok[p];
            const int32_t bj = S.u.a.bal[p];
            // status PREPARED (1) or ACCEPTED (2): the reply is processed
            const int32_t live = (uint32_t)(st.x - MPX_PREPARED) < 2u ? act : 0;
            const int32_t okj = live & io & 1;
            const int32_t nk = live & ((io & 1) ^ 1);
            const int32_t oks = st.y + okj;
            const int32_t c = oks >= half ? okj : 0;                     // acceptOKs+1 > N>>1
            st.y = oks;
            st.x = c ? MPX_COMMITTED : st.x;
            deci |= c;
            st.z += nk;
            const int32_t nb = nk ? bj : INT32_MIN;
            st.w = st.w > nb ? st.w : nb;
        }
        dec = deci != 0;
        if (__ballot(dec) && l == 0) atomicMax(&S.red[0], 1u);
    }
    {  // instances decided by this step (only a lane's own instance can decide)
        const unsigned long long dm = __ballot(dec);
        if (l == 0 && dm) atomicAdd(&S.ndec, (uint32_t)__popcll(dm));
    }
    // executeCommands stops at the first nil instance (nil Cmds); CLASSIC's watermark at the first
    // instance that is not COMMITTED: wave minima, one LDS atomic per wave
    {
        uint32_t fn = (own && (int64_t)t >= lo && (st.x == MPX_STATUS_NIL || !hs)) ? (uint32_t)t : ipg;
        uint32_t fb = (MODE == MPX_MODE_CLASSIC && own && (int64_t)t >= (int64_t)cu_in + 1 &&
                       st.x != MPX_COMMITTED) ? (uint32_t)t : ipg;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t x = __shfl_xor(fn, d), y = __shfl_xor(fb, d);
            fn = fn < x ? fn : x;
            fb = fb < y ? fb : y;
        }
        if (l == 0) {
            if (fn < ipg) atomicMin(&S.firstnil, fn);
            if (MODE == MPX_MODE_CLASSIC && fb < ipg) atomicMin(&S.firstbad, fb);
        }
    }
    __syncthreads();  // B3
    STAMP(2);

    // ---- watermarks and the executed range (uniform) -----------------------------------------------
    int32_t cu = cu_in;
    if (MPX_ABLATE & 32) {
        cu = (int32_t)ipg - 1;
    } else if (MODE == MPX_MODE_MIN) {
        if (S.red[0]) cu = (int32_t)S.red[0] - 1;
    } else if (S.red[0] && (int64_t)cu_in + 1 >= 0 && (int64_t)cu_in + 1 < (int64_t)ipg) {
        cu = (int32_t)S.firstbad - 1;  // updateCommittedUpTo over the final statuses
    }
    int64_t hi = (int64_t)cu;
    if (hi >= (int64_t)ipg) hi = (int64_t)ipg - 1;
    int64_t stop = hi >= lo ? hi + 1 : lo;
    if ((int64_t)S.firstnil < stop && (int64_t)S.firstnil >= lo) stop = S.firstnil;
    const uint32_t x0 = stop > lo ? S.coff[lo] : 0, x1 = stop > lo ? S.coff[stop] : 0;

    // ---- phase 3: slot of every executed command, then the chunk scan of its wave -------------
    // In log order a command's predecessors on its key are: the lower lanes of its chunk on the
    // same slot (a 9-bit ballot match), the wave's earlier chunks (the wave's table, updated by
    // the last lane of each slot in each chunk) and the earlier waves (their tables, after B4).
    // Per command this yields the predecessor (state.Conflict) and the last PUT before it
    // (Execute's GET result); the key's last PUT overall gives its value after the step.
    int64_t cv[kFPer];  // command values, stored to LDS once the lookup has covered their latency
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
        const uint32_t li = cbase + k * kWave;
        cv[k] = ncmd ? ld_stream(b.val + c_lo + (li < clast ? li : clast)) : 0;
    }
    uint32_t ops = 0;  // the four opcodes, one byte each
#pragma unroll
    for (int k = 0; k < kFPer; ++k) ops |= (uint32_t)o[k] << (8 * k);
    const int wv = __builtin_amdgcn_readfirstlane(t / kWave);
    uint16_t* T = S.u.b.tab + wv * kFH;  // this wave's table (the reply image is dead)
#pragma unroll
    for (int k = 0; k < (kFH * 2 / 16 + kWave - 1) / kWave; ++k)  // 16-byte stores clear the wave's table
        if ((kFH * 2 / 16) % kWave == 0 || l + k * kWave < kFH * 2 / 16)
            reinterpret_cast<uint4*>(T)[l + k * kWave] = make_uint4(0u, 0u, 0u, 0u);
    // volatile LDS pointers: every access below is a real ds_* instruction, in program order
#if !MPX_STEP_BALLOT
    typedef __attribute__((address_space(3))) volatile uint8_t lds_u8;
    typedef __attribute__((address_space(3))) volatile unsigned long long lds_u64;
    lds_u8* W = (lds_u8*)(S.u.b.win + wv * kFH);
    lds_u64* PM = (lds_u64*)(S.u.b.pmask + wv * kWave);
    PM[l] = 0ull;
#endif
    const unsigned long long lanebit = 1ull << l;
    const unsigned long long below = lanebit - 1ull;
    const uint32_t wfirst = (uint32_t)wv * kWaveCmds;  // the wave's first command
    int kid[kFPer];
    uint32_t seen[kFPer];  // kTabAny | kTabPut | (1 + last PUT before), within the wave
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
        const uint32_t li = cbase + k * kWave;
        const bool act = li >= x0 && li < x1;
        const unsigned long long key = (unsigned long long)ck[k];
        int kd = -1;
#if MPX_ABLATE & 2
        if (act) kd = (int)fhome<Cfg>(ck[k]);
#else
        if (act && key != kFreeKey) {
            int fresh = 0;
            kd = fast_slot<Cfg>(S, key, fhome<Cfg>(ck[k]), fresh);
        }
#endif
        ebits |= (act && kd < 0) ? kOverflow : 0u;  // table full, or the key INT64_MIN
        const bool live = act && kd >= 0;
        kid[k] = live ? kd : -1;
        const uint32_t sl = live ? (uint32_t)kd : 0u;
        const bool isput = ((ops >> (8 * k)) & 0xffu) == MPX_OP_PUT;
        const unsigned long long livem = __ballot(live);
        if (!livem) {  // uniform: no executed command in this chunk
            seen[k] = 0;
            continue;
        }
        // the chunk's lanes on this lane's slot, through the wave's LDS scratch (LDS executes a
        // wave's instructions in order, so each step sees the previous one complete): every lane
        // writes its id into its slot's byte and one of the ids remains (which one does not
        // matter: it only names the slot's class within the chunk); every lane ORs its bit into
        // its class's mask, reads the mask back, and clears it for the next chunk
        unsigned long long peers = 0;
#if MPX_STEP_BALLOT
        {  // one ballot per slot bit (no LDS scratch: 4 KB less per workgroup, 7 per CU)
            unsigned long long m = livem;
#pragma unroll
            for (int i = 0; i < Cfg::kFHB; ++i) {
                const bool bit = (sl >> i) & 1u;
                const unsigned long long bm = __ballot(bit);
                m &= bit ? bm : ~bm;
            }
            peers = live ? m : 0ull;
        }
#else
        if (live) {
            W[sl] = (uint8_t)l;
            const uint32_t cls = W[sl];
            __hip_atomic_fetch_or((__attribute__((address_space(3))) unsigned long long*)&PM[cls],
                                  lanebit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            peers = PM[cls];
            PM[cls] = 0ull;
        }
#endif
        const unsigned long long putm = __ballot(live && isput);
        const unsigned long long lp_m = peers & below;
        const unsigned long long lput_m = lp_m & putm;
        const uint32_t e = live ? (uint32_t)T[sl] : 0u;
        const uint32_t rl1 = li - (uint32_t)l + 1u - wfirst;  // 1 + wave-relative lane-0 index
        const uint32_t elp = e & kTabLp;                        // wave-relative, 0 = none
        // the predecessor: the highest lower lane on the slot, else the wave's earlier chunks
        const uint32_t hp = 63u - (uint32_t)__clzll(lp_m | 1ull);
        const uint32_t pflags = lp_m ? (kTabAny | (((putm >> hp) & 1ull) ? kTabPut : 0u))
                                     : (e & (kTabAny | kTabPut));
        const uint32_t lpr = lput_m ? rl1 + 63u - (uint32_t)__clzll(lput_m) : elp;
        seen[k] = pflags | (lpr ? lpr + wfirst : 0u);
        if (live && (peers >> l) == 1ull) {  // the chunk's last command on this slot
            const unsigned long long allput = peers & putm;
            const uint32_t gl = allput ? rl1 + 63u - (uint32_t)__clzll(allput) : elp;
            T[sl] = (uint16_t)(kTabAny | (isput ? kTabPut : 0u) | gl);
        }
    }
#pragma unroll
    for (int k = 0; k < kFPer; ++k) S.u.b.cval[cbase + k * kWave] = cv[k];
    if (ebits & kOverflow) atomicOr(&S.flags, 1u);
    __syncthreads();  // B4
    STAMP(3);
    if (S.flags & 1u) {  // table overflow: the general kernel takes the group
        if (pslots) {  // (one-launch step: the step fails)
            if (t == 0) {
                raise_err(err, kErrInval);
                if (totals) (void)__hip_atomic_fetch_add(pslots + g % pk_slots(gridDim.x), 1ull, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
            }
            if (totals && g == gridDim.x - 1) fold_packed(pslots, gridDim.x, totals, err);
        } else if (t == 0) {
            worklist[atomicAdd(wcount, 1u)] = g;
        }
        return;
    }
    // the group stays here: the instance outputs can go now (st_out may alias st_in, so not
    // before this point)
    if (own) {
        if (!(MPX_ABLATE & 16) && touched) st_stream(reinterpret_cast<int4*>(b.st_out) + gi0 + t, st);
        if (b.decided) b.decided[gi0 + t] = dec ? 1 : 0;
    }
    STAMP(4);

    // ---- phase 4: resolve: earlier waves, Execute's result, Conflict --------------------------
    uint32_t fnew = 0;  // bit k: command k is the first PUT of a key new to the table
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
        const uint32_t li = cbase + k * kWave;
        const bool act = kid[k] >= 0;
        if (!__ballot(act)) continue;  // uniform: nothing executed in this chunk
        const uint32_t sl = act ? (uint32_t)kid[k] : 0u;
        uint32_t pf = seen[k] & (kTabAny | kTabPut), lp = seen[k] & kTabLp;
        for (int w2 = wv - 1; w2 >= 0; --w2) {  // earlier waves, latest first
            const uint32_t e = S.u.b.tab[w2 * kFH + sl];
            const uint32_t elp = e & kTabLp;
            pf = pf ? pf : (e & (kTabAny | kTabPut));
            lp = lp ? lp : (elp ? elp + (uint32_t)w2 * kWaveCmds : 0u);
        }
        const bool hasprev = pf != 0;                           // (kTabAny is set with kTabPut)
        const int lastput = (int)lp - 1;                        // -1: none
        const uint32_t op = (ops >> (8 * k)) & 0xffu;
        const bool isput = op == MPX_OP_PUT;
        const bool prevput = (pf & kTabPut) != 0;              // the predecessor is a PUT
        const int src = isput ? (int)li : lastput;              // PUT: own value, GET: last PUT
        const int64_t sv = S.u.b.cval[src >= 0 ? src : 0];
        const uint32_t ti = S.tabidx[sl];
        const bool intab = ti != kNone16;                       // present at the start
        const int64_t at_start =
            Cfg::kFDvalLds ? S.dval[intab ? ti : 0]
                           : (intab && op == MPX_OP_GET && lastput < 0
                                  ? b.kv_val_in[(uint64_t)g * kvpg + ti]
                                  : 0);
        const int64_t r = isput ? sv : (op == MPX_OP_GET ? (lastput >= 0 ? sv : (intab ? at_start : 0)) : 0);
        const bool conf = hasprev && (prevput || isput);      // state.Conflict(prev, this)
        if (act) {
            st_stream(b.ret + c_lo + li, r);
            if (b.conf_prev) st_stream(b.conf_prev + c_lo + li, (uint8_t)(conf ? 1 : 0));
            if (isput && lastput < 0 && !intab) {  // first PUT of a new key: its append rank
                fnew |= 1u << k;
                atomicOr(&S.newbits[li >> 5], 1u << (li & 31));
            }
        }
    }
    __syncthreads();  // B7
    STAMP(5);

    // ---- phase 5: outputs ----------------------------------------------------------------------
    // 1 + command index of the last PUT of the key in slot sl (0: none) over all four waves
    auto last_put = [&](uint32_t sl) {
        uint32_t m = 0;
#pragma unroll
        for (int w2 = 0; w2 < kFWaves; ++w2) {
            const uint32_t x = S.u.b.tab[w2 * kFH + sl] & kTabLp;
            m = x ? x + (uint32_t)w2 * kWaveCmds : m;
        }
        return m;
    };
    int64_t* kko = b.kv_key_out + (uint64_t)g * kvpg;
    int64_t* kvo = b.kv_val_out + (uint64_t)g * kvpg;
#pragma unroll
    for (int k = 0; k < kFTabPer; ++k) {  // original entries stay in place
        const uint32_t e = (uint32_t)t + k * kFT;
        if (!(MPX_ABLATE & 16) && e < kcnt) {
            const uint32_t dl = last_put((uint32_t)tslot[k]);
            kko[e] = (int64_t)S.hkey[tslot[k]];
            kvo[e] = dl ? S.u.b.cval[dl - 1] : (Cfg::kFDvalLds ? S.dval[e] : tv[k]);
        }
    }
    // keys new to the table that hold a value: appended in order of their first PUT, whose
    // rank is a popcount over the first-PUT bitmap (each wave scans the 32 words itself)
    const uint32_t wbits = l < kFCmds / 32 ? S.newbits[l] : 0u;
    const uint32_t pc = __popc(wbits);
    uint32_t incl = pc;
#pragma unroll
    for (int d = 1; d < kFCmds / 32; d <<= 1) {
        const uint32_t x = __shfl_up(incl, d);
        if (l >= d) incl += x;
    }
    const uint32_t excl = incl - pc;
    const uint32_t n_new = (uint32_t)__shfl((int)incl, kFCmds / 32 - 1);
    const uint32_t total = kcnt + n_new;
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {  // the lane of the key's first PUT appends it
        const uint32_t li = cbase + k * kWave;
        const uint32_t base = (uint32_t)__shfl((int)excl, (int)(li >> 5));
        const uint32_t rank = base + __popc(S.newbits[li >> 5] & ((1u << (li & 31)) - 1u));
        if (!(MPX_ABLATE & 16) && ((fnew >> k) & 1u) && kcnt + rank < kvpg) {
            const uint32_t kd = (uint32_t)kid[k];
            kko[kcnt + rank] = (int64_t)S.hkey[kd];
            kvo[kcnt + rank] = S.u.b.cval[last_put(kd) - 1];
        }
    }
    ebits |= (t == 0 && total > kvpg) ? kErrKvFull : 0u;
    if (t < nrep) {
        const uint32_t k = MODE == MPX_MODE_MIN ? S.red[1 + t] : 0u;
        b.peer_out[(uint64_t)g * nrep + t] =
            k ? (int32_t)k - 2 : b.peer_in[(uint64_t)g * nrep + t];  // instance - 1
    }
    if (t == 0) {
        b.committed_out[g] = cu;
        b.executed_out[g] = stop > lo ? (int32_t)(stop - 1) : ex_in;
        b.kv_cnt_out[g] = total < kvpg ? total : kvpg;
        if (b.n_decided) b.n_decided[g] = S.ndec;
    }
    // the step totals: this group's decided instances, executed instances and executed commands
    // into partial slot g % kTotSlots (no-return atomics: nothing waits for them here; the
    // general kernel, a later launch, folds the slots)
    if (tacc && t < 3) {
        const uint32_t v = t == 0 ? S.ndec : (stop > lo ? (t == 1 ? (uint32_t)(stop - lo) : x1 - x0) : 0u);
        if (v)
            (void)__hip_atomic_fetch_add(tacc + (g & (kTotSlots - 1)) * 3 + t, (unsigned long long)v,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (pslots && totals && t == 0)  // one-launch step: the packed word (arrival included)
        (void)__hip_atomic_fetch_add(pslots + g % pk_slots(gridDim.x),
                                     pk_word(S.ndec, stop > lo ? (uint32_t)(stop - lo) : 0u,
                                             stop > lo ? x1 - x0 : 0u),
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ebits &= 0x7FFFFFFFu;
    if (ebits) raise_err(err, ebits);
    if (pslots && totals && g == gridDim.x - 1) fold_packed(pslots, gridDim.x, totals, err);
    STAMP(6);
    STAMP_SPAN();
}

// ======================================= general path =========================================
constexpr int kDCap = 2048;  // distinct keys a group's call may touch (table included)
constexpr int kHCap = 2 * kDCap;
constexpr int kChunk = 1024;
constexpr int kPer = kChunk / kStepBlock;
constexpr int kMaxIpgBits = 8192;

struct GenLds {
    int64_t dkey[kDCap];
    int64_t dval[kDCap];
    uint32_t dfirst[kDCap];
    uint32_t cnt[kDCap];
    uint32_t off[kDCap];
    uint32_t hslot[kHCap];
    int64_t cval[kChunk];
    uint16_t list[kChunk];
    uint8_t dpresent[kDCap];
    uint8_t dseen[kDCap];
    uint32_t dec_bits[kMaxIpgBits / 32];
    uint32_t wsum[kStepBlock / kWave];
    unsigned long long red[1 + MPX_MAX_REPLICAS];
    uint32_t dn, n_orig, ndec, scal[4];
};

template <int MODE>
__device__ void group_general(GenLds& S, const mpx_group_batch& b, uint32_t g, int32_t nrep,
                             uint32_t kvpg, unsigned long long* tacc, uint32_t* err) {
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    const int32_t half = nrep >> 1;
    const uint64_t ipg = b.ipg;
    const uint64_t gi0 = (uint64_t)g * ipg;
    const mpx_inst_state* st_in = b.st_in + gi0;
    mpx_inst_state* st_out = b.st_out + gi0;

    if (t <= MPX_MAX_REPLICAS) S.red[t] = 0;
    for (int i = t; i < kMaxIpgBits / 32; i += kStepBlock) S.dec_bits[i] = 0;
    for (int i = t; i < kHCap; i += kStepBlock) S.hslot[i] = 0;
    if (t == 0) {
        S.dn = 0;
        S.ndec = 0;
    }
    __syncthreads();

    // ---- 1. tally straight from global memory ------------------------------------------------------
    const uint64_t r0 = b.grp_rec_off[g], r1 = b.grp_rec_off[g + 1];
    if (r1 > r0) {
        const uint64_t len = r1 - r0;
        const uint64_t n0 = r0 + len * w / (kStepBlock / kWave);
        const uint64_t n1 = r0 + len * (w + 1) / (kStepBlock / kWave);
        const uint64_t s = find_head(b.recs, n0, r0, r1);
        const uint64_t e = (n1 >= r1) ? r1 : find_head(b.recs, n1, r0, r1);
        if (s < e) {
            TallyOut out{0, 0, false};
            tally_range<MODE>(b.recs, s, e, st_in, st_out, ipg, 0, half, nrep, nullptr, err, 0,
                              out, S.dec_bits);
            if (MODE == MPX_MODE_MIN) {
                if (l == 0 && out.cu_key) atomicMax(&S.red[0], (unsigned long long)out.cu_key);
                if (l < nrep && out.pc_key) atomicMax(&S.red[1 + l], (unsigned long long)out.pc_key);
            } else {
                if (l == 0 && out.any_dec) atomicMax(&S.red[0], 1ull);
            }
        }
    } else if (r1 < r0) {
        raise_err(err, kErrInval);
    }
    __syncthreads();
    if (b.decided)
        for (uint64_t i = t; i < ipg; i += kStepBlock)
            b.decided[gi0 + i] = (S.dec_bits[i >> 5] >> (i & 31)) & 1u;
    if (b.n_decided) {  // popcount of the decided bitmap (bits past ipg stay 0)
        uint32_t c = 0;
        for (uint64_t i = t; i < (ipg + 31) / 32; i += kStepBlock) c += __popc(S.dec_bits[i]);
        if (c) atomicAdd(&S.ndec, c);
    }

    // ---- watermarks --------------------------------------------------------------------------------
    const int32_t cu_in = b.committed_in[g];
    int32_t cu = cu_in;
    if (MPX_ABLATE & 32) {
        cu = (int32_t)ipg - 1;
    } else if (MODE == MPX_MODE_MIN) {
        if (S.red[0]) cu = (int32_t)(uint32_t)(S.red[0] & 0xffffffffull);
        if (t < nrep) {
            const unsigned long long k = S.red[1 + t];
            b.peer_out[(uint64_t)g * nrep + t] =
                k ? (int32_t)(uint32_t)(k & 0xffffffffull) : b.peer_in[(uint64_t)g * nrep + t];
        }
    } else {
        if (t < nrep) b.peer_out[(uint64_t)g * nrep + t] = b.peer_in[(uint64_t)g * nrep + t];
        if (S.red[0]) {
            if (t == 0) S.scal[1] = (uint32_t)ipg;
            __syncthreads();
            const int64_t j0 = (int64_t)cu_in + 1;
            if (j0 >= 0 && (uint64_t)j0 < ipg) {
                for (uint64_t j = (uint64_t)j0 + t; j < ipg; j += kStepBlock) {
                    const bool dec = (S.dec_bits[j >> 5] >> (j & 31)) & 1u;
                    if (!(dec || st_in[j].status == MPX_COMMITTED)) {
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

    // ---- 2. executeCommands: instances exec+1 .. cu while Cmds != nil ------------------------------
    const int32_t ex_in = b.executed_in[g];
    int64_t lo = (int64_t)ex_in + 1;
    int64_t hi = (int64_t)cu;
    if (hi >= (int64_t)ipg) hi = (int64_t)ipg - 1;
    if (lo < 0) lo = 0;
    if (t == 0) S.scal[2] = (uint32_t)(hi + 1 > lo ? hi + 1 : lo);
    __syncthreads();
    if (hi >= lo) {
        for (int64_t i = lo + t; i <= hi; i += kStepBlock) {
            const bool nil = st_in[i].status == MPX_STATUS_NIL || (b.has_cmds && !b.has_cmds[gi0 + i]);
            if (nil) {
                atomicMin(&S.scal[2], (uint32_t)i);
                break;
            }
        }
    }
    __syncthreads();
    const int64_t stop = hi >= lo ? (int64_t)S.scal[2] : lo;
    if (t == 0) {
        b.executed_out[g] = stop > lo ? (int32_t)(stop - 1) : ex_in;
        if (b.n_decided) b.n_decided[g] = S.ndec;
    }
    if (tacc && t == 0) {  // this group's step totals (performed before the caller's ticket)
        unsigned long long* p = tacc + (g & (kTotSlots - 1)) * 3;
        if (S.ndec) atomic_add_done(p, (unsigned long long)S.ndec);
        if (stop > lo) {
            atomic_add_done(p + 1, (unsigned long long)(stop - lo));
            const uint64_t xc = b.cmd_off[gi0 + stop] - b.cmd_off[gi0 + lo];
            if (xc) atomic_add_done(p + 2, (unsigned long long)xc);
        }
    }

    const Dict D{S.dkey, S.dval, S.dfirst, S.cnt, S.hslot, S.dpresent, S.dseen, &S.dn,
                 (uint32_t)kDCap, (uint32_t)kHCap};
    const uint32_t ncnt = b.kv_cnt_in[g];
    if (ncnt > kvpg || ncnt > (uint32_t)kDCap) {
        raise_err(err, kErrInval);
        return;
    }
    for (uint32_t e = t; e < ncnt; e += kStepBlock)
        dict_put_unique(D, e, b.kv_key_in[(uint64_t)g * kvpg + e], b.kv_val_in[(uint64_t)g * kvpg + e]);
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
                    S.cval[li] = b.val[c0 + li];
                    kid[k] = dict_insert(D, b.key[c0 + li]);
                    if (kid[k] >= 0) pos[k] = atomicAdd(&S.cnt[kid[k]], 1u);
                    else raise_err(err, kErrKvFull);
                }
            }
            __syncthreads();
            const uint32_t dn = S.dn < (uint32_t)kDCap ? S.dn : (uint32_t)kDCap;
            block_scan<kDCap / kStepBlock>(S.cnt, S.off, dn, S.wsum);
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const uint32_t li = t + k * kStepBlock;
                if (li < n && kid[k] >= 0)
                    S.list[S.off[kid[k]] + pos[k]] = (uint16_t)((li << 1) | (o[k] == MPX_OP_PUT ? 1u : 0u));
            }
            __syncthreads();
            uint8_t fl[kPer];
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const uint32_t li = t + k * kStepBlock;
                fl[k] = 0;
                if (li >= n || kid[k] < 0) continue;
                int64_t r;
                bool conf;
                fl[k] = resolve_cmd(D, S.off, S.list, S.cval, kid[k], li, o[k], r, conf);
                b.ret[c0 + li] = r;
                if (b.conf_prev) b.conf_prev[c0 + li] = conf ? 1 : 0;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const uint32_t li = t + k * kStepBlock;
                if (li < n && kid[k] >= 0)
                    apply_update(D, kid[k], fl[k], o[k], S.cval[li], (uint32_t)(c0 + li - c_begin),
                                 S.n_orig);
            }
            __syncthreads();
        }
    }
    const uint32_t dn = S.dn < (uint32_t)kDCap ? S.dn : (uint32_t)kDCap;
    table_writeback(D, S.n_orig, dn, b.kv_key_out + (uint64_t)g * kvpg,
                    b.kv_val_out + (uint64_t)g * kvpg, kvpg, &S.scal[0], err);
    if (t == 0) b.kv_cnt_out[g] = S.scal[0] < kvpg ? S.scal[0] : kvpg;
}

// the step totals of group g from its outputs: decided instances, executed instances (the
// executeCommands iterations), executed commands
__device__ __forceinline__ void group_totals(const mpx_group_batch& b, uint32_t g,
                                             unsigned long long& d, unsigned long long& xi,
                                             unsigned long long& xc) {
    d = b.n_decided[g];
    const int64_t ei = b.executed_in[g], eo = b.executed_out[g];
    const int64_t lo = ei + 1 < 0 ? 0 : ei + 1;
    xi = xc = 0;
    if (eo >= lo && eo < (int64_t)b.ipg) {
        const uint64_t gi0 = (uint64_t)g * b.ipg;
        xi = (unsigned long long)(eo - lo + 1);
        xc = b.cmd_off[gi0 + eo + 1] - b.cmd_off[gi0 + lo];
    }
}

// The work list, and (totals != nullptr) the step's totals, so a step is two launches. The fast
// kernel (the previous launch) added every group it kept into the kTotSlots partial slots of the
// control words with no-return atomics; the groups on the list add theirs here. Empty work list
// (the common case): workgroup 0 alone folds the slots (atomic exchanges: read and reset), writes
// the totals and returns; every other workgroup returns at once, whatever it reads. Otherwise
// the first `workers` workgroups run the list (workgroup 0 among them: it has read the count
// before any reset), add their groups' totals with awaited atomics and take a ticket; the last
// zeroes the list count and its ticket and folds the slots.
template <int MODE>
__global__ __launch_bounds__(kStepBlock) void k_group_general(mpx_group_batch b, int32_t nrep,
                                                              uint32_t kvpg,
                                                              const uint32_t* worklist,
                                                              uint32_t* wcount,
                                                              int64_t* totals, uint32_t* err) {
    __shared__ GenLds S;
    __shared__ bool last;
    __shared__ unsigned long long fold[3];
    unsigned long long* part = reinterpret_cast<unsigned long long*>(wcount + 16);
    auto fold_totals = [&]() {  // whole workgroup: the kTotSlots x 3 partials into totals[0..2]
        if (threadIdx.x < 3) fold[threadIdx.x] = 0;
        __syncthreads();
        if (threadIdx.x < kTotSlots * 3) {
            const unsigned long long v = atomic_take(part + threadIdx.x);
            if (v) atomicAdd(&fold[threadIdx.x % 3], v);
        }
        __syncthreads();
        if (threadIdx.x < 3) totals[threadIdx.x] = (int64_t)fold[threadIdx.x];
    };
    static_assert(kTotSlots * 3 <= kStepBlock, "one partial slot word per thread");
    const uint32_t n = *wcount;
    if (n == 0) {
        if (totals && blockIdx.x == 0) fold_totals();
        return;
    }
    const uint32_t workers = n < gridDim.x ? n : gridDim.x;
    if (blockIdx.x >= workers) return;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        group_general<MODE>(S, b, worklist[i], nrep, kvpg, totals ? part : nullptr, err);
        __syncthreads();
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t k = __hip_atomic_fetch_add(wcount + 1, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        last = k == workers - 1;
        if (last) {
            wcount[0] = 0;
            wcount[1] = 0;
        }
    }
    __syncthreads();
    if (last && totals) fold_totals();
}

__global__ void k_fill_worklist(uint32_t* worklist, uint32_t* wcount, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) worklist[i] = i;
    if (i == 0) *wcount = n;
}

namespace {
// a timing event on `stream`; while the stream is being captured into a graph, as an external
// event-record node of the graph, so every replay records it (a plain record inside a capture
// only orders the capture's streams)
void record_timing_event(hipEvent_t ev, hipStream_t stream) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(stream, &cs);
    if (cs == hipStreamCaptureStatusActive)
        (void)hipEventRecordWithFlags(ev, stream, hipEventRecordExternal);
    else
        (void)hipEventRecord(ev, stream);
}

template <int MODE, class Cfg>
void launch_fast(const mpx_group_batch* b, int32_t nrep, uint32_t kvpg, uint32_t* worklist,
                 uint32_t* wcount, unsigned long long* tacc, uint32_t* err, hipStream_t stream,
                 unsigned long long* pslots, int64_t* totals) {
    if (pslots)
        k_group_fast<MODE, Cfg, true><<<b->n_groups, Cfg::kFT, 0, stream>>>(
            *b, nrep, kvpg, worklist, wcount, tacc, err, pslots, totals);
    else
        k_group_fast<MODE, Cfg, false><<<b->n_groups, Cfg::kFT, 0, stream>>>(
            *b, nrep, kvpg, worklist, wcount, tacc, err, nullptr, nullptr);
}
// the smallest fast-path variant the batch's shape fits (0 = none: every group is general)
int fast_variant(int32_t nrep, uint32_t ipg, uint32_t kvpg) {
    const uint64_t recs = (uint64_t)(nrep > 1 ? nrep - 1 : 1) * ipg;  // replies of a full group
    if (ipg <= 256 && recs <= 1024 && kvpg <= 256) return 1;
    if (ipg <= 256 && recs <= 2048 && kvpg <= 256) return 2;
    if (ipg <= 256 && recs <= 1024 && kvpg <= 1024) return 3;
    if (ipg <= 512 && recs <= 2048 && kvpg <= 256) return 5;
    if (ipg <= 512 && recs <= 2048 && kvpg <= 512) return 4;
    return 0;
}
template <int MODE>
void launch_step(const mpx_group_batch* b, int32_t nrep, uint32_t kvpg, uint32_t* worklist,
                 uint32_t* wcount, int64_t* totals, uint32_t* err, hipStream_t stream,
                 hipEvent_t ev0, hipEvent_t ev1, unsigned long long* pslots) {
    // two-launch steps: the step totals' partial slots (control words [16..)), the fast kernel
    // adds the groups it keeps, the general kernel the listed ones and folds them; one-launch
    // steps (pslots): the fast kernel's packed slots and its last workgroup's fold
    unsigned long long* const tacc =
        totals && !pslots ? reinterpret_cast<unsigned long long*>(wcount + 16) : nullptr;
    int64_t* const ptot = pslots ? totals : nullptr;
    if (ev0) record_timing_event(ev0, stream);
    switch (fast_variant(nrep, b->ipg, kvpg)) {
#define MPX_FAST_CASE(n, C)                                                                    \
    case n:                                                                                    \
        launch_fast<MODE, C>(b, nrep, kvpg, worklist, wcount, tacc, err, stream, pslots, ptot); \
        break;
    MPX_FAST_CASE(1, FastBase)
    MPX_FAST_CASE(2, FastRecs)
    MPX_FAST_CASE(3, FastKeys)
    MPX_FAST_CASE(4, FastWide)
    MPX_FAST_CASE(5, FastWide256)
#undef MPX_FAST_CASE
    default:
        k_fill_worklist<<<(b->n_groups + 255) / 256, 256, 0, stream>>>(worklist, wcount,
                                                                       b->n_groups);
    }
    if (ev1) record_timing_event(ev1, stream);
    if (pslots) return;  // (the host checked that a fast variant takes the shape)
    const unsigned gen_grid = b->n_groups < 256 ? b->n_groups : 256;  // one per CU (LDS)
    k_group_general<MODE><<<gen_grid ? gen_grid : 1, kStepBlock, 0, stream>>>(
        *b, nrep, kvpg, worklist, wcount, totals, err);
}
}  // namespace

bool step_one_launch_fits(int32_t nrep, uint32_t ipg, uint32_t kv_per_group) {
    return fast_variant(nrep, ipg, kv_per_group) != 0;
}

hipError_t launch_group_step(int mode, int32_t nrep, uint32_t kv_per_group,
                             const mpx_group_batch* b, uint32_t* worklist, uint32_t* wcount,
                             int64_t* totals, uint32_t* err, hipStream_t stream,
                             hipEvent_t ev0, hipEvent_t ev1, unsigned long long* pslots) {
    if (!b->n_groups)
        return totals ? hipMemsetAsync(totals, 0, 3 * sizeof(int64_t), stream) : hipSuccess;
    if (kv_per_group > (uint32_t)kDCap) return hipErrorInvalidValue;
    if (b->ipg > (uint32_t)kMaxIpgBits) return hipErrorInvalidValue;
    if (pslots && !step_one_launch_fits(nrep, b->ipg, kv_per_group)) return hipErrorInvalidValue;
    if (mode == MPX_MODE_MIN)
        launch_step<MPX_MODE_MIN>(b, nrep, kv_per_group, worklist, wcount, totals, err, stream,
                                  ev0, ev1, pslots);
    else
        launch_step<MPX_MODE_CLASSIC>(b, nrep, kv_per_group, worklist, wcount, totals, err,
                                      stream, ev0, ev1, pslots);
    return hipGetLastError();
}

// per-step totals of a batch: decided instances, executed instances, executed commands. One
// group per lane, a block reduction, one 64-bit atomic per block and counter into the engine's
// accumulators; the last workgroup writes the totals and zeroes the accumulators.
__global__ __launch_bounds__(256) void k_step_totals(mpx_group_batch b, unsigned long long* totals,
                                                     uint32_t* ctl) {
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(ctl + 4);
    __shared__ unsigned long long red[3][kStepBlock / kWave];
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long d = 0, xi = 0, xc = 0;
    if (g < b.n_groups) group_totals(b, g, d, xi, xc);
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) {
        d += __shfl_xor(d, k);
        xi += __shfl_xor(xi, k);
        xc += __shfl_xor(xc, k);
    }
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) {
        red[0][w] = d;
        red[1][w] = xi;
        red[2][w] = xc;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        unsigned long long v = 0;
        for (int k = 0; k < kStepBlock / kWave; ++k) v += red[threadIdx.x][k];
        if (v) atomic_add_done(acc + threadIdx.x, v);
    }
    if (last_workgroup(ctl + 10) && threadIdx.x < 3)
        totals[threadIdx.x] = atomic_take(acc + threadIdx.x);
}

hipError_t launch_step_totals(const mpx_group_batch* b, int64_t* totals, uint32_t* ctl,
                              hipStream_t stream) {
    const uint32_t blocks = b->n_groups ? (b->n_groups + kStepBlock - 1) / kStepBlock : 1;
    k_step_totals<<<blocks, kStepBlock, 0, stream>>>(*b, reinterpret_cast<unsigned long long*>(totals),
                                                     ctl);
    return hipGetLastError();
}

}  // namespace mpx

#if MPX_STAMPS
extern "C" int mpx_debug_stamps(unsigned long long* out16, int reset) {
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(mpx::mpx_stamp_acc), 16 * sizeof(unsigned long long)) != hipSuccess)
        return -3;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(mpx::mpx_stamp_acc), z, sizeof(z)) != hipSuccess) return -3;
    }
    return 0;
}
// every fast workgroup's (start, end) s_memrealtime of the last step, first n of them
extern "C" int mpx_debug_spans(unsigned long long* out, unsigned n) {
    if (n > mpx::kSpanMax) n = mpx::kSpanMax;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpx::mpx_wg_span), (size_t)n * 16) == hipSuccess ? 0 : -3;
}
#endif
