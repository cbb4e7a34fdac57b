// apply_fast.hip — the partitioned apply pipeline of mpx_apply (A5/A6).
//
// Reference: (*state.Command).Execute  src/state/state.go:77-103, applied in log order by
// executeCommands  src/bareminpaxos/bareminpaxos.go:1066-1098; state.Conflict state.go:53-60.
//
// Sequential semantics restated per key: for command i on key k,
//   ret[i]  = PUT: val[i]; GET: val of the last PUT on k before i in this call, else the table
//             value at call start if k is present, else NIL (0); other ops: 0
//   conf[i] = Conflict(previous command on k in this call, command i)
//   table   : k <- val of the last PUT on k in this call
// Commands of different keys never interact, and the table (kvtab.hpp) is cut into 256-slot
// buckets that each hold a closed set of keys. So the log is partitioned by bin (up to 16
// buckets, at least 4 bins) and every bin is resolved in LDS by one workgroup, against its own
// slice of the table, in log order:
//   k_ap_sclear / k_ap_sample / k_ap_select  64K of the chunk's keys are sampled into a hash of
//                 counts; the most frequent keys seen at least hot_min times (at most 127) are HOT:
//                 they skip the partition and are resolved in log order by a per-key max-scan
//                 (below), so a skewed key space cannot pile onto one bin. Index 0 is always the
//                 key INT64_MIN (the table's sentinel, kept in a side slot).
//   k_ap_scatter  persistent (one workgroup per CU, XCD-contiguous tiles, the next tile
//                 prefetched), per 4096-command log tile: a stable per-bin ranking of the cold
//                 commands (per-wave peer masks + wave prefix), the tile's bin-sorted IMAGE of
//                 16-byte records (the key's hash with the command's class in its two top bits -
//                 bin bits the partition implies - and the value) built in LDS and stored whole at
//                 the tile's own place; the tile's row: commands per bin, the bins' image starts,
//                 per hot key the last position of any command and of a PUT; per command its index
//                 in the tile image (ipos, log order)
//   scans         k_ap_scan_part / _top / _bins / _rows over the tile rows: the runs' partition
//                 offsets per tile (sums), hot positions before each tile (maxima)
//   k_ap_runs     the rows transposed into the bin-major run table: per (bin, tile) the run's
//                 partition offset and its image offset
//   k_ap_resolve_list  one workgroup per bin (XCD-contiguous bins): its table slice in LDS (key
//                 hashes, values, state), the bin's records in log order 2048 at a time, gathered
//                 from the tile images through a window of the run table (the next batch
//                 prefetched); every record of a batch at once finds its slot and joins its slot's
//                 list of the batch, then walks the list (or, for a slot with many records, reads
//                 two bitmaps) for its predecessor and last earlier PUT; results stored at the
//                 records' image positions; touched slots written back once
//   k_ap_hot_commit  the hot keys' final value and state
//   k_ap_emit     per tile, log order: the tile's cold results - its own image slots, one
//                 contiguous run - into LDS, read back by ipos; a hot command's from the per-wave
//                 peer scan, the earlier waves' tables and the tile's incoming positions; ret /
//                 conf stored coalesced
// Table traffic is one read and one write of each bin's slice per call instead of one random probe
// per command. New keys: any command on a key the slice does not hold claims a slot for it (a GET
// before the first PUT of a new key is still that PUT's predecessor); slots whose key never
// became present are removed before the write-back (k_ap_resolve_list). Calls of several chunks
// insert every PUT key of the call first, as the fallback pipeline does.
#include "kvtab.hpp"

namespace mpx {

// diagnostic ablation of k_ap_resolve_list (variant builds only): 2 no result stores, 4 one step
// of each list walk (uniform call, round 6: 0.95 -> 0.80 / 0.86 / 0.69 ms for 2 / 4 / 6)
#ifndef MPX_RS_ABL
#define MPX_RS_ABL 0
#endif

constexpr int kTL = 4096;          // commands per log tile
constexpr int kTT = 1024;          // threads of the tile and bin workgroups
constexpr int kTW = kTT / kWave;   // 16 waves
constexpr int kTPer = kTL / kTT;   // 4 commands per thread; wave w owns [256 w, 256 w + 256)
constexpr int kHMax = 128;         // hot keys per chunk, index 0 = INT64_MIN
constexpr int kLgHMax = 7;
constexpr int kHotTab = 512;       // LDS hash of the hot keys (load <= 1/8: probes stay short)
constexpr int kLgMaxBins = 10;
constexpr int kMaxBins = 1 << kLgMaxBins;  // partition bins (super-bins past it)
// bins per super-bin, at most: tables to 2^10 x 2^8 x 4096 = 2^30 slots (the resolve workgroup
// streams its super-bin's records once per bin, so the cost grows with the table past 2^26 slots;
// the sort-based pipeline's result codes stop at 2^29 slots)
constexpr int kLgMaxSub = 8;
// buckets per bin (the resolve workgroup's LDS table: 16 x 256 slots)
constexpr int kLgMaxBPB = 4;
constexpr int kMaxBPB = 1 << kLgMaxBPB;
constexpr int kLgSamples = 16;
constexpr uint32_t kSamples = 1u << kLgSamples;  // (k_ap_sample divides by a shift)
constexpr uint32_t kHotIdx = 0x8000u;  // ipos: hot command (| hot index), else image index
constexpr uint32_t kNoSlot = ~0u;
constexpr unsigned kScatterGrid = 256;  // persistent partition grid: one workgroup per CU
constexpr uint32_t kScanGroups = 256;   // tile groups of the row scan (one workgroup per CU);
                                        // k_ap_scan_top covers 16 x 16 of them per column

static_assert(kScanGroups <= 256, "k_ap_scan_top covers 16 chunks of 16 groups per column");
static_assert((1 << kLgHMax) == kHMax, "hot indices are matched on kLgHMax bits");
static_assert((kTW * kHMax) % kTT == 0, "k_ap_emit clears / scans its per-wave hot tables");
static_assert(kMaxBins <= kTT, "the bin scans take one bin per thread");
static_assert(kSamples % (64 * 256) == 0, "k_ap_sample: whole samples per thread");
static_assert((1 << 17) % (16 * kTT) == 0, "k_ap_select reads the sample table 16 counts per thread at a time");

// LDS slot state of k_ap_resolve_list
constexpr uint8_t kSPresent = 1, kSLastPut = 2, kSTouched = 4, kSValDirty = 8, kSNew = 16,
                  kSWasPresent = 32;

struct ApHot {               // per chunk; written by k_ap_select (+ the scan's totals)
    int64_t key[kHMax];
    int64_t val0[kHMax];     // value at chunk start (present keys)
    uint32_t slot[kHMax];    // table slot, kNoSlot when absent and never inserted
    uint32_t flags[kHMax];   // bit 0 present, bit 1 last op PUT (if touched), bit 2 touched in call
    uint32_t fin_any[kHMax]; // 1 + chunk position of the key's last command (0: none)
    uint32_t fin_put[kHMax]; // 1 + chunk position of the key's last PUT (0: none)
    uint32_t n;              // hot keys, >= 1
    uint32_t restarts;       // bins that ran the two-pass form (diagnostic)
};

// lgsub: tables past kMaxBins bins of 2^lgbpb buckets partition the log into kMaxBins super-bins
// of 2^lgsub bins each; the resolve workgroup of a super-bin takes its bins one after another
// (each pass streams the super-bin's records and resolves those of its bin)
struct ApGeo {
    uint32_t lgnb, lgbpb, lgsub, nbin, lgnbin, rowlen, tiles, ng, tpg;
};

__device__ __forceinline__ uint32_t bin_of(uint64_t h, const ApGeo& g) {
    return bucket_of(h, g.lgnb) >> (g.lgbpb + g.lgsub);
}

// buckets per bin: up to 16, and at least 4 bins (a table has at least 4 buckets): the top two
// bits of a key's hash are then always bits of its bin
__host__ __device__ inline uint32_t lgbpb_for(uint32_t lgnb) {
    const uint32_t x = lgnb >= 2 ? lgnb - 2 : 0;
    return x < (uint32_t)kLgMaxBPB ? x : (uint32_t)kLgMaxBPB;
}

// A partition record is 16 bytes: the key's hash (hash64 is a bijection) with its top two bits -
// bin bits, which the partition itself implies - replaced by the command's class, then the value.
// The resolve compares hashes (its LDS table holds the hashes of its keys) and recovers a key
// only to write a new one to the table (unhash64).
constexpr uint32_t kClsPut = 0, kClsGet = 1, kClsOther = 2;
__device__ __forceinline__ uint32_t op_class(uint32_t op) {
    return op == MPX_OP_PUT ? kClsPut : (op == MPX_OP_GET ? kClsGet : kClsOther);
}
__device__ __forceinline__ uint64_t rec_pack(uint64_t h, uint32_t cls) {
    return (h & ~(3ull << 62)) | ((uint64_t)cls << 62);
}
// the hash of a record of bin `bin` (its top two bits restored from the bin)
__device__ __forceinline__ uint64_t rec_hash(uint64_t x, uint32_t bin, const ApGeo& g) {
    return (x & ~(3ull << 62)) | ((uint64_t)(bin >> (g.lgnbin - 2)) << 62);
}

typedef __attribute__((address_space(3))) volatile uint8_t lds_u8;
typedef __attribute__((address_space(3))) volatile uint16_t lds_u16;
typedef __attribute__((address_space(3))) volatile unsigned long long lds_u64;

// peers of this lane among the active lanes of the wave with the same class id c (< width of W):
// every lane writes its lane id into W[c], reads back the id that remained (one per class), ORs
// its bit into that id's mask and reads the mask back, then the mask is cleared for the next use.
// LDS executes a wave's instructions in order, so each step sees the previous one complete.
__device__ __forceinline__ unsigned long long wave_peers(lds_u8* W, lds_u64* PM, uint32_t c,
                                                         bool act) {
    unsigned long long peers = 0;
    if (act) {
        const int l = lane_id();
        W[c] = (uint8_t)l;
        const uint32_t cls = W[c];
        __hip_atomic_fetch_or((__attribute__((address_space(3))) unsigned long long*)&PM[cls],
                              1ull << l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        peers = PM[cls];
        PM[cls] = 0ull;
    }
    return peers;
}

// the same from one ballot per bit of the class id (c < 2^nbits), without LDS: for few classes,
// or where most lanes share a class (the LDS OR above would serialise on one word)
__device__ __forceinline__ unsigned long long match_bits(uint32_t c, int nbits, bool act) {
    unsigned long long m = __ballot(act);
    for (int i = 0; i < nbits; ++i) {
        const bool bit = (c >> i) & 1u;
        const unsigned long long b = __ballot(bit);
        m &= bit ? b : ~b;
    }
    return act ? m : 0ull;
}

__device__ __forceinline__ int64_t shfl64(int64_t v, int src) {
    return (int64_t)__shfl((long long)v, src);
}

// XCD-aware tile order of a persistent grid (gridDim a multiple of 8): workgroup b runs on XCD
// b % 8; XCD x owns the contiguous tiles [xs, xe) and its workgroups walk them together, so the
// runs that neighbouring tiles read or write in the same partition bin meet in one L2
struct TileWalk {
    uint32_t tile, end, step;
};
__device__ __forceinline__ TileWalk tile_walk(uint32_t tiles) {
    const uint32_t x = blockIdx.x & 7u, i = blockIdx.x >> 3, nper = gridDim.x >> 3;
    const uint32_t per = tiles >> 3, rem = tiles & 7u;
    const uint32_t xs = x * per + (x < rem ? x : rem);
    return TileWalk{xs + i, xs + per + (x < rem ? 1u : 0u), nper};
}
// the same for a one-tile-per-workgroup grid (gridDim == tiles)
__device__ __forceinline__ uint32_t xcd_tile(uint32_t tiles) {
    const uint32_t x = blockIdx.x & 7u, i = blockIdx.x >> 3;
    const uint32_t per = tiles >> 3, rem = tiles & 7u;
    return x * per + (x < rem ? x : rem) + i;
}

// ---- hot keys ---------------------------------------------------------------------------------
struct HotLds {
    int64_t k[kHotTab];
    int8_t h[kHotTab];
};

__device__ __forceinline__ void hot_build(HotLds& s, const ApHot* hot, uint32_t nh) {
    for (int i = threadIdx.x; i < kHotTab; i += blockDim.x) s.k[i] = kSentinel;
    __syncthreads();
    for (uint32_t h = 1 + threadIdx.x; h < nh; h += blockDim.x) {
        const int64_t key = hot->key[h];
        uint32_t p = (uint32_t)(hash64((uint64_t)key) >> 8) & (kHotTab - 1);
        for (;;) {
            const unsigned long long cur =
                atomicCAS(reinterpret_cast<unsigned long long*>(&s.k[p]),
                          (unsigned long long)kSentinel, (unsigned long long)key);
            if (cur == (unsigned long long)kSentinel) {
                s.h[p] = (int8_t)h;
                break;
            }
            p = (p + 1) & (kHotTab - 1);
        }
    }
    __syncthreads();
}

// hot index of a key (hash hk), -1 if cold; two slots per step
__device__ __forceinline__ int hot_find(const HotLds& s, uint32_t nh, int64_t key, uint64_t hk) {
    if (key == kSentinel) return 0;
    if (nh <= 1) return -1;
    uint32_t p = (uint32_t)(hk >> 8) & (kHotTab - 1);
    for (;;) {
        const int64_t c0 = s.k[p], c1 = s.k[(p + 1) & (kHotTab - 1)];
        if (c0 == key) return s.h[p];
        if (c0 == kSentinel) return -1;
        if (c1 == key) return s.h[(p + 1) & (kHotTab - 1)];
        if (c1 == kSentinel) return -1;
        p = (p + 2) & (kHotTab - 1);
    }
}

// Hot-key selection, three small kernels: k_ap_sclear empties the sample table, k_ap_sample
// counts up to 64K sampled keys of the chunk in it (64 workgroups, device-scope CAS / add; a
// sample whose 4-slot probe window is full is dropped: frequent keys arrive early), k_ap_select
// (one workgroup) picks the most frequent keys seen at least hot_min times (at most kHMax - 1)
// and reads their start state. The table has 2x as many slots as the chunk has samples (a power
// of two, at least kGTabMin: select reads it in 16 columns of kTT), so small chunks scan less
constexpr int kGTab = 1 << 17;       // sample table slots, largest
constexpr int kGTabMin = 16 * 1024;  // smallest (kTT threads x 16 loads)
constexpr unsigned kSampGrid = 64;
static_assert(kGTab >= 2 * (int)kSamples && kGTabMin % (16 * 1024) == 0, "sample table sizing");
inline uint32_t gtab_for(uint32_t n) {
    const uint32_t S = n < kSamples ? n : kSamples;
    uint32_t tab = kGTabMin;
    while (tab < 2 * S) tab <<= 1;
    return tab;
}

__global__ __launch_bounds__(256) void k_ap_sclear(int64_t* __restrict__ gk,
                                                   uint32_t* __restrict__ gc, uint32_t tab) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < tab; i += gridDim.x * 256) {
        gk[i] = kSentinel;
        gc[i] = 0;
    }
}

__global__ __launch_bounds__(256) void k_ap_sample(const int64_t* __restrict__ key, uint32_t n,
                                                   uint32_t hot_min, int64_t* __restrict__ gk,
                                                   uint32_t* __restrict__ gc, uint32_t tab) {
    if (!hot_min) return;
    const uint32_t tmask = tab - 1;
    const uint32_t S = n < kSamples ? n : kSamples;
    constexpr int kB = (int)(kSamples / (kSampGrid * 256));  // samples per thread
    int64_t k[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
        const uint32_t i = (blockIdx.x * 256 + threadIdx.x) * kB + u;
        const uint32_t j = S == n ? i : (uint32_t)(((uint64_t)i * n) >> kLgSamples);
        k[u] = i < S ? key[j] : kSentinel;
    }
    const int l = lane_id();
#pragma unroll
    for (int u = 0; u < kB; ++u) {
        // lanes of the wave with the same key act once: the lowest lane of each home-slot class
        // takes every lane whose key equals its own (a hot key is most of the samples, and
        // device-scope atomics on one word serialise); a colliding other key acts alone
        const bool valid = k[u] != kSentinel;
        const uint32_t h0 = (uint32_t)hash64((uint64_t)k[u]) & tmask;
        const unsigned long long cls = match_bits(h0, 16, valid);
        const int lead = valid ? lo_bit(cls) : l;
        const int64_t lk = shfl64(k[u], lead);
        const bool follower = valid && lead != l && lk == k[u];
        const unsigned long long fol = __ballot(follower);
        if (!valid || follower) continue;
        const uint32_t cnt = lead == l ? 1u + (uint32_t)__popcll(fol & cls) : 1u;
        uint32_t p = h0;
        for (int probe = 0; probe < 4; ++probe, p = (p + 1) & tmask) {
            // agent-scope load: a plain one can hit a stale L2 copy of an empty slot that the
            // memory-side CAS has filled
            unsigned long long cur =
                __hip_atomic_load(reinterpret_cast<unsigned long long*>(&gk[p]),
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == (unsigned long long)kSentinel)
                cur = atomicCAS(reinterpret_cast<unsigned long long*>(&gk[p]),
                                (unsigned long long)kSentinel, (unsigned long long)k[u]);
            if (cur == (unsigned long long)kSentinel || (int64_t)cur == k[u]) {
                atomicAdd(&gc[p], cnt);
                break;
            }
        }
    }
}

__global__ __launch_bounds__(kTT) void k_ap_select(KvTable t, const int64_t* __restrict__ gk,
                                                   const uint32_t* __restrict__ gc,
                                                   uint32_t hot_min, uint32_t tab, ApHot* hot) {
    __shared__ int64_t hk[kHMax];
    __shared__ uint32_t sc_hist[kTT];
    __shared__ uint32_t wsum_s[kTW];
    __shared__ uint32_t nh, thr_s;
    const int tid = threadIdx.x;
    const int kPer = (int)(tab / kTT);  // a multiple of 16
    if (tid == 0) nh = 1;
    if (hot_min) {
        // the smallest threshold >= hot_min that leaves at most kHMax - 1 keys: a histogram of
        // the counts (capped at kTT - 1; more than kHMax - 1 keys cannot reach that), then a
        // suffix sum over it
        sc_hist[tid] = 0;
        if (tid == 0) thr_s = kTT;
        __syncthreads();
#pragma unroll 1
        for (int u0 = 0; u0 < kPer; u0 += 16) {  // two passes over the counts (L2): 16 loads in flight
            uint32_t c[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) c[u] = gc[(u0 + u) * kTT + tid];
#pragma unroll
            for (int u = 0; u < 16; ++u)  // counts below hot_min never decide the threshold
                if (c[u] >= hot_min) atomicAdd(&sc_hist[c[u] < (uint32_t)kTT ? c[u] : kTT - 1], 1u);
        }
        __syncthreads();
        {
            // inclusive suffix sum: reverse the index, scan forward
            const int ri = kTT - 1 - tid;
            uint32_t x = sc_hist[ri];
            const int l = lane_id();
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (l >= d) x += y;
            }
            if (l == kWave - 1) wsum_s[tid / kWave] = x;
            __syncthreads();
            uint32_t wb = 0;
            for (int w2 = 0; w2 < tid / kWave; ++w2) wb += wsum_s[w2];
            const uint32_t ge = wb + x;  // keys with count >= ri
            if ((uint32_t)ri >= hot_min && ge <= (uint32_t)kHMax - 1) atomicMin(&thr_s, (uint32_t)ri);
        }
        __syncthreads();
        const uint32_t thr = thr_s;
#pragma unroll 1
        for (int u0 = 0; u0 < kPer; u0 += 16) {
            uint32_t c[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) c[u] = gc[(u0 + u) * kTT + tid];
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (c[u] >= thr) {
                    const uint32_t x = atomicAdd(&nh, 1u);
                    if (x < kHMax) hk[x] = gk[(u0 + u) * kTT + tid];
                }
        }
    }
    __syncthreads();
    const uint32_t H = nh < (uint32_t)kHMax ? nh : (uint32_t)kHMax;
    if (tid == 0) {
        hot->n = H;
        hot->restarts = 0;
    }
    const uint32_t ep = t.epoch[0];
    for (uint32_t h = tid; h < H; h += kTT) {
        const int64_t k = h == 0 ? kSentinel : hk[h];
        const int64_t s = kv_lookup(t, k);
        const uint32_t w = s >= 0 ? t.state[s] : 0u;
        const uint32_t pres = w & kPresent;
        hot->key[h] = k;
        hot->slot[h] = s >= 0 ? (uint32_t)s : kNoSlot;
        hot->flags[h] = pres | ((w >> 2) == ep ? (4u | (w & kLastPut)) : 0u);
        hot->val0[h] = pres ? t.vals[s] : 0;
    }
}

// ---- scan of the tile rows: columns < nbin exclusive sums, the rest exclusive maxima ----------
__device__ __forceinline__ uint32_t col_op(bool sum, uint32_t a, uint32_t b) {
    return sum ? a + b : (a > b ? a : b);
}

// (columns of hot keys past hot->n are all zero and skipped)
__global__ __launch_bounds__(256) void k_ap_scan_part(ApGeo g, const uint32_t* __restrict__ rows,
                                                      uint32_t* __restrict__ part,
                                                      const ApHot* __restrict__ hot) {
    const uint32_t gi = blockIdx.x;
    const uint32_t t0 = gi * g.tpg, t1 = t0 + g.tpg < g.tiles ? t0 + g.tpg : g.tiles;
    const uint32_t cols = g.nbin + 2 * hot->n;
    for (uint32_t c = threadIdx.x; c < cols; c += 256) {
        const bool sum = c < g.nbin;
        uint32_t acc = 0;
        uint32_t tt = t0;
        for (; tt + 8 <= t1; tt += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = rows[(uint64_t)(tt + u) * g.rowlen + c];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc = col_op(sum, acc, v[u]);
        }
        for (; tt < t1; ++tt) acc = col_op(sum, acc, rows[(uint64_t)tt * g.rowlen + c]);
        part[(uint64_t)gi * g.rowlen + c] = acc;
    }
}

// exclusive prefix over the tile groups, 64 columns per workgroup: lane (c, k) of the 16 lanes
// of column c holds groups [16k, 16k + 16); a 16-lane scan of the chunk sums links them
constexpr int kTopCols = kTT / 16;
__global__ __launch_bounds__(kTT) void k_ap_scan_top(ApGeo g, uint32_t* __restrict__ part,
                                                     uint32_t* __restrict__ ctot,
                                                     ApHot* __restrict__ hot) {
    const int tid = threadIdx.x, l = lane_id();
    const int k = l & 15;
    const uint32_t c = blockIdx.x * kTopCols + (uint32_t)(tid / kWave) * 4 + (uint32_t)(l >> 4);
    const uint32_t cols = g.nbin + 2 * hot->n;
    const bool sum = c < g.nbin;
    const bool live = c < cols;
    uint32_t v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const uint32_t gi = (uint32_t)k * 16 + u;
        v[u] = live && gi < g.ng ? part[(uint64_t)gi * g.rowlen + c] : 0u;
    }
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = col_op(sum, acc, v[u]);
    uint32_t x = acc;  // inclusive scan of the chunk results over the 16 lanes of the column
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (k >= d) x = col_op(sum, x, y);
    }
    uint32_t run = (uint32_t)__shfl_up(x, 1);
    if (k == 0) run = 0;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const uint32_t gi = (uint32_t)k * 16 + u;
        if (live && gi < g.ng) part[(uint64_t)gi * g.rowlen + c] = run;
        run = col_op(sum, run, v[u]);
    }
    if (live && k == 15) {
        if (sum) {
            ctot[c] = x;
        } else {
            const uint32_t h = (c - g.nbin) >> 1;
            if ((c - g.nbin) & 1) hot->fin_put[h] = x;
            else hot->fin_any[h] = x;
        }
    }
}

// bin starts: exclusive scan of the bin totals (nbin <= 1024: one per thread)
__global__ __launch_bounds__(kTT) void k_ap_scan_bins(ApGeo g, const uint32_t* __restrict__ ctot,
                                                      uint32_t* __restrict__ bin_start) {
    __shared__ uint32_t wsum[kTW];
    const int tid = threadIdx.x, l = lane_id();
    const uint32_t v = (uint32_t)tid < g.nbin ? ctot[tid] : 0u;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (l >= d) x += y;
    }
    if (l == kWave - 1) wsum[tid / kWave] = x;
    __syncthreads();
    uint32_t wb = 0;
    for (int w2 = 0; w2 < tid / kWave; ++w2) wb += wsum[w2];
    if ((uint32_t)tid < g.nbin) {
        bin_start[tid] = wb + x - v;
        if ((uint32_t)tid == g.nbin - 1) bin_start[g.nbin] = wb + x;
    }
}

__global__ __launch_bounds__(256) void k_ap_scan_rows(ApGeo g, uint32_t* __restrict__ rows,
                                                      const uint32_t* __restrict__ part,
                                                      const uint32_t* __restrict__ bin_start,
                                                      const ApHot* __restrict__ hot) {
    const uint32_t gi = blockIdx.x;
    const uint32_t t0 = gi * g.tpg, t1 = t0 + g.tpg < g.tiles ? t0 + g.tpg : g.tiles;
    const uint32_t cols = g.nbin + 2 * hot->n;
    for (uint32_t c = threadIdx.x; c < cols; c += 256) {
        const bool sum = c < g.nbin;
        uint32_t acc = part[(uint64_t)gi * g.rowlen + c] + (sum ? bin_start[c] : 0u);
        uint32_t tt = t0;
        for (; tt + 8 <= t1; tt += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = rows[(uint64_t)(tt + u) * g.rowlen + c];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                rows[(uint64_t)(tt + u) * g.rowlen + c] = acc;
                acc = col_op(sum, acc, v[u]);
            }
        }
        for (; tt < t1; ++tt) {
            uint32_t* p = rows + (uint64_t)tt * g.rowlen + c;
            const uint32_t x = *p;
            *p = acc;
            acc = col_op(sum, acc, x);
        }
    }
}

// ---- partition ----------------------------------------------------------------------------------
// MPX_SC_LAZYV=1: with hot keys in the chunk, a command's value is loaded only once the command is
// known to be cold (after its hot-key probe, for the current tile), not prefetched for every
// command: a skewed chunk's hot commands (~99 % under zipf) never need theirs in the scatter
// (zipf 1.280 / 1.285 -> 1.256 / 1.246 ms per call, uniform unchanged - it has no hot keys and
// keeps the prefetch; profiles/r05/apply/ab_lazyv_emit_persist.txt)
#ifndef MPX_SC_LAZYV
#define MPX_SC_LAZYV 1
#endif
struct ScatterLds {
    HotLds hl;
    uint32_t lstart[kMaxBins];  // bin start inside the tile image
    uint16_t cw[kTW][kMaxBins]; // per-wave counts -> exclusive prefix over the waves
    uint8_t W[kTW][kMaxBins];
    unsigned long long PM[kTW][kWave];
    int4 img[kTL];              // bin-sorted records of the tile's cold commands
    uint32_t ha[kHMax], hp[kHMax];  // per hot key: 1 + chunk position of its last command / PUT
    uint32_t wsum[kTW];
    uint32_t ncold;
};

// Per 4096-command log tile (persistent, one workgroup per CU, XCD-contiguous tiles, the next
// tile's commands loaded while this one is ranked): the cold commands' stable ranks per bin
// (per-wave LDS peer masks + per-wave counts, prefix over the waves), a bin-sorted image of their
// 16-byte records in LDS, stored out WHOLE at the tile's own place (img[tile * kTL ...]: every
// store coalesced), plus the tile's row: per bin its count (rows, scanned afterwards into the
// runs' partition offsets) and its image start (lrow), per hot key its last command and last PUT
// in the tile. Per command its image index (ipos, log order; hot: kHotIdx | hot index).
__global__ __launch_bounds__(kTT) void k_ap_scatter(ApGeo g, const uint8_t* __restrict__ op,
                                                    const int64_t* __restrict__ key,
                                                    const int64_t* __restrict__ val, uint32_t n,
                                                    uint32_t* __restrict__ rows,
                                                    uint16_t* __restrict__ lrow,
                                                    const ApHot* __restrict__ hot,
                                                    int4* __restrict__ img,
                                                    uint16_t* __restrict__ ipos,
                                                    uint32_t* __restrict__ tcold) {
    __shared__ ScatterLds S;
    const int tid = threadIdx.x, l = lane_id(), w = tid / kWave;
    const uint32_t nh = hot->n;
    uint32_t* cw32 = reinterpret_cast<uint32_t*>(&S.cw[0][0]);
    for (int i = tid; i < kTW * kMaxBins / 2; i += kTT) cw32[i] = 0u;
    S.PM[w][l] = 0ull;
    if (tid < kHMax) S.ha[tid] = S.hp[tid] = 0u;
    hot_build(S.hl, hot, nh);
    TileWalk tw = tile_walk(g.tiles);
    const uint32_t wofs = (uint32_t)w * (kWave * kTPer) + (uint32_t)l;
    // this tile's commands in registers; the next tile's are loaded while this one is ranked
    uint32_t o[kTPer];  // 32-bit: byte-packed ops make the compiler wait for the prefetch early
    int64_t k[kTPer], v[kTPer];
    const bool lazy = MPX_SC_LAZYV && nh > 1;  // (uniform over the grid)
    auto load = [&](uint32_t tile, uint32_t* o_, int64_t* k_, int64_t* v_) {
#pragma unroll
        for (int r = 0; r < kTPer; ++r) {
            const uint32_t j = tile * (uint32_t)kTL + wofs + r * kWave;
            const bool in = tile < tw.end && j < n;
            o_[r] = in ? op[j] : 0;
            k_[r] = in ? key[j] : 0;
            v_[r] = in && !lazy ? val[j] : 0;
        }
    };
    load(tw.tile, o, k, v);
    lds_u8* W = (lds_u8*)&S.W[w][0];
    lds_u64* PM = (lds_u64*)&S.PM[w][0];
    lds_u16* CW = (lds_u16*)&S.cw[w][0];
    const unsigned long long below = (1ull << l) - 1ull;
    for (; tw.tile < tw.end; tw.tile += tw.step) {
        const uint32_t tile = tw.tile;
        const uint32_t j0 = tile * (uint32_t)kTL + wofs;
        uint32_t no[kTPer];
        int64_t nk[kTPer], nv[kTPer];
        load(tile + tw.step, no, nk, nv);
        uint32_t bin[kTPer], rank[kTPer];
        uint64_t hs[kTPer];  // the keys' hashes: the records carry them instead of the keys
        bool cold[kTPer];
#pragma unroll
        for (int r = 0; r < kTPer; ++r) {
            const uint32_t j = j0 + r * kWave;
            const bool in = j < n;
            const uint64_t h = hash64((uint64_t)k[r]);
            hs[r] = h;
            const int hh = in ? hot_find(S.hl, nh, k[r], h) : -1;
            const bool hotc = in && hh >= 0;
            if (hotc) ipos[j] = (uint16_t)(kHotIdx | (uint32_t)hh);
            cold[r] = in && hh < 0;
            if (lazy && cold[r]) v[r] = val[j];  // (used after the scans below)
            if (__ballot(hotc)) {
                // per hot key of the round: its last command and its last PUT, one LDS atomic each
                const bool put = hotc && o[r] == MPX_OP_PUT;
                const unsigned long long peers = match_bits((uint32_t)hh, kLgHMax, hotc);
                const unsigned long long puts = peers & __ballot(put);
                if (hotc && hi_bit(peers) == l) atomicMax(&S.ha[hh], j + 1);
                if (put && hi_bit(puts) == l) atomicMax(&S.hp[hh], j + 1);
            }
            bin[r] = cold[r] ? bin_of(h, g) : 0u;
            rank[r] = 0;
            if (!__ballot(cold[r])) continue;
            const unsigned long long peers = wave_peers(W, PM, bin[r], cold[r]);
            if (cold[r]) {
                const uint32_t base = CW[bin[r]];
                rank[r] = base + (uint32_t)__popcll(peers & below);
                if ((peers >> l) == 1ull) CW[bin[r]] = (uint16_t)(base + (uint32_t)__popcll(peers));
            }
        }
        __syncthreads();
        // per bin: exclusive prefix over the waves, the tile's count per bin
        uint32_t* row = rows + (uint64_t)tile * g.rowlen;
        for (uint32_t b = tid; b < g.nbin; b += kTT) {
            uint32_t x[kTW];  // all loads first: the stores below may alias them
#pragma unroll
            for (int w2 = 0; w2 < kTW; ++w2) x[w2] = S.cw[w2][b];
            uint32_t s = 0;
#pragma unroll
            for (int w2 = 0; w2 < kTW; ++w2) {
                S.cw[w2][b] = (uint16_t)s;
                s += x[w2];
            }
            S.lstart[b] = s;
            row[b] = s;
        }
        if (tid < kHMax) {
            row[g.nbin + 2 * tid] = S.ha[tid];
            row[g.nbin + 2 * tid + 1] = S.hp[tid];
            S.ha[tid] = S.hp[tid] = 0u;  // (read above by this thread only)
        }
        __syncthreads();
        {  // exclusive scan of the counts over the bins (nbin <= 1024: one per thread)
            const uint32_t c = (uint32_t)tid < g.nbin ? S.lstart[tid] : 0u;
            uint32_t x = c;
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (l >= d) x += y;
            }
            if (l == kWave - 1) S.wsum[w] = x;
            __syncthreads();
            uint32_t wb = 0;
            for (int w2 = 0; w2 < w; ++w2) wb += S.wsum[w2];
            if ((uint32_t)tid < g.nbin) {
                S.lstart[tid] = wb + x - c;
                lrow[(uint64_t)tile * g.nbin + tid] = (uint16_t)(wb + x - c);
            }
            if (tid == kTT - 1) S.ncold = wb + x;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kTPer; ++r) {
            if (!cold[r]) continue;
            const uint32_t b = bin[r];
            const uint32_t wr = S.cw[w][b] + rank[r];
            const uint32_t ip = S.lstart[b] + wr;
            const uint64_t x = rec_pack(hs[r], op_class(o[r]));
            S.img[ip] = make_int4((int)(uint32_t)x, (int)(uint32_t)(x >> 32),
                                  (int)(uint32_t)v[r], (int)(uint32_t)((uint64_t)v[r] >> 32));
            ipos[j0 + r * kWave] = (uint16_t)ip;
        }
        __syncthreads();
        // the image out whole: a wave stores its 64 slots when any of them holds a record (the
        // slots past the tile's cold commands are the tile's own, never read)
        const uint32_t nc = S.ncold;
        if (tid == 0) tcold[tile] = nc;
        int4* dst = img + (uint64_t)tile * kTL;
#pragma unroll
        for (int u = 0; u < kTPer; ++u) {
            const uint32_t i = tid + u * kTT;
            if (i - (uint32_t)l < nc) dst[i] = S.img[i];
        }
        for (int i = tid; i < kTW * kMaxBins / 2; i += kTT) cw32[i] = 0u;  // next tile's counts
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kTPer; ++r) {
            o[r] = no[r];
            k[r] = nk[r];
            v[r] = nv[r];
        }
    }
}

// The bin-major run table of the resolve: for bin b and tile t, run (t, b) = the tile's records of
// bin b, at partition positions [roff(t, b), roff(t + 1, b)) (the scanned rows; the bin's end
// after the last tile) and at image positions tile * kTL + lrow(t, b) + ...: runs[b][t] = {roff,
// image start - roff} (so a partition position q of the run lives at img[q + .y], 32-bit wrap).
// A transpose through LDS: 64 tiles x 64 bins per 256-thread workgroup.
constexpr int kRunT = 64, kRunB = 64;
__global__ __launch_bounds__(256) void k_ap_runs(ApGeo g, const uint32_t* __restrict__ rows,
                                                 const uint16_t* __restrict__ lrow,
                                                 uint2* __restrict__ runs) {
    __shared__ uint2 T[kRunB][kRunT + 1];
    const uint32_t t0 = blockIdx.x * kRunT, b0 = blockIdx.y * kRunB;
    const int tid = threadIdx.x;
    // read: 4 tiles x 64 bins per pass (lane = bin)
    for (int u = tid; u < kRunT * kRunB; u += 256) {
        const uint32_t tt = (uint32_t)u / kRunB, bb = (uint32_t)u % kRunB;
        const uint32_t t = t0 + tt, b = b0 + bb;
        if (t < g.tiles && b < g.nbin) {
            const uint32_t ro = rows[(uint64_t)t * g.rowlen + b];
            const uint32_t ls = lrow[(uint64_t)t * g.nbin + b];
            T[bb][tt] = make_uint2(ro, t * (uint32_t)kTL + ls - ro);
        }
    }
    __syncthreads();
    // write: 4 bins x 64 tiles per pass (lane = tile)
    for (int u = tid; u < kRunT * kRunB; u += 256) {
        const uint32_t bb = (uint32_t)u / kRunT, tt = (uint32_t)u % kRunT;
        const uint32_t t = t0 + tt, b = b0 + bb;
        if (t < g.tiles && b < g.nbin) runs[(uint64_t)b * g.tiles + t] = T[bb][tt];
    }
}

__device__ __forceinline__ int64_t kv_lo_hi(int lo, int hi) {
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// ---- per-bin resolve -------------------------------------------------------------------------
// One workgroup per bin, every record of a batch at once instead of 64 per wave and round:
//   P1  each record finds its slot in the bin's LDS table (a command on a key the table does not
//       hold claims a slot for it, PUT or not: a GET before the first PUT of a new key must still
//       be that PUT's predecessor) and pushes itself onto the slot's list of the batch (one LDS
//       exchange on a head word tagged with the batch; its link keeps the previous head)
//   P2  each record walks its slot's list (every record of the batch on its key, in push order):
//       the highest index below its own is its predecessor (state.Conflict), the highest PUT
//       below it its GET's source, none above it makes it the slot's last; the slot's state at
//       batch start covers what the batch does not. Results are stored in partition order
//       (coalesced). The slot's last record keeps the slot's new state
//   P3  the last records write the new states (after a barrier: P2 read the old ones)
// A slot claimed by commands that never PUT (a "phantom": the key stays absent) is removed at
// write-back and the bucket's new keys are placed again, so the table stays a linear-probing
// table of the present keys. A bucket that runs out of slots re-runs the bin in the two-pass form
// (every PUT key inserted first; other commands on absent keys then have no PUT in the call and
// resolve to 0 without a slot).
#ifndef MPX_RL_PER
#define MPX_RL_PER 2
#endif
// result stores: plain (default: the emit reads them back soon, through L2) or nontemporal
#ifndef MPX_RL_NT
#define MPX_RL_NT 0
#endif
// MPX_RES16=1: a command's result travels from the resolve to the emit as ONE 16-byte record
// (ret, conf) instead of an 8-byte ret and a separate conf byte: the emit's gather of the
// tile's ~4-record runs is then one request per run instead of two, for 7 more bytes per
// command written and read (uniform 2.09 -> 2.07 ms per call, zipf neutral;
// profiles/r05/apply/ab_res16.txt). OFF by default: the padding costs 0.93 GB of HBM traffic
// per uniform call (7.40 vs 6.47 GB, 4.16 x the algorithmic bytes instead of 3.64 x) for 1 %
#ifndef MPX_RES16
#define MPX_RES16 0
#endif
// MPX_RES_IMG=1: the resolve stores each result at its record's IMAGE position (the tile's own
// slots, the runs of the records' gather), so the emit reads its tile's results in one
// contiguous run instead of gathering them run by run from partition order
#ifndef MPX_RL_XCD
#define MPX_RL_XCD 1
#endif
#ifndef MPX_RES_IMG
#define MPX_RES_IMG 1
#endif
// diagnostic build: wave 0's clock per phase of k_ap_resolve_list, printed by bin 0
#ifndef MPX_RL_STAMP
#define MPX_RL_STAMP 0
#endif
#if MPX_RL_STAMP
#define RL_STAMP(k)                                              \
    do {                                                         \
        const unsigned long long _c = clock64();                 \
        if (tid == 0) S.rph[k] += _c - rl_c0;                    \
        rl_c0 = _c;                                              \
    } while (0)
#else
#define RL_STAMP(k) do {} while (0)
#endif
constexpr int kLT = 1024;                 // threads of the list-resolve workgroup
constexpr int kLW = kLT / kWave;
constexpr int kLPer = MPX_RL_PER;         // records per thread and batch
constexpr int kLB = kLT * kLPer;          // records per batch
constexpr int kLSlots = kMaxBPB * kSB;    // table slots of a bin
constexpr uint32_t kLIdx = 13;            // bits of 1 + a batch index
constexpr uint32_t kLIdxMask = (1u << kLIdx) - 1u;
constexpr uint32_t kLTagMax = (1u << (32 - kLIdx)) - 1u;
constexpr uint32_t kFOverflow = 4u;
constexpr int kLWin = kLT;                // tiles of the run window (one per thread)
static_assert(kLB < (1 << kLIdx) && kLB <= 0x7FFF, "links hold 1 + a batch index below the PUT bit");

// A slot with more than kLHeavyMin records in a batch (a warm key: walking its list would cost
// O(count^2)) is HEAVY: its records set their bits in a bitmap over the batch (and a bitmap of
// its PUTs), one wave scans each bitmap's words for the last set bit at or before every word, and
// a record's predecessor / last PUT before it is then a masked word plus one prefix entry. At most
// kLHeavy heavy slots per batch (more walk their lists).
constexpr uint32_t kLHeavyMin = 16;
constexpr int kLHeavy = 8;
constexpr int kLWords = kLB / 32;
static_assert(kLB % 32 == 0 && kLWords <= 2 * kWave, "a wave scans a heavy bitmap, two words a lane");

struct ListLds {
    int64_t tk[kLSlots];
    int64_t tv[kLSlots];
    // (one word past the slots: the target of the records without a slot, so the pushes and
    // counts need no branch)
    uint32_t head[kLSlots + 2];  // per slot: (batch tag << kLIdx) | (1 + the last record pushed)
    uint32_t cnt[2][kLSlots / 2 + 1];  // per batch parity, two 16-bit slot counts a word
    uint8_t ts[kLSlots];
    uint16_t link[kLB];      // per record: (PUT << 15) | (1 + the record pushed before it)
    int64_t bval[kLB];       // per record: its value (read for PUTs)
    uint32_t hb[kLHeavy][kLWords];  // heavy slots: the batch's records on it, bit per record
    uint32_t hp[kLHeavy][kLWords];  //   ... its PUTs
    int32_t la[kLHeavy][kLWords];   //   the last record at or before each word (-1: none)
    int32_t lp[kLHeavy][kLWords];   //   the last PUT at or before each word
    uint32_t hslot[kLHeavy];
    uint32_t nheavy[2];
    uint32_t flags;
    // the run window: tiles [wt0, wt0 + kLWin) of the bin's run table, their runs' partition
    // starts (wr[kLWin]: the start of the run after the window, the bin's end past the last
    // tile) and image offsets. A batch's runs as marks: per batch parity a bit per record that
    // starts a run or a 64-record segment (MB), the run's image offset at each mark (D)
    uint32_t wr[kLWin + 1];
    uint32_t wd[kLWin];
    uint32_t MB[2][kLB / 32];
    uint32_t D[kLB];
#if MPX_RL_STAMP
    unsigned long long rph[8];
#endif
};

__global__ __launch_bounds__(kLT) void k_ap_resolve_list(ApGeo g, KvTable t,
                                                         const uint32_t* __restrict__ bin_start,
                                                         const uint2* __restrict__ runs,
                                                         const int4* __restrict__ img,
                                                         int64_t* __restrict__ r_ret,
                                                         uint8_t* __restrict__ r_conf, uint32_t spare,
                                                         ApHot* hot, uint32_t* err) {
    __shared__ ListLds S;
    const int tid = threadIdx.x, l = lane_id(), w = tid / kWave;
    const uint32_t bpb = 1u << g.lgbpb;
    // XCD-contiguous bins (workgroup b runs on XCD b % 8): the bins one XCD resolves side by side
    // are neighbours, so their runs of a tile image - adjacent in it - meet in that XCD's L2: the
    // gathers' shared lines and the results' partial lines are merged there, not in HBM
    const uint32_t bin = MPX_RL_XCD ? xcd_tile(g.nbin) : blockIdx.x;
    const uint32_t nslot = bpb * kSB;
    const uint32_t nsub = 1u << g.lgsub;
    const uint32_t ep = t.epoch[0];
    const uint32_t r0 = bin_start[bin], r1 = bin_start[bin + 1];
    if (r0 == r1) return;  // no records: nothing read, nothing touched
    // the LDS table holds hashes; a free slot holds the hash of INT64_MIN (the sentinel key,
    // which never reaches a bin: it is always hot index 0)
    const int64_t kHS = (int64_t)hash64((uint64_t)kSentinel);
    // The bin's records in partition order are its runs (one per tile, bin-major run table):
    // partition position q of run u lives at img[q + wd[u]]. A batch's image positions are
    // written into P by the window's tiles (a run longer than 32 records of the batch by its
    // wave); a batch past the window's last run moves the window on (workgroup-uniform).
    const uint2* brun = runs + (uint64_t)bin * g.tiles;
    uint32_t wt0 = 0;
    auto load_win = [&](uint32_t t0) {  // (every thread; the caller's barrier publishes it)
        wt0 = t0;
        for (uint32_t u = tid; u <= (uint32_t)kLWin; u += kLT) {
            const uint32_t tt = t0 + u;
            const uint2 x = tt < g.tiles ? brun[tt] : make_uint2(r1, 0u);
            S.wr[u] = x.x;
            if (u < (uint32_t)kLWin) S.wd[u] = x.y;
        }
    };
    // the marks of batch [base, base + kLB) into MB[mp] / D (every thread; barriers inside when
    // the batch runs past the window)
    auto expand = [&](uint32_t base, uint32_t mp) {
        const uint32_t end = base + kLB < r1 ? base + kLB : r1;
        for (;;) {
            for (uint32_t u = tid; u < (uint32_t)kLWin; u += kLT) {
                const uint32_t ra = S.wr[u], re = S.wr[u + 1], d = S.wd[u];
                const uint32_t a = ra > base ? ra : base, e = re < end ? re : end;
                for (uint32_t x = a - base; a < e && x < e - base; x = (x | 63u) + 1u) {
                    atomicOr(&S.MB[mp][x >> 5], 1u << (x & 31));
                    S.D[x] = d;
                }
            }
            if (S.wr[kLWin] >= end) break;
            __syncthreads();  // the window is read
            load_win(wt0 + kLWin);
            __syncthreads();
        }
    };
    // after the marks' barrier: the image position of the thread's record i of batch `base` (nb
    // records; past them the last one's) - the last mark at or before it in its 64-record segment
    auto locate = [&](uint32_t base, uint32_t mp, uint32_t nb, uint32_t i) {
        const uint32_t x = i < nb ? i : nb - 1;
        const uint32_t sg = x >> 6, bit = x & 63u;
        const unsigned long long w =
            ((unsigned long long)S.MB[mp][2 * sg + 1] << 32) | S.MB[mp][2 * sg];
        const unsigned long long mk = bit == 63u ? ~0ull : (2ull << bit) - 1ull;
        const uint32_t m = (sg << 6) + 63u - (uint32_t)__clzll((long long)(w & mk));
        return base + x + S.D[m];
    };
    for (uint32_t sub = 0; sub < nsub; ++sub) {
        const uint64_t gbase = ((((uint64_t)bin << g.lgsub) | sub) * bpb) * kSB;
        auto member = [&](uint64_t h) {
            return ((bucket_of(h, g.lgnb) >> g.lgbpb) & (nsub - 1)) == sub;
        };
        bool rerun = false;
        for (int mode = 0; mode < 2; ++mode) {
            if (mode == 1 && !rerun) break;
            __syncthreads();  // the previous pass is done with the LDS
            for (uint32_t i = tid; i < nslot; i += kLT) {
                const int64_t key = t.keys[gbase + i];
                S.tk[i] = key == kSentinel ? kHS : (int64_t)hash64((uint64_t)key);
                S.tv[i] = t.vals[gbase + i];
                const uint32_t x = t.state[gbase + i];
                const uint8_t pres = (uint8_t)(x & kPresent);
                S.ts[i] = (uint8_t)(pres | (pres ? kSWasPresent : 0) |
                                    ((x >> 2) == ep ? (kSTouched | (x & kLastPut)) : 0u));
                S.head[i] = 0u;
            }
            for (uint32_t i = tid; i < (uint32_t)(2 * (kLSlots / 2 + 1)); i += kLT) (&S.cnt[0][0])[i] = 0u;
            for (uint32_t i = tid; i < (uint32_t)(kLHeavy * kLWords); i += kLT) {
                (&S.hb[0][0])[i] = 0u;
                (&S.hp[0][0])[i] = 0u;
            }
            if (tid == 0) {
                S.flags = 0;
                S.nheavy[0] = S.nheavy[1] = 0;
            }
            __syncthreads();
            if (mode == 1) {  // two-pass form: every PUT key of the bin first
                if (tid == 0) atomicAdd(&hot->restarts, 1u);
                for (uint32_t q = 0, tt = tid, qe = 0, d = 0;; ++q) {  // thread: tiles tid + kLT k
                    while (q >= qe && tt < g.tiles) {  // the next nonempty run of this thread
                        const uint2 x = brun[tt];
                        qe = tt + 1 < g.tiles ? brun[tt + 1].x : r1;
                        q = x.x;
                        d = x.y;
                        tt += kLT;
                    }
                    if (q >= qe) break;
                    const int4 kv = img[q + d];
                    const uint64_t x = (uint64_t)kv_lo_hi(kv.x, kv.y);
                    if ((uint32_t)(x >> 62) != kClsPut) continue;
                    const uint64_t h = rec_hash(x, bin, g);
                    const int64_t k = (int64_t)h;
                    if (!member(h)) continue;
                    const uint32_t bb = (bucket_of(h, g.lgnb) & (bpb - 1)) * kSB;
                    uint32_t p = home_of(h);
                    bool done = false;
                    for (int probe = 0; probe < kSB && !done; ++probe) {
                        const unsigned long long cur =
                            atomicCAS(reinterpret_cast<unsigned long long*>(&S.tk[bb + p]),
                                      (unsigned long long)kHS, (unsigned long long)k);
                        if (cur == (unsigned long long)kHS) {
                            S.ts[bb + p] |= kSNew;
                            done = true;
                        } else if ((int64_t)cur == k) {
                            done = true;
                        }
                        p = (p + 1) & (kSB - 1);
                    }
                    if (!done) raise_err(err, kErrKvFull);
                }
                __syncthreads();
            }
            __syncthreads();  // (the pre-insert loop's window use is over)
            load_win(0);
            for (uint32_t i = tid; i < (uint32_t)(2 * kLB / 32); i += kLT) (&S.MB[0][0])[i] = 0u;
            __syncthreads();
            expand(r0, 1u);  // (the first batch's tag is 1)
            __syncthreads();
            int4 kv[kLPer];
            uint32_t nxp[kLPer];  // the loaded batch's image positions
            {
                const uint32_t nb1 = r1 - r0 < (uint32_t)kLB ? r1 - r0 : (uint32_t)kLB;
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    const uint32_t i = hh * kLT + tid;
                    nxp[hh] = locate(r0, 1u, nb1, i);
                    kv[hh] = img[nxp[hh]];
                }
            }
            uint32_t tag = 0;
#if MPX_RL_STAMP
            if (tid < 8) S.rph[tid] = 0;
            unsigned long long rl_c0 = clock64();
#endif
            for (uint32_t base = r0; base < r1; base += kLB) {
                if (++tag == kLTagMax) {  // (after 2^19 batches) heads of old tags would match
                    for (uint32_t i = tid; i < nslot; i += kLT) S.head[i] = 0u;
                    __syncthreads();
                    tag = 1;
                }
                const uint32_t par = tag & 1u;
                // ---- P1: slot, push ----
                // (the thread's records side by side: the common path is straight-line code, so
                // their LDS round trips overlap; a probe past 4 slots and a claim run after)
                int sl[kLPer];
                int64_t v[kLPer], k[kLPer];
                uint32_t cl[kLPer];  // bit 0 a record of this pass, bit 1 PUT, bit 2 GET
                uint32_t bbs[kLPer], ps[kLPer];
                int64_t c[kLPer][4];
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    const uint32_t i = hh * kLT + tid;
                    const uint64_t x = (uint64_t)kv_lo_hi(kv[hh].x, kv[hh].y);
                    const uint32_t cls = (uint32_t)(x >> 62);
                    const uint64_t h = rec_hash(x, bin, g);
                    k[hh] = (int64_t)h;  // (the table is probed by hash)
                    v[hh] = kv_lo_hi(kv[hh].z, kv[hh].w);
                    const bool live = base + i < r1 && member(h);
                    cl[hh] = (live ? 1u : 0u) | (cls == kClsPut ? 2u : 0u) |
                             (cls == kClsGet ? 4u : 0u);
                    bbs[hh] = (bucket_of(h, g.lgnb) & (bpb - 1)) * kSB;
                    ps[hh] = home_of(h);
#pragma unroll
                    for (int u = 0; u < 4; ++u) c[hh][u] = S.tk[bbs[hh] + ((ps[hh] + u) & (kSB - 1))];
                }
                // first probe step; -1: look further (no hit and no free slot among the 4), -2:
                // absent (p = the first free slot)
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    int hit = -1, stop = -1;
#pragma unroll
                    for (int u = 3; u >= 0; --u) {
                        if (c[hh][u] == k[hh]) hit = u;
                        if (c[hh][u] == kHS) stop = u;
                    }
                    int s = -1;
                    if (hit >= 0 && (stop < 0 || hit < stop)) s = (int)((ps[hh] + hit) & (kSB - 1));
                    else if (stop >= 0) {
                        s = -2;
                        ps[hh] = (ps[hh] + stop) & (kSB - 1);
                    } else {
                        ps[hh] = (ps[hh] + 4) & (kSB - 1);
                    }
                    sl[hh] = (cl[hh] & 1u) ? s : -3;  // -3: not a record of this pass
                }
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    if (sl[hh] != -1) continue;  // rare: a long probe
                    const uint32_t bb = bbs[hh];
                    uint32_t p = ps[hh];
                    int s = -2;
                    for (int step = 1; step < kSB / 4; ++step) {
                        int64_t cc[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) cc[u] = S.tk[bb + ((p + u) & (kSB - 1))];
                        int hit = -1, stop = -1;
#pragma unroll
                        for (int u = 3; u >= 0; --u) {
                            if (cc[u] == k[hh]) hit = u;
                            if (cc[u] == kHS) stop = u;
                        }
                        if (hit >= 0 && (stop < 0 || hit < stop)) {
                            s = (int)((p + hit) & (kSB - 1));
                            break;
                        }
                        if (stop >= 0) {
                            p = (p + stop) & (kSB - 1);
                            break;
                        }
                        p = (p + 4) & (kSB - 1);
                    }
                    ps[hh] = p;
                    sl[hh] = s;
                }
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    if (sl[hh] != -2) continue;  // absent: claim a slot (any op in the one-pass form)
                    const bool isput = (cl[hh] & 2u) != 0;
                    int s = -1;
                    if (mode == 0 || isput) {
                        const uint32_t bb = bbs[hh];
                        uint32_t p = ps[hh];
                        for (int probe = 0; probe < kSB; ++probe) {
                            const unsigned long long cur =
                                atomicCAS(reinterpret_cast<unsigned long long*>(&S.tk[bb + p]),
                                          (unsigned long long)kHS, (unsigned long long)k[hh]);
                            if (cur == (unsigned long long)kHS) {
                                s = (int)p;
                                S.ts[bb + p] |= kSNew;
                                break;
                            }
                            if ((int64_t)cur == k[hh]) {
                                s = (int)p;
                                break;
                            }
                            p = (p + 1) & (kSB - 1);
                        }
                        if (s < 0) {
                            if (mode == 0) atomicOr(&S.flags, kFOverflow);
                            else raise_err(err, kErrKvFull);
                        }
                    }
                    sl[hh] = s;
                }
                // (branch-free: a record without a slot pushes onto and counts in the spare word)
                uint32_t olds[kLPer];
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    const uint32_t i = hh * kLT + tid;
                    sl[hh] = sl[hh] >= 0 ? (int)(bbs[hh] + (uint32_t)sl[hh]) : -1;
                    const uint32_t x = sl[hh] >= 0 ? (uint32_t)sl[hh] : (uint32_t)kLSlots;
                    olds[hh] = atomicExch(&S.head[x], (tag << kLIdx) | (i + 1u));
                }
                uint32_t cnts[kLPer];
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    const uint32_t i = hh * kLT + tid;
                    const uint32_t x = sl[hh] >= 0 ? (uint32_t)sl[hh] : (uint32_t)kLSlots;
                    const bool isput = (cl[hh] & 2u) != 0;
                    const uint32_t pv = (olds[hh] >> kLIdx) == tag ? (olds[hh] & kLIdxMask) : 0u;
                    S.link[i] = (uint16_t)((isput ? 0x8000u : 0u) | pv);
                    S.bval[i] = v[hh];  // (read for PUTs only)
                    const uint32_t sh = 16u * (x & 1u);
                    cnts[hh] = (atomicAdd(&S.cnt[par][x >> 1], 1u << sh) >> sh) & 0xFFFFu;
                }
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    if (sl[hh] >= 0 && cnts[hh] == kLHeavyMin) {  // the slot turns heavy
                        const uint32_t hx = atomicAdd(&S.nheavy[par], 1u);
                        if (hx < (uint32_t)kLHeavy) S.hslot[hx] = (uint32_t)sl[hh];
                    }
                }
                // the next batch's image positions (batch parity par ^ 1: the one this batch
                // was loaded through is read no more), then its records load while this one
                // resolves
                const bool more = base + kLB < r1;  // (uniform)
                RL_STAMP(6);
                if (more) expand(base + kLB, par ^ 1u);
                RL_STAMP(0);
                __syncthreads();
                RL_STAMP(1);
                uint32_t cur[kLPer];  // this batch's image positions (its results' places)
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) cur[hh] = nxp[hh];
                if (more) {
                    const uint32_t nb1 = r1 - (base + kLB) < (uint32_t)kLB ? r1 - (base + kLB) : (uint32_t)kLB;
#pragma unroll
                    for (int hh = 0; hh < kLPer; ++hh) {  // (clamped, not guarded: no branch)
                        const uint32_t i = hh * kLT + tid;
                        nxp[hh] = locate(base + kLB, par ^ 1u, nb1, i);
                        kv[hh] = img[nxp[hh]];
                    }
                }
                // ---- heavy slots: bitmaps, then their prefix maxima (uniform branch) ----
                const uint32_t nh0 = S.nheavy[par];
                const uint32_t nh = nh0 < (uint32_t)kLHeavy ? nh0 : (uint32_t)kLHeavy;
                // (cl bits 4..7: 1 + the heavy index of the record's slot, 0: walk its list)
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    if (!nh || sl[hh] < 0) continue;
                    const uint32_t x = (uint32_t)sl[hh];
                    const uint32_t c = (S.cnt[par][x >> 1] >> (16u * (x & 1u))) & 0xFFFFu;
                    if (c <= kLHeavyMin) continue;
                    int hx = -1;
                    for (uint32_t q = 0; q < nh; ++q)
                        if (S.hslot[q] == x) hx = (int)q;
                    if (hx >= 0) {
                        const uint32_t i = hh * kLT + tid;
                        cl[hh] |= (uint32_t)(hx + 1) << 4;
                        atomicOr(&S.hb[hx][i >> 5], 1u << (i & 31));
                        if (cl[hh] & 2u) atomicOr(&S.hp[hx][i >> 5], 1u << (i & 31));
                    }
                }
                if (nh) {
                    __syncthreads();
                    if ((uint32_t)w < nh) {  // wave w: heavy slot w's prefix maxima over the words
                        int a0 = -1, a1 = -1, p0 = -1, p1 = -1;
                        if (l < kLWords) {  // (kLWords < 64 for batches under 2048 records)
                            const uint32_t b0 = S.hb[w][l], q0 = S.hp[w][l];
                            a0 = b0 ? l * 32 + hi_bit(b0) : -1;
                            p0 = q0 ? l * 32 + hi_bit(q0) : -1;
                        }
                        if (l + kWave < kLWords) {
                            const uint32_t b1 = S.hb[w][l + kWave], q1 = S.hp[w][l + kWave];
                            a1 = b1 ? (l + kWave) * 32 + hi_bit(b1) : -1;
                            p1 = q1 ? (l + kWave) * 32 + hi_bit(q1) : -1;
                        }
#pragma unroll
                        for (int d = 1; d < kWave; d <<= 1) {
                            const int ya0 = __shfl_up(a0, d), yp0 = __shfl_up(p0, d);
                            const int ya1 = __shfl_up(a1, d), yp1 = __shfl_up(p1, d);
                            if (l >= d) {
                                a0 = a0 > ya0 ? a0 : ya0;
                                p0 = p0 > yp0 ? p0 : yp0;
                                a1 = a1 > ya1 ? a1 : ya1;
                                p1 = p1 > yp1 ? p1 : yp1;
                            }
                        }
                        const int ta = __shfl(a0, kWave - 1), tp = __shfl(p0, kWave - 1);
                        if (l < kLWords) {
                            S.la[w][l] = a0;
                            S.lp[w][l] = p0;
                        }
                        if (l + kWave < kLWords) {
                            S.la[w][l + kWave] = a1 > ta ? a1 : ta;
                            S.lp[w][l + kWave] = p1 > tp ? p1 : tp;
                        }
                    }
                    __syncthreads();
                }
                RL_STAMP(2);
                // ---- P2: walk, results ----
                // (the thread's lists walked side by side: one round issues the next link of
                // each, so a round trip serves all three)
                uint32_t j1[kLPer];
                uint32_t stt[kLPer];
                int64_t tabv[kLPer];
                int prev[kLPer], lastput[kLPer];
                uint32_t fl[kLPer];  // bit 0 the predecessor is a PUT, bit 1 a later record
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    const int x = sl[hh] >= 0 ? sl[hh] : 0;
                    const uint32_t hw = S.head[x];  // (unconditional: no branch around the load)
                    j1[hh] = sl[hh] >= 0 && !(cl[hh] >> 4) ? (hw & kLIdxMask) : 0u;
                    stt[hh] = S.ts[x];
                    tabv[hh] = S.tv[x];
                    prev[hh] = lastput[hh] = -1;
                    fl[hh] = 0;
                }
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    if (!(cl[hh] >> 4)) continue;  // heavy: the bitmaps
                    const uint32_t i = hh * kLT + tid;
                    const int hx = (int)(cl[hh] >> 4) - 1;
                    const uint32_t wd = i >> 5, mk = (1u << (i & 31)) - 1u;
                    const uint32_t ba = S.hb[hx][wd] & mk, bp = S.hp[hx][wd] & mk;
                    prev[hh] = ba ? (int)(wd * 32 + hi_bit(ba)) : (wd ? S.la[hx][wd - 1] : -1);
                    lastput[hh] = bp ? (int)(wd * 32 + hi_bit(bp)) : (wd ? S.lp[hx][wd - 1] : -1);
                    fl[hh] = (prev[hh] >= 0 && prev[hh] == lastput[hh] ? 1u : 0u) |
                             (S.la[hx][kLWords - 1] > (int)i ? 2u : 0u);
                }
                for (;;) {
                    uint32_t any = 0;
#pragma unroll
                    for (int hh = 0; hh < kLPer; ++hh) any |= j1[hh];
                    if (!any) break;
                    uint32_t lk[kLPer];
#pragma unroll
                    for (int hh = 0; hh < kLPer; ++hh) lk[hh] = S.link[j1[hh] ? j1[hh] - 1u : 0u];
#pragma unroll
                    for (int hh = 0; hh < kLPer; ++hh) {
                        if (!j1[hh]) continue;
                        const uint32_t i = hh * kLT + tid;
                        const uint32_t j = j1[hh] - 1u;
                        const bool pj = (lk[hh] >> 15) != 0;
                        if (j < i) {
                            if ((int)j > prev[hh]) {
                                prev[hh] = (int)j;
                                fl[hh] = (fl[hh] & ~1u) | (pj ? 1u : 0u);
                            }
                            if (pj && (int)j > lastput[hh]) lastput[hh] = (int)j;
                        } else if (j > i) {
                            fl[hh] |= 2u;
                        }
                        j1[hh] = lk[hh] & 0x7FFFu;
                    }
                    if (MPX_RS_ABL & 4) break;  // (diagnostic: one step of each list)
                }
                int64_t lpv[kLPer];
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) lpv[hh] = S.bval[lastput[hh] >= 0 ? lastput[hh] : 0];
                uint32_t nst = 0;  // byte hh: the new state of record hh's slot (0: not its last)
                int64_t nval[kLPer];
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    const uint32_t i = hh * kLT + tid;
                    nval[hh] = 0;
                    const bool isput = (cl[hh] & 2u) != 0, isget = (cl[hh] & 4u) != 0;
                    int64_t ret = 0;
                    bool conf = false;
                    if (sl[hh] >= 0) {
                        const uint32_t st0 = stt[hh];
                        const bool hl = lastput[hh] >= 0;
                        const bool hasprev = prev[hh] >= 0 || (st0 & kSTouched) != 0;
                        const bool pput = prev[hh] >= 0 ? (fl[hh] & 1u) != 0 : (st0 & kSLastPut) != 0;
                        ret = isput ? v[hh]
                                    : (isget ? (hl ? lpv[hh] : ((st0 & kSPresent) ? tabv[hh] : 0)) : 0);
                        conf = hasprev && (pput || isput);
                        if (!(fl[hh] & 2u)) {  // the slot's last record of the batch: its new state
                            uint32_t ns = (st0 & (kSPresent | kSValDirty | kSNew | kSWasPresent)) |
                                          kSTouched | (isput ? kSLastPut : 0);
                            if (isput || hl) ns |= kSPresent | kSValDirty;
                            nst |= ns << (8 * hh);
                            nval[hh] = isput ? v[hh] : (hl ? lpv[hh] : tabv[hh]);
                        }
                    }
                    // (a record of this pass without a slot: the two-pass form's key that is
                    // absent and never PUT in the call - NIL, no conflict)
                    // (every record stores, those not of this pass to the spare slot past the chunk:
                    // a fixed count, so the wait for the next batch, loaded before these stores,
                    // does not wait for them)
#if MPX_RES_IMG
                    const uint32_t dst = (cl[hh] & 1u) ? cur[hh] : spare;
#else
                    const uint32_t dst = (cl[hh] & 1u) ? base + i : spare;
#endif
                    if (!(MPX_RS_ABL & 2)) {
#if MPX_RES16
                        reinterpret_cast<int4*>(r_ret)[dst] =
                            make_int4((int)(uint32_t)ret, (int)(uint32_t)((uint64_t)ret >> 32),
                                      conf ? 1 : 0, 0);
#elif MPX_RL_NT
                        st_stream(r_ret + dst, ret);
                        st_stream(r_conf + dst, (uint8_t)(conf ? 1 : 0));
#else
                        r_ret[dst] = ret;
                        r_conf[dst] = conf ? 1 : 0;
#endif
                    }
                }
                // this batch's marks are read (after the last barrier): cleared for the batch after
                // next (marked after the next barrier)
                if (tid < kLB / 32) S.MB[par][tid] = 0u;
                RL_STAMP(3);
                __syncthreads();
                RL_STAMP(4);
                // ---- P3: the slots' new states; this parity's counters and bitmaps cleared (its
                // next batch comes after the next batch's first barrier) ----
#pragma unroll
                for (int hh = 0; hh < kLPer; ++hh) {
                    const uint8_t ns = (uint8_t)(nst >> (8 * hh));
                    if (ns) {  // (a last record's state has kSTouched)
                        S.ts[sl[hh]] = ns;
                        if (ns & kSValDirty) S.tv[sl[hh]] = nval[hh];
                    }
                    if (sl[hh] >= 0) S.cnt[par][(uint32_t)sl[hh] >> 1] = 0u;
                }
                if (nh && (uint32_t)w < nh) {
                    if (l < kLWords) {
                        S.hb[w][l] = 0u;
                        S.hp[w][l] = 0u;
                    }
                    if (l + kWave < kLWords) {
                        S.hb[w][l + kWave] = 0u;
                        S.hp[w][l + kWave] = 0u;
                    }
                }
                if (tid == 0) {
                    S.nheavy[par] = 0u;
                    S.cnt[par][kLSlots / 2] = 0u;
                }
                RL_STAMP(5);
            }
            __syncthreads();
#if MPX_RL_STAMP
            if (bin == 0 && sub == 0 && tid == 0)
                printf("RL_STAMP bin0 mode %d recs %u batches %u: P1 %llu expand %llu bar1 %llu heavy %llu P2 %llu bar2 %llu P3 %llu\n",
                       mode, r1 - r0, tag, S.rph[6], S.rph[0], S.rph[1], S.rph[2], S.rph[3], S.rph[4], S.rph[5]);
#endif
            if (mode == 0) rerun = (S.flags & kFOverflow) != 0;
        }
        // ---- phantoms out: a bucket holding slots whose keys never became present has them
        // removed and its new keys placed again (existing keys never move: every slot of their
        // probe chains was occupied before this call). Wave w takes bucket w.
        for (uint32_t b = (uint32_t)w; b < bpb; b += kLW) {
            int64_t* T = S.tk + b * kSB;
            int64_t* V = S.tv + b * kSB;
            uint8_t* TS = S.ts + b * kSB;
            uint8_t sv[kSB / kWave];
            bool ph = false;
#pragma unroll
            for (int u = 0; u < kSB / kWave; ++u) {
                sv[u] = TS[l + u * kWave];
                ph |= (sv[u] & kSNew) && !(sv[u] & kSPresent);
            }
            if (!__ballot(ph)) continue;
            int64_t kk[kSB / kWave], vv[kSB / kWave];
#pragma unroll
            for (int u = 0; u < kSB / kWave; ++u) {
                kk[u] = T[l + u * kWave];
                vv[u] = V[l + u * kWave];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll
            for (int u = 0; u < kSB / kWave; ++u) {
                if (sv[u] & kSNew) {
                    T[l + u * kWave] = kHS;
                    TS[l + u * kWave] = 0;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll
            for (int u = 0; u < kSB / kWave; ++u) {
                if ((sv[u] & kSNew) && (sv[u] & kSPresent)) {
                    uint32_t p = home_of((uint64_t)kk[u]);
                    for (int probe = 0; probe < kSB; ++probe) {
                        const unsigned long long cur =
                            atomicCAS(reinterpret_cast<unsigned long long*>(&T[p]),
                                      (unsigned long long)kHS, (unsigned long long)kk[u]);
                        if (cur == (unsigned long long)kHS) {
                            V[p] = vv[u];
                            TS[p] = sv[u];
                            break;
                        }
                        p = (p + 1) & (kSB - 1);
                    }
                }
            }
        }
        __syncthreads();
        // write back the touched slots; count the keys that became present
        uint32_t added = 0;
        for (uint32_t i = tid; i < nslot; i += kLT) {
            const uint8_t s = S.ts[i];
            if (s & kSNew) t.keys[gbase + i] = (int64_t)unhash64((uint64_t)S.tk[i]);
            if (s & kSValDirty) t.vals[gbase + i] = S.tv[i];
            if (s & kSTouched) t.state[gbase + i] = (ep << 2) | (s & (kPresent | kLastPut));
            added += ((s & kSPresent) && !(s & kSWasPresent)) ? 1u : 0u;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) added += __shfl_xor(added, d);
        if (l == 0 && added) atomicAdd(t.n_present, (unsigned long long)added);
        __syncthreads();  // the next sub-bin reloads the LDS table
    }
}

// ---- hot keys: final state ----------------------------------------------------------------------
__global__ void k_ap_hot_commit(KvTable t, const int64_t* __restrict__ val, const ApHot* hot,
                                uint32_t* err) {
    const uint32_t h = threadIdx.x;
    if (h >= hot->n) return;
    const uint32_t a = hot->fin_any[h], p = hot->fin_put[h];
    if (!a) return;
    uint32_t slot = hot->slot[h];
    const uint32_t fl = hot->flags[h];
    if (slot == kNoSlot) {
        if (!p) return;  // GET / other ops of an absent key: nothing to record
        const int64_t s = kv_insert(t, hot->key[h], err);
        if (s < 0) return;
        slot = (uint32_t)s;
    }
    const uint32_t ep = t.epoch[0];
    if (p) t.vals[slot] = val[p - 1];
    t.state[slot] = (ep << 2) | (a == p ? kLastPut : 0u) | ((fl & kPresent) || p ? kPresent : 0u);
    if (!(fl & kPresent) && p) atomicAdd(t.n_present, 1ull);
}

// ---- log-order results --------------------------------------------------------------------------
struct EmitLds {
    uint2 T[kTW][kHMax];   // per wave and hot key: 1 + position of the last command / last PUT
    uint2 TP[kTW][kHMax];  // the same over the earlier waves of the tile
    uint2 inc[kHMax];      // over the earlier tiles
    int64_t hval[kHMax];
    uint32_t hfl[kHMax];
    int64_t iret[kTL];     // the tile's cold results in image order (bin runs)
    uint8_t iconf[kTL];
    uint16_t lst[kMaxBins];  // per bin: image start of the tile's run
    uint32_t dof[kMaxBins];  //          partition start of the run - image start
    uint32_t wsum[kTW];
};

__global__ __launch_bounds__(kTT) void k_ap_emit(ApGeo g, const uint8_t* __restrict__ op,
                                                 const int64_t* __restrict__ val, uint32_t n,
                                                 const uint16_t* __restrict__ ipos,
                                                 const uint32_t* __restrict__ tcold,
                                                 const int64_t* __restrict__ r_ret,
                                                 const uint8_t* __restrict__ r_conf,
                                                 const uint32_t* __restrict__ rows,
                                                 const uint32_t* __restrict__ bin_start,
                                                 const ApHot* __restrict__ hot,
                                                 int64_t* __restrict__ ret,
                                                 uint8_t* __restrict__ conf) {
    __shared__ EmitLds S;
    const int tid = threadIdx.x, l = lane_id(), w = tid / kWave;
    for (int i = l; i < kHMax; i += kWave) S.T[w][i] = make_uint2(0u, 0u);  // own row: no barrier
    const uint32_t tile = xcd_tile(g.tiles);
    if (tid < kHMax) {
        const uint32_t* row = rows + (uint64_t)tile * g.rowlen + g.nbin;
        S.inc[tid] = make_uint2(row[2 * tid], row[2 * tid + 1]);
        S.hval[tid] = hot->val0[tid];
        S.hfl[tid] = hot->flags[tid];
    }
    const uint32_t jw = tile * (uint32_t)kTL + (uint32_t)w * (kWave * kTPer);
    uint32_t p[kTPer];
    int64_t rv[kTPer];
    uint8_t cf[kTPer];
    uint32_t o[kTPer];
#pragma unroll
    for (int r = 0; r < kTPer; ++r) {
        const uint32_t j = jw + r * kWave + l;
        p[r] = j < n ? ipos[j] : 0u;
    }
    // the cold results, lanes over the tile image: consecutive lanes read consecutive positions of
    // one bin run (the gather in command order touched one line per lane)
#if MPX_RES_IMG
    {  // the tile's results in image order are its own slots: one contiguous run
        const uint32_t nc = tcold[tile];
        const uint64_t r0 = (uint64_t)tile * kTL;
        int64_t xr[kTPer];
        uint8_t c[kTPer];
#pragma unroll
        for (int u = 0; u < kTPer; ++u) {
            const uint32_t i = tid + u * kTT;
            const bool any = i - (uint32_t)l < nc;  // (wave-uniform)
#if MPX_RES16
            const int4 rr = any ? reinterpret_cast<const int4*>(r_ret)[r0 + i] : make_int4(0, 0, 0, 0);
            xr[u] = kv_lo_hi(rr.x, rr.y);
            c[u] = (uint8_t)rr.z;
#else
            xr[u] = any ? r_ret[r0 + i] : 0;
            c[u] = any ? r_conf[r0 + i] : 0;
#endif
        }
#pragma unroll
        for (int u = 0; u < kTPer; ++u) {
            const uint32_t i = tid + u * kTT;
            if (i < nc) {
                S.iret[i] = xr[u];
                S.iconf[i] = c[u];
            }
        }
    }
#else
    {
        // the tile's run of bin b starts at partition position rows[tile][b] and ends at the next
        // tile's start (the bin's end after the last tile); its image start is the exclusive
        // scan of the run lengths over the bins. An image position's run: a binary search of the
        // runs' image starts (the last one at or before it; an empty run starts where the next
        // one does, so the search never ends on one)
        uint32_t rof = 0, cnt = 0;
        if ((uint32_t)tid < g.nbin) {
            rof = rows[(uint64_t)tile * g.rowlen + tid];
            const uint32_t nx = tile + 1 < g.tiles ? rows[(uint64_t)(tile + 1) * g.rowlen + tid]
                                                   : bin_start[tid + 1];
            cnt = nx - rof;
        }
        uint32_t x = cnt;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if (l >= d) x += y;
        }
        if (l == kWave - 1) S.wsum[w] = x;
        __syncthreads();
        uint32_t wb = 0, nc = 0;
#pragma unroll
        for (int w2 = 0; w2 < kTW; ++w2) {
            const uint32_t ws = S.wsum[w2];
            wb += w2 < w ? ws : 0u;
            nc += ws;
        }
        if ((uint32_t)tid < g.nbin) {
            const uint32_t lst = wb + x - cnt;
            S.lst[tid] = (uint16_t)lst;
            S.dof[tid] = rof - lst;
        }
        __syncthreads();
        uint32_t lo[kTPer];
#pragma unroll
        for (int u = 0; u < kTPer; ++u) lo[u] = 0;
        // (the searches side by side; a wave whose positions are all past the tile's cold
        // commands skips them: a skewed chunk's tiles have few)
        const uint32_t nsearch = nc > (uint32_t)(tid - l) ? (nc - (uint32_t)(tid - l) + kTT - 1) / kTT : 0u;
        for (uint32_t half = nsearch ? g.nbin >> 1 : 0u; half; half >>= 1) {
#pragma unroll
            for (int u = 0; u < kTPer; ++u) {
                if ((uint32_t)u >= nsearch) continue;  // (wave-uniform)
                const uint32_t i = tid + u * kTT;
                lo[u] = S.lst[lo[u] + half] <= i ? lo[u] + half : lo[u];
            }
        }
        uint32_t q[kTPer];
#pragma unroll
        for (int u = 0; u < kTPer; ++u) q[u] = S.dof[lo[u]] + tid + u * kTT;
        int64_t xr[kTPer];
        uint8_t c[kTPer];
#pragma unroll
        for (int u = 0; u < kTPer; ++u) {
            const uint32_t i = tid + u * kTT;
#if MPX_RES16
            const int4 rr = i < nc ? reinterpret_cast<const int4*>(r_ret)[q[u]] : make_int4(0, 0, 0, 0);
            xr[u] = kv_lo_hi(rr.x, rr.y);
            c[u] = (uint8_t)rr.z;
#else
            xr[u] = i < nc ? r_ret[q[u]] : 0;
            c[u] = i < nc ? r_conf[q[u]] : 0;
#endif
        }
#pragma unroll
        for (int u = 0; u < kTPer; ++u) {
            const uint32_t i = tid + u * kTT;
            if (i < nc) {
                S.iret[i] = xr[u];
                S.iconf[i] = c[u];
            }
        }
    }
#endif
#pragma unroll
    for (int r = 0; r < kTPer; ++r) {
        const uint32_t j = jw + r * kWave + l;
        const bool in = j < n;
        const bool hotc = in && (p[r] & kHotIdx);
        o[r] = hotc ? op[j] : 0u;
        rv[r] = hotc ? val[j] : 0;
        cf[r] = 0;
    }
    const unsigned long long below = (1ull << l) - 1ull;
    uint32_t pa[kTPer], pp[kTPer];
#pragma unroll
    for (int r = 0; r < kTPer; ++r) {
        const uint32_t j = jw + r * kWave + l;
        const bool hotc = j < n && (p[r] & kHotIdx);
        pa[r] = 0;
        pp[r] = 0;
        if (!__ballot(hotc)) continue;
        const uint32_t h = hotc ? (p[r] & ~kHotIdx) : 0u;
        const unsigned long long peers = match_bits(h, kLgHMax, hotc);
        const unsigned long long putm = __ballot(hotc && o[r] == MPX_OP_PUT);
        if (hotc) {
            const uint2 tr = S.T[w][h];
            const unsigned long long lp = peers & below, lput = lp & putm;
            const uint32_t jb = jw + r * kWave + 1;  // 1 + position of lane 0
            pa[r] = lp ? jb + (uint32_t)hi_bit(lp) : tr.x;
            pp[r] = lput ? jb + (uint32_t)hi_bit(lput) : tr.y;
            if ((peers >> l) == 1ull) {
                const unsigned long long allput = peers & putm;
                S.T[w][h] = make_uint2(jb + (uint32_t)l, allput ? jb + (uint32_t)hi_bit(allput) : tr.y);
            }
        }
    }
    bool mine = false;  // any hot command among this thread's
#pragma unroll
    for (int r = 0; r < kTPer; ++r) mine |= jw + r * kWave + l < n && (p[r] & kHotIdx);
    if (!__syncthreads_or(mine)) goto emit_out;  // also publishes the staged cold results
    for (int i = tid; i < kTW * kHMax; i += kTT) {
        const int ww = i / kHMax, hh = i % kHMax;
        uint2 m = make_uint2(0u, 0u);
        for (int w2 = 0; w2 < ww; ++w2) {
            const uint2 x = S.T[w2][hh];
            m.x = m.x > x.x ? m.x : x.x;
            m.y = m.y > x.y ? m.y : x.y;
        }
        S.TP[ww][hh] = m;
    }
    __syncthreads();
emit_out:
#pragma unroll
    for (int r = 0; r < kTPer; ++r) {
        const uint32_t j = jw + r * kWave + l;
        if (j >= n) continue;
        if (p[r] & kHotIdx) {
            const uint32_t h = p[r] & ~kHotIdx;
            const uint2 tp = S.TP[w][h], ic = S.inc[h];
            uint32_t a = pa[r] > tp.x ? pa[r] : tp.x;
            a = a > ic.x ? a : ic.x;
            uint32_t q = pp[r] > tp.y ? pp[r] : tp.y;
            q = q > ic.y ? q : ic.y;
            const uint32_t fl = S.hfl[h];
            const bool hasprev = a != 0 || (fl & 4u);
            const bool prevput = a ? a == q : (fl & kLastPut) != 0;
            const bool isput = o[r] == MPX_OP_PUT, isget = o[r] == MPX_OP_GET;
            const int64_t x = isput ? rv[r]
                                    : (isget ? (q ? val[q - 1] : ((fl & kPresent) ? S.hval[h] : 0))
                                             : 0);
            rv[r] = x;
            cf[r] = hasprev && (prevput || isput) ? 1 : 0;
        } else {
            rv[r] = S.iret[p[r]];
            cf[r] = S.iconf[p[r]];
        }
        st_stream(ret + j, rv[r]);
        if (conf) st_stream(conf + j, cf[r]);
    }
}

// ---- launcher ---------------------------------------------------------------------------------
namespace {
struct FastLayout {
    uint64_t gk, gc, rows, part, ctot, bin_start, img, lrow, runs, ipos, tcold, r_ret, r_conf, hot,
        total;
};

ApGeo geo_for(const KvTable& t, uint64_t n) {
    ApGeo g{};
    g.lgnb = t.lgnb;
    g.lgbpb = lgbpb_for(t.lgnb);
    const uint32_t lgbins = t.lgnb - g.lgbpb;
    g.lgsub = lgbins > (uint32_t)kLgMaxBins ? lgbins - (uint32_t)kLgMaxBins : 0u;
    g.lgnbin = lgbins - g.lgsub;
    g.nbin = 1u << g.lgnbin;
    g.rowlen = g.nbin + 2 * kHMax;
    g.tiles = (uint32_t)((n + kTL - 1) / kTL);
    if (!g.tiles) g.tiles = 1;
    g.ng = g.tiles < kScanGroups ? g.tiles : kScanGroups;
    g.tpg = (g.tiles + g.ng - 1) / g.ng;
    g.ng = (g.tiles + g.tpg - 1) / g.tpg;
    return g;
}

FastLayout fast_layout(const KvTable& t, uint64_t c) {
    const ApGeo g = geo_for(t, c);
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    FastLayout L{};
    uint64_t o = 0;
    L.gk = o; o += al((uint64_t)kGTab * 8);
    L.gc = o; o += al((uint64_t)kGTab * 4);
    L.rows = o; o += al((uint64_t)g.tiles * g.rowlen * 4);
    L.part = o; o += al((uint64_t)kScanGroups * g.rowlen * 4);
    L.ctot = o; o += al((uint64_t)g.nbin * 4);
    L.bin_start = o; o += al(((uint64_t)g.nbin + 1) * 4);
    L.img = o; o += al((uint64_t)g.tiles * kTL * 16);
    L.lrow = o; o += al((uint64_t)g.tiles * g.nbin * 2);
    L.runs = o; o += al((uint64_t)g.tiles * g.nbin * 8);
    L.ipos = o; o += al(c * 2);
    L.tcold = o; o += al((uint64_t)g.tiles * 4);
    // results: at partition or image positions, + the spare result (see k_ap_resolve_list)
    const uint64_t nres = (MPX_RES_IMG ? (uint64_t)g.tiles * kTL : c) + 1;
    L.r_ret = o; o += al(nres * (MPX_RES16 ? 16 : 8));
    L.r_conf = o; o += MPX_RES16 ? 0 : al(nres);
    L.hot = o; o += al(sizeof(ApHot));
    L.total = o;
    return L;
}
}  // namespace

bool apply_fast_ok(const KvTable& t) {
    return t.lgnb >= 2 && t.lgnb - lgbpb_for(t.lgnb) <= (uint32_t)(kLgMaxBins + kLgMaxSub);
}

uint64_t apply_fast_work_bytes(const KvTable& t, uint64_t c) { return fast_layout(t, c).total; }

__global__ __launch_bounds__(256) void k_ap_preinsert(KvTable t, const uint8_t* __restrict__ op,
                                                      const int64_t* __restrict__ key, uint64_t m,
                                                      uint32_t* err) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride)
        if (op[i] == MPX_OP_PUT && key[i] != kSentinel) kv_insert(t, key[i], err);
}

hipError_t launch_apply_fast(KvTable& t, const uint8_t* op, const int64_t* key, const int64_t* val,
                             uint64_t m, int64_t* ret, uint8_t* conf, uint64_t C, ApplyWork& w,
                             uint32_t hot_min, uint32_t* err, hipStream_t stream) {
    if (C >= (1ull << 31)) return hipErrorInvalidValue;
    const FastLayout L = fast_layout(t, C);
    if (w.bytes < L.total) return hipErrorInvalidValue;
    char* b = (char*)w.base;
    int64_t* gk = (int64_t*)(b + L.gk);
    uint32_t* gc = (uint32_t*)(b + L.gc);
    uint32_t* rows = (uint32_t*)(b + L.rows);
    uint32_t* part = (uint32_t*)(b + L.part);
    uint32_t* ctot = (uint32_t*)(b + L.ctot);
    uint32_t* bin_start = (uint32_t*)(b + L.bin_start);
    int4* img = (int4*)(b + L.img);
    uint16_t* lrow = (uint16_t*)(b + L.lrow);
    uint2* runs = (uint2*)(b + L.runs);
    uint16_t* ipos = (uint16_t*)(b + L.ipos);
    uint32_t* tcold = (uint32_t*)(b + L.tcold);
    int64_t* r_ret = (int64_t*)(b + L.r_ret);
    uint8_t* r_conf = (uint8_t*)(b + L.r_conf);
    ApHot* hot = (ApHot*)(b + L.hot);

    if (const hipError_t er = launch_epoch_next(t, nullptr, stream); er != hipSuccess) return er;
    if (C < m) {
        const uint64_t blocks = (m + 255) / 256;
        k_ap_preinsert<<<(unsigned)(blocks > 8192 ? 8192 : blocks), 256, 0, stream>>>(t, op, key,
                                                                                     m, err);
    }
    // scratch for the r_conf writes when the caller wants no conf: still written (cheap)
    for (uint64_t c0 = 0; c0 < m; c0 += C) {
        const uint32_t n = (uint32_t)(m - c0 < C ? m - c0 : C);
        const ApGeo g = geo_for(t, n);
        const uint32_t tab = gtab_for(n);
        if (hot_min) {
            k_ap_sclear<<<kSampGrid, 256, 0, stream>>>(gk, gc, tab);
            k_ap_sample<<<kSampGrid, 256, 0, stream>>>(key + c0, n, hot_min, gk, gc, tab);
        }
        k_ap_select<<<1, kTT, 0, stream>>>(t, gk, gc, hot_min, tab, hot);
        k_ap_scatter<<<kScatterGrid, kTT, 0, stream>>>(g, op + c0, key + c0, val + c0, n, rows,
                                                       lrow, hot, img, ipos, tcold);
        k_ap_scan_part<<<g.ng, 256, 0, stream>>>(g, rows, part, hot);
        k_ap_scan_top<<<(g.rowlen + kTopCols - 1) / kTopCols, kTT, 0, stream>>>(g, part, ctot, hot);
        k_ap_scan_bins<<<1, kTT, 0, stream>>>(g, ctot, bin_start);
        k_ap_scan_rows<<<g.ng, 256, 0, stream>>>(g, rows, part, bin_start, hot);
        k_ap_runs<<<dim3((g.tiles + kRunT - 1) / kRunT, (g.nbin + kRunB - 1) / kRunB), 256, 0,
                    stream>>>(g, rows, lrow, runs);
        const uint32_t spare = MPX_RES_IMG ? g.tiles * (uint32_t)kTL : (uint32_t)C;
        k_ap_resolve_list<<<g.nbin, kLT, 0, stream>>>(g, t, bin_start, runs, img, r_ret, r_conf,
                                                      spare, hot, err);
        k_ap_hot_commit<<<1, kHMax, 0, stream>>>(t, val + c0, hot, err);
        k_ap_emit<<<g.tiles, kTT, 0, stream>>>(g, op + c0, val + c0, n, ipos, tcold, r_ret, r_conf, rows,
                                               bin_start, hot, ret + c0, conf ? conf + c0 : nullptr);
    }
    return hipGetLastError();
}

}  // namespace mpx
