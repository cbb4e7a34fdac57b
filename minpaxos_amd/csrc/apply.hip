// apply.hip — the engine's device KV table (clear / import / export), the sort-based apply
// pipeline used for tables past apply_fast.hip's bin limit and small calls (and as its A/B
// reference, mpx_config.apply_path = MPX_APPLY_SORTED), the dispatcher of mpx_apply, and
// state.ConflictBatch (A5/A6).
//
// Reference: (*state.Command).Execute  src/state/state.go:77-103, applied in log order by
// executeCommands  src/bareminpaxos/bareminpaxos.go:1066-1098; state.Conflict state.go:53-60;
// state.ConflictBatch state.go:62-71.
//
// Sequential semantics restated per key: for command i on key k,
//   ret[i]  = PUT: val[i]; GET: val of the last PUT on k before i in this call, else the
//             table value at call start if k is present, else NIL (0); other ops: 0
//   conf[i] = Conflict(previous command on k in this call, command i)
//   table   : k <- val of the last PUT on k in this call
// Only keys that are PUT in this call or already present can change any output, so:
//   0. k_epoch_next       a new call epoch (device counter, so captured graphs stay correct)
//   1. k_kv_insert_puts   insert every PUT key of the whole call (one 64-bit CAS per probe; the
//                         key INT64_MIN is kept in a side slot so the table needs no key state)
// then the log is cut into chunks of C commands, processed in order; per chunk:
//   2. k_kv_lookup        sort key (slot << 32 | j << 2 | op class) of every command j of the
//                         chunk (absent, never-PUT keys: ret 0, conf 0 now, sorted last)
//   1+2 in a one-chunk call (the default): k_kv_index writes every sort key in one pass (PUTs
//                         insert, the other commands probe concurrently), k_kv_reprobe redoes the
//                         probes that missed once every insert is done
//   3. radix sort on the slot bits - stable, so log order within a slot; the op class rides in
//                         the key's low bits
//   4-5. segmented inclusive max-scan by slot of (q if PUT else -1) -> last PUT at or before q
//                         in its slot; its items are computed from the sorted keys as the scan
//                         reads them, so nothing but the scan's output is materialised
//   6. k_apply_finish     a 32-bit result code per command (conf bit + where its ret comes
//                         from); a slot's first command in the chunk takes its predecessor
//                         from the table's per-slot state word (epoch-tagged)
//   7. radix sort of (command index, code) pairs on the index bits above the low 12: the codes
//                         back in log order up to blocks of 4096 commands
//   8. k_apply_emit       per block of 4096: places the codes by the low index bits in LDS, then
//                         log order ret / conf; a GET's value is gathered from val[] or the table
//   9. k_apply_commit     the last command of each slot in the chunk updates value + state
// Random access is the cost driver (a uniform key stream is a random permutation of the log):
// a command-indexed scatter of results costs HBM a read-modify-write per partial line, so the
// results travel back by a second radix sort instead; what stays random is one table probe per
// command (2), one per PUT (1) and one value gather per GET (8), all reads. Chunks only bound
// the scratch memory.
// Steps 3, 5 and 7 use the engine's own device primitives (radix.hpp: stable LSD radix sort;
// scan.hpp: the segmented max-scan as a scan of (slot, position) pairs).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "kvtab.hpp"
#include "radix.hpp"
#include "scan.hpp"

namespace mpx {

// op class carried in the low 2 bits of a sort key
constexpr uint32_t kClsOther = 0, kClsPut = 1, kClsGet = 2;

__global__ void k_kv_fill(KvTable t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= t.cap; s += stride) {
        t.keys[s] = kSentinel;
        t.state[s] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *t.n_present = 0;
        t.epoch[1] = 0;  // k_epoch_next's completion counter (a stale count after a fault)
    }
}

// A new call epoch in one launch: epoch[0] = the current call epoch; when it would reach
// kEpochMax every slot's tag is cleared and it restarts at 1. Every block reads the old epoch
// before it counts itself done in epoch[1] (0 between calls); the last block to finish writes the
// new one, so no block can see it early. Also zeroes the call's miss counter (k_kv_index).
__global__ void k_epoch_next(KvTable t, uint32_t* n_miss) {
    if (n_miss && blockIdx.x == 0 && threadIdx.x == 0) *n_miss = 0;
    const uint32_t e0 = t.epoch[0];
    const bool wrap = e0 + 1 >= kEpochMax;
    if (wrap) {
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= t.cap; s += stride)
            t.state[s] &= kPresent;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&t.epoch[1], 1u) == gridDim.x - 1) {
            atomicExch(&t.epoch[1], 0u);
            atomicExch(&t.epoch[0], wrap ? 1u : e0 + 1);
        }
    }
}

hipError_t launch_epoch_next(KvTable& t, uint32_t* n_miss, hipStream_t stream) {
    // few blocks: their completion atomics on one word serialise (1024 blocks cost ~15 us per
    // call); the sweep they share runs once per 2^30 calls
    k_epoch_next<<<32, 256, 0, stream>>>(t, n_miss);
    return hipGetLastError();
}

hipError_t launch_kv_clear(KvTable& t, hipStream_t stream) {
    k_kv_fill<<<1024, 256, 0, stream>>>(t);
    return hipGetLastError();
}

__global__ void k_kv_import_insert(KvTable t, const int64_t* __restrict__ keys, uint64_t n,
                                   uint32_t* err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) kv_insert(t, keys[i], err);
}

__global__ void k_kv_import_set(KvTable t, const int64_t* __restrict__ keys,
                                const int64_t* __restrict__ vals, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t s = kv_lookup(t, keys[i]);
    if (s < 0) return;
    t.vals[s] = vals[i];
    if ((atomicOr(&t.state[s], kPresent) & kPresent) == 0u) atomicAdd(t.n_present, 1ull);
}

hipError_t launch_kv_import(KvTable& t, const int64_t* keys, const int64_t* vals, uint64_t n,
                            uint32_t* err, hipStream_t stream) {
    if (!n) return hipSuccess;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    k_kv_import_insert<<<blocks, 256, 0, stream>>>(t, keys, n, err);
    k_kv_import_set<<<blocks, 256, 0, stream>>>(t, keys, vals, n);
    return hipGetLastError();
}

__global__ void k_kv_export(KvTable t, int64_t* __restrict__ keys, int64_t* __restrict__ vals,
                            uint64_t cap_out, unsigned long long* counter) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= t.cap; s += stride) {
        if (t.state[s] & kPresent) {
            const unsigned long long pos = atomicAdd(counter, 1ull);
            if (pos < cap_out) {
                keys[pos] = s == t.cap ? kSentinel : t.keys[s];
                vals[pos] = t.vals[s];
            }
        }
    }
}

__global__ void k_zero_u64(unsigned long long* p) { *p = 0; }

hipError_t launch_kv_export(KvTable& t, int64_t* keys, int64_t* vals, uint64_t cap,
                            unsigned long long* counter, hipStream_t stream) {
    k_zero_u64<<<1, 1, 0, stream>>>(counter);
    k_kv_export<<<1024, 256, 0, stream>>>(t, keys, vals, cap, counter);
    return hipGetLastError();
}

// ---- the apply pipeline -------------------------------------------------------------------
// multi-chunk calls: insert every PUT key of the whole call before any chunk is looked up
__global__ __launch_bounds__(256) void k_kv_insert_puts(KvTable t, const uint8_t* __restrict__ op,
                                                        const int64_t* __restrict__ key,
                                                        uint64_t m, uint32_t* err) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride)
        if (op[i] == MPX_OP_PUT) kv_insert(t, key[i], err);
}

__device__ __forceinline__ uint32_t op_class(uint8_t o) {
    return o == MPX_OP_PUT ? kClsPut : (o == MPX_OP_GET ? kClsGet : kClsOther);
}

// probes while other lanes insert read the key words with plain (L2-cached) loads: a slot's key
// changes at most once per call (empty -> key), so a key read is final and only "empty" can be
// stale - an insert then claims the slot with the CAS (which returns the true word), a probe's
// miss is re-probed by k_kv_reprobe after the pass. MPX_INDEX_PLAIN=0: relaxed agent-scope
// atomic loads instead (they bypass the XCD's L2).
#ifndef MPX_INDEX_PLAIN
#define MPX_INDEX_PLAIN 0
#endif
__device__ __forceinline__ unsigned long long probe_load(const int64_t* p) {
#if MPX_INDEX_PLAIN
    return (unsigned long long)*p;
#else
    return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
#endif
}
// the two probe loops resumed at slot s whose key `cur` was already loaded (k_kv_index issues
// the first probe of several commands together)
// (probes stay inside the key's 256-slot bucket, kvtab.hpp)
__device__ __forceinline__ uint64_t next_in_bucket(uint64_t s) {
    return (s & ~(uint64_t)(kSB - 1)) | ((s + 1) & (kSB - 1));
}
__device__ __forceinline__ uint64_t first_slot(const KvTable& t, int64_t key) {
    const uint64_t h = hash64((uint64_t)key);
    return ((uint64_t)bucket_of(h, t.lgnb) << kLgSB) | home_of(h);
}
__device__ __forceinline__ int64_t kv_insert_from(const KvTable& t, int64_t key, uint64_t s,
                                                  unsigned long long cur, uint32_t* err) {
    for (int probe = 0; probe < kSB; ++probe) {
        unsigned long long* slot = reinterpret_cast<unsigned long long*>(t.keys + s);
        if (probe) cur = probe_load(t.keys + s);
        if (cur == (unsigned long long)kSentinel) {
            cur = atomicCAS(slot, (unsigned long long)kSentinel, (unsigned long long)key);
            if (cur == (unsigned long long)kSentinel) return (int64_t)s;  // claimed
        }
        if ((int64_t)cur == key) return (int64_t)s;
        s = next_in_bucket(s);
    }
    raise_err(err, kErrKvFull);
    return -1;
}

__device__ __forceinline__ int64_t kv_probe_racy_from(const KvTable& t, int64_t key, uint64_t s,
                                                      unsigned long long cur) {
    for (int probe = 0; probe < kSB; ++probe) {
        if (probe) cur = probe_load(t.keys + s);
        if ((int64_t)cur == key) return (int64_t)s;
        if ((int64_t)cur == kSentinel) return -1;
        s = next_in_bucket(s);
    }
    return -1;
}

// one-chunk calls: the sort key of every command in one pass, so every lane probes (the split
// insert / lookup passes left half the lanes of each wave idle). PUTs insert; the others probe
// concurrently and append a miss to `miss` (one counter atomic per wave). Each lane takes
// kIndexUnroll commands per round and issues their first probes together.
#ifndef MPX_INDEX_UNROLL
#define MPX_INDEX_UNROLL 2
#endif
constexpr int kIndexUnroll = MPX_INDEX_UNROLL;
__global__ __launch_bounds__(256) void k_kv_index(KvTable t, const uint8_t* __restrict__ op,
                                                  const int64_t* __restrict__ key, uint64_t m,
                                                  uint32_t* err, uint64_t* __restrict__ skey,
                                                  uint32_t* __restrict__ miss,
                                                  uint32_t* __restrict__ n_miss) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * kIndexUnroll;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x * kIndexUnroll; i0 < m; i0 += stride) {
        uint8_t o[kIndexUnroll];
        int64_t k[kIndexUnroll];
        uint64_t h[kIndexUnroll];
        unsigned long long cur[kIndexUnroll];
#pragma unroll
        for (int u = 0; u < kIndexUnroll; ++u) {
            const uint64_t i = i0 + (uint64_t)u * blockDim.x + threadIdx.x;
            o[u] = i < m ? op[i] : 0;
            k[u] = i < m ? key[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < kIndexUnroll; ++u) {
            const uint64_t i = i0 + (uint64_t)u * blockDim.x + threadIdx.x;
            h[u] = first_slot(t, k[u]);
            cur[u] = i < m && k[u] != kSentinel ? probe_load(t.keys + h[u]) : 0ull;
        }
#pragma unroll
        for (int u = 0; u < kIndexUnroll; ++u) {
            const uint64_t i = i0 + (uint64_t)u * blockDim.x + threadIdx.x;
            bool missed = false;
            if (i < m) {
                int64_t s;
                if (k[u] == kSentinel) {
                    s = (int64_t)t.cap;  // side slot
                } else if (o[u] == MPX_OP_PUT) {
                    s = kv_insert_from(t, k[u], h[u], cur[u], err);
                    if (s < 0) s = (int64_t)t.cap + 1;  // full table: the call fails
                } else {
                    s = kv_probe_racy_from(t, k[u], h[u], cur[u]);
                    missed = s < 0;
                }
                if (!missed) skey[i] = ((uint64_t)s << 32) | (i << 2) | op_class(o[u]);
            }
            const uint64_t bal = __ballot(missed);
            if (bal) {
                uint32_t base = 0;
                if (lane_id() == 0) base = atomicAdd(n_miss, (uint32_t)__popcll(bal));
                base = __shfl(base, 0);
                if (missed) miss[base + __popcll(bal & ((1ull << lane_id()) - 1))] = (uint32_t)i;
            }
        }
    }
}

// after every insert of the call: the missed probes again (an absent key that no PUT of the
// call inserted gets slot cap+1: its outputs are zero)
__global__ __launch_bounds__(256) void k_kv_reprobe(KvTable t, const uint8_t* __restrict__ op,
                                                    const int64_t* __restrict__ key,
                                                    const uint32_t* __restrict__ miss,
                                                    const uint32_t* __restrict__ n_miss,
                                                    uint64_t* __restrict__ skey) {
    const uint32_t n = *n_miss;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += stride) {
        const uint64_t j = miss[x];
        const int64_t s = kv_lookup(t, key[j]);
        const uint64_t sl = s < 0 ? t.cap + 1 : (uint64_t)s;
        skey[j] = (sl << 32) | (j << 2) | op_class(op[j]);
    }
}

// sort key of chunk command j: slot << 32 | j << 2 | class; an absent key that is never PUT in
// this call gets slot cap+1 (sorts last; its outputs are zero: GET -> NIL, and no conflict since
// nothing before or after it on that key in this call is a PUT)
__global__ __launch_bounds__(256) void k_kv_lookup(KvTable t, const uint8_t* __restrict__ op,
                                                   const int64_t* __restrict__ key, uint64_t n,
                                                   uint64_t* __restrict__ skey) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        const uint8_t o = op[j];
        const int64_t s = kv_lookup(t, key[j]);
        const uint64_t sl = s < 0 ? t.cap + 1 : (uint64_t)s;
        skey[j] = (sl << 32) | (j << 2) | op_class(o);
    }
}

__device__ __forceinline__ uint32_t sk_index(uint64_t k) { return (uint32_t)k >> 2; }
__device__ __forceinline__ uint32_t sk_class(uint64_t k) { return (uint32_t)k & 3u; }

// the segmented max-scan reads its keys (slots) and values (own position if PUT, else -1)
// straight from the sorted keys: no materialised slot / position arrays. Its items are
// (slot, value) pairs; combining an earlier a with a later b keeps b's slot and takes the max
// only within one slot (associative over slot-sorted items, scan.hpp's contract)
__device__ __forceinline__ uint32_t sk_slot(uint64_t k) { return (uint32_t)(k >> 32); }
struct SlotPos {
    uint32_t slot;
    int32_t pos;
};
struct SegMax {
    static constexpr bool kCommutes = false;  // segmented: order matters
    __device__ __forceinline__ SlotPos operator()(SlotPos a, SlotPos b) const {
        return SlotPos{b.slot, a.slot == b.slot && a.pos > b.pos ? a.pos : b.pos};
    }
};
struct PutPosIn {
    const uint64_t* skey;
    __device__ __forceinline__ SlotPos operator()(uint64_t q) const {
        const uint64_t k = skey[q];
        return SlotPos{sk_slot(k), ((uint32_t)k & 3u) == kClsPut ? (int32_t)q : -1};
    }
};
struct LastPutOut {  // lps[q] = the last PUT at or before q in its slot (inclusive)
    int32_t* lps;
    __device__ __forceinline__ void operator()(uint64_t q, SlotPos ex, SlotPos x) const {
        lps[q] = SegMax{}(ex, x).pos;
    }
};

// per sorted position q: the command's chunk index and a 32-bit result code
//   bit 31 conf | bits 29-30 kind | bits 0-28 payload
//   kind 0: ret 0 (other ops, GET of an absent key); 1: ret = own val (PUT);
//   2: ret = val of chunk command `payload` (the last PUT before it in this chunk);
//   3: ret = table value of slot `payload` at chunk start (no PUT before it in this chunk)
// The codes are sorted back to log order (k_apply_emit reads them sequentially), so no
// command-indexed store is ever scattered: a random partial-line store costs HBM a
// read-modify-write, a radix pass over 8 bytes does not.
constexpr uint32_t kCodeConf = 1u << 31;
constexpr uint32_t kKindShift = 29;
constexpr uint32_t kPayloadMask = (1u << kKindShift) - 1u;
constexpr uint32_t kKindZero = 0, kKindOwn = 1, kKindLog = 2, kKindTable = 3;

// kUnroll positions per lane per round, loads of a round issued together (memory-level
// parallelism: each round's loads are one dependent chain per lane otherwise)
constexpr int kUnroll = 4;

__global__ __launch_bounds__(256) void k_apply_finish(KvTable t, const uint64_t* __restrict__ skey,
                                                      const int32_t* __restrict__ lps, uint64_t n,
                                                      uint32_t* __restrict__ jkey,
                                                      uint32_t* __restrict__ code) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * kUnroll;
    const uint32_t none = (uint32_t)(t.cap + 1);
    const uint32_t ep = t.epoch[0];
    for (uint64_t q0 = (uint64_t)blockIdx.x * blockDim.x * kUnroll + threadIdx.x; q0 < n;
         q0 += stride) {
        uint64_t k[kUnroll], kp[kUnroll], kq[kUnroll];
        int32_t pp[kUnroll];
        uint32_t st[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {  // round 1: the sorted neighbours
            const uint64_t q = q0 + (uint64_t)u * blockDim.x;
            const bool in = q < n;
            k[u] = in ? skey[q] : ~0ull;
            kp[u] = in && q > 0 ? skey[q - 1] : ~0ull;
            pp[u] = in && q > 0 ? lps[q - 1] : -1;
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {  // round 2: slot state word, last PUT's key
            const uint32_t sl = sk_slot(k[u]);
            const bool live = k[u] != ~0ull && sl != none;
            const bool in_chunk = live && sk_slot(kp[u]) == sl;
            if (!in_chunk) pp[u] = -1;  // last PUT strictly before q, within the slot's run
            const bool get = sk_class(k[u]) == kClsGet;
            st[u] = live && (!in_chunk || (get && pp[u] < 0)) ? t.state[sl] : 0u;
            kq[u] = live && get && pp[u] >= 0 ? skey[pp[u]] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint64_t q = q0 + (uint64_t)u * blockDim.x;
            if (q >= n) continue;
            const uint32_t sl = sk_slot(k[u]);
            jkey[q] = sk_index(k[u]);
            if (sl == none) {
                code[q] = 0;
                continue;
            }
            const uint32_t c = sk_class(k[u]);
            const bool in_chunk = q > 0 && sk_slot(kp[u]) == sl;
            const bool prev = in_chunk || (st[u] >> 2) == ep;
            const bool prev_put = in_chunk ? sk_class(kp[u]) == kClsPut : prev && (st[u] & kLastPut);
            uint32_t x = kKindZero << kKindShift;
            if (c == kClsPut) x = kKindOwn << kKindShift;
            else if (c == kClsGet && pp[u] >= 0) x = (kKindLog << kKindShift) | sk_index(kq[u]);
            else if (c == kClsGet && (st[u] & kPresent)) x = (kKindTable << kKindShift) | sl;
            code[q] = x | (prev && (prev_put || c == kClsPut) ? kCodeConf : 0u);
        }
    }
}

// log order: the caller's ret / conf from the sorted-back codes (before the chunk commits, so
// kind 3 still reads the chunk-start table value). The back-sort only orders by j >> kEmitBits:
// block g receives exactly the kEmitGroup codes of commands [g * kEmitGroup, (g+1) * kEmitGroup)
// in some order and places them by j's low bits in LDS (saves two of the four radix passes).
constexpr int kEmitBits = 12;
constexpr int kEmitGroup = 1 << kEmitBits;
__global__ __launch_bounds__(256) void k_apply_emit(KvTable t, const uint32_t* __restrict__ jkey,
                                                    const uint32_t* __restrict__ code, uint64_t n,
                                                    const int64_t* __restrict__ val,
                                                    int64_t* __restrict__ ret,
                                                    uint8_t* __restrict__ conf) {
    __shared__ uint32_t lc[kEmitGroup];
    const uint64_t g0 = (uint64_t)blockIdx.x * kEmitGroup;
    const uint32_t cnt = (uint32_t)(n - g0 < (uint64_t)kEmitGroup ? n - g0 : kEmitGroup);
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x)
        lc[jkey[g0 + i] & (kEmitGroup - 1)] = code[g0 + i];
    __syncthreads();
    // kEmitUnroll commands per lane per round: their (random) value gathers are all issued
    // before the first store, so each lane keeps several loads in flight
    constexpr int kEmitUnroll = 4;
    for (uint32_t i0 = threadIdx.x; i0 < cnt; i0 += kEmitUnroll * blockDim.x) {
        uint32_t x[kEmitUnroll];
        int64_t r[kEmitUnroll];
#pragma unroll
        for (int u = 0; u < kEmitUnroll; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            x[u] = i < cnt ? lc[i] : 0u;
            const uint32_t kind = (x[u] >> kKindShift) & 3u, p = x[u] & kPayloadMask;
            const int64_t* src = kind == kKindOwn ? val + g0 + i
                                 : kind == kKindLog ? val + p
                                 : kind == kKindTable ? t.vals + p
                                 : nullptr;
            r[u] = src ? *src : 0;
        }
#pragma unroll
        for (int u = 0; u < kEmitUnroll; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            if (i < cnt) {
                ret[g0 + i] = r[u];
                if (conf) conf[g0 + i] = (uint8_t)(x[u] >> 31);
            }
        }
    }
}

// the last command of every slot in the chunk writes the slot's value (if the chunk PUT it) and
// its state word, after every read of the chunk-start state is done (previous kernels)
__global__ __launch_bounds__(256) void k_apply_commit(KvTable t, const uint64_t* __restrict__ skey,
                                                      const int32_t* __restrict__ lps, uint64_t n,
                                                      const int64_t* __restrict__ val) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * kUnroll;
    const uint32_t none = (uint32_t)(t.cap + 1);
    const uint32_t ep = t.epoch[0];
    unsigned long long added = 0;
    for (uint64_t q0 = (uint64_t)blockIdx.x * blockDim.x * kUnroll + threadIdx.x; q0 < n;
         q0 += stride) {
        uint64_t k[kUnroll], kq[kUnroll];
        int32_t pp[kUnroll];
        bool last[kUnroll];
        uint32_t old[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {  // round 1: is q its slot's last command?
            const uint64_t q = q0 + (uint64_t)u * blockDim.x;
            k[u] = q < n ? skey[q] : 0ull;
            const uint64_t kn = q + 1 < n ? skey[q + 1] : ~0ull;
            last[u] = q < n && sk_slot(k[u]) != none && sk_slot(kn) != sk_slot(k[u]);
            pp[u] = last[u] ? lps[q] : -1;
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {  // round 2: old state, last PUT's key
            old[u] = last[u] ? t.state[sk_slot(k[u])] : 0u;
            kq[u] = pp[u] >= 0 ? skey[pp[u]] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            if (!last[u]) continue;
            const uint32_t sl = sk_slot(k[u]);
            uint32_t present = old[u] & kPresent;
            if (pp[u] >= 0) {
                t.vals[sl] = val[sk_index(kq[u])];
                added += present ? 0 : 1;
                present = kPresent;
            }
            t.state[sl] = (ep << 2) | (sk_class(k[u]) == kClsPut ? kLastPut : 0u) | present;
        }
    }
    // one counter atomic per wave
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) added += __shfl_xor(added, d);
    if (lane_id() == 0 && added) atomicAdd(t.n_present, added);
}

namespace {
struct WorkLayout {
    uint64_t skey_a, skey_b, lps, jkey, code, jkey_b, code_b, n_miss, tmp, tmp_bytes, total;
};
WorkLayout layout(uint64_t m) {
    const uint64_t sort_tmp = radix_scratch_bytes<uint64_t, RsNoValue>(m);
    const uint64_t scan_tmp = scan_scratch_bytes<SlotPos>(m);
    const uint64_t back_tmp = radix_scratch_bytes<uint32_t, uint32_t>(m);
    uint64_t t = sort_tmp > scan_tmp ? sort_tmp : scan_tmp;
    t = t > back_tmp ? t : back_tmp;
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    WorkLayout w;
    uint64_t o = 0;
    w.skey_a = o; o += al(m * 8);
    w.skey_b = o; o += al(m * 8);
    w.lps = o; o += al(m * 4);
    w.jkey = o; o += al(m * 4);
    w.code = o; o += al(m * 4);
    w.jkey_b = o; o += al(m * 4);
    w.code_b = o; o += al(m * 4);
    w.n_miss = o; o += al(4);
    w.tmp_bytes = al(t);
    w.tmp = o; o += w.tmp_bytes;
    w.total = o;
    return w;
}

unsigned grid_for(uint64_t n) {
    uint64_t b = (n + 255) / 256;
    return (unsigned)(b > 8192 ? 8192 : (b ? b : 1));
}

unsigned bits_for(uint64_t x) {  // bits to represent every value < x
    unsigned b = 1;
    while ((1ull << b) < x) ++b;
    return b;
}
}  // namespace

uint64_t apply_chunk_commands(uint64_t chunk, uint64_t m) {
    const uint64_t c = chunk ? chunk : kApplyChunkDefault;
    return m < c ? (m ? m : 1) : c;
}

namespace {
// Which pipeline runs a call of m commands (the handle's ApplyOpts). The partitioned pipeline has
// a fixed cost of about a dozen dependent launches plus a pass over every bin that received
// records, so AUTO sends calls below fast_min commands (default kFastMinDefault, the measured
// crossover) to the sort-based one. SORTED / PARTITIONED force a pipeline at any size (the
// partitioned one where the table geometry allows it). All give identical results.
constexpr uint64_t kFastMinDefault = 16384;
uint64_t fast_min(const KvTable& t, const ApplyOpts& o) {  // partitioned from this many commands
    if (!apply_fast_ok(t) || o.path == MPX_APPLY_SORTED) return UINT64_MAX;
    if (o.path == MPX_APPLY_PARTITIONED) return 0;
    return o.fast_min ? o.fast_min : kFastMinDefault;
}
bool use_fast(const KvTable& t, const ApplyOpts& o, uint64_t m) { return m >= fast_min(t, o); }
// calls of at most MPX_APPLY_SMALL_MAX commands run the one-launch kernel (apply_small.hip)
// unless a multi-launch pipeline is forced
bool use_small(const ApplyOpts& o, uint64_t m) {
    return m <= MPX_APPLY_SMALL_MAX && (o.path == MPX_APPLY_AUTO || o.path == MPX_APPLY_SMALL);
}
uint32_t hot_min(const ApplyOpts& o) {  // sample count (of 64K) that makes a key hot; 0 = none
    return o.hot_min == MPX_APPLY_NO_HOT ? 0u : (o.hot_min ? o.hot_min : 5u);
}
}  // namespace

bool apply_is_one_launch(const ApplyOpts& o, uint64_t m) { return m && use_small(o, m); }

uint64_t apply_work_bytes(const KvTable& t, const ApplyOpts& o, uint64_t m) {
    if (use_small(o, m)) return 0;
    const uint64_t C = apply_chunk_commands(o.chunk, m);
    return use_fast(t, o, m) ? apply_fast_work_bytes(t, C) : layout(C).total;
}

// Every m <= max_m must fit: each pipeline's need grows with m, so the largest call on either
// side of the size switch bounds them all.
uint64_t apply_reserve_bytes(const KvTable& t, const ApplyOpts& o, uint64_t max_m) {
    uint64_t b = apply_work_bytes(t, o, max_m);
    const uint64_t thr = fast_min(t, o);
    if (thr > 1 && thr <= max_m) b = std::max(b, apply_work_bytes(t, o, thr - 1));
    const uint64_t small_end = MPX_APPLY_SMALL_MAX;  // the first size past the small kernel
    if (use_small(o, small_end) && small_end < max_m)
        b = std::max(b, apply_work_bytes(t, o, small_end + 1));
    return b;
}

hipError_t launch_apply(KvTable& t, const uint8_t* op, const int64_t* key, const int64_t* val,
                        uint64_t m, int64_t* ret, uint8_t* conf, const ApplyOpts& o, ApplyWork& w,
                        uint32_t* err, hipStream_t stream) {
    if (!m) return hipSuccess;
    if (use_small(o, m)) return launch_apply_small(t, op, key, val, m, ret, conf, err, stream);
    const uint64_t C = apply_chunk_commands(o.chunk, m);
    if (use_fast(t, o, m))
        return launch_apply_fast(t, op, key, val, m, ret, conf, C, w, hot_min(o), err, stream);
    // result codes carry a chunk index or a slot in 29 bits
    if (C > kPayloadMask || t.cap + 1 > kPayloadMask) return hipErrorInvalidValue;
    const WorkLayout L = layout(C);
    if (w.bytes < L.total) return hipErrorInvalidValue;
    char* b = (char*)w.base;
    uint64_t* skey_a = (uint64_t*)(b + L.skey_a);
    uint64_t* skey_b = (uint64_t*)(b + L.skey_b);
    int32_t* lps = (int32_t*)(b + L.lps);
    uint32_t* jkey = (uint32_t*)(b + L.jkey);
    uint32_t* code = (uint32_t*)(b + L.code);
    uint32_t* jkey_b = (uint32_t*)(b + L.jkey_b);
    uint32_t* code_b = (uint32_t*)(b + L.code_b);
    void* tmp = b + L.tmp;
    const unsigned slot_bits = bits_for(t.cap + 2);

    uint32_t* n_miss = (uint32_t*)(b + L.n_miss);
    if (const hipError_t er = launch_epoch_next(t, n_miss, stream); er != hipSuccess) return er;
    // one chunk: one pass writes every sort key (PUTs insert, the rest probe; misses re-probed
    // after the pass, through lps as the miss list - lps is not live until the scan)
    const bool one = C >= m;
    if (one) {
        k_kv_index<<<grid_for(m), 256, 0, stream>>>(t, op, key, m, err, skey_a, (uint32_t*)lps,
                                                    n_miss);
        k_kv_reprobe<<<grid_for(m), 256, 0, stream>>>(t, op, key, (const uint32_t*)lps, n_miss,
                                                      skey_a);
    } else {
        k_kv_insert_puts<<<grid_for(m), 256, 0, stream>>>(t, op, key, m, err);
    }
    for (uint64_t c0 = 0; c0 < m; c0 += C) {
        const uint64_t n = m - c0 < C ? m - c0 : C;
        const unsigned g = grid_for(n);
        if (!one)
            k_kv_lookup<<<g, 256, 0, stream>>>(t, op + c0, key + c0, n, skey_a);
        hipError_t r = radix_sort<uint64_t, RsNoValue>(skey_a, skey_b, nullptr, nullptr, n, 32u,
                                                       32u + slot_bits, tmp, L.tmp_bytes, stream);
        if (r != hipSuccess) return r;
        r = device_scan(PutPosIn{skey_b}, LastPutOut{lps}, n, SegMax{},
                        SlotPos{0xFFFFFFFFu, -1}, (SlotPos*)tmp, stream);
        if (r != hipSuccess) return r;
        k_apply_finish<<<g, 256, 0, stream>>>(t, skey_b, lps, n, jkey, code);
        const unsigned jb = bits_for(n);
        const uint32_t *jk = jkey, *cd = code;  // one emit group: LDS placement alone suffices
        if (jb > (unsigned)kEmitBits) {
            r = radix_sort<uint32_t, uint32_t>(jkey, jkey_b, code, code_b, n, (unsigned)kEmitBits,
                                               jb, tmp, L.tmp_bytes, stream);
            if (r != hipSuccess) return r;
            jk = jkey_b;
            cd = code_b;
        }
        const unsigned eg = (unsigned)((n + kEmitGroup - 1) / kEmitGroup);
        k_apply_emit<<<eg, 256, 0, stream>>>(t, jk, cd, n, val + c0, ret + c0,
                                             conf ? conf + c0 : nullptr);
        k_apply_commit<<<g, 256, 0, stream>>>(t, skey_b, lps, n, val + c0);
    }
    return hipGetLastError();
}

// ---- state.ConflictBatch over consecutive instances ------------------------------------------
// ConflictBatch(b1, b2) (state.go:62-71) = some pair (c1 in b1, c2 in b2) with the same key and a
// PUT among the two. A workgroup takes 256 consecutive pairs, i.e. one contiguous command range.
// Its 258 offsets are read once (one coalesced load, into LDS); when the range fits kStage
// commands its keys are staged in LDS by 16-byte loads and its op bytes by 16-byte loads (every
// load of the tile issued before the first LDS write; the loads start at the 16-byte boundary at
// or below the range, the bytes before it are never read back). A lane then takes one pair when
// both instances have at most kSmall commands (MAX_BATCH-sized instances are rare) and tests all
// |b1| x |b2| products in registers. The wave then takes its larger pairs one at a time, lanes
// striding over the products with an early exit on the first hit.
// (4: the products of two 4-command instances in registers take 16 key registers, not 32, and
// the kernel runs at higher occupancy; pairs with more commands take the wave path)
#ifndef MPX_CONF_SMALL
#define MPX_CONF_SMALL 4
#endif
constexpr int kSmall = MPX_CONF_SMALL;
constexpr int kConfBlock = 256;
#ifndef MPX_CONF_STAGE
#define MPX_CONF_STAGE 1534
#endif
constexpr int kStage = MPX_CONF_STAGE;  // staged commands: 12 KB of keys with the slack, 8 workgroups per CU
constexpr int kStageKV = (kStage + 2) / 2;  // 16-byte key vectors: the range + one key of slack
constexpr int kStageOV = (kStage + 30) / 16;  // 16-byte op vectors: the range + 15 bytes of slack
constexpr int kKeyRounds = (kStageKV + kConfBlock - 1) / kConfBlock;

template <typename KeyAt, typename PutAt>
__device__ __forceinline__ bool small_pair(uint64_t a0, uint64_t na, uint64_t a1, uint64_t nb,
                                           KeyAt key_at, PutAt put_at) {
    int64_t ka[kSmall], kb[kSmall];
    uint32_t pa = 0, pb = 0;  // PUT bits
#pragma unroll
    for (int i = 0; i < kSmall; ++i) {
        const bool ia = (uint64_t)i < na, ib = (uint64_t)i < nb;
        ka[i] = ia ? key_at(a0 + i) : 0;
        kb[i] = ib ? key_at(a1 + i) : 0;
        pa |= (ia && put_at(a0 + i) ? 1u : 0u) << i;
        pb |= (ib && put_at(a1 + i) ? 1u : 0u) << i;
    }
    bool hit = false;
#pragma unroll
    for (int i = 0; i < kSmall; ++i)
#pragma unroll
        for (int j = 0; j < kSmall; ++j)
            hit |= (uint64_t)i < na && (uint64_t)j < nb && ka[i] == kb[j] &&
                   (((pa >> i) | (pb >> j)) & 1u);
    return hit;
}

// small_pair over the LDS-staged range: the low key halves compared first, the high halves read
// only for the (rare) pairs whose low halves meet
__device__ __forceinline__ bool small_pair_lds(uint32_t a0, uint64_t na, uint32_t a1, uint64_t nb,
                                               const uint32_t* slo, const uint32_t* shi,
                                               const uint8_t* so) {
    uint32_t ka[kSmall], kb[kSmall];
    uint32_t pa = 0, pb = 0;  // PUT bits
#pragma unroll
    for (int i = 0; i < kSmall; ++i) {
        const bool ia = (uint64_t)i < na, ib = (uint64_t)i < nb;
        ka[i] = ia ? slo[a0 + i] : 0u;
        kb[i] = ib ? slo[a1 + i] : 0u;
        pa |= (ia && so[a0 + i] == MPX_OP_PUT ? 1u : 0u) << i;
        pb |= (ib && so[a1 + i] == MPX_OP_PUT ? 1u : 0u) << i;
    }
    uint32_t cand = 0;  // bit 4i + j: low halves equal and a PUT among the two
#pragma unroll
    for (int i = 0; i < kSmall; ++i)
#pragma unroll
        for (int j = 0; j < kSmall; ++j)
            cand |= ((uint64_t)i < na && (uint64_t)j < nb && ka[i] == kb[j] &&
                     (((pa >> i) | (pb >> j)) & 1u))
                        ? 1u << (kSmall * i + j)
                        : 0u;
    while (cand) {
        const int b = __builtin_ctz(cand);
        cand &= cand - 1;
        if (shi[a0 + b / kSmall] == shi[a1 + b % kSmall]) return true;
    }
    return false;
}

__global__ __launch_bounds__(kConfBlock) void k_conflict_batch(const uint8_t* __restrict__ op,
                                                               const int64_t* __restrict__ key,
                                                               const uint64_t* __restrict__ off,
                                                               uint64_t n_pairs,
                                                               uint8_t* __restrict__ out) {
    __shared__ uint64_t soff[kConfBlock + 2];
    // the keys as two 32-bit planes (a lane's instance lies ~4 keys past its neighbour's: 8-byte
    // reads would hit every 8th bank pair, 32-bit ones every 4th), the high halves read only on a
    // low-half match
    __shared__ uint2 slo2[kStageKV], shi2[kStageKV];
    __shared__ int4 so4[kStageOV];
    const uint64_t p0 = (uint64_t)blockIdx.x * kConfBlock;
    const int t = threadIdx.x;
    const uint32_t np = n_pairs - p0 < (uint64_t)kConfBlock ? (uint32_t)(n_pairs - p0)
                                                            : (uint32_t)kConfBlock;
    // off[p0 .. p0 + np + 1]: np + 2 entries
    {
        const bool x = t < 2 && kConfBlock + t < (int)np + 2;
        const uint64_t o = off[p0 + min((uint32_t)t, np + 1)];
        const uint64_t ox = x ? off[p0 + kConfBlock + t] : 0;
        if ((uint32_t)t < np + 2) soff[t] = o;
        if (x) soff[kConfBlock + t] = ox;
    }
    __syncthreads();
    const uint64_t c_lo = soff[0], c_hi = soff[np + 1];
    // vector bases at or below the range, 16-byte aligned (pointer arithmetic, so the loads
    // stay global ones): ksh keys / osh op bytes of slack before c_lo
    const uint32_t ksh = (uint32_t)(((uintptr_t)(key + c_lo) >> 3) & 1);
    const uint32_t osh = (uint32_t)((uintptr_t)(op + c_lo) & 15);
    const int4* kv = (const int4*)(key + c_lo - ksh);
    const int4* ov = (const int4*)(op + c_lo - osh);
    const uint64_t span = c_hi - c_lo;
    const bool staged = span <= (uint64_t)kStage;  // uniform over the workgroup
    static_assert(kKeyRounds == 3 || kKeyRounds == 4, "three or four key vectors per thread");
    if (staged) {
        const uint32_t nkv = (uint32_t)((span + ksh + 1) >> 1);
        const uint32_t nov = (uint32_t)((span + osh + 15) >> 4);
        if (nkv) {  // (clamped, unconditional loads: the tile's vectors all in flight at once)
            const uint32_t i0 = (uint32_t)t, i1 = i0 + kConfBlock, i2 = i1 + kConfBlock,
                           i3 = i2 + kConfBlock;
            const int4 k0 = kv[min(i0, nkv - 1)], k1 = kv[min(i1, nkv - 1)],
                       k2 = kv[min(i2, nkv - 1)],
                       k3 = kKeyRounds > 3 ? kv[min(i3, nkv - 1)] : make_int4(0, 0, 0, 0);
            const int4 o0 = ov[min(i0, nov - 1)];
            auto put = [&](uint32_t i, int4 x) {
                if (i < nkv) {
                    slo2[i] = make_uint2((uint32_t)x.x, (uint32_t)x.z);
                    shi2[i] = make_uint2((uint32_t)x.y, (uint32_t)x.w);
                }
            };
            put(i0, k0);
            put(i1, k1);
            put(i2, k2);
            if (kKeyRounds > 3) put(i3, k3);
            if (i0 < nov) so4[i0] = o0;
        }
        __syncthreads();
    }
    const bool live = (uint32_t)t < np;
    const uint64_t a0 = soff[t], a1 = soff[t + 1], b1 = soff[t + 2];
    const uint64_t na = a1 - a0, nb = b1 - a1;
    const bool small = live && na <= (uint64_t)kSmall && nb <= (uint64_t)kSmall;
    if (small) {
        bool hit;
        if (staged) {
            const uint32_t* slo = (const uint32_t*)slo2 + ksh;
            const uint32_t* shi = (const uint32_t*)shi2 + ksh;
            const uint8_t* so = (const uint8_t*)so4 + osh;
            hit = small_pair_lds(a0 - c_lo, na, a1 - c_lo, nb, slo, shi, so);
        } else {
            hit = small_pair(a0, na, a1, nb, [&](uint64_t i) { return key[i]; },
                             [&](uint64_t i) { return op[i] == MPX_OP_PUT; });
        }
        out[p0 + t] = hit ? 1 : 0;
    }
    // the wave's larger pairs, one at a time
    const int l = lane_id();
    unsigned long long big = __ballot(live && !small);
    while (big) {
        const int src = __ffsll((long long)big) - 1;
        big &= big - 1;
        const uint64_t x0 = (uint64_t)__shfl((long long)a0, src);
        const uint64_t x1 = (uint64_t)__shfl((long long)a1, src);
        const uint64_t y1 = (uint64_t)__shfl((long long)b1, src);
        const uint64_t xa = x1 - x0, xb = y1 - x1, tot = xa * xb;
        bool hit = false;
        for (uint64_t base = 0; base < tot; base += kWave) {
            const uint64_t x = base + l;
            bool h = false;
            if (x < tot) {
                const uint64_t i = x0 + x / xb, j = x1 + x % xb;
                h = key[i] == key[j] && (op[i] == MPX_OP_PUT || op[j] == MPX_OP_PUT);
            }
            if (__ballot(h)) {
                hit = true;
                break;
            }
        }
        if (l == src) out[p0 + t] = hit ? 1 : 0;
    }
}

hipError_t launch_conflict_batch(const uint8_t* op, const int64_t* key, const uint64_t* inst_off,
                                 uint64_t n_inst, uint8_t* out, hipStream_t stream) {
    if (n_inst < 2) return hipSuccess;
    const uint64_t pairs = n_inst - 1;
    k_conflict_batch<<<dim3((unsigned)((pairs + kConfBlock - 1) / kConfBlock)), kConfBlock, 0,
                       stream>>>(op, key, inst_off, pairs, out);
    return hipGetLastError();
}

}  // namespace mpx
