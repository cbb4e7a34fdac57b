// apply.hip — batched state-machine apply against the engine's device KV table (A5/A6).
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
//   1. k_kv_insert_puts   insert every PUT key (one 64-bit CAS per probe; the key value
//                         INT64_MIN is kept in a side slot so the table needs no state word)
//   2. k_kv_lookup        slot of every command (absent, never-PUT keys: ret 0, conf 0 now)
//   3. radix sort of (slot << 32 | i) on the slot bits — stable, so log order within a slot
//   4. k_apply_mark       per sorted position q: slot[q], lp[q] = q if PUT else -1
//   5. segmented inclusive max-scan of lp by slot  -> last PUT at or before q in its slot
//   6. k_apply_finish     ret / conf per command; the last PUT of each slot updates the table
// Steps 3 and 5 use rocPRIM device primitives (stable LSD radix sort, look-back scan_by_key).
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "common.hpp"
#include "kernels.hpp"

namespace mpx {

constexpr int64_t kSentinel = INT64_MIN;

__device__ __forceinline__ uint64_t hash64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

// table arrays hold cap+1 entries; entry cap is the side slot of key INT64_MIN
__device__ __forceinline__ int64_t kv_insert(const KvTable& t, int64_t key, uint32_t* err) {
    if (key == kSentinel) return (int64_t)t.cap;
    const uint64_t mask = t.cap - 1;
    uint64_t s = hash64((uint64_t)key) & mask;
    for (uint64_t probe = 0; probe < t.cap; ++probe, s = (s + 1) & mask) {
        unsigned long long* slot = reinterpret_cast<unsigned long long*>(t.keys + s);
        unsigned long long cur = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == (unsigned long long)kSentinel) {
            cur = atomicCAS(slot, (unsigned long long)kSentinel, (unsigned long long)key);
            if (cur == (unsigned long long)kSentinel) return (int64_t)s;  // claimed
        }
        if ((int64_t)cur == key) return (int64_t)s;
    }
    raise_err(err, kErrKvFull);
    return -1;
}

// lookup after all inserts of this call have finished (previous kernel): plain loads
__device__ __forceinline__ int64_t kv_lookup(const KvTable& t, int64_t key) {
    if (key == kSentinel) return (int64_t)t.cap;
    const uint64_t mask = t.cap - 1;
    uint64_t s = hash64((uint64_t)key) & mask;
    for (uint64_t probe = 0; probe < t.cap; ++probe, s = (s + 1) & mask) {
        const int64_t cur = t.keys[s];
        if (cur == key) return (int64_t)s;
        if (cur == kSentinel) return -1;
    }
    return -1;
}

__global__ void k_kv_fill(KvTable t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= t.cap; s += stride) {
        t.keys[s] = kSentinel;
        t.state[s] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *t.n_present = 0;
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
    if (atomicExch(&t.state[s], 1u) == 0u) atomicAdd(t.n_present, 1ull);
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
        if (t.state[s]) {
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
__global__ __launch_bounds__(256) void k_kv_insert_puts(KvTable t, const uint8_t* __restrict__ op,
                                                        const int64_t* __restrict__ key,
                                                        uint64_t m, uint32_t* err) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride)
        if (op[i] == MPX_OP_PUT) kv_insert(t, key[i], err);
}

// slot of every command -> sort keys (slot << 32 | i); NONE slot = cap+1 sorts last
__global__ __launch_bounds__(256) void k_kv_lookup(KvTable t, const int64_t* __restrict__ key,
                                                   uint64_t m, uint64_t* __restrict__ skey,
                                                   int64_t* __restrict__ ret,
                                                   uint8_t* __restrict__ conf) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
        const int64_t s = kv_lookup(t, key[i]);
        const uint64_t sl = s < 0 ? t.cap + 1 : (uint64_t)s;
        skey[i] = (sl << 32) | i;
        if (s < 0) {  // never PUT in this call and absent: GET -> NIL, no conflicts
            ret[i] = 0;
            if (conf) conf[i] = 0;
        }
    }
}

__global__ __launch_bounds__(256) void k_apply_mark(const uint64_t* __restrict__ skey, uint64_t m,
                                                    const uint8_t* __restrict__ op,
                                                    uint32_t* __restrict__ sslot,
                                                    int32_t* __restrict__ lp) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += stride) {
        const uint64_t k = skey[q];
        const uint32_t i = (uint32_t)k;
        sslot[q] = (uint32_t)(k >> 32);
        lp[q] = op[i] == MPX_OP_PUT ? (int32_t)q : -1;
    }
}

__global__ __launch_bounds__(256) void k_apply_finish(
    KvTable t, const uint64_t* __restrict__ skey, const uint32_t* __restrict__ sslot,
    const int32_t* __restrict__ lps, uint64_t m, const uint8_t* __restrict__ op,
    const int64_t* __restrict__ val, int64_t* __restrict__ ret, uint8_t* __restrict__ conf) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t none = (uint32_t)(t.cap + 1);
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += stride) {
        const uint32_t sl = sslot[q];
        if (sl == none) continue;
        const uint32_t i = (uint32_t)skey[q];
        const uint8_t o = op[i];
        const bool has_prev = q > 0 && sslot[q - 1] == sl;
        if (conf) {
            bool c = false;
            if (has_prev) {
                const uint8_t po = op[(uint32_t)skey[q - 1]];
                c = (po == MPX_OP_PUT) || (o == MPX_OP_PUT);
            }
            conf[i] = c;
        }
        int64_t r = 0;
        if (o == MPX_OP_PUT) {
            r = val[i];
        } else if (o == MPX_OP_GET) {
            const int32_t pp = has_prev ? lps[q - 1] : -1;  // last PUT strictly before q
            if (pp >= 0) r = val[(uint32_t)skey[pp]];
            else if (t.state[sl]) r = t.vals[sl];
        }
        ret[i] = r;
    }
}

// the last PUT of every slot writes the table (after every read of the start value is done)
__global__ __launch_bounds__(256) void k_apply_commit(KvTable t, const uint64_t* __restrict__ skey,
                                                      const uint32_t* __restrict__ sslot,
                                                      const int32_t* __restrict__ lps, uint64_t m,
                                                      const int64_t* __restrict__ val) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t none = (uint32_t)(t.cap + 1);
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += stride) {
        const uint32_t sl = sslot[q];
        if (sl == none) continue;
        const bool seg_end = (q + 1 == m) || sslot[q + 1] != sl;
        if (!seg_end) continue;
        const int32_t pp = lps[q];
        if (pp < 0) continue;
        t.vals[sl] = val[(uint32_t)skey[pp]];
        if (t.state[sl] == 0) {
            t.state[sl] = 1;
            atomicAdd(t.n_present, 1ull);
        }
    }
}

namespace {
struct WorkLayout {
    uint64_t skey_a, skey_b, sslot, lp, lps, tmp, tmp_bytes, total;
};
WorkLayout layout(uint64_t m) {
    size_t sort_tmp = 0, scan_tmp = 0;
    (void)rocprim::radix_sort_keys(nullptr, sort_tmp, (uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)m,
                             32u, 64u);
    (void)rocprim::inclusive_scan_by_key(nullptr, scan_tmp, (uint32_t*)nullptr, (int32_t*)nullptr,
                                   (int32_t*)nullptr, (size_t)m, rocprim::maximum<int32_t>(),
                                   rocprim::equal_to<uint32_t>());
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    WorkLayout w;
    uint64_t o = 0;
    w.skey_a = o; o += al(m * 8);
    w.skey_b = o; o += al(m * 8);
    w.sslot = o; o += al(m * 4);
    w.lp = o; o += al(m * 4);
    w.lps = o; o += al(m * 4);
    w.tmp_bytes = al(sort_tmp > scan_tmp ? sort_tmp : scan_tmp);
    w.tmp = o; o += w.tmp_bytes;
    w.total = o;
    return w;
}
}  // namespace

uint64_t apply_work_bytes(uint64_t m) { return layout(m < 1 ? 1 : m).total; }

hipError_t launch_apply(KvTable& t, const uint8_t* op, const int64_t* key, const int64_t* val,
                        uint64_t m, int64_t* ret, uint8_t* conf, ApplyWork& w, uint32_t* err,
                        hipStream_t stream) {
    if (!m) return hipSuccess;
    const WorkLayout L = layout(m);
    if (w.bytes < L.total) return hipErrorInvalidValue;
    char* b = (char*)w.base;
    uint64_t* skey_a = (uint64_t*)(b + L.skey_a);
    uint64_t* skey_b = (uint64_t*)(b + L.skey_b);
    uint32_t* sslot = (uint32_t*)(b + L.sslot);
    int32_t* lp = (int32_t*)(b + L.lp);
    int32_t* lps = (int32_t*)(b + L.lps);
    void* tmp = b + L.tmp;
    size_t tmp_bytes = L.tmp_bytes;
    unsigned blocks = (unsigned)((m + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    k_kv_insert_puts<<<blocks, 256, 0, stream>>>(t, op, key, m, err);
    k_kv_lookup<<<blocks, 256, 0, stream>>>(t, key, m, skey_a, ret, conf);
    unsigned bits = 1;
    while ((1ull << bits) <= t.cap + 1) ++bits;
    hipError_t r = rocprim::radix_sort_keys(tmp, tmp_bytes, skey_a, skey_b, (size_t)m, 32u,
                                            32u + bits, stream);
    if (r != hipSuccess) return r;
    k_apply_mark<<<blocks, 256, 0, stream>>>(skey_b, m, op, sslot, lp);
    tmp_bytes = L.tmp_bytes;
    r = rocprim::inclusive_scan_by_key(tmp, tmp_bytes, sslot, lp, lps, (size_t)m,
                                       rocprim::maximum<int32_t>(), rocprim::equal_to<uint32_t>(),
                                       stream);
    if (r != hipSuccess) return r;
    k_apply_finish<<<blocks, 256, 0, stream>>>(t, skey_b, sslot, lps, m, op, val, ret, conf);
    k_apply_commit<<<blocks, 256, 0, stream>>>(t, skey_b, sslot, lps, m, val);
    return hipGetLastError();
}

// ---- state.ConflictBatch over consecutive instances ------------------------------------------
// one wave per instance pair; lanes stride over the |A| x |B| pairs, early exit on a hit
__global__ __launch_bounds__(256) void k_conflict_batch(const uint8_t* __restrict__ op,
                                                        const int64_t* __restrict__ key,
                                                        const uint64_t* __restrict__ off,
                                                        uint64_t n_pairs, uint8_t* __restrict__ out) {
    const uint64_t pair = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    if (pair >= n_pairs) return;
    const int l = lane_id();
    const uint64_t a0 = off[pair], a1 = off[pair + 1], b1 = off[pair + 2];
    const uint64_t na = a1 - a0, nb = b1 - a1, tot = na * nb;
    bool hit = false;
    for (uint64_t base = 0; base < tot; base += kWave) {
        const uint64_t x = base + l;
        if (x < tot) {
            const uint64_t a = a0 + x / nb, b = a1 + x % nb;
            hit = key[a] == key[b] && (op[a] == MPX_OP_PUT || op[b] == MPX_OP_PUT);
        }
        if (ballot(hit)) {
            hit = true;
            break;
        }
    }
    if (l == 0) out[pair] = hit ? 1 : 0;
}

hipError_t launch_conflict_batch(const uint8_t* op, const int64_t* key, const uint64_t* inst_off,
                                 uint64_t n_inst, uint8_t* out, hipStream_t stream) {
    if (n_inst < 2) return hipSuccess;
    const uint64_t pairs = n_inst - 1;
    const uint64_t blocks = (pairs * kWave + 255) / 256;
    k_conflict_batch<<<dim3((unsigned)blocks), 256, 0, stream>>>(op, key, inst_off, pairs, out);
    return hipGetLastError();
}

}  // namespace mpx
