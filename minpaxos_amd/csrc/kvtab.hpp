// kvtab.hpp — addressing of the engine's device KV table (mpx_apply's state.State.Store).
//
// The table is cap / 256 buckets of 256 slots; a key lives in bucket hash >> (64 - lgnb) and
// probes linearly from slot hash & 255 WITHIN its bucket. A bucket is therefore a closed hash
// table of its own, which is what lets the apply pipeline (apply_fast.hip) hold a bucket in one
// wave's LDS and resolve every command of its keys without touching the table in HBM. Buckets are
// grouped into bins of up to 16 (one workgroup of 16 waves per bin). The key INT64_MIN is the
// empty-slot sentinel and lives in the side slot `cap`.
#pragma once
#include "common.hpp"

namespace mpx {

constexpr int64_t kSentinel = INT64_MIN;
constexpr int kSB = 256;  // slots per bucket
constexpr int kLgSB = 8;
// per-slot state word: bit 0 present (has a value); bit 1 the last command on the slot in call
// epoch (word >> 2) was a PUT. Epochs start at 1, so a cleared word (0) is "untouched".
constexpr uint32_t kPresent = 1u;
constexpr uint32_t kLastPut = 2u;
constexpr uint32_t kEpochMax = kKvEpochMax;

__device__ __forceinline__ uint64_t hash64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

// the inverse of hash64 (every step of the finalizer is a bijection): the partitioned apply moves
// keys as their hashes and recovers a key only where it writes one to the table
__device__ __forceinline__ uint64_t unhash64(uint64_t x) {
    x ^= (x >> 31) ^ (x >> 62);
    x *= 0x319642B2D24D8EC3ull;  // 0x94D049BB133111EB^-1 mod 2^64
    x ^= (x >> 27) ^ (x >> 54);
    x *= 0x96DE1B173F119089ull;  // 0xBF58476D1CE4E5B9^-1 mod 2^64
    x ^= (x >> 30) ^ (x >> 60);
    return x;
}

__device__ __forceinline__ uint32_t bucket_of(uint64_t h, uint32_t lgnb) {
    return lgnb ? (uint32_t)(h >> (64 - lgnb)) : 0u;
}
__device__ __forceinline__ uint32_t home_of(uint64_t h) { return (uint32_t)h & (kSB - 1); }

// insert-or-find with one 64-bit CAS per claimed slot (concurrent inserters of the same or other
// keys are safe); -1 and kErrKvFull when the key's bucket is full
__device__ __forceinline__ int64_t kv_insert(const KvTable& t, int64_t key, uint32_t* err) {
    if (key == kSentinel) return (int64_t)t.cap;
    const uint64_t h = hash64((uint64_t)key);
    const uint64_t base = (uint64_t)bucket_of(h, t.lgnb) << kLgSB;
    uint32_t s = home_of(h);
    for (int probe = 0; probe < kSB; ++probe, s = (s + 1) & (kSB - 1)) {
        unsigned long long* slot = reinterpret_cast<unsigned long long*>(t.keys + base + s);
        unsigned long long cur = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == (unsigned long long)kSentinel) {
            cur = atomicCAS(slot, (unsigned long long)kSentinel, (unsigned long long)key);
            if (cur == (unsigned long long)kSentinel) return (int64_t)(base + s);  // claimed
        }
        if ((int64_t)cur == key) return (int64_t)(base + s);
    }
    raise_err(err, kErrKvFull);
    return -1;
}

// lookup after every insert of this call has finished (a previous kernel): plain loads
__device__ __forceinline__ int64_t kv_lookup(const KvTable& t, int64_t key) {
    if (key == kSentinel) return (int64_t)t.cap;
    const uint64_t h = hash64((uint64_t)key);
    const uint64_t base = (uint64_t)bucket_of(h, t.lgnb) << kLgSB;
    uint32_t s = home_of(h);
    for (int probe = 0; probe < kSB; ++probe, s = (s + 1) & (kSB - 1)) {
        const int64_t cur = t.keys[base + s];
        if (cur == key) return (int64_t)(base + s);
        if (cur == kSentinel) return -1;
    }
    return -1;
}

}  // namespace mpx
