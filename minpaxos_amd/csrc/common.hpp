// common.hpp — shared device helpers for the gfx950 kernels (wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mpx.h"
#include "kernels.hpp"

namespace mpx {

constexpr int kWave = 64;

// Streaming-access policy of once-read inputs and once-written outputs (records, instance
// state, commands, results): MPX_NT bit 0 = nontemporal loads, bit 1 = nontemporal stores.
// Both together measured 3-5 % faster on the fused group step than default-policy accesses
// (tools/ab_step.py, same process); loads alone were slower.
#ifndef MPX_NT
#define MPX_NT 3
#endif
template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
#if MPX_NT & 1
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
template <typename T>
__device__ __forceinline__ void st_stream(T* p, T v) {
#if MPX_NT & 2
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
typedef int v4i_t __attribute__((ext_vector_type(4)));
template <>
__device__ __forceinline__ int4 ld_stream<int4>(const int4* p) {
#if MPX_NT & 1
    const v4i_t x = __builtin_nontemporal_load(reinterpret_cast<const v4i_t*>(p));
    return make_int4(x.x, x.y, x.z, x.w);
#else
    return *p;
#endif
}
typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
template <>
__device__ __forceinline__ uint4 ld_stream<uint4>(const uint4* p) {
#if MPX_NT & 1
    const v4u_t x = __builtin_nontemporal_load(reinterpret_cast<const v4u_t*>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
#else
    return *p;
#endif
}
template <>
__device__ __forceinline__ void st_stream<uint4>(uint4* p, uint4 v) {
#if MPX_NT & 2
    v4u_t x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4u_t*>(p));
#else
    *p = v;
#endif
}
template <>
__device__ __forceinline__ void st_stream<int4>(int4* p, int4 v) {
#if MPX_NT & 2
    v4i_t x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4i_t*>(p));
#else
    *p = v;
#endif
}


__device__ __forceinline__ int lane_id() { return __lane_id(); }

// mask of lanes 0..l inclusive
__device__ __forceinline__ uint64_t lanes_upto(int l) {
    return l >= 63 ? ~0ull : ((2ull << l) - 1ull);
}
// mask of lanes 0..l-1
__device__ __forceinline__ uint64_t lanes_below(int l) { return l <= 0 ? 0ull : ((1ull << l) - 1ull); }

__device__ __forceinline__ int hi_bit(uint64_t m) { return 63 - __clzll((long long)m); }
__device__ __forceinline__ int lo_bit(uint64_t m) { return __ffsll((long long)m) - 1; }
__device__ __forceinline__ int popc(uint64_t m) { return __popcll(m); }

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

template <typename T>
__device__ __forceinline__ T readlane(T v, int l);
template <>
__device__ __forceinline__ int32_t readlane<int32_t>(int32_t v, int l) {
    return __builtin_amdgcn_readlane(v, l);
}
template <>
__device__ __forceinline__ uint32_t readlane<uint32_t>(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

__device__ __forceinline__ void raise_err(uint32_t* err, uint32_t bit) {
    if (err) atomicOr(err, bit);
}

// ---- last-workgroup-done without cache maintenance ------------------------------------------
// A workgroup hands its partial results to the grid's last workgroup through device-scope
// atomics on engine-owned control words, then takes a ticket. On gfx950 an agent-scope release
// fence (__threadfence) writes back the XCD's whole L2 (buffer_wbl2 sc1) and the acquire side
// invalidates it, in every workgroup: measured +40 us on a 1024-workgroup tally. Instead each
// contribution is an atomic whose RETURN the thread waits for - it has then been performed at the
// device's coherence point - before the barrier that precedes the ticket, so the ticket cannot
// overtake it; the last workgroup reads (and resets) the accumulators with atomics as well.
__device__ __forceinline__ void atomic_max_done(uint32_t* p, uint32_t v) {
    const uint32_t old = __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(old) : "memory");
}
__device__ __forceinline__ void atomic_add_done(unsigned long long* p, unsigned long long v) {
    const unsigned long long old =
        __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(old) : "memory");
}
__device__ __forceinline__ void atomic_add_done(uint32_t* p, uint32_t v) {
    const uint32_t old = __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(old) : "memory");
}
__device__ __forceinline__ uint32_t atomic_take(uint32_t* p) {  // read and reset to 0
    return __hip_atomic_exchange(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long atomic_take(unsigned long long* p) {
    return __hip_atomic_exchange(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// true in the grid's last workgroup to get here (all threads call; the ticket is reset there)
__device__ __forceinline__ bool last_workgroup(uint32_t* ticket) {
    __shared__ bool last;
    __syncthreads();  // every contribution of the workgroup has been performed
    if (threadIdx.x == 0) {
        const uint32_t k =
            __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = k == gridDim.x - 1;
        if (last) (void)atomic_take(ticket);
    }
    __syncthreads();
    return last;
}

// Segmented inclusive max-scan over the wave. `head` marks the first lane of a segment.
// Lanes before the first head of the wave form an open segment (no head).
__device__ __forceinline__ int32_t seg_max_scan(int32_t v, bool head) {
    const int l = lane_id();
    int f = head ? 1 : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int32_t t = __shfl_up(v, d);
        int tf = __shfl_up(f, d);
        if (l >= d && !f) {
            v = v > t ? v : t;
            f |= tf;
        }
    }
    return v;
}

// Wave-wide max of a u64 key held by the lanes in `active` (others contribute 0).
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint64_t t = __shfl_xor(v, d);
        v = v > t ? v : t;
    }
    return v;
}

}  // namespace mpx
