// mall_probe.hip — how random 8/16-byte stores and loads behave when their footprint is a window
// that fits the XCD L2s / the 256 MB Infinity Cache, against the same traffic spread over a
// buffer far larger than it. Calibration for the apply pipeline's design, not part
// of the engine.
//   seq_store        : 64M u64 coalesced stores (512 MB)
//   rand_store_full  : 64M u64 stores, a random permutation of the whole 512 MB
//   rand_store_win W : the same 512 MB written window by window (one launch per W-element window),
//                      a random permutation inside each window
//   rand_load_win W  : 64M u64 loads, random inside each window, stored coalesced
//   rand_u8_win W    : 64M byte stores, random inside each window
//   rand_rec16_win W : 32M 16-byte records, random inside each window
//   table_load T     : 64M u64 loads from random slots of a T-element table (the index probe)
// Build: hipcc -O3 --offload-arch=gfx950 tools/mall_probe.hip -o tools/mall_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

// a bijection of [0, 2^bits)
__device__ __forceinline__ uint32_t perm(uint32_t i, int bits) {
    const uint32_t m = bits >= 32 ? ~0u : (1u << bits) - 1u;
    uint32_t x = (i * 0x9E3779B1u) & m;
    x ^= x >> (bits / 2 + 1);
    x = (x * 0x85EBCA6Bu) & m;
    x ^= x >> (bits / 2);
    return x & m;
}

constexpr int U = 4;

__global__ __launch_bounds__(256) void k_seq_store(uint64_t* out, uint32_t n) {
    const uint32_t base = (blockIdx.x * 256u) * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * 256u;
        if (i < n) out[i] = i;
    }
}

__global__ __launch_bounds__(256) void k_rand_store(uint64_t* out, uint32_t n, int bits) {
    const uint32_t base = (blockIdx.x * 256u) * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * 256u;
        if (i < n) out[perm(i, bits)] = i;
    }
}

__global__ __launch_bounds__(256) void k_rand_load(const uint64_t* in, uint64_t* out, uint32_t n,
                                                   int bits) {
    const uint32_t base = (blockIdx.x * 256u) * U + threadIdx.x;
    uint64_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * 256u;
        v[u] = i < n ? in[perm(i, bits)] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * 256u;
        if (i < n) out[i] = v[u];
    }
}

__global__ __launch_bounds__(256) void k_rand_u8(uint8_t* out, uint32_t n, int bits) {
    const uint32_t base = (blockIdx.x * 256u) * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * 256u;
        if (i < n) out[perm(i, bits)] = (uint8_t)i;
    }
}

__global__ __launch_bounds__(256) void k_rand_rec16(int4* out, uint32_t n, int bits) {
    const uint32_t base = (blockIdx.x * 256u) * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * 256u;
        if (i < n) out[perm(i, bits)] = make_int4(i, i, i, i);
    }
}

__global__ __launch_bounds__(256) void k_table_load(const uint64_t* tab, uint64_t* out, uint32_t n,
                                                    int tbits) {
    const uint32_t base = (blockIdx.x * 256u) * U + threadIdx.x;
    uint64_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * 256u;
        v[u] = i < n ? tab[perm(i * 2654435761u, 32) >> (32 - tbits)] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = base + u * 256u;
        if (i < n) out[i] = v[u];
    }
}

template <class F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    f();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

static unsigned blocks(uint32_t n) { return (n + 256 * U - 1) / (256 * U); }

int main() {
    const uint32_t N = 1u << 26;  // 64M elements
    const int reps = 5;
    uint64_t *a, *b;
    CHK(hipMalloc(&a, (size_t)N * 8));
    CHK(hipMalloc(&b, (size_t)N * 8));
    CHK(hipMemset(a, 1, (size_t)N * 8));
    CHK(hipMemset(b, 0, (size_t)N * 8));
    auto line = [](const char* name, long w, float ms) {
        printf("{\"test\": \"%s\", \"window\": %ld, \"ms\": %.4f, \"Gops\": %.2f}\n", name, w, ms,
               (double)(1u << 26) / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    line("seq_store", N, time_ms([&] { k_seq_store<<<blocks(N), 256>>>(a, N); }, reps));
    line("rand_store_full", N, time_ms([&] { k_rand_store<<<blocks(N), 256>>>(a, N, 26); }, reps));
    for (int wb = 18; wb <= 24; ++wb) {
        const uint32_t W = 1u << wb;
        line("rand_store_win", W, time_ms([&] {
                 for (uint32_t w0 = 0; w0 < N; w0 += W) k_rand_store<<<blocks(W), 256>>>(a + w0, W, wb);
             }, reps));
    }
    line("rand_load_full", N, time_ms([&] { k_rand_load<<<blocks(N), 256>>>(a, b, N, 26); }, reps));
    for (int wb = 18; wb <= 24; wb += 2) {
        const uint32_t W = 1u << wb;
        line("rand_load_win", W, time_ms([&] {
                 for (uint32_t w0 = 0; w0 < N; w0 += W)
                     k_rand_load<<<blocks(W), 256>>>(a + w0, b + w0, W, wb);
             }, reps));
    }
    uint8_t* c = (uint8_t*)a;
    line("rand_u8_full", N, time_ms([&] { k_rand_u8<<<blocks(N), 256>>>(c, N, 26); }, reps));
    for (int wb = 20; wb <= 24; wb += 2) {
        const uint32_t W = 1u << wb;
        line("rand_u8_win", W, time_ms([&] {
                 for (uint32_t w0 = 0; w0 < N; w0 += W) k_rand_u8<<<blocks(W), 256>>>(c + w0, W, wb);
             }, reps));
    }
    int4* r = (int4*)a;  // 32M records of 16 B = 512 MB
    const uint32_t NR = N / 2;
    line("rand_rec16_full", NR, time_ms([&] { k_rand_rec16<<<blocks(NR), 256>>>(r, NR, 25); }, reps));
    for (int wb = 18; wb <= 22; wb += 2) {
        const uint32_t W = 1u << wb;
        line("rand_rec16_win", W, time_ms([&] {
                 for (uint32_t w0 = 0; w0 < NR; w0 += W) k_rand_rec16<<<blocks(W), 256>>>(r + w0, W, wb);
             }, reps));
    }
    for (int tb = 18; tb <= 24; tb += 2)
        line("table_load", 1l << tb,
             time_ms([&] { k_table_load<<<blocks(N), 256>>>(a, b, N, tb); }, reps));
    CHK(hipGetLastError());
    CHK(hipFree(a));
    CHK(hipFree(b));
    return 0;
}
