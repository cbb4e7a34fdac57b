// hbm_ceiling.hip — practical HBM ceiling of this MI355X for the engine's stream mixes.
//
// Not part of the engine: a calibration for DESIGN.md's roofline table. It times plain streaming
// kernels (16-byte nontemporal loads / stores, grid-stride, 4 independent loads in flight per
// lane) over buffers far larger than the 256 MB Infinity Cache:
//   read      : sum of R bytes (one 4-byte store per workgroup)
//   write     : W bytes of a constant
//   copy      : R bytes in, R bytes out
//   mix R:W   : the group step's ratio (2.79 GB fetched : 1.13 GB written per launch, rocprofv3
//               FETCH_SIZE / WRITE_SIZE in profiles/r01), coalesced 5 int4 in : 2 int4 out
// Build: hipcc -O3 --offload-arch=gfx950 tools/hbm_ceiling.hip -o tools/hbm_ceiling
// Run (GPU box): tools/hbm_ceiling  -> one JSON line per kernel, bytes / average launch time.
#include <hip/hip_runtime.h>

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

typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int4 ld(const int4* p) {
    const v4i_t x = __builtin_nontemporal_load(reinterpret_cast<const v4i_t*>(p));
    return make_int4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void st(int4* p, int4 v) {
    v4i_t x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4i_t*>(p));
}

__global__ __launch_bounds__(256) void k_read(const int4* __restrict__ in, size_t n,
                                              int* __restrict__ out) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    int acc = 0;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const int4 a = ld(in + i), b = ld(in + i + stride), c = ld(in + i + 2 * stride),
                   d = ld(in + i + 3 * stride);
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^
               d.z ^ d.w;
    }
    for (; i < n; i += stride) {
        const int4 a = ld(in + i);
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x7fffffff) out[blockIdx.x] = acc;  // keeps the loads alive
}

__global__ __launch_bounds__(256) void k_write(int4* __restrict__ out, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const int4 v = make_int4(1, 2, 3, 4);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) st(out + i, v);
}

__global__ __launch_bounds__(256) void k_copy(const int4* __restrict__ in, int4* __restrict__ out,
                                              size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const int4 a = ld(in + i), b = ld(in + i + stride), c = ld(in + i + 2 * stride),
                   d = ld(in + i + 3 * stride);
        st(out + i, a);
        st(out + i + stride, b);
        st(out + i + 2 * stride, c);
        st(out + i + 3 * stride, d);
    }
    for (; i < n; i += stride) st(out + i, ld(in + i));
}

// the group step's read:write ratio, coalesced: unit u reads int4 u + k*U of `in` (k < 5) and
// writes int4 u + k*U of `out` (k < 2), U = units
__global__ __launch_bounds__(256) void k_mix(const int4* __restrict__ in, int4* __restrict__ out,
                                             size_t U) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x; u < U; u += stride) {
        const int4 a = ld(in + u), b = ld(in + u + U), c = ld(in + u + 2 * U),
                   d = ld(in + u + 3 * U), e = ld(in + u + 4 * U);
        st(out + u, make_int4(a.x ^ c.x, a.y ^ c.y, a.z ^ e.z, a.w ^ e.w));
        st(out + u + U, make_int4(b.x ^ d.x, b.y ^ d.y, b.z ^ d.z, b.w ^ d.w));
    }
}

template <class F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    f();
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

int main() {
    const size_t R = 2800ull << 20, W = 1120ull << 20;  // about the group step's bytes
    const int reps = 20;
    int4 *in, *out;
    int* sink;
    CHK(hipMalloc(&in, R));
    CHK(hipMalloc(&out, R));
    CHK(hipMalloc(&sink, 1 << 20));
    CHK(hipMemset(in, 1, R));
    CHK(hipMemset(out, 0, R));
    const unsigned grid = 256 * 32;  // 8192 workgroups of 256: 32 waves per CU resident
    auto line = [](const char* name, double bytes, float ms) {
        printf("{\"kernel\": \"%s\", \"bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}\n", name, bytes,
               ms, bytes / (ms * 1e-3) / 1e9);
    };
    float ms = time_ms([&] { k_read<<<grid, 256>>>(in, R / 16, sink); }, reps);
    line("read", (double)R, ms);
    ms = time_ms([&] { k_write<<<grid, 256>>>(out, W / 16); }, reps);
    line("write", (double)W, ms);
    const size_t C = 1600ull << 20;
    ms = time_ms([&] { k_copy<<<grid, 256>>>(in, out, C / 16); }, reps);
    line("copy", 2.0 * C, ms);
    const size_t U = W / 32;  // units of 5 int4 in, 2 int4 out
    ms = time_ms([&] { k_mix<<<grid, 256>>>(in, out, U); }, reps);
    line("mix_5r_2w", (double)U * 16 * 7, ms);
    ms = time_ms([&] { k_mix<<<U / 256, 256>>>(in, out, U); }, reps);  // one unit per lane
    line("mix_5r_2w_flat", (double)U * 16 * 7, ms);
    CHK(hipGetLastError());
    CHK(hipFree(in));
    CHK(hipFree(out));
    CHK(hipFree(sink));
    return 0;
}
