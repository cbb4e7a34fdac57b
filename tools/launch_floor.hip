// launch_floor.hip: the device-time floor of a replica-sized apply call on this GPU.
// Events around 1/2/3 empty launches, and around one kernel doing d dependent random 8-byte loads
// per thread (5000 threads, a 20 MB table: the replica path's round trips), d = 1..6.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_empty(int* out) { if (threadIdx.x == 1024) out[0] = 1; }
__global__ void k_chase(const uint64_t* __restrict__ tab, uint64_t mask, int n, int d, uint64_t* out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    uint64_t x = (uint64_t)p * 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < d; ++i) x = __hip_atomic_load(&tab[(x >> 17) & mask], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + x;
    out[p] = x;
}
__global__ void k_fill(uint64_t* tab, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        tab[i] = i * 0xBF58476D1CE4E5B9ull;
}
static float med(std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }
int main() {
    int* o; uint64_t *tab, *out;
    const uint64_t n = 1u << 21;  // 16 MB of 8-byte words (the 1M-slot table's keys + vals)
    CK(hipMalloc(&o, 4)); CK(hipMalloc(&tab, n * 8)); CK(hipMalloc(&out, 1 << 20));
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    k_fill<<<1024, 256, 0, s>>>(tab, n);
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int nk = 1; nk <= 3; ++nk) {
        std::vector<float> t;
        for (int r = 0; r < 200; ++r) {
            CK(hipEventRecord(a, s));
            for (int k = 0; k < nk; ++k) k_empty<<<20, 256, 0, s>>>(o);
            CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); if (r >= 20) t.push_back(ms * 1000);
        }
        printf("empty launches %d: median %.2f us\n", nk, med(t));
    }
    for (int d = 0; d <= 6; ++d) {
        std::vector<float> t;
        for (int r = 0; r < 200; ++r) {
            CK(hipEventRecord(a, s));
            k_chase<<<20, 256, 0, s>>>(tab, n - 1, 5000, d, out);
            CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); if (r >= 20) t.push_back(ms * 1000);
        }
        printf("chase 5000 threads x %d dependent loads: median %.2f us\n", d, med(t));
    }
    for (int d = 0; d <= 6; d += 2) {
        std::vector<float> t;
        for (int r = 0; r < 200; ++r) {
            CK(hipEventRecord(a, s));
            k_chase<<<5, 1024, 0, s>>>(tab, n - 1, 5000, d, out);
            CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); if (r >= 20) t.push_back(ms * 1000);
        }
        printf("chase 5 x 1024 threads x %d dependent loads: median %.2f us\n", d, med(t));
    }
    return 0;
}
