// tally.hip — accept tally kernels for one instance log (configs 2 and the single-group API).
#include "kernels.hpp"
#include "tally.hpp"

namespace mpx {

// One wave per tile of kTallyTile records; tiles are shifted to instance boundaries so an
// instance is always tallied by exactly one wave.
constexpr uint64_t kTallyTile = 512;
constexpr int kTallyBlock = 256;

// red layout (u64): [0] MIN last-crossing key | CLASSIC any-decided flag
//                   [1..N] MIN peer-commit keys ; [17] CLASSIC first non-committed index
constexpr int kRedFirstBad = 1 + MPX_MAX_REPLICAS;

template <int MODE>
__global__ __launch_bounds__(kTallyBlock) void k_accept_tally(
    const mpx_accept_reply* __restrict__ recs, uint64_t n, const mpx_inst_state* __restrict__ st_in,
    mpx_inst_state* __restrict__ st_out, uint64_t n_inst, int32_t base, int32_t half, int32_t nrep,
    unsigned long long* __restrict__ red, uint8_t* __restrict__ decided, uint32_t* err) {
    const uint64_t wave = ((uint64_t)blockIdx.x * kTallyBlock + threadIdx.x) / kWave;
    const uint64_t s0 = wave * kTallyTile;
    if (s0 >= n) return;
    const uint64_t e0 = s0 + kTallyTile;
    const uint64_t s = find_head(recs, s0, 0, n);
    const uint64_t e = e0 >= n ? n : find_head(recs, e0, 0, n);
    if (s >= e) return;
    TallyOut out{0, 0, false};
    tally_range<MODE>(recs, s, e, st_in, st_out, n_inst, base, half, nrep, decided, err, 0, out);
    const int l = lane_id();
    if (MODE == MPX_MODE_MIN) {
        if (l == 0 && out.cu_key) atomicMax(&red[0], (unsigned long long)out.cu_key);
        if (l < nrep && out.pc_key) atomicMax(&red[1 + l], (unsigned long long)out.pc_key);
    } else {
        if (l == 0 && out.any_dec) atomicMax(&red[0], 1ull);
    }
}

__global__ void k_tally_init(unsigned long long* red, uint64_t n_inst) {
    const int t = threadIdx.x;
    if (t < kRedFirstBad) red[t] = 0;
    if (t == kRedFirstBad) red[t] = n_inst;
}

// CLASSIC updateCommittedUpTo (paxos.go:259-264) over the final statuses: find the first
// instance >= committedUpTo+1 that is not COMMITTED (final COMMITTED <=> st_in COMMITTED or
// decided in this call).
__global__ __launch_bounds__(256) void k_classic_first_bad(
    const mpx_inst_state* __restrict__ st, const uint8_t* __restrict__ decided, uint64_t n_inst,
    int32_t base, const int32_t* __restrict__ scalars, unsigned long long* __restrict__ red) {
    if (red[0] == 0) return;  // no crossing in this call: committedUpTo unchanged
    const int64_t j0 = (int64_t)scalars[0] + 1 - base;
    if (j0 < 0 || (uint64_t)j0 >= n_inst) return;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)j0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_inst;
         j += stride) {
        const unsigned long long fb = __hip_atomic_load(&red[kRedFirstBad], __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        if (j >= fb) break;
        const bool committed = st[j].status == MPX_COMMITTED || (decided && decided[j]);
        if (!committed) atomicMin(&red[kRedFirstBad], (unsigned long long)j);
    }
}

template <int MODE>
__global__ void k_tally_finalize(const unsigned long long* __restrict__ red, int32_t* scalars,
                                 int32_t nrep, uint64_t n_inst, int32_t base) {
    if (threadIdx.x != 0) return;
    if (MODE == MPX_MODE_MIN) {
        if (red[0]) scalars[0] = (int32_t)(uint32_t)(red[0] & 0xffffffffull);
        for (int j = 0; j < nrep; ++j)
            if (red[1 + j]) scalars[1 + j] = (int32_t)(uint32_t)(red[1 + j] & 0xffffffffull);
    } else {
        if (red[0] == 0) return;
        const int64_t j0 = (int64_t)scalars[0] + 1 - base;
        if (j0 < 0 || (uint64_t)j0 >= n_inst) return;
        const uint64_t fb = red[kRedFirstBad];  // first non-committed (n_inst if none)
        scalars[0] = (int32_t)(base + (int64_t)fb - 1);
    }
}

hipError_t launch_accept_tally(int mode, const mpx_accept_reply* recs, uint64_t n,
                               const mpx_inst_state* st_in, mpx_inst_state* st_out,
                               uint64_t n_inst, int32_t base, int32_t nrep, int32_t* scalars,
                               uint8_t* decided, unsigned long long* red, uint32_t* err,
                               hipStream_t stream) {
    const int32_t half = nrep >> 1;
    k_tally_init<<<1, 64, 0, stream>>>(red, n_inst);
    if (decided && n_inst) (void)hipMemsetAsync(decided, 0, n_inst, stream);
    if (n) {
        const uint64_t waves = (n + kTallyTile - 1) / kTallyTile;
        const uint64_t blocks = (waves * kWave + kTallyBlock - 1) / kTallyBlock;
        if (mode == MPX_MODE_MIN)
            k_accept_tally<MPX_MODE_MIN><<<dim3((unsigned)blocks), kTallyBlock, 0, stream>>>(
                recs, n, st_in, st_out, n_inst, base, half, nrep, red, decided, err);
        else
            k_accept_tally<MPX_MODE_CLASSIC><<<dim3((unsigned)blocks), kTallyBlock, 0, stream>>>(
                recs, n, st_in, st_out, n_inst, base, half, nrep, red, decided, err);
    }
    if (mode == MPX_MODE_MIN) {
        k_tally_finalize<MPX_MODE_MIN><<<1, 64, 0, stream>>>(red, scalars, nrep, n_inst, base);
    } else {
        if (n_inst) {
            uint64_t blocks = (n_inst + 255) / 256;
            if (blocks > 2048) blocks = 2048;
            k_classic_first_bad<<<dim3((unsigned)blocks), 256, 0, stream>>>(st_in, decided, n_inst,
                                                                             base, scalars, red);
        }
        k_tally_finalize<MPX_MODE_CLASSIC><<<1, 64, 0, stream>>>(red, scalars, nrep, n_inst,
                                                                 base);
    }
    return hipGetLastError();
}

// Standalone CLASSIC watermark over a status window (mpx_committed_prefix).
__global__ void k_prefix_mark(unsigned long long* red) { red[0] = 1; }

hipError_t launch_committed_prefix(const mpx_inst_state* st, uint64_t n_inst, int32_t base,
                                   int32_t* scalars, unsigned long long* red, hipStream_t stream) {
    k_tally_init<<<1, 64, 0, stream>>>(red, n_inst);
    k_prefix_mark<<<1, 1, 0, stream>>>(red);
    if (n_inst) {
        uint64_t blocks = (n_inst + 255) / 256;
        if (blocks > 2048) blocks = 2048;
        k_classic_first_bad<<<dim3((unsigned)blocks), 256, 0, stream>>>(st, nullptr, n_inst, base,
                                                                         scalars, red);
    }
    k_tally_finalize<MPX_MODE_CLASSIC><<<1, 64, 0, stream>>>(red, scalars, 0, n_inst, base);
    return hipGetLastError();
}

}  // namespace mpx
