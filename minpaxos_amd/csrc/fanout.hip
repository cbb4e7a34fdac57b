// fanout.hip — client reply fan-out.
//
// Reference: the leader answers every command of a decided instance with a
// genericsmrproto.ProposeReplyTS{OK, CommandId, Value, Timestamp, Leader}
// (genericsmrproto.go:31-37) written to the proposing client's connection:
//   at decide time  bareminpaxos.go:1030-1042 (Value = state.NIL, unless -dreply)
//   at apply time   bareminpaxos.go:1076-1084 (Value = Execute's return, with -dreply)
// through genericsmr.(*Replica).ReplyProposeTS (genericsmr.go:529-535), whose Marshal
// (gsmrprotomarsh.go:702-732) writes 25 bytes: OK u8, CommandId i32, Value i64, Timestamp i64,
// Leader i32, little endian, no frame code.
// The engine takes a batch of replies in execution order and produces, for every client
// connection, the exact byte run its bufio.Writer would receive: a stable partition by client
// (per-client order = execution order).
// Up to kFanMaxClients connections: a one-pass counting sort fused with the encoding.
//   k_fan_count    workgroup b counts the clients of its contiguous slice of replies (LDS
//                  histogram) into hist[client][b] (client-major)
//   exclusive scan of hist: the first output record of every (client, workgroup)
//   k_fan_scatter  workgroup b walks its slice in tiles of kFanTile replies: each wave ranks its
//                  segment's replies per client (match over the client bits, per-wave LDS
//                  counters - stable), the workgroup turns the ranks into positions of a
//                  client-sorted tile image in LDS and encodes the 25-byte replies there, then
//                  copies every client's run of the image to its place in that client's output
//                  run with dword stores (head and tail bytes of a run with byte stores).
// HBM: the replies are read twice (count, scatter) and the output written once, coalesced in
// runs; nothing is gathered at random. More connections: a radix sort (radix.hpp) of the client
// id with the reply index as payload, then each block gathers 256 replies, assembles their
// encodings in LDS and stores the 6400-byte run with 16-byte vector stores.
// client_off[c] = byte offset of client c's run; client_off[n_clients] = 25 n.
#include <cstring>

#include "common.hpp"
#include "kernels.hpp"
#include "radix.hpp"
#include "scan.hpp"

namespace mpx {

namespace {
constexpr int kFanBlock = 256;
constexpr int kRecBytes = 25;

unsigned bits_for_clients(uint32_t c) {  // bits to represent every client id < c
    unsigned b = 1;
    while ((1ull << b) < c) ++b;
    return b;
}
}  // namespace

// the radix sort's input: client id and reply index of every reply
__global__ __launch_bounds__(256) void k_fan_keys(const mpx_reply_rec* __restrict__ recs, uint64_t n,
                                                 uint32_t* __restrict__ keys,
                                                 uint32_t* __restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    keys[i] = recs[i].client;
    idx[i] = (uint32_t)i;
}

// exclusive scan of the client-major histogram: the first output record of every (client, slice)
struct HistIn {
    const uint32_t* h;
    __device__ __forceinline__ uint32_t operator()(uint64_t i) const { return h[i]; }
};
struct FirstOut {
    uint32_t* first;
    __device__ __forceinline__ void operator()(uint64_t i, uint32_t ex, uint32_t) const {
        first[i] = ex;
    }
};

template <bool kAligned>
__global__ __launch_bounds__(kFanBlock) void k_fan_encode(
    const mpx_reply_rec* __restrict__ recs, const uint32_t* __restrict__ skeys,
    const uint32_t* __restrict__ perm, uint64_t n, uint32_t n_clients, uint8_t ok, int32_t leader,
    uint8_t* __restrict__ out, uint64_t* __restrict__ client_off, uint32_t* err) {
    __shared__ __attribute__((aligned(16))) uint8_t S[kFanBlock * kRecBytes];
    const uint64_t q0 = (uint64_t)blockIdx.x * kFanBlock;
    const uint64_t q = q0 + threadIdx.x;
    const uint32_t cnt = (uint32_t)(n - q0 < (uint64_t)kFanBlock ? n - q0 : kFanBlock);
    if (q < n) {
        const mpx_reply_rec r = recs[perm[q]];
        uint8_t* b = S + threadIdx.x * kRecBytes;
        b[0] = ok;
        const uint32_t cid = (uint32_t)r.command_id;
        const uint64_t v = (uint64_t)r.value, ts = (uint64_t)r.timestamp;
        const uint32_t ld = (uint32_t)leader;
#pragma unroll
        for (int k = 0; k < 4; ++k) b[1 + k] = (uint8_t)(cid >> (8 * k));
#pragma unroll
        for (int k = 0; k < 8; ++k) b[5 + k] = (uint8_t)(v >> (8 * k));
#pragma unroll
        for (int k = 0; k < 8; ++k) b[13 + k] = (uint8_t)(ts >> (8 * k));
#pragma unroll
        for (int k = 0; k < 4; ++k) b[21 + k] = (uint8_t)(ld >> (8 * k));
        // client run boundaries: every client id in (previous key, this key] starts here. A
        // client id >= n_clients (sorted on its low bits only) fails the call; it is clamped so
        // no offset outside client_off is ever written.
        if (r.client >= n_clients) raise_err(err, kErrInval);
        const int64_t c = skeys[q] < n_clients ? (int64_t)skeys[q] : (int64_t)n_clients - 1;
        const int64_t prev = q == 0 ? -1
                                    : (skeys[q - 1] < n_clients ? (int64_t)skeys[q - 1]
                                                                : (int64_t)n_clients - 1);
        for (int64_t x = prev + 1; x <= c; ++x) client_off[x] = q * kRecBytes;
        if (q + 1 == n)
            for (uint64_t x = (uint64_t)c + 1; x <= n_clients; ++x) client_off[x] = n * kRecBytes;
    }
    __syncthreads();
    const uint32_t bytes = cnt * kRecBytes;
    uint8_t* dst = out + q0 * kRecBytes;
    if (kAligned) {  // q0 * 25 is a multiple of 16: full 16-byte vectors, then the tail
        const uint32_t nv = bytes / 16;
        for (uint32_t i = threadIdx.x; i < nv; i += kFanBlock)
            st_stream(reinterpret_cast<uint4*>(dst) + i, reinterpret_cast<const uint4*>(S)[i]);
        for (uint32_t i = nv * 16 + threadIdx.x; i < bytes; i += kFanBlock) dst[i] = S[i];
    } else {
        for (uint32_t i = threadIdx.x; i < bytes; i += kFanBlock) dst[i] = S[i];
    }
}

__global__ void k_fan_empty(uint64_t* client_off, uint32_t n_clients) {
    for (uint32_t x = threadIdx.x; x <= n_clients; x += blockDim.x) client_off[x] = 0;
}

// ---- counting-sort path (n_clients <= kFanMaxClients) ------------------------------------------
#ifndef MPX_FAN_ABLATE
#define MPX_FAN_ABLATE 0  // diagnostic builds only: 1 no write-out, 2 no encode, 8 no stores
#endif
#ifndef MPX_FAN_UNROLL
#define MPX_FAN_UNROLL 2
#endif
constexpr uint32_t kFanMaxClients = 1024;
constexpr int kFanThreads = 512;
constexpr int kFanWaves = kFanThreads / kWave;        // 8
#ifndef MPX_FAN_PER
#define MPX_FAN_PER 8
#endif
constexpr int kFanPer = MPX_FAN_PER;                  // replies per lane per tile
constexpr int kFanSeg = kFanPer * kWave;              // 512 replies per wave segment
constexpr int kFanTile = kFanSeg * kFanWaves;         // 4096 replies per tile
constexpr uint32_t kFanMaxSlices = 1024;              // workgroups (client-major histogram columns)
constexpr int kSlotWords = 7;                         // image slot: 25 bytes + 3 pad


struct FanPlan {
    uint32_t slices;     // workgroups
    uint64_t per_slice;  // replies per workgroup (a multiple of kFanTile)
};
FanPlan fan_plan(uint64_t n) {
    const uint64_t tiles = (n + kFanTile - 1) / kFanTile;
    const uint64_t slices = tiles < kFanMaxSlices ? (tiles ? tiles : 1) : kFanMaxSlices;
    const uint64_t tiles_per = (tiles + slices - 1) / slices;
    FanPlan p;
    p.per_slice = (tiles_per ? tiles_per : 1) * kFanTile;
    p.slices = (uint32_t)((n + p.per_slice - 1) / p.per_slice);
    if (!p.slices) p.slices = 1;
    return p;
}

__device__ __forceinline__ uint32_t fan_client(uint32_t c, uint32_t n_clients, uint32_t* err) {
    if (c >= n_clients) {  // the call fails; clamped so nothing lands outside the output
        raise_err(err, kErrInval);
        return n_clients - 1;
    }
    return c;
}

__global__ __launch_bounds__(kFanThreads) void k_fan_count(const mpx_reply_rec* __restrict__ recs,
                                                           uint64_t n, uint64_t per_slice,
                                                           uint32_t n_clients, uint32_t slices,
                                                           uint32_t* __restrict__ hist,
                                                           uint32_t* err) {
    __shared__ uint32_t cnt[kFanMaxClients];
    for (uint32_t c = threadIdx.x; c < n_clients; c += kFanThreads) cnt[c] = 0;
    __syncthreads();
    const uint64_t r0 = (uint64_t)blockIdx.x * per_slice;
    const uint64_t r1 = n - r0 < per_slice ? n : r0 + per_slice;
    const uint32_t* cl = reinterpret_cast<const uint32_t*>(recs) + 5;  // client word of record 0
    for (uint64_t i = r0 + threadIdx.x; i < r1; i += kFanThreads)
        atomicAdd(&cnt[fan_client(cl[i * 6], n_clients, err)], 1u);
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < n_clients; c += kFanThreads)
        hist[(uint64_t)c * slices + blockIdx.x] = cnt[c];
}

// exclusive scan of (a, b) pairs over n <= 2 * kFanThreads entries held in LDS, in place;
// returns the totals (every thread)
__device__ __forceinline__ uint2 fan_block_scan2(uint32_t* a, uint32_t* b, uint32_t n,
                                                 uint32_t* wsum /* 2 * kFanWaves */) {
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    const uint32_t i0 = 2 * t, i1 = 2 * t + 1;
    const uint32_t a0 = i0 < n ? a[i0] : 0, a1 = i1 < n ? a[i1] : 0;
    const uint32_t b0 = i0 < n ? b[i0] : 0, b1 = i1 < n ? b[i1] : 0;
    uint32_t sa = a0 + a1, sb = b0 + b1;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t ta = __shfl_up(sa, d), tb = __shfl_up(sb, d);
        if (l >= d) {
            sa += ta;
            sb += tb;
        }
    }
    if (l == kWave - 1) {
        wsum[w] = sa;
        wsum[kFanWaves + w] = sb;
    }
    __syncthreads();
    uint32_t pa = 0, pb = 0, ta = 0, tb = 0;
#pragma unroll
    for (int x = 0; x < kFanWaves; ++x) {
        if (x < w) {
            pa += wsum[x];
            pb += wsum[kFanWaves + x];
        }
        ta += wsum[x];
        tb += wsum[kFanWaves + x];
    }
    // exclusive prefix of entry i0 = inclusive of this thread minus its own pair
    const uint32_t ea = pa + sa - (a0 + a1), eb = pb + sb - (b0 + b1);
    __syncthreads();  // every entry read before any is overwritten
    if (i0 < n) {
        a[i0] = ea;
        b[i0] = eb;
    }
    if (i1 < n) {
        a[i1] = ea + a0;
        b[i1] = eb + b0;
    }
    __syncthreads();
    return make_uint2(ta, tb);
}

__global__ __launch_bounds__(kFanThreads) void k_fan_scatter(
    const mpx_reply_rec* __restrict__ recs, uint64_t n, uint64_t per_slice, uint32_t n_clients,
    uint32_t slices, const uint32_t* __restrict__ first, uint8_t ok, int32_t leader,
    uint8_t* __restrict__ out, uint64_t* __restrict__ client_off, uint32_t* err) {
    __shared__ uint32_t img[(kFanTile + 1) * kSlotWords];      // client-sorted 28-byte slots
    __shared__ uint16_t wcnt[kFanWaves][kFanMaxClients];       // per-wave counts -> prefixes
    __shared__ uint16_t sc[kFanTile];                          // client of image slot
    __shared__ uint32_t base[kFanMaxClients];                  // next output record per client
    // a client's output region of this slice is contiguous and filled tile by tile, so the
    // bytes of a run's last, partial output dword wait here (carry: bit 31 valid, low 3 bytes)
    // for the client's next run to complete the dword: only whole dwords are stored inside a
    // slice, bytewise stores remain only at the slice's two ends
    __shared__ uint32_t carry[kFanMaxClients];
    __shared__ uint32_t carry_in[kFanMaxClients];              // carry at the tile's start
    __shared__ uint32_t tstart[kFanMaxClients];                // client's run in the tile image
    __shared__ uint32_t tcnt[kFanMaxClients];
    __shared__ uint32_t wsum[2 * kFanWaves];
    const int t = threadIdx.x, l = lane_id(), w = t / kWave;
    const uint32_t C = n_clients;
    unsigned cbits = 1;
    while ((1u << cbits) < C) ++cbits;
    for (uint32_t c = t; c < C; c += kFanThreads) {
        base[c] = first[(uint64_t)c * slices + blockIdx.x];
        carry[c] = 0;
        if (blockIdx.x == 0) client_off[c] = (uint64_t)base[c] * kRecBytes;
    }
    if (blockIdx.x == 0 && t == 0) client_off[C] = n * kRecBytes;
    const uint64_t r0 = (uint64_t)blockIdx.x * per_slice;
    const uint64_t r1 = n - r0 < per_slice ? n : r0 + per_slice;
    const uint32_t out_mis = (uint32_t)((uintptr_t)out & 3u);
    // the wave's segment of a tile: reply k*64+l of segment w, coalesced per k; the next tile's
    // replies are loaded while this tile is ranked, encoded and written
    mpx_reply_rec nxt[kFanPer];
    auto load_tile = [&](uint64_t t0) {
        const uint32_t nt = (uint32_t)(r1 - t0 < (uint64_t)kFanTile ? r1 - t0 : kFanTile);
#pragma unroll
        for (int k = 0; k < kFanPer; ++k) {
            const uint32_t j = w * kFanSeg + k * kWave + l;
            if (j < nt) nxt[k] = recs[t0 + j];
        }
    };
    if (r0 < r1) load_tile(r0);
    for (uint64_t t0 = r0; t0 < r1; t0 += kFanTile) {
        const uint32_t nt = (uint32_t)(r1 - t0 < (uint64_t)kFanTile ? r1 - t0 : kFanTile);
        for (uint32_t x = t; x < kFanWaves * C; x += kFanThreads) wcnt[x / C][x % C] = 0;
        mpx_reply_rec rec[kFanPer];
        uint32_t cl[kFanPer], lr[kFanPer];
#pragma unroll
        for (int k = 0; k < kFanPer; ++k) {
            const uint32_t j = w * kFanSeg + k * kWave + l;
            rec[k] = nxt[k];
            cl[k] = j < nt ? fan_client(rec[k].client, C, err) : 0u;
        }
        if (t0 + kFanTile < r1) load_tile(t0 + kFanTile);
        __syncthreads();
        // stable rank within the wave's segment: lanes with the same client in one round
        // (match over the client bits), rounds in order, per-wave LDS counters
#pragma unroll
        for (int k = 0; k < kFanPer; ++k) {
            const uint32_t j = w * kFanSeg + k * kWave + l;
            const bool v = j < nt;
            uint64_t peers = __ballot(v);
            for (unsigned bit = 0; bit < cbits; ++bit) {
                const uint64_t b = __ballot((cl[k] >> bit) & 1u);
                peers &= ((cl[k] >> bit) & 1u) ? b : ~b;
            }
            const uint32_t before = v ? wcnt[w][cl[k]] : 0u;
            lr[k] = before + (uint32_t)popc(peers & lanes_below(l));
            if (v && (peers & lanes_below(l)) == 0)  // the round's first lane of this client
                wcnt[w][cl[k]] = (uint16_t)(before + popc(peers));
        }
        __syncthreads();
        // per client: the waves' exclusive prefixes and the tile count
        for (uint32_t c = t; c < C; c += kFanThreads) {
            uint32_t run = 0;
#pragma unroll
            for (int x = 0; x < kFanWaves; ++x) {
                const uint32_t k = wcnt[x][c];
                wcnt[x][c] = (uint16_t)run;
                run += k;
            }
            tcnt[c] = run;
            tstart[c] = run;
        }
        __syncthreads();
        (void)fan_block_scan2(tstart, tcnt, C, wsum);  // tcnt scanned too; restored below
        for (uint32_t c = t; c < C; c += kFanThreads)
            tcnt[c] = (c + 1 < C ? tstart[c + 1] : nt) - tstart[c];
        __syncthreads();
        // encode into the tile image at the reply's client-sorted position
#pragma unroll
        for (int k = 0; k < kFanPer; ++k) {
            const uint32_t j = w * kFanSeg + k * kWave + l;
            if (j >= nt) continue;
            const uint32_t pos = tstart[cl[k]] + wcnt[w][cl[k]] + lr[k];
            sc[pos] = (uint16_t)cl[k];
            if (pos == tstart[cl[k]]) carry_in[cl[k]] = carry[cl[k]];  // before any update
            if (MPX_FAN_ABLATE & 2) continue;
            // OK u8, CommandId i32, Value i64, Timestamp i64, Leader i32 (little endian)
            const uint32_t cid = (uint32_t)rec[k].command_id, ld = (uint32_t)leader;
            const uint64_t v = (uint64_t)rec[k].value, ts = (uint64_t)rec[k].timestamp;
            uint32_t* d = img + pos * kSlotWords;
            d[0] = (uint32_t)ok | (cid << 8);
            d[1] = (cid >> 24) | ((uint32_t)v << 8);
            d[2] = (uint32_t)(v >> 24);
            d[3] = (uint32_t)(v >> 56) | ((uint32_t)ts << 8);
            d[4] = (uint32_t)(ts >> 24);
            d[5] = (uint32_t)(ts >> 56) | (ld << 8);
            d[6] = ld >> 24;
        }
        __syncthreads();
        // write-out by image position s: the reply's output bytes [d, d+25) own every aligned
        // output dword that starts inside them (bytes past 25 come from the next reply of the
        // run); the dword running past the end of the client's run goes to the carry, and the
        // first reply of a run completes the dword the carry started (or, at the slice's start,
        // stores its head bytes one by one)
#pragma unroll MPX_FAN_UNROLL
        for (uint32_t s = t; s < ((MPX_FAN_ABLATE & 1) ? 0u : nt); s += kFanThreads) {
            const uint32_t c = sc[s];
            const uint32_t S = tstart[c];                        // run's first image slot
            const uint64_t d = ((uint64_t)base[c] + (s - S)) * kRecBytes;  // output offset
            const uint32_t rem = (tcnt[c] - (s - S)) * kRecBytes;  // bytes from d to the run end
            const uint32_t head = (4u - (uint32_t)((d + out_mis) & 3u)) & 3u;
            uint8_t* const od = out + d;
            // B = the reply's 25 bytes then 7 bytes of the next slot (pad when s is last)
            uint32_t B[8];
            const uint32_t* r = img + s * kSlotWords;
#pragma unroll
            for (int q = 0; q < 6; ++q) B[q] = r[q];
            const uint32_t n0 = r[kSlotWords], n1 = r[kSlotWords + 1];
            B[6] = (r[6] & 0xFFu) | (n0 << 8);
            B[7] = (n0 >> 24) | (n1 << 8);
            if (s == S && head) {
                const uint32_t cin = carry_in[c];
                if (cin >> 31) {  // carry bytes [d-(4-head), d) + the first head bytes
                    const uint32_t pre = 4 - head;
                    const uint32_t v = (cin & ((1u << (8 * pre)) - 1u)) | (B[0] << (8 * pre));
                    *reinterpret_cast<uint32_t*>(od - pre) = v;
                } else {
                    for (uint32_t q = 0; q < head; ++q) od[q] = (uint8_t)(B[0] >> (8 * q));
                }
            }
#pragma unroll
            for (uint32_t q = 0; q < 7; ++q) {
                const uint32_t o = head + 4 * q;  // output dword at d + o (aligned)
                if (o >= (uint32_t)kRecBytes) break;
                const uint32_t v = __builtin_amdgcn_alignbyte(B[q + 1], B[q], head);
                if (o + 4 <= rem) {
                    if (!(MPX_FAN_ABLATE & 8)) *reinterpret_cast<uint32_t*>(od + o) = v;
                } else if (o < rem) {  // the run's last reply: its partial dword waits
                    const uint32_t nb = rem - o;
                    carry[c] = 0x80000000u | (v & ((1u << (8 * nb)) - 1u));
                }
            }
            if (rem == (uint32_t)kRecBytes && ((d + kRecBytes + out_mis) & 3u) == 0)
                carry[c] = 0x80000000u;
        }
        __syncthreads();
        for (uint32_t c = t; c < C; c += kFanThreads) base[c] += tcnt[c];
        // (the next tile's first barrier orders these updates before their readers)
    }
    __syncthreads();
    // the slice's end: every client's pending partial dword, bytewise (the next slice's first
    // run of that client writes the rest of the dword the same way)
    for (uint32_t c = t; c < C; c += kFanThreads) {
        const uint32_t cv = carry[c];
        const uint64_t end = (uint64_t)base[c] * kRecBytes;
        const uint32_t nb = (uint32_t)((end + out_mis) & 3u);
        if ((cv >> 31) && nb)
            for (uint32_t b = 0; b < nb; ++b) out[end - nb + b] = (uint8_t)(cv >> (8 * b));
    }
}

uint64_t fanout_work_bytes(uint64_t n) {
    const uint64_t m = n ? n : 1;
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t radix = 4 * al(m * 4) + al(radix_scratch_bytes<uint32_t, uint32_t>(m));
    const uint64_t h = (uint64_t)kFanMaxClients * fan_plan(m).slices;
    const uint64_t counting = 2 * al(h * 4) + al(scan_scratch_bytes<uint32_t>(h));
    return radix > counting ? radix : counting;
}

hipError_t launch_encode_replies(const mpx_reply_rec* recs, uint64_t n, uint32_t n_clients,
                                 uint8_t ok, int32_t leader, uint8_t* out, uint64_t* client_off,
                                 void* work, uint64_t work_bytes, uint32_t* err,
                                 hipStream_t stream) {
    if (!n_clients || n >= (1ull << 32)) return hipErrorInvalidValue;
    if (work_bytes < fanout_work_bytes(n)) return hipErrorInvalidValue;
    if (n == 0) {
        k_fan_empty<<<1, 256, 0, stream>>>(client_off, n_clients);
        return hipGetLastError();
    }
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    char* w = (char*)work;
    if (n_clients <= kFanMaxClients) {
        const FanPlan p = fan_plan(n);
        const uint64_t h = (uint64_t)n_clients * p.slices;
        uint32_t* hist = (uint32_t*)w;
        uint32_t* first = (uint32_t*)(w + al(h * 4));
        uint32_t* tmp = (uint32_t*)(w + 2 * al(h * 4));
        k_fan_count<<<p.slices, kFanThreads, 0, stream>>>(recs, n, p.per_slice, n_clients,
                                                          p.slices, hist, err);
        const hipError_t r = device_scan(HistIn{hist}, FirstOut{first}, h, ScanSum32{}, 0u, tmp,
                                         stream);
        if (r != hipSuccess) return r;
        k_fan_scatter<<<p.slices, kFanThreads, 0, stream>>>(recs, n, p.per_slice, n_clients,
                                                            p.slices, first, ok, leader, out,
                                                            client_off, err);
        return hipGetLastError();
    }
    uint32_t* skeys = (uint32_t*)w;
    uint32_t* perm = (uint32_t*)(w + al(n * 4));
    uint32_t* keys_in = (uint32_t*)(w + 2 * al(n * 4));
    uint32_t* idx_in = (uint32_t*)(w + 3 * al(n * 4));
    void* tmp = w + 4 * al(n * 4);
    const uint64_t tmp_bytes = work_bytes - 4 * al(n * 4);
    k_fan_keys<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(recs, n, keys_in, idx_in);
    const hipError_t r = radix_sort(keys_in, skeys, idx_in, perm, n, 0u,
                                    bits_for_clients(n_clients), tmp, tmp_bytes, stream);
    if (r != hipSuccess) return r;
    const unsigned blocks = (unsigned)((n + kFanBlock - 1) / kFanBlock);
    if (((uintptr_t)out & 15) == 0)
        k_fan_encode<true><<<blocks, kFanBlock, 0, stream>>>(recs, skeys, perm, n, n_clients, ok,
                                                             leader, out, client_off, err);
    else
        k_fan_encode<false><<<blocks, kFanBlock, 0, stream>>>(recs, skeys, perm, n, n_clients, ok,
                                                              leader, out, client_off, err);
    return hipGetLastError();
}

}  // namespace mpx
