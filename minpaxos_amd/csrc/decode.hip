// decode.hip — batched peer-stream framing + AcceptReply decode.
//
// Reference: genericsmr.(*Replica).replicaListener  src/genericsmr/genericsmr.go:402-446 reads
// one peer connection as a sequence of frames [code u8][body]: GENERIC_SMR_BEACON (6) and
// GENERIC_SMR_BEACON_REPLY (7) carry an 8-byte timestamp; codes 8..13 are the RPCs registered by
// bareminpaxos.NewReplica (bareminpaxos.go:108-113; rpcCode starts at
// GENERIC_SMR_BEACON_REPLY+1, genericsmr.go:92): Prepare (12-byte body,
// minpaxosprotomarsh.go:259-270), Accept (variable, :470-507), Commit (variable, :648-672),
// CommitShort (16, :737-749), PrepareReply (variable, :352-387), AcceptReply (13, :545-580).
// Any other code is logged and skipped (genericsmr.go:440-442), so it is a 1-byte frame.
// AcceptReply bodies decode into mpx_accept_reply (Instance, OK, Ballot, Id; little endian);
// every other fixed-size frame is reported as (offset, code) for the host. Framing stops at the
// first variable-length frame (the host parses it and calls again past it) or at a frame that
// runs past the end of the buffer (a partial read: the host keeps the tail).
//
// Framing is sequential by nature (each frame's start depends on every earlier length). The
// engine makes it data parallel with entry maps: a frame that starts in a 128-byte chunk ends at
// most 16 bytes into the next one (the longest fixed frame is 17 bytes), so a chunk's behaviour
// is a function from its entry offset (0..16) to (exit offset into the next chunk | stop
// position, AcceptReplies and other frames passed on the way). Each lane computes its chunk's
// 17-entry map with a register-window DP over the chunk's bytes (the possible lengths are 1, 9,
// 13, 14 and 17, so the DP only looks back at fixed distances). Maps compose associatively: a
// workgroup reduces its 128 chunk maps to a 16 KB tile map (tree in LDS), 256 tile maps reduce
// to a group map, one block walks the group maps from entry 0, and the down-sweeps hand every
// tile, then every chunk, its true entry and output offsets; the chunks then emit their records.
// HBM traffic: the stream is read twice (maps, emit), the records written once; the maps are
// 204 bytes per 16 KB tile plus a 16-byte exit map per 128-byte chunk, which the emit pass reads
// instead of recomputing the DP.
#include "common.hpp"
#include "kernels.hpp"

#ifndef MPX_DEC_DBL_TREE  // timing probe build: the tile tree computed twice
#define MPX_DEC_DBL_TREE 0
#endif

namespace mpx {

namespace {

constexpr int kChunk = 128;                // bytes per lane
constexpr int kTileLanes = 128;            // lanes per tile workgroup
constexpr int kTileBytes = kChunk * kTileLanes;
constexpr int kEntries = 17;               // entry offsets 0..16
constexpr int kGroupTiles = 256;           // tile maps per group
constexpr uint32_t kDead = 0xFFFFFFFFu;    // tile / chunk past the stop of the frame chain

// frame length by code, code byte included (0 = variable-length frame: stop); codes 6..13 from
// a byte-lane table, everything else is a 1-byte unknown frame
constexpr uint64_t kLenLut = 9ull | (9ull << 8) | (13ull << 16) | (0ull << 24) | (0ull << 32) |
                             (17ull << 40) | (0ull << 48) | (14ull << 56);
__device__ __forceinline__ uint32_t frame_len(uint32_t code) {
    const uint32_t i = code - (uint32_t)MPX_PEER_BEACON;
    const uint32_t in = 0u - (uint32_t)(i < 8u);
    return (((uint32_t)(kLenLut >> ((i & 7u) * 8u)) & 0xFFu) & in) | (1u & ~in);
}
static_assert(MPX_PEER_BEACON == 6 && MPX_PEER_BEACON_REPLY == 7 && MPX_PEER_PREPARE == 8 &&
                  MPX_PEER_ACCEPT == 9 && MPX_PEER_COMMIT == 10 && MPX_PEER_COMMIT_SHORT == 11 &&
                  MPX_PEER_PREPARE_REPLY == 12 && MPX_PEER_ACCEPT_REPLY == 13,
              "kLenLut is laid out for codes 6..13");

// lane-map entry (u32): [0..6] pos (exit offset into the next chunk, or stop offset in the
// chunk), [7] stop, [8..11] AcceptReplies (<= 128/14), [12..19] other frames (<= 128)
constexpr uint32_t kLStop = 1u << 7;
__device__ __forceinline__ uint32_t l_pos(uint32_t x) { return x & 0x7Fu; }
__device__ __forceinline__ uint32_t l_ar(uint32_t x) { return (x >> 8) & 0xFu; }
__device__ __forceinline__ uint32_t l_oth(uint32_t x) { return (x >> 12) & 0xFFu; }
static_assert(kChunk <= 128, "lane-map fields are sized for 128-byte chunks");

// tile-level entry (u64): [0..15] pos (exit offset, or stop offset from the tile start),
// [16] stop, [17..32] AcceptReplies, [33..48] other frames
constexpr uint64_t kTStop = 1ull << 16;
__device__ __forceinline__ uint64_t t_make(uint32_t pos, bool stop, uint32_t ar, uint32_t oth) {
    return (uint64_t)pos | (stop ? kTStop : 0ull) | ((uint64_t)ar << 17) | ((uint64_t)oth << 33);
}
__device__ __forceinline__ uint32_t t_pos(uint64_t x) { return (uint32_t)x & 0xFFFFu; }
__device__ __forceinline__ bool t_stop(uint64_t x) { return (x & kTStop) != 0; }
__device__ __forceinline__ uint32_t t_ar(uint64_t x) { return (uint32_t)(x >> 17) & 0xFFFFu; }
__device__ __forceinline__ uint32_t t_oth(uint64_t x) { return (uint32_t)(x >> 33) & 0xFFFFu; }
// a, then the map b of the chunks right after a's
__device__ __forceinline__ uint64_t t_compose(uint64_t a, const uint64_t* b) {
    if (t_stop(a)) return a;
    const uint64_t y = b[t_pos(a)];
    return (y & 0x1FFFFull) | ((uint64_t)(t_ar(a) + t_ar(y)) << 17) |
           ((uint64_t)(t_oth(a) + t_oth(y)) << 33);
}

// The lane's chunk -> its 17 map entries (w[k] = entry k) by a backward DP over the
// chunk's positions: dp[p] = frame p reaches past the chunk ? exit : dp[p + len(p)] + frame p.
// Before step p the window holds w[k] = dp[p+1+k]; the lengths are compile-time offsets into it.
// kEdge: the chunk ends within 17 bytes of the end of the buffer, so positions past the end and
// frames running past it must be checked (every other chunk skips both tests).
template <bool kEdge>
__device__ __forceinline__ void lane_map_dp(const uint32_t (&wd)[kChunk / 4], uint32_t c0,
                                            uint32_t len,
                                            uint32_t (&w)[kEntries]) {
#pragma unroll
    for (int k = 0; k < kEntries; ++k) w[k] = 0;
#pragma unroll
    for (int p = kChunk - 1; p >= 0; --p) {
        // branch-free: every select below is a mask, so the unrolled loop stays straight-line
        // code and the window shift is pure register renaming
        const uint32_t code = (wd[p >> 2] >> ((p & 3) * 8)) & 0xFFu;
        const uint32_t fl = frame_len(code);
        uint32_t stop = (uint32_t)(fl == 0);
        if (kEdge) stop |= (uint32_t)(c0 + (uint32_t)p >= len) | (uint32_t)(c0 + (uint32_t)p + fl > len);
        const uint32_t inc = (1u << 12) - (uint32_t)(code == MPX_PEER_ACCEPT_REPLY) * ((1u << 12) - (1u << 8));
        uint32_t nx = (w[13] & (0u - (uint32_t)(fl == 14))) | (w[8] & (0u - (uint32_t)(fl == 9))) |
                      (w[12] & (0u - (uint32_t)(fl == 13))) | (w[16] & (0u - (uint32_t)(fl == 17))) |
                      (w[0] & (0u - (uint32_t)(fl == 1)));
        if (p + 17 > kChunk) {  // compile time: only the last 17 positions can leave the chunk
            const uint32_t out = 0u - (uint32_t)((uint32_t)p + fl >= (uint32_t)kChunk);
            nx = (nx & ~out) | (((uint32_t)p + fl - kChunk) & out);
        }
        const uint32_t sm = 0u - stop;
        const uint32_t d = (((uint32_t)p | kLStop) & sm) | ((nx + inc) & ~sm);
#pragma unroll
        for (int k = kEntries - 1; k > 0; --k) w[k] = w[k - 1];
        w[0] = d;
    }
}

__device__ __forceinline__ void lane_map(const uint32_t (&wd)[kChunk / 4], uint64_t c0,
                                         uint64_t len,
                                         uint32_t (&w)[kEntries]) {
    if (c0 + kChunk + kEntries > len) lane_map_dp<true>(wd, (uint32_t)c0, (uint32_t)len, w);
    else lane_map_dp<false>(wd, (uint32_t)c0, (uint32_t)len, w);
}

__device__ __forceinline__ void load_chunk(const uint8_t* __restrict__ buf, uint64_t len,
                                           uint64_t c0, uint32_t (&wd)[kChunk / 4]) {
    if (c0 + kChunk <= len) {
        const uint4* s = reinterpret_cast<const uint4*>(buf + c0);
#pragma unroll
        for (int i = 0; i < kChunk / 16; ++i) {
            const uint4 v = s[i];  // default policy: the emit pass reads the stream again
            wd[4 * i] = v.x;
            wd[4 * i + 1] = v.y;
            wd[4 * i + 2] = v.z;
            wd[4 * i + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kChunk / 4; ++i) {
            uint32_t x = 0;
            for (int b = 0; b < 4; ++b) {
                const uint64_t a = c0 + 4 * i + b;
                if (a < len) x |= (uint32_t)buf[a] << (8 * b);
            }
            wd[i] = x;
        }
    }
}

__device__ __forceinline__ int level_base(int k) { return 2 * kTileLanes - (2 * kTileLanes >> k); }
constexpr int kLevels = 7;  // log2(kTileLanes)

// The reduction of a tile's 128 lane maps to the tile map, in place over one level of storage
// (the map kernel needs only the root; the emit pass keeps its own tree of exit offsets): level
// k's row j = compose(row 2j, row 2j+1) of level k-1, every task of a level computed into
// registers before any row is overwritten. 17 KB of LDS instead of a whole tree's 35 KB: five
// waves per SIMD instead of two (1.66 -> 1.44 ms per config-2-sized stream).
struct TileRow {
    uint64_t m[kTileLanes][kEntries];
};
__device__ void tile_reduce(TileRow& T, const uint32_t (&w)[kEntries]) {
    const int l = threadIdx.x;
#pragma unroll
    for (int e = 0; e < kEntries; ++e) {
        const uint32_t x = w[e];
        const bool st = (x & kLStop) != 0;
        const uint32_t pos = st ? (uint32_t)(l * kChunk) + l_pos(x) : l_pos(x);
        T.m[l][e] = t_make(pos, st, l_ar(x), l_oth(x));
    }
    __syncthreads();
    constexpr int kMaxTasks = (kTileLanes / 2 * kEntries + kTileLanes - 1) / kTileLanes;
#pragma unroll
    for (int k = 1; k <= kLevels; ++k) {
        const int total = (kTileLanes >> k) * kEntries;
        uint64_t r[kMaxTasks];
#pragma unroll
        for (int i = 0; i < kMaxTasks; ++i) {
            const int t = l + i * kTileLanes;
            if (t < total) {
                const int j = t / kEntries;
                r[i] = t_compose(T.m[2 * j][t % kEntries], T.m[2 * j + 1]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kMaxTasks; ++i) {
            const int t = l + i * kTileLanes;
            if (t < total) T.m[t / kEntries][t % kEntries] = r[i];
        }
        __syncthreads();
    }
}

// map entry across tiles: pos (bit 31 = stop: absolute stop position in bits 0..30; else exit
// offset into the next tile), AcceptReplies and other frames passed
struct GEntry {
    uint32_t pos, ar, oth;
};
constexpr uint32_t kGStop = 1u << 31;

}  // namespace

// ---- pass A: tile maps -------------------------------------------------------------------------
// exit map of a chunk for the emit pass: 6 bits per entry (exit offset, or kXStop), entries
// 0..9 in the low 64 bits, 10..16 in the high 64 bits
constexpr uint32_t kXStop = 63u;
__device__ __forceinline__ ulonglong2 pack_exits(const uint32_t (&w)[kEntries]) {
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int e = 0; e < kEntries; ++e) {
        const uint64_t x = (w[e] & kLStop) ? kXStop : l_pos(w[e]);
        if (e < 10) lo |= x << (6 * e);
        else hi |= x << (6 * (e - 10));
    }
    return make_ulonglong2(lo, hi);
}

__global__ __launch_bounds__(kTileLanes) void k_dec_tile_maps(const uint8_t* __restrict__ buf,
                                                              uint64_t len,
                                                              GEntry* __restrict__ tmap,
                                                              ulonglong2* __restrict__ xmap) {
    __shared__ TileRow T;
    const uint64_t t0 = (uint64_t)blockIdx.x * kTileBytes;
    const uint64_t c0 = t0 + (uint64_t)threadIdx.x * kChunk;
    uint32_t wd[kChunk / 4], w[kEntries];
    load_chunk(buf, len, c0, wd);
    lane_map(wd, c0, len, w);
    xmap[(uint64_t)blockIdx.x * kTileLanes + threadIdx.x] = pack_exits(w);
#ifdef MPX_DEC_ABLATE_TREE
    if (threadIdx.x < kEntries) {  // timing ablation only: skips the tile tree (wrong results)
        tmap[(uint64_t)blockIdx.x * kEntries + threadIdx.x] = GEntry{w[threadIdx.x] & 15u, 0, 0};
        return;
    }
    return;
#endif
#if MPX_DEC_DBL_TREE  // timing probe: the tile tree twice (same result)
    tile_reduce(T, w);
    __syncthreads();
#endif
    tile_reduce(T, w);
    if (threadIdx.x < kEntries) {
        const uint64_t x = T.m[0][threadIdx.x];
        GEntry g;
        g.pos = t_stop(x) ? (kGStop | (uint32_t)(t0 + t_pos(x))) : t_pos(x);
        g.ar = t_ar(x);
        g.oth = t_oth(x);
        tmap[(uint64_t)blockIdx.x * kEntries + threadIdx.x] = g;
    }
}

// The map walks of passes B1-B3 follow 256 maps in kDParts parts of 32 side by side: thread
// (q, e) takes entry e through part q (8 x 17 chains of 32 dependent LDS reads instead of 17 of
// 256), one thread chains the 8 part maps from the run's entry, and 8 threads then walk their
// parts from their part's entry where every map's entry is wanted (gres, tres).
constexpr int kDParts = 8;
constexpr uint32_t kDPer = kGroupTiles / kDParts;
__device__ __forceinline__ void dec_part_maps(const GEntry (*S)[kEntries], uint32_t n,
                                              GEntry (*Q)[kEntries]) {
    const uint32_t t = threadIdx.x;
    if (t < (uint32_t)(kDParts * kEntries)) {
        const uint32_t q = t / kEntries, e = t % kEntries;
        const uint32_t t0 = q * kDPer, t1 = min(t0 + kDPer, n);
        GEntry a{e, 0, 0};
        for (uint32_t k = t0; k < t1 && !(a.pos & kGStop); ++k) {
            const GEntry y = S[k][a.pos];
            a = GEntry{y.pos, a.ar + y.ar, a.oth + y.oth};
        }
        Q[q][e] = a;
    }
}
// thread 0: the parts' entries from the run's entry r (pos kDead: past the stop); returns the
// state after the run ({pos, ar, oth} with pos = kGStop | stop position once stopped)
__device__ __forceinline__ GEntry dec_part_entries(const GEntry (*Q)[kEntries], GEntry r, GEntry* PE) {
    for (int q = 0; q < kDParts; ++q) {
        PE[q] = (r.pos & kGStop) ? GEntry{kDead, r.ar, r.oth} : r;
        if (!(r.pos & kGStop)) {
            const GEntry y = Q[q][r.pos];
            r = GEntry{y.pos, r.ar + y.ar, r.oth + y.oth};
        }
    }
    return r;
}
// threads q < kDParts: part q's maps from its entry, out[k] = {entry, ar, oth before map k}
// (kDead entries past the stop)
__device__ __forceinline__ void dec_part_walk(const GEntry (*S)[kEntries], uint32_t n,
                                              const GEntry* PE, GEntry* out, bool keep_counts) {
    const uint32_t q = threadIdx.x;
    if (q >= (uint32_t)kDParts) return;
    const uint32_t t0 = q * kDPer, t1 = min(t0 + kDPer, n);
    uint32_t e = PE[q].pos, ar = PE[q].ar, oth = PE[q].oth;
    bool dead = e == kDead;
    for (uint32_t k = t0; k < t1; ++k) {
        if (dead) {
            out[k] = keep_counts ? GEntry{kDead, ar, oth} : GEntry{kDead, 0, 0};
            continue;
        }
        out[k] = GEntry{e, ar, oth};
        const GEntry x = S[k][e];
        ar += x.ar;
        oth += x.oth;
        if (x.pos & kGStop) dead = true;
        else e = x.pos;
    }
}

// ---- pass B1: group maps (a group = 256 consecutive tiles) ----------------------------------
__global__ __launch_bounds__(256) void k_dec_group_maps(const GEntry* __restrict__ tmap,
                                                        uint32_t n_tiles,
                                                        GEntry* __restrict__ gmap) {
    __shared__ GEntry S[kGroupTiles][kEntries];
    __shared__ GEntry Q[kDParts][kEntries];
    const uint32_t g = blockIdx.x, first = g * kGroupTiles;
    const uint32_t nt = min((uint32_t)kGroupTiles, n_tiles - first);
    for (uint32_t i = threadIdx.x; i < nt * kEntries; i += blockDim.x)
        (&S[0][0])[i] = tmap[(uint64_t)first * kEntries + i];
    __syncthreads();
    dec_part_maps(S, nt, Q);
    __syncthreads();
    if (threadIdx.x < kEntries) {
        GEntry a{threadIdx.x, 0, 0};
#pragma unroll
        for (int q = 0; q < kDParts; ++q)
            if (!(a.pos & kGStop)) {
                const GEntry y = Q[q][a.pos];
                a = GEntry{y.pos, a.ar + y.ar, a.oth + y.oth};
            }
        gmap[(uint64_t)g * kEntries + threadIdx.x] = a;
    }
}

// ---- pass B2: the true chain through the group maps from entry 0 (one block; the maps are
// staged in LDS 256 groups at a time, followed in parts) --------------------------------------
// gres[g] = {entry of group g (kDead past the stop), AcceptReplies before it, others before it}
__global__ __launch_bounds__(256) void k_dec_walk(const GEntry* __restrict__ gmap,
                                                  uint32_t n_groups, uint64_t len,
                                                  const uint8_t* __restrict__ buf,
                                                  GEntry* __restrict__ gres,
                                                  mpx_decode_result* __restrict__ res) {
    __shared__ GEntry S[kGroupTiles][kEntries];
    __shared__ GEntry Q[kDParts][kEntries];
    __shared__ GEntry PE[kDParts];
    __shared__ GEntry cur;  // the chain's state before the batch: {entry | kGStop stop, ar, oth}
    if (threadIdx.x == 0) cur = GEntry{0, 0, 0};
    for (uint32_t b0 = 0; b0 < n_groups; b0 += kGroupTiles) {
        const uint32_t nb = min((uint32_t)kGroupTiles, n_groups - b0);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nb * kEntries; i += blockDim.x)
            (&S[0][0])[i] = gmap[(uint64_t)b0 * kEntries + i];
        __syncthreads();
        dec_part_maps(S, nb, Q);
        __syncthreads();
        if (threadIdx.x == 0) cur = dec_part_entries(Q, cur, PE);
        __syncthreads();
        dec_part_walk(S, nb, PE, gres + b0, true);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // the chain always stops inside the last tile at the latest (position len)
        const uint64_t stop = (cur.pos & kGStop) ? (uint64_t)(cur.pos & ~kGStop) : len;
        res->consumed = stop;
        res->n_accept_replies = cur.ar;
        res->n_other = cur.oth;
        int32_t why = MPX_DECODE_END, code = -1;
        if (stop < len) {
            code = buf[stop];
            why = frame_len((uint32_t)code) == 0 ? MPX_DECODE_VARIABLE : MPX_DECODE_PARTIAL;
        }
        res->stop_reason = why;
        res->stop_code = code;
    }
}

// ---- pass B3: tile entries inside each group (the group's tile maps followed in parts) -------
__global__ __launch_bounds__(256) void k_dec_tile_entries(const GEntry* __restrict__ tmap,
                                                          uint32_t n_tiles,
                                                          const GEntry* __restrict__ gres,
                                                          GEntry* __restrict__ tres) {
    __shared__ GEntry S[kGroupTiles][kEntries];
    __shared__ GEntry Q[kDParts][kEntries];
    __shared__ GEntry PE[kDParts];
    const uint32_t g = blockIdx.x, first = g * kGroupTiles;
    const uint32_t nt = min((uint32_t)kGroupTiles, n_tiles - first);
    const GEntry r = gres[g];
    if (r.pos == kDead) {
        for (uint32_t t = threadIdx.x; t < nt; t += blockDim.x) tres[first + t] = GEntry{kDead, 0, 0};
        return;
    }
    for (uint32_t i = threadIdx.x; i < nt * kEntries; i += blockDim.x)
        (&S[0][0])[i] = tmap[(uint64_t)first * kEntries + i];
    __syncthreads();
    dec_part_maps(S, nt, Q);
    __syncthreads();
    if (threadIdx.x == 0) dec_part_entries(Q, r, PE);
    __syncthreads();
    dec_part_walk(S, nt, PE, tres + first, false);
}

// ---- pass C: chunk entries (tree over the stored exit maps) and record emission -------------
// The tile's bytes are staged in LDS; the true chain is walked per chunk twice (count, then
// emit at the offsets of a block-wide exclusive scan of the counts).
constexpr int kXPad = 20;  // bytes per exit map in LDS (17 used)
#ifndef MPX_DEC_EMIT_REG
#define MPX_DEC_EMIT_REG 1
#endif
constexpr int kDecRegAR = 10;          // a 128-byte chunk starts at most 10 AcceptReply frames
constexpr uint32_t kDecRegCap = 1024;  // staged records per LDS pass (the tile image's space)
// The staged tile image: 4 pad bytes after every 128-byte chunk (MPX_DEC_PAD), so the lanes -
// one per chunk, at similar offsets - read 64 LDS banks instead of two (as the stream emit)
#ifndef MPX_DEC_PAD
#define MPX_DEC_PAD 1
#endif
__device__ __forceinline__ uint32_t dpofs(uint32_t o) { return MPX_DEC_PAD ? o + ((o >> 7) << 2) : o; }
constexpr int kDecImg = kTileBytes + 32 + (MPX_DEC_PAD ? 4 * (kTileLanes + 1) : 0) + 16;
__device__ __forceinline__ void dimg_put(uint8_t* B, int i, const uint4 v) {
    if (MPX_DEC_PAD) {
        uint32_t* w = reinterpret_cast<uint32_t*>(B) + 4 * i + (i >> 3);
        w[0] = v.x;
        w[1] = v.y;
        w[2] = v.z;
        w[3] = v.w;
    } else {
        reinterpret_cast<uint4*>(B)[i] = v;
    }
}
// 4 bytes at tile offset o from two aligned dword reads, each at its image position
__device__ __forceinline__ int32_t lds_le32(const uint8_t* B, uint32_t o) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(B);
    const uint32_t d = o >> 2, sh = o & 3u;
    const uint32_t d0 = MPX_DEC_PAD ? d + (d >> 5) : d, d1 = MPX_DEC_PAD ? d + 1 + ((d + 1) >> 5) : d + 1;
    const uint64_t x = ((uint64_t)w[d1] << 32) | w[d0];
    return (int32_t)(uint32_t)(x >> (8 * sh));
}
__global__ __launch_bounds__(kTileLanes) void k_dec_emit(
    const uint8_t* __restrict__ buf, uint64_t len, const GEntry* __restrict__ tres,
    const ulonglong2* __restrict__ xmap, mpx_accept_reply* __restrict__ ar_out, uint64_t ar_cap,
    mpx_peer_frame* __restrict__ oth_out, uint64_t oth_cap) {
#ifndef MPX_DEC_EMIT_UNION
#define MPX_DEC_EMIT_UNION 1
#endif
    __shared__ uint8_t E[2 * kTileLanes - 1];  // entry per tree node (kXStop = dead)
#if MPX_DEC_EMIT_UNION
    // the exit-map tree is dead once every chunk has its entry: the tile's bytes (loaded into
    // registers meanwhile) take its LDS, 16.7 KB per workgroup instead of 21.8 KB
    constexpr int kVec = ((kTileBytes + 32) / 16 + kTileLanes - 1) / kTileLanes;
    static_assert((2 * kTileLanes - 1) * kXPad <= kTileBytes + 32, "the tree fits the tile image");
    __shared__ __attribute__((aligned(16))) uint8_t B[kDecImg];
    uint8_t(*const X)[kXPad] = reinterpret_cast<uint8_t(*)[kXPad]>(B);
#else
    __shared__ uint8_t X[2 * kTileLanes - 1][kXPad];
    __shared__ __attribute__((aligned(16))) uint8_t B[kDecImg];
#endif
    __shared__ uint32_t wsum[kTileLanes / kWave];
    const GEntry r = tres[blockIdx.x];
    if (r.pos == kDead) return;  // uniform per block
    const uint64_t t0 = (uint64_t)blockIdx.x * kTileBytes;
    const int l = threadIdx.x;
    // stage the tile (+32 bytes of the next) in LDS (with the union: into registers now, into
    // LDS after the down-sweep)
    auto tile_vec = [&](int i) {
        const uint64_t a = t0 + (uint64_t)i * 16;
        uint4 v;
        if (a + 16 <= len) {
            v = *reinterpret_cast<const uint4*>(buf + a);
        } else {
            uint32_t q[4] = {0, 0, 0, 0};
            for (int b = 0; b < 16; ++b)
                if (a + b < len) q[b >> 2] |= (uint32_t)buf[a + b] << (8 * (b & 3));
            v = make_uint4(q[0], q[1], q[2], q[3]);
        }
        return v;
    };
#if MPX_DEC_EMIT_UNION
    uint4 tv[kVec];
    if (t0 + (uint64_t)kVec * kTileLanes * 16 <= len) {
        // interior tile (block-uniform): every load in flight together, no per-load branch
        // (whose join waited out each load in turn); lanes past the window reload its last
        // vector, which the stores below skip
        const uint4* src = reinterpret_cast<const uint4*>(buf + t0);
#pragma unroll
        for (int k = 0; k < kVec; ++k) tv[k] = src[min(l + k * kTileLanes, (kTileBytes + 32) / 16 - 1)];
    } else {
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int i = l + k * kTileLanes;
            tv[k] = i < (kTileBytes + 32) / 16 ? tile_vec(i) : make_uint4(0, 0, 0, 0);
        }
    }
#else
    for (int i = l; i < (kTileBytes + 32) / 16; i += kTileLanes)
        dimg_put(B, i, tile_vec(i));
#endif
    {
        const ulonglong2 m = xmap[(uint64_t)blockIdx.x * kTileLanes + l];
#pragma unroll
        for (int e = 0; e < kEntries; ++e)
            X[l][e] = (uint8_t)((e < 10 ? m.x >> (6 * e) : m.y >> (6 * (e - 10))) & 63u);
    }
    __syncthreads();
    for (int k = 1; k <= kLevels; ++k) {
        const int nodes = kTileLanes >> k;
        const int src = level_base(k - 1), dst = level_base(k);
        for (int t = l; t < nodes * kEntries; t += kTileLanes) {
            const int j = t / kEntries, e = t % kEntries;
            const uint8_t a = X[src + 2 * j][e];
            X[dst + j][e] = a == kXStop ? (uint8_t)kXStop : X[src + 2 * j + 1][a];
        }
        __syncthreads();
    }
    if (l == 0) E[level_base(kLevels)] = (uint8_t)r.pos;
    __syncthreads();
    for (int k = kLevels; k >= 1; --k) {
        const int nodes = kTileLanes >> k;
        const int src = level_base(k), dst = level_base(k - 1);
        if (l < nodes) {
            const uint8_t e = E[src + l];
            E[dst + 2 * l] = e;
            E[dst + 2 * l + 1] = e == kXStop ? (uint8_t)kXStop : X[dst + 2 * l][e];
        }
        __syncthreads();
    }
    const uint32_t e = E[l];
#if MPX_DEC_EMIT_UNION
    __syncthreads();  // every lane has read its tree nodes: the tile's bytes take the tree's LDS
#pragma unroll
    for (int k = 0; k < kVec; ++k) {
        const int i = l + k * kTileLanes;
        if (i < (kTileBytes + 32) / 16) dimg_put(B, i, tv[k]);
    }
    __syncthreads();
#endif
    // walk 1: frames starting in this chunk on the true chain
    const uint32_t base = (uint32_t)l * kChunk;  // chunk start within the tile
    const uint64_t tl = len - t0;               // bytes of the buffer from the tile start
    uint32_t n_ar = 0, n_oth = 0;
    if (e != kXStop) {
        for (uint32_t p = base + e; p < base + kChunk;) {
            const uint32_t code = B[dpofs(p)];
            const uint32_t fl = frame_len(code);
            if ((uint64_t)p >= tl || fl == 0 || (uint64_t)p + fl > tl) break;
            if (code == MPX_PEER_ACCEPT_REPLY) ++n_ar;
            else ++n_oth;
            p += fl;
        }
    }
    // block exclusive scan of (n_ar | n_oth << 16)
    uint32_t v = n_ar | (n_oth << 16), inc = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d);
        if (lane_id() >= d) inc += t;
    }
    if (lane_id() == kWave - 1) wsum[l / kWave] = inc;
    __syncthreads();
    uint32_t pre = inc - v;
    for (int w2 = 0; w2 < l / kWave; ++w2) pre += wsum[w2];
    uint64_t ar_i = r.ar + (pre & 0xFFFFu), oth_i = r.oth + (pre >> 16);
    // walk 2, one frame at p: an AcceptReply comes back in rec (is_ar), any other frame is stored
    // here; live = false after the chunk's last frame
    auto frame = [&](uint32_t& p, bool& live, bool& is_ar, uint4& rec) {
        is_ar = false;
        const uint32_t code = B[dpofs(p)];
        const uint32_t fl = frame_len(code);
        if ((uint64_t)p >= tl || fl == 0 || (uint64_t)p + fl > tl) {
            live = false;
            return;
        }
        if (code == MPX_PEER_ACCEPT_REPLY) {  // Instance, OK, Ballot, Id (little endian)
            rec = make_uint4((uint32_t)lds_le32(B, p + 1), (uint32_t)lds_le32(B, p + 6),
                             (uint32_t)lds_le32(B, p + 10), (uint32_t)B[dpofs(p + 5)]);
            is_ar = true;
        } else {
            if (oth_i < oth_cap) {
                mpx_peer_frame f;
                f.offset = (uint32_t)(t0 + p);
                f.code = (uint8_t)code;
                f.pad[0] = f.pad[1] = f.pad[2] = 0;
                oth_out[oth_i] = f;
            }
            ++oth_i;
        }
        p += fl;
        live = p < base + kChunk;
    };
    uint4* const ar4 = reinterpret_cast<uint4*>(ar_out);  // mpx_accept_reply as 4 dwords
    uint32_t p = base + e;
    bool live = e != kXStop;
    bool is_ar;
    uint4 rec;
#if MPX_DEC_EMIT_REG
    // the first kDecRegAR frames with their AcceptReplies in registers, then (the tile image dead)
    // through LDS, so the tile's AcceptReplies leave as coalesced runs (stream.hip k_sd_emit)
    uint32_t tot_ar = 0;
    for (int w2 = 0; w2 < kTileLanes / kWave; ++w2) tot_ar += wsum[w2] & 0xFFFFu;
    const uint64_t ar0 = r.ar;
    uint4 rr[kDecRegAR];
    uint32_t rl[kDecRegAR];  // tile-local index, ~0 = none
#pragma clang loop unroll(full)
    for (int it = 0; it < kDecRegAR; ++it) {
        rl[it] = ~0u;
        if (live) {
            frame(p, live, is_ar, rec);
            if (is_ar) {
                rr[it] = rec;
                rl[it] = ar_i < ar_cap ? (uint32_t)(ar_i - ar0) : ~0u;
                ++ar_i;
            }
        }
    }
    if (__syncthreads_or(live)) {  // a chunk with more frames: every record stored directly
#pragma unroll
        for (int it = 0; it < kDecRegAR; ++it)
            if (rl[it] != ~0u) ar4[ar0 + rl[it]] = rr[it];
        while (live) {
            frame(p, live, is_ar, rec);
            if (is_ar) {
                if (ar_i < ar_cap) ar4[ar_i] = rec;
                ++ar_i;
            }
        }
        return;
    }
    uint4* const R = reinterpret_cast<uint4*>(B);
    for (uint32_t ph = 0; ph < tot_ar; ph += kDecRegCap) {
#pragma unroll
        for (int it = 0; it < kDecRegAR; ++it)
            if (rl[it] - ph < kDecRegCap) R[rl[it] - ph] = rr[it];
        __syncthreads();
        const uint32_t hi = tot_ar - ph < kDecRegCap ? tot_ar : ph + kDecRegCap;
        for (uint32_t i = ph + (uint32_t)l; i < hi; i += kTileLanes)
            if (ar0 + i < ar_cap) ar4[ar0 + i] = R[i - ph];
        __syncthreads();
    }
#else
    while (live) {
        frame(p, live, is_ar, rec);
        if (is_ar) {
            if (ar_i < ar_cap) ar4[ar_i] = rec;
            ++ar_i;
        }
    }
#endif
}

__global__ void k_dec_empty(mpx_decode_result* res) {
    res->consumed = 0;
    res->n_accept_replies = 0;
    res->n_other = 0;
    res->stop_reason = MPX_DECODE_END;
    res->stop_code = -1;
}

uint64_t decode_work_bytes(uint64_t len) {
    const uint64_t tiles = (len + kTileBytes - 1) / kTileBytes;
    const uint64_t groups = (tiles + kGroupTiles - 1) / kGroupTiles;
    return (tiles * (kEntries + 1) + groups * (kEntries + 1)) * sizeof(GEntry) +
           tiles * kTileLanes * sizeof(ulonglong2) + 256;
}

hipError_t launch_decode_peer_stream(const uint8_t* buf, uint64_t len, mpx_accept_reply* ar_out,
                                     uint64_t ar_cap, mpx_peer_frame* oth_out, uint64_t oth_cap,
                                     mpx_decode_result* res, void* work, uint64_t work_bytes,
                                     hipStream_t stream) {
    if (len > (uint64_t)MPX_DECODE_MAX_BYTES) return hipErrorInvalidValue;
    if (work_bytes < decode_work_bytes(len)) return hipErrorInvalidValue;
    if (len == 0) {
        k_dec_empty<<<1, 1, 0, stream>>>(res);
        return hipGetLastError();
    }
    const uint32_t tiles = (uint32_t)((len + kTileBytes - 1) / kTileBytes);
    const uint32_t groups = (tiles + kGroupTiles - 1) / kGroupTiles;
    GEntry* tmap = (GEntry*)work;
    GEntry* tres = tmap + (uint64_t)tiles * kEntries;
    GEntry* gmap = tres + tiles;
    GEntry* gres = gmap + (uint64_t)groups * kEntries;
    ulonglong2* xmap = (ulonglong2*)(((uintptr_t)(gres + groups) + 15) & ~(uintptr_t)15);
    k_dec_tile_maps<<<tiles, kTileLanes, 0, stream>>>(buf, len, tmap, xmap);
    k_dec_group_maps<<<groups, 256, 0, stream>>>(tmap, tiles, gmap);
    k_dec_walk<<<1, 256, 0, stream>>>(gmap, groups, len, buf, gres, res);
    k_dec_tile_entries<<<groups, 256, 0, stream>>>(tmap, tiles, gres, tres);
    k_dec_emit<<<tiles, kTileLanes, 0, stream>>>(buf, len, tres, xmap, ar_out, ar_cap, oth_out,
                                                 oth_cap);
    return hipGetLastError();
}

}  // namespace mpx
