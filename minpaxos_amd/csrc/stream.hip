// stream.hip — full peer-stream framing: fixed AND variable-length frames, MIN or CLASSIC wire
// (mpx_decode_stream, and mpx_decode_peer_stream as its MIN,
// stop-at-variable special case).
//
// Reference: genericsmr.(*Replica).replicaListener src/genericsmr/genericsmr.go:402-446 reads a
// connection as frames [code u8][body]; the body of a variable-length message (Accept, Commit,
// PrepareReply) is a fixed header, a binary.PutVarint slice length, 17-byte Commands and, for
// MIN Accept / PrepareReply, a CatchUpLog of Instances (8 bytes + V(k) + 17k each)
// (minpaxosprotomarsh.go:126-153, :352-387, :470-507, :648-672; paxosprotomarsh.go:152-176,
// :244-270, :403-430). Layout table in include/mpx.h.
//
// Framing is a chain: each frame's start depends on every earlier length. The engine makes it
// data parallel with POSITION maps: a 128-byte chunk maps each entry offset e in [0, 64) (where
// a frame that started before the chunk can end) to the offset its chain leaves the chunk at
// (an entry of the next chunk), or to "terminal". A lane computes its chunk's map with a backward
// DP over the chunk's bytes in LDS: D[p] = D[p + len(frame at p)]; a variable-length frame's
// length comes from a bounded parse of its varints. Terminals are: the end of the buffer, a
// frame running past it, a malformed varint / negative length, and a frame landing more than
// 63 bytes into the next chunk (LONG: rare - catch-up logs, large batches). Maps compose
// associatively: a workgroup reduces its 128 chunk maps to a 16 KB tile map, a group of 256
// tile maps to a group map, one block walks the group maps from the entry, classifies the
// terminal it reaches exactly, and the down-sweeps give every tile, then every chunk, its true
// entry. The count pass walks each chunk's frames on the true chain and counts them per record
// kind, a scan gives every tile its output offsets, and the emit pass walks again and writes
// the records. A LONG terminal is decoded too and ends the call (MPX_DECODE_LONG): the next
// call starts at its end (the host form loops).
// Chains from different entries merge within a few frames, so a tile whose 64 chains all leave
// its first 8 chunks at one entry X (or die there) - nearly every tile of a real stream - has
// chunk entries past those 8 chunks that do not depend on its entry: the framing pass stores
// them with group 0's 8 chunk maps as the tile's TileEnt (640 bytes) instead of its 128 chunk
// maps (8 KB), and the count pass and the walk read that (MPX_SD_TENT).
// HBM traffic per stream byte: 1 read (maps) + 1 read (count) + 1 read (emit) + 0.04 (TileEnt
// write and read), records written once.
#include "common.hpp"
#include "kernels.hpp"


namespace mpx {

namespace {

constexpr int kC = 128;                 // bytes per chunk (one lane)
constexpr int kE = MPX_DECODE_WINDOW;   // entry offsets per chunk map
constexpr int kTL = 128;                // chunks (lanes) per tile
constexpr int kTB = kC * kTL;           // tile bytes
constexpr int kGT = 256;                // tiles per group
#ifndef MPX_SD_VARLDS
#define MPX_SD_VARLDS 1
#endif
constexpr int kDRow = kC + 4;           // LDS row of a chunk's DP (bank-conflict padding)
constexpr int kTEnt = 8 * kE + kTL + 16;  // a tile's TileEnt bytes (+ chunks 8..127's counts)
#ifndef MPX_SD_WPE  // k_sd_tile_maps' waves per SIMD bound (its VGPR budget)
#define MPX_SD_WPE 5
#endif
#ifndef MPX_SD_TCNT  // converged tiles: chunks 8..127 counted by the framing pass (needs TENT)
#define MPX_SD_TCNT 1
#endif
#ifndef MPX_SD_TENT
#define MPX_SD_TENT 1
#endif
#ifndef MPX_SD_PRMARK  // PrepareReplies marked 0x60 in the landing table: a position mask, no loads
#define MPX_SD_PRMARK 0
#endif
#ifndef MPX_SD_TENT_NOCONV  // test build: every tile takes the unconverged path
#define MPX_SD_TENT_NOCONV 0
#endif
constexpr uint8_t kTerm = 0xFF;         // terminal (tree levels >= 1, tile / group maps)
constexpr uint8_t kDeadE = 0xFF;        // no entry (past the stop)
static_assert(kE == 64 && kE + kC <= 255, "u8 DP encoding: landings < kC + kE, 0xFF terminal");

enum { kOk = 0, kPartial = 1, kMalformed = 2, kBeyond = 3 };


// fixed frame length by code (code byte included), 0 = variable-length message
__host__ __device__ __forceinline__ uint32_t flen(uint32_t code, int proto) {
    switch (code) {
    case MPX_PEER_BEACON:
    case MPX_PEER_BEACON_REPLY: return 9;
    case MPX_PEER_PREPARE: return proto == MPX_MODE_MIN ? 13 : 14;
    case MPX_PEER_COMMIT_SHORT: return 17;
    case MPX_PEER_ACCEPT_REPLY: return proto == MPX_MODE_MIN ? 14 : 10;
    case MPX_PEER_ACCEPT:
    case MPX_PEER_COMMIT:
    case MPX_PEER_PREPARE_REPLY: return 0;
    default: return 1;
    }
}

// bytes of the stream: an LDS-staged window [lo, hi) (relative positions), global otherwise
// The staged tile image of the count and emit passes: 4 pad bytes after every 128-byte chunk
// (MPX_SD_PAD), so the lanes - one per chunk, at similar offsets - read 64 different banks
// instead of two (the emit pass's SQ pass: 72 % of its LDS cycles were bank conflicts).
#ifndef MPX_SD_PAD
#define MPX_SD_PAD 1
#endif
__host__ __device__ __forceinline__ uint32_t pofs(uint32_t o) {  // image offset of stream offset o
    return MPX_SD_PAD ? o + ((o >> 7) << 2) : o;
}
struct Bytes {
    const uint8_t* g;
    const uint8_t* s;
    uint64_t lo, hi;
    bool padded;  // s is a padded tile image (pofs)
    __host__ __device__ __forceinline__ uint32_t operator()(uint64_t i) const {
        if (i >= lo && i < hi) return s[padded ? pofs((uint32_t)(i - lo)) : (uint32_t)(i - lo)];
        return g[i];
    }
};

struct VarInfo {
    uint32_t len, n_cmds, cmds_off, n_log, log_off;  // offsets relative to the call's base
};

// binary.ReadVarint at *pos (len: end of the buffer; limit: give up past it)
__host__ __device__ __forceinline__ int read_varint(const Bytes& by, uint64_t len, uint64_t limit,
                                           uint64_t* pos, int64_t* out) {
    uint64_t x = 0;
    uint32_t s = 0;
    for (int i = 0; i < 10; ++i) {
        if (*pos >= len) return kPartial;
        if (*pos >= limit) return kBeyond;
        const uint32_t b = by((*pos)++);
        if (b < 0x80u) {
            if (i == 9 && b > 1u) return kMalformed;  // errOverflow
            x |= (uint64_t)b << s;
            *out = (int64_t)(x >> 1) ^ -(int64_t)(x & 1ull);
            return kOk;
        }
        x |= (uint64_t)(b & 0x7fu) << s;
        s += 7;
    }
    return kMalformed;
}

__host__ __device__ __forceinline__ int skip_cmds(uint64_t len, uint64_t limit, uint64_t* pos, int64_t n) {
    if (n < 0) return kMalformed;  // make() panics
    if ((uint64_t)n > (len - *pos) / 17) return kPartial;
    *pos += 17 * (uint64_t)n;
    return *pos > limit ? kBeyond : kOk;
}

// the variable-length message at p; the parse gives up (kBeyond) once it passes `limit`.
// Returns the status in .st and the frame in .f (valid when .st == kOk).
struct VarRes {
    int st;
    VarInfo f;
};
// the Command slice: where it starts and how long it is (header + V(n))
struct VarHead {
    int st;
    uint32_t hdr_end, n;
};
__host__ __device__ __forceinline__ uint32_t var_hdr(uint32_t code, int proto) {
    if (proto == MPX_MODE_MIN) return code == MPX_PEER_ACCEPT ? 16 : code == MPX_PEER_COMMIT ? 12 : 17;
    return code == MPX_PEER_PREPARE_REPLY ? 9 : 12;
}
__host__ __device__ __forceinline__ VarHead var_head(const Bytes& by, uint64_t len,
                                                     uint64_t limit, uint64_t p, int proto) {
    VarHead h{kOk, 0, 0};
    uint64_t pos = p + 1 + var_hdr(by(p), proto);
    if (pos > len) { h.st = kPartial; return h; }
    if (pos > limit) { h.st = kBeyond; return h; }
    int64_t n = 0;
    h.st = read_varint(by, len, limit, &pos, &n);
    if (h.st == kOk && n < 0) h.st = kMalformed;
    h.hdr_end = (uint32_t)pos;
    h.n = (uint32_t)n;
    return h;
}
// the variable-length message at p; the parse gives up (kBeyond) once it passes `limit`.
// Returns the status in .st and the frame in .f (valid when .st == kOk).
__host__ __device__ __forceinline__ VarRes parse_var(const Bytes& by, uint64_t len,
                                                     uint64_t limit, uint64_t p, int proto) {
    VarRes r{kOk, {0, 0, 0, 0, 0}};
    const uint32_t code = by(p);
    const VarHead h = var_head(by, len, limit, p, proto);
    if (h.st != kOk) {
        r.st = h.st;
        return r;
    }
    uint64_t pos = h.hdr_end;
    int st = skip_cmds(len, limit, &pos, (int64_t)h.n);
    uint64_t log_off = pos;
    int64_t m = 0;
    if (st == kOk && proto == MPX_MODE_MIN && code != MPX_PEER_COMMIT) {  // CatchUpLog
        st = read_varint(by, len, limit, &pos, &m);
        if (st == kOk && m < 0) st = kMalformed;
        if (st == kOk && (uint64_t)m > (len - pos) / 9) st = kPartial;
        log_off = pos;
        for (int64_t i = 0; st == kOk && i < m; ++i) {  // Instance: Ballot, Status, V(k), k Commands
            if (pos + 8 > len) {
                st = kPartial;
                break;
            }
            pos += 8;
            int64_t k = 0;
            st = read_varint(by, len, limit, &pos, &k);
            if (st == kOk) st = skip_cmds(len, limit, &pos, k);
        }
    }
    r.st = st;
    // the slice header again from its own parse (kept apart from the loop above)
    const VarHead h2 = var_head(by, len, limit, p, proto);
    r.f = VarInfo{(uint32_t)(pos - p), h2.n, h2.hdr_end, (uint32_t)m, (uint32_t)log_off};
    return r;
}

struct SParams {
    const uint8_t* buf;  // base of the call (16-byte aligned)
    uint64_t len;        // bytes from base
    uint64_t pos_base;   // offset of base in the caller's buffer (for record offsets)
    uint32_t entry0;     // the chain starts at base + entry0 (< 16)
    int proto;
    int legacy;          // stop at variable-length messages (mpx_decode_peer_stream)
};

// ---- workspace ----------------------------------------------------------------------------
struct Work {
    uint8_t* cmap;             // [tiles * kTL][kE] chunk maps (MPX_SD_TENT: converged tiles skip them)
    uint8_t* tconv;            // [tiles][kTEnt] TileEnt: group 0's chunk maps, then [0] converged,
                               // [1] X, [8..127] the chunk entries from X (MPX_SD_TENT)
    uint8_t* tmap;             // [tiles][kE]
    uint8_t* tent;             // [tiles] true entry (kDeadE past the stop)
    uint8_t* gmap;             // [groups][kE]
    uint8_t* gent;             // [groups]
    uint32_t* tcnt;            // [tiles][4] records of each kind the tile emits (k_sd_count)
    uint32_t* tpre;            // [tiles][4] exclusive prefixes of tcnt within 1024 tiles
    uint32_t* btot;            // [tiles / 1024][4] totals of the scan's workgroups
    uint32_t* boff;            // [tiles / 1024][4] their exclusive prefixes
    uint32_t* ticket;          // the scan's last-workgroup ticket (zeroed per call)
    uint2* cinfo;              // [tiles][kTL] per chunk: .x = entry, .y = its 4 record counts
                               // (u8 each; k_sd_count -> k_sd_emit)
    uint64_t* stop;            // [0] stop position, [1] next, [2] reason, [3..7] VarInfo of a
                               // LONG stop frame, [8..11] the call's input counts
};

uint64_t n_tiles_of(uint64_t len) { return (len + kTB - 1) / kTB; }

}  // namespace

// ---- pass A: chunk maps and tile maps --------------------------------------------------------
// frame length by code from a byte-lane table (codes 6..13; 0 = variable-length message,
// anything else a 1-byte frame); the two wire formats differ in Prepare and AcceptReply
constexpr uint64_t kLutMin = 9ull | (9ull << 8) | (13ull << 16) | (0ull << 24) | (0ull << 32) |
                             (17ull << 40) | (0ull << 48) | (14ull << 56);
constexpr uint64_t kLutClassic = 9ull | (9ull << 8) | (14ull << 16) | (0ull << 24) |
                                 (0ull << 32) | (17ull << 40) | (0ull << 48) | (10ull << 56);
__device__ __forceinline__ uint32_t lut_len(uint64_t lut, uint32_t code) {
    const uint32_t i = code - (uint32_t)MPX_PEER_BEACON;
    const uint32_t in = 0u - (uint32_t)(i < 8u);
    return (((uint32_t)(lut >> ((i & 7u) * 8u)) & 0xFFu) & in) | (1u & ~in);
}


// The DP's byte per position p (dp_enc): the landing q = p + length of the frame at p, which
// is < kC for a landing inside the chunk (its value is D[q]), in [kC, kC + kE) for an exit (bit 7
// set, bit 6 clear: exit q - kC), and 0xFF for a terminal at p. The chunk map stores an exit as
// its offset (< kE) and a terminal as 0x7F (>= kE): the walk, the one reader of a terminal's
// position, re-scans its stop chunk (chunk_terminal).
//
// Phase 2a: the landings of the fixed-length frames, four positions per dword of chunk bytes.
// v_perm_b32 looks the four codes up in an 8-byte table of length - 1 (kVarMark for a variable
// message) indexed by code - MPX_PEER_BEACON; every other code selects 0x00 or 0xFF, cleared to
// 0 (a 1-byte frame); the positions are added bytewise (no carries: <= 0x40 + 128). Returns the
// dword of landings; *var gets bit 6 of every variable-message byte (var_bits: the one table
// value with bit 6 set - fixed lengths are at most 17 - so one AND, where round 6's first form,
// 0x7F, needed a zero-byte test).
constexpr uint32_t kVarMark = 0x40;
__device__ __forceinline__ uint32_t var_bits(uint32_t y2) { return y2 & 0x40404040u; }
__device__ __forceinline__ uint32_t dp_landings(uint32_t w, uint32_t lut_lo, uint32_t lut_hi,
                                                uint32_t pos4, uint32_t* var) {
    const uint32_t h = w & 0x80808080u;
    const uint32_t sel = (((w | 0x80808080u) - 0x06060606u) ^ 0x80808080u) | h;  // code - 6
    const uint32_t y = __builtin_amdgcn_perm(lut_hi, lut_lo, sel);
    const uint32_t hb = y & 0x80808080u;
    // 0xFF bytes (out of the table) -> 0: y ^ hb ^ (hb - (hb >> 7)) (the two masks are disjoint;
    // one v_bitop3_b32 - the AND-NOT-OR form compiled to four ops)
    const uint32_t y2 = __builtin_amdgcn_bitop3_b32(y, hb, hb - (hb >> 7), 0x96);
    *var = var_bits(y2);
    return y2 + pos4;
}
static_assert(MPX_PEER_BEACON == 6, "dp_landings indexes the table by code - 6");

// 0xFF in every byte whose bit 7 is set (bytes of 0x80 / 0x00)
__device__ __forceinline__ uint32_t byte_mask(uint32_t b7) { return b7 | (b7 - (b7 >> 7)); }

// binary.ReadVarint's unsigned part at *pos (relative), every read below e; false = a failure
// (past e, or malformed: errOverflow / more than 10 bytes)
template <class ByteAt>
__host__ __device__ __forceinline__ bool uvarint_at(const ByteAt& R, uint32_t* pos, uint32_t e, uint64_t* x) {
    uint64_t v = 0;
    uint32_t sh = 0;
#pragma unroll 1
    for (int i = 0; i < 10; ++i) {
        if (*pos >= e) return false;
        const uint32_t b = R(*pos);
        ++*pos;
        if (b < 0x80u) {
            if (i == 9 && b > 1u) return false;
            *x = v | ((uint64_t)b << sh);
            return true;
        }
        v |= (uint64_t)(b & 0x7fu) << sh;
        sh += 7;
    }
    return false;
}
// The landing (relative to the chunk) of the variable-length message at p, or 0xFF: exactly
// "parse_var(limit = c0 + kC + kE - 1) is kOk and the frame ends before kC + kE" (every other
// outcome - partial, malformed, past the limit - is a terminal), restated for that one question:
// e = min(len - c0, kC + kE - 1) bounds every read and the frame's end, a zigzag varint is
// negative iff odd, and a catch-up log of m instances needs at least 9m bytes (so m beyond what
// is left ends at a terminal however its instances parse). No VarInfo, no second header parse,
// 32-bit positions: the DP parses every byte 9 / 10 / 12 of the stream as a frame start.
template <class ByteAt>
__host__ __device__ __forceinline__ uint32_t var_land(const ByteAt& R, uint32_t p, uint32_t e, int proto) {
    const uint32_t code = R(p);
    uint32_t pos = p + 1 + var_hdr(code, proto);
    if (pos > e) return 0xFFu;
    uint64_t x;
    if (!uvarint_at(R, &pos, e, &x) || (x & 1u)) return 0xFFu;  // n < 0: make() panics
    if ((x >> 1) > (uint64_t)((e - pos) / 17)) return 0xFFu;
    pos += 17 * (uint32_t)(x >> 1);
    if (proto == MPX_MODE_MIN && code != MPX_PEER_COMMIT) {  // CatchUpLog
        if (!uvarint_at(R, &pos, e, &x) || (x & 1u)) return 0xFFu;
        if ((x >> 1) > (uint64_t)((e - pos) / 9)) return 0xFFu;
#pragma unroll 1
        for (uint32_t m = (uint32_t)(x >> 1); m; --m) {  // Instance: Ballot, Status, V(k), k Commands
            if (pos + 8 > e) return 0xFFu;
            pos += 8;
            if (!uvarint_at(R, &pos, e, &x) || (x & 1u)) return 0xFFu;
            if ((x >> 1) > (uint64_t)((e - pos) / 17)) return 0xFFu;
            pos += 17 * (uint32_t)(x >> 1);
        }
    }
    return pos;
}

// Phase 2a' (a chunk holding a variable-message code byte - any byte 9, 10 or 12, at the
// positions of other frames' payload too: ~12 per 64 chunks of the bench's MIN stream, runs of
// ~9 per chunk where an instance number has such a byte): the bounded parse of each, D[p] = the
// frame's landing, or 0xFF: a terminal (unparseable, landing kE or more bytes into the next
// chunk, or legacy mode, which stops at every variable-length message).
// The wave's positions are one task list: each lane's positions were its own serial loop, so a
// wave took as many rounds as its busiest lane, each as long as its deepest parse (catch-up
// logs over zero-rich payload: ~20 dependent reads). Tasks (lane << 7 | position, u16) go to
// T[kVarTasks] (the workgroup's G, free until the DP is done); lane j parses tasks j, j + 64,
// ... The parse reads the rows' raw bytes (MPX_SD_VARLDS, written before the landings; a chunk's
// next-chunk bytes from the next row when that is the same wave's, else through L2), so a row's
// raw bytes must outlive every parse of the wave: the results wait in registers (a byte per
// round) and are stored after the last round. More than kVarTasks positions (a var-dense wave)
// go a window at a time, bytes through L2, results stored at once. The loops stay rolled: an
// unrolled form was ~30 KB of code. Round 6 (profiles/r06/stream/): MIN 0.63-0.65 -> 0.47-0.51
// ms per k_sd_tile_maps call, CLASSIC 0.44-0.46 -> 0.34-0.36 with the leaner DP init and
// var_land; the rows-vs-L2 choice measured within noise (SD_STAMP still shows 10-80K cycles of
// a wave's ~12 parses: dependent reads in a wave that shares its SIMD with three others).
constexpr uint32_t kVarTasks = 256;
static_assert(kVarTasks <= 4 * 64, "a byte of q per round");
struct TileBytes {  // a chunk's bytes [0, kC + kE): its row and the next row (null: L2)
    const uint8_t* row;
    const uint8_t* next;
    const uint8_t* g;  // the chunk's first byte in global memory
    __host__ __device__ __forceinline__ uint32_t operator()(uint32_t i) const {
        if (i < (uint32_t)kC) return row ? row[i] : g[i];
        return next ? next[i - kC] : g[i];
    }
};
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t var_wave(const SParams P, uint64_t t0, uint64_t m_lo, uint64_t m_hi,
                                          uint8_t (*D)[kDRow], uint16_t* T) {
    const uint32_t ln = threadIdx.x & 63u, w0 = threadIdx.x & ~63u;
    const uint32_t cnt = (uint32_t)(__popcll(m_lo) + __popcll(m_hi));
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d, 64);
        if (ln >= (uint32_t)d) incl += t;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    const bool lds = MPX_SD_VARLDS && total <= kVarTasks;
    for (uint32_t base = 0; base < total; base += kVarTasks) {
        const uint32_t n = min(total - base, kVarTasks);
        uint32_t o = incl - cnt;  // this lane's first task index
        if (o < base + n && o + cnt > base) {
            for (int h = 0; h < 2; ++h) {
                uint64_t m = h ? m_hi : m_lo;
                while (m) {
                    const uint32_t p = (uint32_t)(__ffsll((long long)m) - 1 + 64 * h);
                    m &= m - 1;
                    if (o >= base && o < base + n) T[o - base] = (uint16_t)((ln << 7) | p);
                    ++o;
                }
            }
        }
        wave_sync();
        uint32_t q = 0;  // the rounds' results, a byte each (at most 4 rounds), stored after the last
#pragma unroll 1
        for (uint32_t j = ln; j < ((n + 63u) & ~63u); j += 64) {
            uint32_t v = 0xFFu;
            if (j < n && !P.legacy) {
                const uint32_t tk = T[j], src = w0 + (tk >> 7), p = tk & 127u;
                const uint64_t cs = t0 + (uint64_t)src * kC;
                const uint32_t e = (uint32_t)min(P.len - cs, (uint64_t)(kC + kE - 1));
                const TileBytes R{lds ? D[src] : nullptr, lds && (src & 63u) != 63u ? D[src + 1] : nullptr,
                                  P.buf + cs};
                v = var_land(R, p, e, P.proto);
            }
            if (lds) {
                q |= v << (8 * (j >> 6));
            } else if (j < n) {
                const uint32_t tk = T[j];
                D[w0 + (tk >> 7)][tk & 127u] = (uint8_t)v;
            }
        }
        if (lds) {
            wave_sync();
#pragma unroll 1
            for (uint32_t j = ln; j < n; j += 64) {
                const uint32_t tk = T[j];
                D[w0 + (tk >> 7)][tk & 127u] = (uint8_t)(q >> (8 * (j >> 6)));
            }
        }
        wave_sync();
    }
    return total;
}

// the table of dp_landings for a protocol (kLutMin / kLutClassic: lengths by code - 6)
__host__ __device__ constexpr uint64_t dp_table(uint64_t lut) {
    uint64_t e = 0;
    for (int i = 0; i < 8; ++i) {
        const uint64_t fl = (lut >> (8 * i)) & 0xFFu;
        const uint64_t vm = MPX_SD_PRMARK && i == MPX_PEER_PREPARE_REPLY - MPX_PEER_BEACON ? kVarMark | 0x20u : kVarMark;
        e |= (fl ? fl - 1 : vm) << (8 * i);
    }
    return e;
}

// Phase 2b: the backward DP over the chunk's positions, in the lane's LDS row, with every
// position a pointer: a position whose value is final (an exit or a terminal, bit 7 of its
// landing byte) gets that value written to its own row byte first and points at itself. The
// row is the landings with bit 7 flipped (an exit 128 + e becomes e, a terminal 0xFF becomes
// 0x7F, the rest is overwritten by the DP) and the self-pointers one v_perm_b32 mask (the sign
// bits of the four bytes) and one bitwise select: 4 VALU ops per dword instead of the ~17 of
// round 4's form, which kept each terminal's position (kE + p). A position is then a byte
// extract, the LDS read of its landing's value (already final: landings lie ahead) and the LDS
// write of its own: ~3 VALU ops. Round 3's 64-register window compiled to ~45 VALU ops per
// position and round 4's LDS form with a per-position length lookup and selects to ~25 (the
// DP is issue-bound at 4 cycles per wave64 VALU op); the same DP with bit-mask selects in
// place of the self-pointers (~11 ops) measured 2 % slower (stream 1.90 -> 1.65 / 1.62 ms
// MIN, 1.62 -> 1.44 / 1.41 CLASSIC, profiles/r04/stream/ab_dp_self.txt).
__device__ __forceinline__ void chunk_dp_self(uint32_t (&pw)[kC / 4], uint8_t* D) {
    uint32_t* row = reinterpret_cast<uint32_t*>(D);
#pragma unroll
    for (int i = 0; i < kC / 4; ++i) {
        const uint32_t x = pw[i];
        // 0xFF per final byte: v_perm_b32 selectors 8..11 replicate bit 15 / 31 / 47 / 63 of
        // {x, x << 8}, i.e. bit 7 of bytes 0, 2 (of x << 8) and 1, 3 (of x)
        const uint32_t fmask = __builtin_amdgcn_perm(x, x << 8, 0x0B090A08u);
        const uint32_t self = (uint32_t)(4 * i) * 0x01010101u + 0x03020100u;
        row[i] = x ^ 0x80808080u;
        pw[i] = (x & ~fmask) | (self & fmask);
    }
#pragma unroll
    for (int p = kC - 1; p >= 0; --p) D[p] = D[(pw[p >> 2] >> ((p & 3) * 8)) & 0xFFu];
}

// 16 groups of 8 chunks: G[g][e] = where entry e of chunk 8g leaves chunk 8g+7 (kTerm: a
// terminal on the way); X[c][e] are chunk maps with terminals as kTerm or >= kE. A thread
// follows its 8 (group, entry) chains one chunk at a time, so 8 LDS reads are in flight per
// step instead of one chain of 64 dependent reads (branch-free: a terminal reads entry 0's
// byte and stays terminal).
__device__ __forceinline__ void chunk_groups(const uint8_t* X, int xstride, uint8_t (*G)[kE]) {
    constexpr int kTasks = (kTL / 8) * kE / kTL;
    static_assert((kTL / 8) * kE % kTL == 0, "whole tasks per thread");
    uint32_t x[kTasks];
#pragma unroll
    for (int j = 0; j < kTasks; ++j) x[j] = (uint32_t)((threadIdx.x + j * kTL) % kE);
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int j = 0; j < kTasks; ++j) {
            const int g = (threadIdx.x + j * kTL) / kE;
            const uint32_t y = X[(8 * g + c) * xstride + (x[j] & (uint32_t)(kE - 1))];
            x[j] = (x[j] | y) >= (uint32_t)kE ? (uint32_t)kTerm : y;
        }
#pragma unroll
    for (int j = 0; j < kTasks; ++j) {
        const int t = threadIdx.x + j * kTL;
        G[t / kE][t % kE] = (uint8_t)x[j];
    }
}

// diagnostic build (-DMPX_SD_STAMP=1): one wave's clock per phase of k_sd_tile_maps, printed
// for a few sample workgroups
#ifndef MPX_SD_STAMP
#define MPX_SD_STAMP 0
#endif
#if MPX_SD_STAMP
#define SD_STAMP(k) sd_t[k] = clock64()
#else
#define SD_STAMP(k) do {} while (0)
#endif

// a lane's chunk map (64 bytes of its row) into the chunk-map array
__device__ __forceinline__ void store_chunk_map(const Work& W, uint32_t tile, const uint8_t* row) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(row);
    uint4* dst = reinterpret_cast<uint4*>(W.cmap + ((uint64_t)tile * kTL + threadIdx.x) * kE);
#pragma unroll
    for (int i = 0; i < kE / 16; ++i)
        dst[i] = make_uint4(src[4 * i], src[4 * i + 1], src[4 * i + 2], src[4 * i + 3]);
}

__global__ __launch_bounds__(kTL) __attribute__((amdgpu_waves_per_eu(MPX_SD_WPE))) void k_sd_tile_maps(SParams P, Work W) {
#if MPX_SD_STAMP
    unsigned long long sd_t[8];
    sd_t[0] = clock64();
#endif
    // the chunk's bytes (raw, for the variable-message parses), the landings, the parses, then
    // the DP, all in the lane's row; rows padded to an odd dword count so the 64 lanes of a
    // wave, each on its own row, hit 64 different banks (a 128-byte stride put every lane on two)
    __shared__ __attribute__((aligned(16))) uint8_t D[kTL][kDRow];
    __shared__ __attribute__((aligned(16))) uint8_t G[kTL / 8][kE];
    static_assert(kTL / 8 * kE >= 2 * kVarTasks * 2, "the var task lists fit G");
    const int l = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * kTB;
    const uint64_t c0 = t0 + (uint64_t)l * kC;
    uint32_t wd[kC / 4];
    if (c0 + kC <= P.len) {
        const uint4* s4 = reinterpret_cast<const uint4*>(P.buf + c0);
#pragma unroll
        for (int i = 0; i < kC / 16; ++i) {
            const uint4 v = s4[i];  // default policy: the emit pass reads the stream again
            wd[4 * i] = v.x;
            wd[4 * i + 1] = v.y;
            wd[4 * i + 2] = v.z;
            wd[4 * i + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kC / 4; ++i) {
            uint32_t x = 0;
            for (int b = 0; b < 4; ++b) {
                const uint64_t a = c0 + 4 * i + b;
                if (a < P.len) x |= (uint32_t)P.buf[a] << (8 * b);
            }
            wd[i] = x;
        }
    }
#if MPX_SD_VARLDS
    {   // the raw chunk into its row (the variable-message parse's bytes; wave-local readers)
        uint32_t* row = reinterpret_cast<uint32_t*>(D[l]);
#pragma unroll
        for (int i = 0; i < kC / 4; ++i) row[i] = wd[i];
    }
#endif
    const uint64_t tab = P.proto == MPX_MODE_MIN ? dp_table(kLutMin) : dp_table(kLutClassic);
    const uint32_t tab_lo = (uint32_t)tab, tab_hi = (uint32_t)(tab >> 32);
    uint32_t any_var = 0;  // bit 6 of the chunk's variable-message bytes, OR-ed
#pragma unroll
    for (int i = 0; i < kC / 4; ++i) {
        uint32_t vb;
        const uint32_t pos4 = (uint32_t)(4 * i + 1) * 0x01010101u + 0x03020100u;
        wd[i] = dp_landings(wd[i], tab_lo, tab_hi, pos4, &vb);
        any_var |= vb;
    }
    SD_STAMP(1);
    uint64_t m_lo = 0, m_hi = 0;  // the chunk's variable-message positions (kept for the counts)
#if MPX_SD_PRMARK
    uint64_t r_lo = 0, r_hi = 0;  // its PrepareReplies' (bit 5 of the table value)
#endif
    {
        const bool wv = __ballot(any_var != 0) != 0;  // (wave-uniform)
        uint16_t* T = reinterpret_cast<uint16_t*>(&G[0][0]) + (l >> 6) * kVarTasks;
        if (any_var) {  // positions from the landings (a variable message's is its position + 1 + kVarMark)
#pragma unroll
            for (int i = 0; i < kC / 4; ++i) {
                const uint32_t pos4 = (uint32_t)(4 * i + 1) * 0x01010101u + 0x03020100u;
#if MPX_SD_PRMARK
                // bit 0 of a byte: variable message, bit 4: PrepareReply; gathered to two nibbles
                const uint32_t d = wd[i] - pos4;
                const uint32_t z = ((d >> 6) & 0x01010101u) | ((d >> 1) & 0x10101010u);
                const uint32_t c = (z | (z >> 7) | (z >> 14) | (z >> 21));
                const uint64_t nib = c & 0xFu, rnib = (c >> 4) & 0xFu;
                if (i < 16) { m_lo |= nib << (4 * i); r_lo |= rnib << (4 * i); }
                else { m_hi |= nib << (4 * (i - 16)); r_hi |= rnib << (4 * (i - 16)); }
#else
                const uint32_t t = var_bits(wd[i] - pos4) >> 6;  // 0x01 per variable-message byte
                const uint64_t nib = (uint64_t)((t | (t >> 7) | (t >> 14) | (t >> 21)) & 0xFu);
                if (i < 16) m_lo |= nib << (4 * i); else m_hi |= nib << (4 * (i - 16));
#endif
            }
        }
        const uint32_t vt = wv ? var_wave(P, t0, m_lo, m_hi, D, T) : 0u;
#if MPX_SD_STAMP
        sd_t[7] = vt;
#else
        (void)vt;
#endif
    }
    if (any_var) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(D[l]);
#pragma unroll
        for (int i = 0; i < kC / 4; ++i) {
            const uint32_t pos4 = (uint32_t)(4 * i + 1) * 0x01010101u + 0x03020100u;
            const uint32_t vm = byte_mask(var_bits(wd[i] - pos4) << 1);
            wd[i] = (wd[i] & ~vm) | (row[i] & vm);
        }
    }
    SD_STAMP(2);
    if (c0 + kC + 17 + kE > P.len) {  // the end of the buffer: terminals (rare, per position)
#pragma unroll
        for (int p = 0; p < kC; ++p) {
            const uint32_t sh = (p & 3) * 8, x = (wd[p >> 2] >> sh) & 0xFFu;
            const uint64_t a = c0 + (uint64_t)p;
            if (a >= P.len || (x < 0xC0u && a + (x - (uint32_t)p) > P.len)) wd[p >> 2] |= 0xFFu << sh;
        }
    }
    SD_STAMP(3);
    chunk_dp_self(wd, D[l]);
    SD_STAMP(4);
#if !MPX_SD_TENT
    store_chunk_map(W, blockIdx.x, D[l]);
#endif
    __syncthreads();
    SD_STAMP(5);
    chunk_groups(&D[0][0], kDRow, G);
    __syncthreads();
#if MPX_SD_TENT
    {   // the tile's entry table (TileEnt): whether every chain from the 64 tile entries that
        // leaves group 0 (chunks 0..7) leaves it at one entry X, and the chunk entries from X on
        // TE (the entry row, 128 bytes) and GEs (the 16 group entries) live in the rows' 4 pad
        // bytes (rows 0..31 and 32..35): 144 more bytes of LDS would cost a workgroup per CU
        static_assert(kDRow - kC == 4 && kTL / 4 + kTL / 8 / 4 <= kTL, "pad bytes for TE / GEs");
        auto TE = [&](uint32_t k) -> uint8_t& { return D[k >> 2][kC + (k & 3)]; };
        auto GEs = [&](uint32_t g) -> uint8_t& { return D[kTL / 4 + (g >> 2)][kC + (g & 3)]; };
        if (l < kE) {  // wave 0: the live exits' min and max
            const uint32_t v = G[0][l], live = v < (uint32_t)kE;
            uint32_t mn = live ? v : 0xFFu, mx = live ? v : 0u;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                mn = min(mn, (uint32_t)__shfl_xor(mn, d));
                mx = max(mx, (uint32_t)__shfl_xor(mx, d));
            }
            if (l == 0) {
                const bool conv = (mn == 0xFFu || mn == mx) && !MPX_SD_TENT_NOCONV;
                TE(0) = conv ? 1 : 0;
                TE(1) = (uint8_t)(conv ? mn : 0xFFu);  // X (kDeadE: no chain leaves group 0)
                uint32_t x = conv ? mn : (uint32_t)kDeadE;
                for (int g = 1; g < kTL / 8; ++g) {  // the group entries from X
                    GEs(g) = (uint8_t)x;
                    x = x == kDeadE ? kDeadE : G[g][x];
                }
            }
        }
        __syncthreads();
        const bool conv = TE(0) != 0;
        if (conv && l >= 1 && l < kTL / 8) {  // chunk entries inside groups 1..15
            uint32_t x = GEs(l);
            for (int c = 0; c < 8; ++c) {
                TE(8 * l + c) = (uint8_t)x;
                const uint32_t y = x == kDeadE ? kDeadE : D[8 * l + c][x];
                x = y < (uint32_t)kE ? y : kDeadE;
            }
        }
        __syncthreads();
        uint8_t* te = W.tconv + (uint64_t)blockIdx.x * kTEnt;
        if (conv) {  // group 0's 8 chunk maps and the entry row: 640 bytes instead of 8 KB
            if (l < 8 * kE / 16) {
                const uint32_t* src = reinterpret_cast<const uint32_t*>(D[l >> 2]) + 4 * (l & 3);
                reinterpret_cast<uint4*>(te)[l] = make_uint4(src[0], src[1], src[2], src[3]);
            } else if (l < (8 * kE + kTL) / 16) {  // 16 entry bytes: four rows' pad dwords
                const int r = 4 * (l - 8 * kE / 16);
                auto pad = [&](int k) { return *reinterpret_cast<const uint32_t*>(&D[r + k][kC]); };
                reinterpret_cast<uint4*>(te)[l] = make_uint4(pad(0), pad(1), pad(2), pad(3));
            }
        } else {
            if (l == 0) te[8 * kE] = 0;
            store_chunk_map(W, blockIdx.x, D[l]);
        }
    }
#endif
    {  // the tile map: the first and second 8 group maps composed by two halves of the
       // workgroup side by side, then entry l through both
        static_assert(kTL == 2 * kE && kTL / 8 == 16, "two halves of 8 group maps");
        const int h = l / kE, e = l % kE;
        uint32_t x = (uint32_t)e;
#pragma unroll
        for (int g = 0; g < 8; ++g) x = x >= (uint32_t)kE ? (uint32_t)kTerm : G[8 * h + g][x & (kE - 1)];
        __syncthreads();
        G[h][e] = (uint8_t)x;  // (rows 0 and 1 were read by this thread's half only before)
        __syncthreads();
        if (l < kE) {
            const uint32_t y = G[0][l];
            W.tmap[(uint64_t)blockIdx.x * kE + l] =
                (uint8_t)(y >= (uint32_t)kE ? (uint32_t)kTerm : G[1][y]);
        }
#if MPX_SD_TENT && MPX_SD_TCNT
        // A converged tile's chunks 8..127 lie on one chain whatever the tile's entry: count
        // their frames here (the count pass then reads 8 chunks of bytes instead of 128). Each
        // lane walks its chunk from its entry through the DP's pointers (landing, or itself for a
        // frame leaving the chunk), written over its row once every value read is done; a
        // frame's kind by its length (an AcceptReply's is unique among the fixed frames) or the
        // variable-message mask; a variable message's code through L2 (PrepareReply or not).
        // Only the stop tile can meet a terminal on this chain, and the count pass redoes it.
        auto TE = [&](uint32_t k) -> uint8_t& { return D[k >> 2][kC + (k & 3)]; };
        if (TE(0) != 0) {  // converged (block-uniform)
            uint32_t ex = kDeadE;  // where the lane's chain leaves its chunk
            if (l == kTL - 1) {
                const uint32_t e = TE(kTL - 1);
                const uint32_t v = e < (uint32_t)kE ? D[kTL - 1][e] : kDeadE;
                ex = v < (uint32_t)kE ? v : kDeadE;
            } else if (l >= 8) {
                ex = TE(l + 1);
            }
            const uint32_t ent = l >= 8 ? TE(l) : kDeadE;
            __syncthreads();  // every value row read (TileEnt, chunk maps, the walk's entries)
            uint32_t* row = reinterpret_cast<uint32_t*>(D[l]);
#pragma unroll
            for (int i = 0; i < kC / 4; ++i) row[i] = wd[i];  // the pointers
            const uint32_t ar_len = flen(MPX_PEER_ACCEPT_REPLY, P.proto);
            uint32_t cnt[4] = {0, 0, 0, 0};  // AcceptReplies, PrepareReplies, variable, other
            for (uint32_t x = ent; x < (uint32_t)kC;) {
                const uint32_t q = D[l][x];
                const uint32_t len = q != x ? q - x : kC + ex - x;
                const bool var = ((x < 64 ? m_lo >> x : m_hi >> (x - 64)) & 1ull) != 0;
                if (var) {
                    cnt[2]++;
#if MPX_SD_PRMARK
                    cnt[1] += (uint32_t)((x < 64 ? r_lo >> x : r_hi >> (x - 64)) & 1ull);
#else
                    cnt[1] += P.buf[c0 + x] == MPX_PEER_PREPARE_REPLY ? 1u : 0u;
#endif
                } else {
                    cnt[len == ar_len ? 0 : 3]++;
                }
                if (q == x) break;
                x = q;
            }
            if (l >= 8)
                W.cinfo[(uint64_t)blockIdx.x * kTL + l] =
                    make_uint2(ent, cnt[0] | (cnt[1] << 8) | (cnt[2] << 16) | (cnt[3] << 24));
            uint32_t* ws = reinterpret_cast<uint32_t*>(&G[0][0]);  // (free: the tile map is out)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t x = cnt[k];
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
                if (lane_id() == 0) ws[4 * (l / kWave) + k] = x;
            }
            __syncthreads();
            if (l < 4) {
                uint32_t x = 0;
                for (int w = 0; w < kTL / kWave; ++w) x += ws[4 * w + l];
                reinterpret_cast<uint32_t*>(W.tconv + (uint64_t)blockIdx.x * kTEnt + 8 * kE + kTL)[l] = x;
            }
        }
#endif
#if MPX_SD_STAMP
        SD_STAMP(6);
        if ((blockIdx.x & 2047) == 1025 && (l & 63) == 0)
            printf("SD_STAMP blk %u wave %d: land %llu var %llu (tasks %llu) eob %llu dp %llu store+bar %llu groups+tmap %llu\n",
                   blockIdx.x, l >> 6, sd_t[1] - sd_t[0], sd_t[2] - sd_t[1], sd_t[7], sd_t[3] - sd_t[2],
                   sd_t[4] - sd_t[3], sd_t[5] - sd_t[4], sd_t[6] - sd_t[5]);
#endif
    }
}

// n bytes (a multiple of 16; both ends 16-byte aligned) from global memory into LDS, 16 per load
// (the maps were staged a byte per load: 256 dependent-issue loads per thread)
__device__ __forceinline__ void stage16(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                        uint32_t n) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    const uint4* g = reinterpret_cast<const uint4*>(src);
    for (uint32_t i = threadIdx.x; i < n / 16; i += blockDim.x) d[i] = g[i];
}

// ---- pass B1: group maps --------------------------------------------------------------------
// The group's 256 tile maps in kParts parts of 32: thread (q, e) follows entry e through part
// q (8 chains of 32 dependent LDS reads side by side instead of one of 256), then entry e runs
// through the 8 part maps.
constexpr int kParts = 8;
constexpr int kPartTiles = kGT / kParts;
__device__ __forceinline__ void part_maps(const uint8_t (*S)[kE], uint32_t nt, uint8_t (*Q)[kE]) {
    const uint32_t q = threadIdx.x / kE, e = threadIdx.x % kE;
    const uint32_t t0 = q * kPartTiles, t1 = min(t0 + (uint32_t)kPartTiles, nt);
    uint32_t x = e;
    for (uint32_t t = t0; t < t1; ++t) x = x >= (uint32_t)kE ? (uint32_t)kTerm : S[t][x];
    Q[q][e] = (uint8_t)x;
}
__global__ __launch_bounds__(kParts * kE) void k_sd_group_maps(Work W, uint32_t n_tiles) {
    __shared__ __attribute__((aligned(16))) uint8_t S[kGT][kE];
    __shared__ uint8_t Q[kParts][kE];
    const uint32_t g = blockIdx.x, first = g * kGT;
    const uint32_t nt = min((uint32_t)kGT, n_tiles - first);
    stage16(&S[0][0], W.tmap + (uint64_t)first * kE, nt * kE);
    __syncthreads();
    part_maps(S, nt, Q);
    __syncthreads();
    if (threadIdx.x < kE) {
        uint32_t x = threadIdx.x;
#pragma unroll
        for (int q = 0; q < kParts; ++q) x = x >= (uint32_t)kE ? (uint32_t)kTerm : Q[q][x];
        W.gmap[(uint64_t)g * kE + threadIdx.x] = (uint8_t)x;
    }
}

// ---- pass B2: the true chain over the group maps, then the exact stop ------------------------
// One block of kParts x 64 threads. The group maps are staged 256 at a time and followed in
// parts (part_maps; one thread chains the 8 part maps, 8 threads walk their parts writing the
// group entries); at the terminal group the block descends the same way to the terminal tile
// and chunk, then thread 0 classifies the frame at the terminal byte and writes the result.
// The run's first map at which the chain from entry e0 reaches a terminal: part maps, the parts
// chained by thread 0, then thread 0 walks the terminal part. S[k][e] >= kE is a terminal (kTerm
// in tile / group maps, 0x7F in chunk maps). Thread 0 gets (map index, entry into it,
// the terminal value); every chain reaches one (at the latest the end of the buffer).
__device__ __forceinline__ void first_terminal(const uint8_t (*S)[kE], uint32_t n, uint32_t e0,
                                               uint8_t (*Q)[kE], uint32_t* k_out,
                                               uint32_t* e_out, uint32_t* v_out) {
    part_maps(S, n, Q);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t e = e0, q = 0;
        for (; q < (uint32_t)kParts - 1; ++q) {
            const uint32_t x = Q[q][e];
            if (x >= (uint32_t)kE) break;
            e = x;
        }
        const uint32_t t1 = min((q + 1) * (uint32_t)kPartTiles, n);
        uint32_t k = q * kPartTiles, v = kTerm;
        for (; k < t1; ++k) {
            v = S[k][e];
            if (v >= (uint32_t)kE) break;
            e = v;
        }
        *k_out = k;
        *e_out = e;
        *v_out = v;
    }
}
// The position in the chunk at c0 where the chain entering at e reaches its terminal, by the
// rules k_sd_tile_maps' DP applies (the chunk maps store a terminal without its position): the
// end of the buffer, a frame past it, a legacy-mode or unparseable variable-length message, or
// one landing kE or more bytes into the next chunk. Thread 0 of the walk, once per call.
__device__ uint32_t chunk_terminal(const SParams& P, uint64_t c0, uint32_t e) {
    const Bytes by{P.buf, nullptr, 0, 0};
    uint32_t p = e;
    while (p < (uint32_t)kC) {  // p increases: every frame is at least a byte
        const uint64_t a = c0 + p;
        if (a >= P.len) return p;
        const uint32_t code = P.buf[a];
        uint32_t fl = flen(code, P.proto);
        if (!fl) {
            if (P.legacy) return p;
            const VarRes r = parse_var(by, P.len, c0 + kC + kE - 1, a, P.proto);
            if (r.st != kOk || p + r.f.len >= (uint32_t)(kC + kE)) return p;
            fl = r.f.len;
        }
        if (a + fl > P.len) return p;
        p += fl;
    }
    return p;  // (an exit: not reached for a chain the maps end at a terminal)
}

__global__ __launch_bounds__(kParts * kE) void k_sd_walk(SParams P, Work W, uint32_t n_tiles,
                                                         uint32_t n_groups, mpx_stream_result* res) {
    __shared__ __attribute__((aligned(16))) uint8_t S[kGT][kE];
    __shared__ uint8_t Q[kParts][kE];
    __shared__ uint8_t PE[kParts];
    __shared__ uint32_t st[3];  // entry, terminal group (n_groups = none), its entry
    __shared__ uint32_t fk[3];  // first_terminal's result
    const int t = threadIdx.x;
    if (t == 0) {
        st[0] = P.entry0;
        st[1] = n_groups;
        st[2] = 0;
        // the input counts, for the emit pass (which overwrites *res with the totals)
        W.stop[8] = res->n_accept_replies;
        W.stop[9] = res->n_prepare_replies;
        W.stop[10] = res->n_var;
        W.stop[11] = res->n_other;
    }
    for (uint32_t b0 = 0; b0 < n_groups; b0 += kGT) {
        const uint32_t nb = min((uint32_t)kGT, n_groups - b0);
        __syncthreads();
        if (st[1] != n_groups) {  // past the terminal: the rest is dead
            for (uint32_t g = t; g < nb; g += blockDim.x) W.gent[b0 + g] = kDeadE;
            continue;
        }
        stage16(&S[0][0], W.gmap + (uint64_t)b0 * kE, nb * kE);
        __syncthreads();
        part_maps(S, nb, Q);
        __syncthreads();
        if (t == 0) {  // the parts' entries (kDeadE after the part that reaches the terminal)
            uint32_t e = st[0];
            for (int q = 0; q < kParts; ++q) {
                PE[q] = (uint8_t)e;
                e = e >= (uint32_t)kE ? (uint32_t)kDeadE : Q[q][e];
            }
            st[0] = e;  // the next batch's entry (unused once a terminal is found)
        }
        __syncthreads();
        if (t < kParts) {  // part t's group entries; the part with the terminal records it
            const uint32_t g0 = t * kPartTiles, g1 = min(g0 + (uint32_t)kPartTiles, nb);
            uint32_t e = PE[t];
            for (uint32_t g = g0; g < g1; ++g) {
                W.gent[b0 + g] = (uint8_t)e;
                if (e >= (uint32_t)kE) continue;
                const uint32_t x = S[g][e];
                if (x >= (uint32_t)kE) {
                    st[1] = b0 + g;
                    st[2] = e;
                }
                e = x >= (uint32_t)kE ? (uint32_t)kDeadE : x;
            }
        }
    }
    __syncthreads();
    // the terminal tile within group gs
    const uint32_t gs = st[1];
    const uint32_t first = gs * kGT, nt = min((uint32_t)kGT, n_tiles - first);
    stage16(&S[0][0], W.tmap + (uint64_t)first * kE, nt * kE);
    __syncthreads();
    first_terminal(S, nt, st[2], Q, &fk[0], &fk[1], &fk[2]);
    __syncthreads();
    const uint32_t ts = first + fk[0];
    const uint32_t te = fk[1];
    __syncthreads();
    // the terminal chunk within the tile: a converged tile's TileEnt (group 0's chunk maps, then
    // the chunk entries from X), else its 128 chunk maps (8 KB) over S
#if MPX_SD_TENT
    for (uint32_t i = t; i < (uint32_t)kTEnt / 16; i += blockDim.x)
        reinterpret_cast<uint4*>(&S[0][0])[i] =
            reinterpret_cast<const uint4*>(W.tconv + (uint64_t)ts * kTEnt)[i];
    __syncthreads();
    const bool conv = S[8][0] != 0;
    __syncthreads();
    if (conv) {
        const uint8_t* E = &S[8][0];
        if (t == 0) fk[2] = kTL - 1;
        __syncthreads();
        // past group 0 the chain ends in the first chunk whose successor is dead
        if (t >= 8 && t < kTL - 1 && E[t] != kDeadE && E[t + 1] == kDeadE) atomicMin(&fk[2], t);
        __syncthreads();
        if (t == 0) {
            uint32_t x = te, c = 0;
            for (; c < 8; ++c) {  // the chain dies in group 0, or leaves it at X = E[8]
                const uint32_t y = S[c][x];
                if (y >= (uint32_t)kE) break;
                x = y;
            }
            if (c == 8) {
                c = fk[2];
                x = E[c];
            }
            fk[0] = c;
            fk[1] = x;
        }
    } else
#endif
    {
        for (uint32_t i = t; i < (uint32_t)kTL * kE / 16; i += blockDim.x)
            reinterpret_cast<uint4*>(&S[0][0])[i] =
                reinterpret_cast<const uint4*>(W.cmap + (uint64_t)ts * kTL * kE)[i];
        __syncthreads();
        first_terminal(S, kTL, te, Q, &fk[0], &fk[1], &fk[2]);
    }
    __syncthreads();
    if (t == 0) {
        const uint32_t cs = fk[0];
        const uint64_t cb = (uint64_t)ts * kTB + (uint64_t)cs * kC;
        const uint64_t s = cb + chunk_terminal(P, cb, fk[1]);  // terminal byte
        int32_t why, code = -1;
        uint64_t next = s;
        VarInfo f{0, 0, 0, 0, 0};
        if (s >= P.len) {
            why = MPX_DECODE_END;
        } else {
            code = P.buf[s];
            const uint32_t fl = flen((uint32_t)code, P.proto);
            if (fl) {
                why = MPX_DECODE_PARTIAL;  // a fixed frame past the end (the only fixed terminal)
            } else if (P.legacy) {
                why = MPX_DECODE_VARIABLE;
            } else {
                const VarRes r = parse_var(Bytes{P.buf, nullptr, 0, 0}, P.len, ~0ull, s, P.proto);
                why = r.st == kOk ? MPX_DECODE_LONG : r.st == kPartial ? MPX_DECODE_PARTIAL
                                                                      : MPX_DECODE_MALFORMED;
                if (r.st == kOk) {
                    f = r.f;
                    next = s + f.len;
                }
            }
        }
        res->consumed = P.pos_base + (why == MPX_DECODE_END ? P.len : s);
        res->next = P.pos_base + next;
        res->stop_reason = why;
        res->stop_code = code;
        W.stop[0] = s;
        W.stop[1] = next;
        W.stop[2] = (uint64_t)(uint32_t)why;
        W.stop[3] = f.len;
        W.stop[4] = f.n_cmds;
        W.stop[5] = f.cmds_off;
        W.stop[6] = f.n_log;
        W.stop[7] = f.log_off;
    }
}

// ---- pass B3: tile entries inside each group ---------------------------------------------------
__global__ __launch_bounds__(kParts * kE) void k_sd_tile_entries(Work W, uint32_t n_tiles) {
    __shared__ __attribute__((aligned(16))) uint8_t S[kGT][kE];
    __shared__ uint8_t Q[kParts][kE];
    __shared__ uint8_t E[kParts];
    const uint32_t g = blockIdx.x, first = g * kGT;
    const uint32_t nt = min((uint32_t)kGT, n_tiles - first);
    const uint8_t r = W.gent[g];
    if (r == kDeadE) {
        for (uint32_t t = threadIdx.x; t < nt; t += blockDim.x) W.tent[first + t] = kDeadE;
        return;
    }
    stage16(&S[0][0], W.tmap + (uint64_t)first * kE, nt * kE);
    __syncthreads();
    part_maps(S, nt, Q);  // (as in k_sd_group_maps: the parts' maps, then the parts' entries)
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x = r;
        for (int q = 0; q < kParts; ++q) {
            E[q] = (uint8_t)x;
            x = x >= (uint32_t)kE ? (uint32_t)kDeadE : Q[q][x];  // kTerm == kDeadE
        }
    }
    __syncthreads();
    if (threadIdx.x < kParts) {  // part q's tiles from its entry
        const uint32_t q = threadIdx.x, t0 = q * kPartTiles, t1 = min(t0 + (uint32_t)kPartTiles, nt);
        uint32_t e = E[q];
        for (uint32_t t = t0; t < t1; ++t) {
            W.tent[first + t] = (uint8_t)e;
            e = e >= (uint32_t)kE ? (uint32_t)kDeadE : S[t][e];  // the tiles after are dead
        }
    }
}

// ---- pass C: chunk entries, counts, look-back, records ----------------------------------------
struct Outs {
    mpx_accept_reply* ar;
    uint64_t ar_cap;
    void* prep;
    uint64_t prep_cap;
    mpx_var_frame* var;
    uint64_t var_cap;
    mpx_peer_frame* oth;
    uint64_t oth_cap;
};

__device__ __forceinline__ int32_t le32(const Bytes& by, uint64_t i) {
    return (int32_t)(by(i) | (by(i + 1) << 8) | (by(i + 2) << 16) | (by(i + 3) << 24));
}
// 4 bytes at stream offset o of a (padded) tile image from two aligned dword reads (each dword
// at its own image position: a field may straddle a chunk's pad)
__device__ __forceinline__ int32_t lds_le32(const uint8_t* B, uint32_t o) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(B);
    const uint32_t d = o >> 2, sh = o & 3u;
    const uint32_t d0 = MPX_SD_PAD ? d + (d >> 5) : d, d1 = MPX_SD_PAD ? d + 1 + ((d + 1) >> 5) : d + 1;
    const uint64_t x = ((uint64_t)w[d1] << 32) | w[d0];
    return (int32_t)(uint32_t)(x >> (8 * sh));
}
// the image's bytes: kTB + kE stream bytes, a pad per chunk (kTL + 1 chunks started), and the
// second dword lds_le32 may read past the last byte
constexpr int kImg = kTB + kE + (MPX_SD_PAD ? 4 * (kTL + 1) : 0) + 16;
// 16 stream bytes (piece i of the tile) into the image: a piece never crosses a chunk
__device__ __forceinline__ void img_put(uint8_t* B, int i, const uint4 v) {
    if (MPX_SD_PAD) {
        uint32_t* w = reinterpret_cast<uint32_t*>(B) + 4 * i + (i >> 3);
        w[0] = v.x;
        w[1] = v.y;
        w[2] = v.z;
        w[3] = v.w;
    } else {
        reinterpret_cast<uint4*>(B)[i] = v;
    }
}

// the tile's chunk entries: the tile's true entry through its chunk maps (X, in LDS)
__device__ __forceinline__ void chunk_entries(uint32_t ent, uint8_t (*X)[kE], uint8_t (*G)[kE],
                                              uint8_t* GE, uint8_t* En) {
    const int l = threadIdx.x;
    chunk_groups(&X[0][0], kE, G);
    __syncthreads();
    if (l == 0) {  // group entries from the tile's entry
        uint32_t x = ent;
        for (int g = 0; g < kTL / 8; ++g) {
            GE[g] = (uint8_t)x;
            x = x == kDeadE ? kDeadE : G[g][x];
        }
    }
    __syncthreads();
    if (l < kTL / 8) {  // chunk entries inside each group
        uint32_t x = GE[l];
        for (int c = 0; c < 8; ++c) {
            En[8 * l + c] = (uint8_t)x;
            const uint32_t y = x == kDeadE ? kDeadE : X[8 * l + c][x];
            x = y < (uint32_t)kE ? y : kDeadE;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void load_chunk_maps(const Work& W, uint32_t tile, uint8_t (*X)[kE]) {
    // the 8 KB of chunk maps: a lane's four loads in flight together, then the LDS stores
    const uint4* src = reinterpret_cast<const uint4*>(W.cmap + (uint64_t)tile * kTL * kE);
    constexpr int kN = kTL * kE / 16 / kTL;
    static_assert(kTL * kE / 16 % kTL == 0, "whole vectors per lane");
    uint4 v[kN];
#pragma unroll
    for (int k = 0; k < kN; ++k) v[k] = src[threadIdx.x + k * kTL];
#pragma unroll
    for (int k = 0; k < kN; ++k) reinterpret_cast<uint4*>(&X[0][0])[threadIdx.x + k * kTL] = v[k];
}

// frames of the lane's chunk on the true chain, by kind: AcceptReplies, PrepareReplies, variable
// messages, other fixed frames (every frame before the stop is complete and in the window).
// code_at(a): the byte at stream position a.
template <class CodeAt>
__device__ __forceinline__ void chunk_counts(uint32_t e, uint64_t c0, uint64_t stop, bool long_stop,
                                             const SParams& P, const Bytes& by, CodeAt code_at,
                                             uint32_t (&cnt)[4]) {
    const uint64_t lut = P.proto == MPX_MODE_MIN ? kLutMin : kLutClassic;
    if (e == kDeadE) return;
    for (uint64_t a = c0 + e; a < c0 + kC;) {
        const uint32_t code = code_at(a);
        if (a == stop) {
            if (long_stop) {
                cnt[2]++;
                cnt[1] += code == MPX_PEER_PREPARE_REPLY ? 1u : 0u;
            }
            break;
        }
        uint32_t fl = lut_len(lut, code);
        if (fl == 0) {
            fl = parse_var(by, P.len, ~0ull, a, P.proto).f.len;
            cnt[2]++;
            cnt[1] += code == MPX_PEER_PREPARE_REPLY ? 1u : 0u;
        } else {
            cnt[code == MPX_PEER_ACCEPT_REPLY ? 0 : 3]++;
        }
        a += fl;
    }
}

// pass C1: every tile's record counts (the emit pass takes its output indices from their
// exclusive scan; a decoupled look-back across the ~1500 tiles in flight waited on device-scope
// loads, which bypass the XCDs' L2s)
// the tile's bytes [t0, t0 + kTB + kE) into LDS (zero past len)
__device__ __forceinline__ void stage_tile(const SParams& P, uint64_t t0, uint8_t* B) {
    for (int i = threadIdx.x; i < (kTB + kE) / 16; i += kTL) {
        const uint64_t a = t0 + (uint64_t)i * 16;
        uint4 v;
        if (a + 16 <= P.len) {
            v = *reinterpret_cast<const uint4*>(P.buf + a);
        } else {
            uint32_t q[4] = {0, 0, 0, 0};
            for (int b = 0; b < 16; ++b)
                if (a + b < P.len) q[b >> 2] |= (uint32_t)P.buf[a + b] << (8 * (b & 3));
            v = make_uint4(q[0], q[1], q[2], q[3]);
        }
        img_put(B, i, v);
    }
}

// the tile's bytes for stage_tile, loaded into registers (kStageVec 16-byte pieces per lane)
constexpr int kStageVec = ((kTB + kE) / 16 + kTL - 1) / kTL;
__device__ __forceinline__ void load_tile_regs(const SParams& P, uint64_t t0, uint4 (&v)[kStageVec]) {
    if (t0 + (uint64_t)kStageVec * kTL * 16 <= P.len) {
        // interior tile (block-uniform): one basic block of loads, all in flight together (with
        // the edge checks below per load, the compiler waited out each load at the branch join);
        // only the last vector is partial: its lanes past the window reload the window's last
        // vector (no branch, whose join would wait for every load; the stores skip them)
        const uint4* src = reinterpret_cast<const uint4*>(P.buf + t0);
        const int l = threadIdx.x;
        __builtin_assume(l < kTL);
#pragma unroll
        for (int k = 0; k < kStageVec; ++k) v[k] = src[min(l + k * kTL, (kTB + kE) / 16 - 1)];
        return;
    }
#pragma unroll
    for (int k = 0; k < kStageVec; ++k) {
        const int i = threadIdx.x + k * kTL;
        const uint64_t a = t0 + (uint64_t)i * 16;
        if (i >= (kTB + kE) / 16) {
            v[k] = make_uint4(0, 0, 0, 0);
        } else if (a + 16 <= P.len) {
            v[k] = *reinterpret_cast<const uint4*>(P.buf + a);
        } else {
            uint32_t q[4] = {0, 0, 0, 0};
            for (int b = 0; b < 16; ++b)
                if (a + b < P.len) q[b >> 2] |= (uint32_t)P.buf[a + b] << (8 * (b & 3));
            v[k] = make_uint4(q[0], q[1], q[2], q[3]);
        }
    }
}

#ifndef MPX_SD_COUNT_UNION
#define MPX_SD_COUNT_UNION 1
#endif
__global__ __launch_bounds__(kTL) void k_sd_count(SParams P, Work W) {
#if MPX_SD_COUNT_UNION
    // the chunk maps are dead once the chunk entries are known: the tile's bytes (loaded into
    // registers meanwhile) take their LDS, so a workgroup needs 16.5 KB instead of 24.5 KB
    // (and the group maps of an unconverged tile's chunk entries take the bytes after X)
    __shared__ __attribute__((aligned(16))) uint8_t U[kImg];
    uint8_t* const B = U;
    uint8_t(*const X)[kE] = reinterpret_cast<uint8_t(*)[kE]>(U);
    uint8_t(*const G)[kE] = reinterpret_cast<uint8_t(*)[kE]>(U + kTL * kE);
    static_assert(kTL * kE + kTL / 8 * kE <= kImg, "X and G fit the image");
#else
    __shared__ __attribute__((aligned(16))) uint8_t B[kImg];
    __shared__ __attribute__((aligned(16))) uint8_t X[kTL][kE];
    __shared__ uint8_t G[kTL / 8][kE];
#endif
    __shared__ uint8_t GE[kTL / 8];
    __shared__ uint8_t En[kTL];
    __shared__ uint32_t wsum[kTL / kWave][4];
    const int l = threadIdx.x;
    const uint32_t tile = blockIdx.x;
    const uint8_t ent = W.tent[tile];
#if MPX_SD_TENT && MPX_SD_TCNT
    const bool conv_tile = W.tconv[(uint64_t)tile * kTEnt + 8 * kE] != 0;
    const bool stop_tile = W.stop[0] / kTB == tile;
#endif
    if (ent == kDeadE) {
        if (l < 4) W.tcnt[4 * (uint64_t)tile + l] = 0;
        return;
    }
#if MPX_SD_TENT && MPX_SD_TCNT
    if (conv_tile && !stop_tile) return;  // k_sd_count_conv's
#endif
    const uint64_t t0 = (uint64_t)tile * kTB;
#if MPX_SD_COUNT_UNION
#if MPX_SD_TENT
    // the TileEnt's loads first (needed first), then the tile's, all in flight together; a
    // converged tile (the common case) needs no chunk maps past group 0
    uint4 tev = make_uint4(0, 0, 0, 0);
    if (l < kTEnt / 16) tev = reinterpret_cast<const uint4*>(W.tconv + (uint64_t)tile * kTEnt)[l];
    uint4 tv[kStageVec];
    load_tile_regs(P, t0, tv);
    if (l < kTEnt / 16) reinterpret_cast<uint4*>(&X[0][0])[l] = tev;
    __syncthreads();
    if (X[8][0] != 0) {  // converged (block-uniform)
        if (l == 0) {  // group 0 from the tile's entry; the rest is the entry row or dead
            uint32_t x = ent;
            for (int c = 0; c < 8; ++c) {
                En[c] = (uint8_t)x;
                const uint32_t y = x == kDeadE ? kDeadE : X[c][x];
                x = y < (uint32_t)kE ? y : kDeadE;
            }
            GE[0] = x != kDeadE;
        }
        __syncthreads();
        if (l >= 8) En[l] = GE[0] ? X[8][l] : kDeadE;
        __syncthreads();
    } else {  // (rare: chains still apart after group 0) the 8 KB of chunk maps
        const uint4* csrc = reinterpret_cast<const uint4*>(W.cmap + (uint64_t)tile * kTL * kE);
        __syncthreads();  // (every thread has read the flag)
#pragma unroll 1
        for (int k = 0; k < kTL * kE / 16 / kTL; ++k)
            reinterpret_cast<uint4*>(&X[0][0])[l + k * kTL] = csrc[l + k * kTL];
        __syncthreads();
        chunk_entries(ent, X, G, GE, En);  // (ends with a barrier: X is dead)
    }
#else
    // the chunk maps' loads first (needed first), then the tile's, all in flight together
    constexpr int kCm = kTL * kE / 16 / kTL;
    uint4 cm[kCm];
    const uint4* csrc = reinterpret_cast<const uint4*>(W.cmap + (uint64_t)tile * kTL * kE);
#pragma unroll
    for (int k = 0; k < kCm; ++k) cm[k] = csrc[l + k * kTL];
    uint4 tv[kStageVec];
    load_tile_regs(P, t0, tv);
#pragma unroll
    for (int k = 0; k < kCm; ++k) reinterpret_cast<uint4*>(&X[0][0])[l + k * kTL] = cm[k];
    __syncthreads();
    chunk_entries(ent, X, G, GE, En);  // (ends with a barrier: X is dead)
#endif
#pragma unroll
    for (int k = 0; k < kStageVec; ++k) {
        const int i = l + k * kTL;
        if (i < (kTB + kE) / 16) img_put(B, i, tv[k]);
    }
    __syncthreads();
#else
    stage_tile(P, t0, B);
    load_chunk_maps(W, tile, X);
    __syncthreads();
    chunk_entries(ent, X, G, GE, En);
#endif
    const uint64_t c0 = t0 + (uint64_t)l * kC;
    const Bytes by{P.buf, B, t0, t0 + kTB + kE < P.len ? t0 + kTB + kE : P.len, MPX_SD_PAD != 0};
    uint32_t cnt[4] = {0, 0, 0, 0};
    chunk_counts(En[l], c0, W.stop[0], (int)W.stop[2] == MPX_DECODE_LONG, P, by,
                 [&](uint64_t a) { return (uint32_t)B[pofs((uint32_t)(a - t0))]; }, cnt);
    W.cinfo[(uint64_t)tile * kTL + l] =
        make_uint2(En[l], cnt[0] | (cnt[1] << 8) | (cnt[2] << 16) | (cnt[3] << 24));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t x = cnt[k];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
        if (lane_id() == 0) wsum[l / kWave][k] = x;
    }
    __syncthreads();
    if (l < 4) {
        uint32_t x = 0;
        for (int w = 0; w < kTL / kWave; ++w) x += wsum[w][l];
        W.tcnt[4 * (uint64_t)tile + l] = x;
    }
}

// pass C1': a converged tile (not the stop tile): chunks 8..127 were counted by the framing
// pass (their cinfo and the four totals at the end of the TileEnt), so one wave resolves the
// entries of chunks 0..7 from group 0's maps and walks those 8 chunks: 1.2 KB of the tile's bytes
// read instead of 16 KB (the count pass re-read every stream byte: 0.94 GB of the MIN bench's
// 2.07 x traffic)
constexpr int kCcVec = (9 * kC) / 16;  // chunks 0..8 (chunk 7's frames may end in chunk 8)
__global__ __launch_bounds__(kWave) void k_sd_count_conv(SParams P, Work W) {
    __shared__ __attribute__((aligned(16))) uint8_t TEs[kTEnt];
    __shared__ __attribute__((aligned(16))) uint8_t B[9 * kC + 16];
    __shared__ uint8_t En[8];
    const int l = threadIdx.x;
    const uint32_t tile = blockIdx.x;
    const uint8_t ent = W.tent[tile];
    const uint8_t* te = W.tconv + (uint64_t)tile * kTEnt;
    const bool conv_tile = te[8 * kE] != 0;
    const bool stop_tile = W.stop[0] / kTB == tile;
    if (ent == kDeadE || !conv_tile || stop_tile) return;  // k_sd_count's
    const uint64_t t0 = (uint64_t)tile * kTB;
    // (not the stop tile: the stream goes on past this tile, so all of its bytes exist)
    const uint4* tsrc = reinterpret_cast<const uint4*>(te);
    const uint4* bsrc = reinterpret_cast<const uint4*>(P.buf + t0);
    const uint4 tv = l < kTEnt / 16 ? tsrc[l] : make_uint4(0, 0, 0, 0);
    const uint4 b0 = bsrc[l];
    const uint4 b1 = l + kWave < kCcVec ? bsrc[l + kWave] : make_uint4(0, 0, 0, 0);
    if (l < kTEnt / 16) reinterpret_cast<uint4*>(TEs)[l] = tv;
    reinterpret_cast<uint4*>(B)[l] = b0;
    if (l + kWave < kCcVec) reinterpret_cast<uint4*>(B)[l + kWave] = b1;
    __syncthreads();
    if (l == 0) {  // group 0 from the tile's entry (it leaves group 0 at X: not the stop tile)
        uint32_t x = ent;
        for (int c = 0; c < 8; ++c) {
            En[c] = (uint8_t)x;
            const uint32_t y = x == kDeadE ? kDeadE : TEs[c * kE + x];
            x = y < (uint32_t)kE ? y : kDeadE;
        }
    }
    __syncthreads();
    uint32_t cnt[4] = {0, 0, 0, 0};
    if (l < 8) {
        const Bytes by{P.buf, B, t0, t0 + 9 * kC};
        chunk_counts(En[l], t0 + (uint64_t)l * kC, W.stop[0], false, P, by,
                     [&](uint64_t a) { return (uint32_t)B[a - t0]; }, cnt);
        W.cinfo[(uint64_t)tile * kTL + l] =
            make_uint2(En[l], cnt[0] | (cnt[1] << 8) | (cnt[2] << 16) | (cnt[3] << 24));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t x = cnt[k];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
        cnt[k] = x;
    }
    if (l < 4) {
        const uint32_t rest = reinterpret_cast<const uint32_t*>(TEs + 8 * kE + kTL)[l];
        W.tcnt[4 * (uint64_t)tile + l] = (l == 0 ? cnt[0] : l == 1 ? cnt[1] : l == 2 ? cnt[2] : cnt[3]) + rest;
    }
}

// pass C2: exclusive scan of the tile counts: a workgroup scans 1024 tiles (coalesced) and
// publishes its total; the last workgroup to finish scans the totals into per-workgroup offsets
// (tile prefix = tpre[tile] + boff[tile / kScanT])
constexpr int kScanT = 1024;
__global__ __launch_bounds__(kScanT) void k_sd_scan(Work W, uint32_t n_tiles) {
    __shared__ uint32_t ws[kScanT / kWave][4];
    __shared__ bool last;
    const int t = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * kScanT + t;
    uint4 c = make_uint4(0, 0, 0, 0);
    if (i < n_tiles) c = reinterpret_cast<const uint4*>(W.tcnt)[i];
    uint32_t v[4] = {c.x, c.y, c.z, c.w}, ex[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t x = v[k];
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if (lane_id() >= d) x += y;
        }
        if (lane_id() == kWave - 1) ws[t / kWave][k] = x;
        ex[k] = x - v[k];
    }
    __syncthreads();
    uint32_t tot[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (int w = 0; w < kScanT / kWave; ++w) {
            ex[k] += w < t / kWave ? ws[w][k] : 0u;
            tot[k] += ws[w][k];
        }
    if (i < n_tiles) reinterpret_cast<uint4*>(W.tpre)[i] = make_uint4(ex[0], ex[1], ex[2], ex[3]);
    if (t == 0) {
        reinterpret_cast<uint4*>(W.btot)[blockIdx.x] = make_uint4(tot[0], tot[1], tot[2], tot[3]);
        __threadfence();
        last = atomicAdd(W.ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    // the workgroup offsets (at most 128 workgroups: 2^31 bytes / 16 KB tiles / 1024)
    const uint32_t nb = gridDim.x;
    uint32_t b[4] = {0, 0, 0, 0};
    if ((uint32_t)t < nb)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            b[k] = __hip_atomic_load(W.btot + 4 * t + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t x = b[k];
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if (lane_id() >= d) x += y;
        }
        if (lane_id() == kWave - 1) ws[t / kWave][k] = x;
        ex[k] = x - b[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (int w = 0; w < t / kWave; ++w) ex[k] += ws[w][k];
    if ((uint32_t)t < nb)
        reinterpret_cast<uint4*>(W.boff)[t] = make_uint4(ex[0], ex[1], ex[2], ex[3]);
    if (t == 0) *W.ticket = 0;
}

#ifndef MPX_SD_EMIT_REG
#define MPX_SD_EMIT_REG 1
#endif
// frames whose AcceptReplies a lane keeps in registers for the staged stores (a 128-byte chunk
// starts at most 10 MIN AcceptReply frames; 13 would cost a wave per SIMD of occupancy, so a
// tile with a longer chunk - CLASSIC's 10-byte frames back to back - stores directly), and the
// tile's records per LDS pass
constexpr int kRegAR = 10;
constexpr uint32_t kRegCap = 1024;
__global__ __launch_bounds__(kTL) void k_sd_emit(SParams P, Work W, Outs O, uint32_t n_tiles,
                                                 mpx_stream_result* res) {
    __shared__ __attribute__((aligned(16))) uint8_t B[kImg];
    __shared__ uint32_t wsum[kTL / kWave][4];
    static_assert(kImg / 16 >= kRegCap, "a pass of staged records fits the tile image");
    const int l = threadIdx.x;
    const uint32_t tile = blockIdx.x;
    const uint8_t ent = W.tent[tile];
    if (ent == kDeadE) return;  // every tile after the stop tile, never one before it
    const uint64_t t0 = (uint64_t)tile * kTB;
    // the tile's bytes. MIN wire: all of a lane's 16-byte loads issued before the first LDS
    // store (the load-store loop of stage_tile waits out each load in turn, 9 round trips per
    // lane): emit 574 -> 447 us. CLASSIC's 10-byte AcceptReply frames overflow the register
    // staging (kRegAR) and take the direct-store path, which ran 678 -> 727 us with the loads
    // batched (profiles/r04/stream/ab_tile_loads.txt), so it keeps the loop.
    if (P.proto == MPX_MODE_MIN) {
        uint4 tv[kStageVec];
        load_tile_regs(P, t0, tv);
#pragma unroll
        for (int k = 0; k < kStageVec; ++k) {
            const int i = l + k * kTL;
            if (i < (kTB + kE) / 16) img_put(B, i, tv[k]);
        }
    } else {
        stage_tile(P, t0, B);
    }
    const uint2 ci = W.cinfo[(uint64_t)tile * kTL + l];  // entry and counts (k_sd_count)
    __syncthreads();
    const uint32_t e = ci.x;
    const uint64_t stop = W.stop[0];
    const int why = (int)W.stop[2];
    const bool long_stop = why == MPX_DECODE_LONG;
    const Bytes by{P.buf, B, t0, t0 + kTB + kE < P.len ? t0 + kTB + kE : P.len, MPX_SD_PAD != 0};
    const uint64_t c0 = t0 + (uint64_t)l * kC;
    const uint32_t cnt[4] = {ci.y & 0xFFu, (ci.y >> 8) & 0xFFu, (ci.y >> 16) & 0xFFu, ci.y >> 24};
    const uint64_t lut = P.proto == MPX_MODE_MIN ? kLutMin : kLutClassic;
    // block exclusive scan of the four counts
    uint32_t incl[4], tot[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t x = cnt[k];
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if (lane_id() >= d) x += y;
        }
        incl[k] = x;
        if (lane_id() == kWave - 1) wsum[l / kWave][k] = x;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t before = 0, all = 0;
        for (int w = 0; w < kTL / kWave; ++w) {
            before += w < l / kWave ? wsum[w][k] : 0u;
            all += wsum[w][k];
        }
        incl[k] = incl[k] - cnt[k] + before;  // exclusive within the tile
        tot[k] = all;
    }
    uint64_t idx[4];
    const uint64_t base[4] = {W.stop[8], W.stop[9], W.stop[10], W.stop[11]};
    uint32_t tp[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        tp[k] = W.tpre[4 * (uint64_t)tile + k] + W.boff[4 * (uint64_t)(tile / kScanT) + k];
        idx[k] = base[k] + tp[k] + incl[k];
    }
    // the stop tile (the one holding the terminal byte, at the latest position len) owns the
    // totals: every later tile is dead
    if (stop / kTB == tile && l == 0) {
        res->n_accept_replies = base[0] + tp[0] + tot[0];
        res->n_prepare_replies = base[1] + tp[1] + tot[1];
        res->n_var = base[2] + tp[2] + tot[2];
        res->n_other = base[3] + tp[3] + tot[3];
    }
    const uint64_t ar0 = base[0] + tp[0];  // the tile's first AcceptReply
    // walk 2, one frame at a: an AcceptReply comes back in rec (is_ar), every other record is
    // stored here; live = false after the chunk's last frame
    auto frame = [&](uint64_t& a, bool& live, bool& is_ar, uint4& rec) {
        is_ar = false;
        const uint32_t code = B[pofs((uint32_t)(a - t0))];
        uint32_t fl = lut_len(lut, code);
        const bool at_stop = a == stop;
        if (at_stop && !long_stop) {
            live = false;
            return;
        }
        if (fl == 0) {
            VarInfo f;
            if (at_stop) {
                f = VarInfo{(uint32_t)W.stop[3], (uint32_t)W.stop[4], (uint32_t)W.stop[5],
                            (uint32_t)W.stop[6], (uint32_t)W.stop[7]};
            } else {
                f = parse_var(by, P.len, ~0ull, a, P.proto).f;
            }
            fl = f.len;
            if (code == MPX_PEER_PREPARE_REPLY) {
                if (idx[1] < O.prep_cap) {
                    if (P.proto == MPX_MODE_MIN) {  // Id, Instance, OK, Ballot, LastCommitted
                        mpx_prepare_reply_min r;
                        r.id = le32(by, a + 1);
                        r.instance = le32(by, a + 5);
                        r.ok = by(a + 9);
                        r.ballot = le32(by, a + 10);
                        r.last_committed = le32(by, a + 14);
                        r.value_id = (uint32_t)idx[2];
                        static_cast<mpx_prepare_reply_min*>(O.prep)[idx[1]] = r;
                    } else {  // Instance, OK, Ballot
                        mpx_prepare_reply r;
                        r.instance = le32(by, a + 1);
                        r.ok = by(a + 5);
                        r.ballot = le32(by, a + 6);
                        r.value_id = (uint32_t)idx[2];
                        static_cast<mpx_prepare_reply*>(O.prep)[idx[1]] = r;
                    }
                }
                ++idx[1];
            }
            if (idx[2] < O.var_cap) {
                mpx_var_frame v;
                v.offset = (uint32_t)(P.pos_base + a);
                v.length = f.len;
                v.n_cmds = f.n_cmds;
                v.cmds_off = (uint32_t)(P.pos_base + f.cmds_off);
                v.n_log = f.n_log;
                v.log_off = (uint32_t)(P.pos_base + f.log_off);
                v.code = (uint8_t)code;
#pragma unroll
                for (int k = 0; k < 7; ++k) v.pad[k] = 0;
                O.var[idx[2]] = v;
            }
            ++idx[2];
            if (at_stop) {
                live = false;
                return;
            }
        } else if (code == MPX_PEER_ACCEPT_REPLY) {
            // a complete fixed frame, inside the LDS window: Instance, OK, Ballot, Id
            const uint32_t o = (uint32_t)(a - t0);
            rec = make_uint4((uint32_t)lds_le32(B, o + 1), (uint32_t)lds_le32(B, o + 6),
                             P.proto == MPX_MODE_MIN ? (uint32_t)lds_le32(B, o + 10) : 0xFFFFFFFFu,
                             (uint32_t)B[pofs(o + 5)]);
            is_ar = true;
        } else {
            if (idx[3] < O.oth_cap) {
                mpx_peer_frame f;
                f.offset = (uint32_t)(P.pos_base + a);
                f.code = (uint8_t)code;
                f.pad[0] = f.pad[1] = f.pad[2] = 0;
                O.oth[idx[3]] = f;
            }
            ++idx[3];
        }
        a += fl;
        live = a < c0 + kC;
    };
    uint4* const ar4 = reinterpret_cast<uint4*>(O.ar);  // mpx_accept_reply as 4 dwords
    uint64_t a = c0 + e;
    bool live = e != kDeadE;
    bool is_ar;
    uint4 rec;
#if MPX_SD_EMIT_REG
    // the lane's first kRegAR frames with their AcceptReplies held in registers ...
    uint4 rr[kRegAR];
    uint32_t rl[kRegAR];  // tile-local index, ~0 = none
#pragma clang loop unroll(full)
    for (int it = 0; it < kRegAR; ++it) {
        rl[it] = ~0u;
        if (live) {
            frame(a, live, is_ar, rec);
            if (is_ar) {
                rr[it] = rec;
                rl[it] = idx[0] < O.ar_cap ? (uint32_t)(idx[0] - ar0) : ~0u;
                ++idx[0];
            }
        }
    }
    if (__syncthreads_or(live)) {  // a chunk with more frames: every record stored directly
#pragma unroll
        for (int it = 0; it < kRegAR; ++it)
            if (rl[it] != ~0u) ar4[ar0 + rl[it]] = rr[it];
        while (live) {
            frame(a, live, is_ar, rec);
            if (is_ar) {
                if (idx[0] < O.ar_cap) ar4[idx[0]] = rec;
                ++idx[0];
            }
        }
        return;
    }
    // ... then through LDS (the tile image is dead: every lane has left its walk) in passes of
    // kRegCap, so the tile's AcceptReplies leave as one coalesced run instead of a 16-byte store
    // per lane and frame 150 bytes apart
    uint4* const R = reinterpret_cast<uint4*>(B);
    for (uint32_t ph = 0; ph < tot[0]; ph += kRegCap) {
#pragma unroll
        for (int it = 0; it < kRegAR; ++it)
            if (rl[it] - ph < kRegCap) R[rl[it] - ph] = rr[it];
        __syncthreads();
        const uint32_t hi = tot[0] - ph < kRegCap ? tot[0] : ph + kRegCap;
        for (uint32_t i = ph + (uint32_t)l; i < hi; i += kTL)
            if (ar0 + i < O.ar_cap) ar4[ar0 + i] = R[i - ph];
        __syncthreads();
    }
#else
    while (live) {
        frame(a, live, is_ar, rec);
        if (is_ar) {
            if (idx[0] < O.ar_cap) ar4[idx[0]] = rec;
            ++idx[0];
        }
    }
#endif
}

// an empty call ([start, len) holds no byte): END, counts unchanged
__global__ void k_sd_empty(mpx_stream_result* res, uint64_t at) {
    res->consumed = at;
    res->next = at;
    res->stop_reason = MPX_DECODE_END;
    res->stop_code = -1;
}

// ---- host side ----------------------------------------------------------------------------
namespace {
struct Layout {
    uint64_t cmap, tconv, tmap, tent, gmap, gent, tcnt, tpre, btot, boff, ticket, cinfo, stop, total;
};
Layout layout_of(uint64_t len) {
    const uint64_t tiles = n_tiles_of(len + 16), groups = (tiles + kGT - 1) / kGT;
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    Layout L{};
    uint64_t o = 0;
    L.cmap = o; o += al(tiles * kTL * kE);
    L.tconv = o; o += al(tiles * kTEnt);
    L.tmap = o; o += al(tiles * kE);
    L.tent = o; o += al(tiles);
    L.gmap = o; o += al(groups * kE);
    L.gent = o; o += al(groups);
    L.tcnt = o; o += al(tiles * 16);
    L.tpre = o; o += al(tiles * 16);
    L.btot = o; o += al((tiles / 1024 + 1) * 16);
    L.boff = o; o += al((tiles / 1024 + 1) * 16);
    L.ticket = o; o += al(4);
    L.cinfo = o; o += al(tiles * kTL * 8);
    L.stop = o; o += al(12 * 8);
    L.total = o;
    return L;
}
}  // namespace

uint64_t stream_work_bytes(uint64_t len) { return layout_of(len).total; }

hipError_t launch_decode_stream(int proto, int legacy, const uint8_t* buf, uint64_t len,
                                uint64_t start, const StreamOuts& outs, mpx_stream_result* res,
                                void* work, uint64_t work_bytes, hipStream_t stream) {
    if (len > (uint64_t)MPX_DECODE_MAX_BYTES || start > len) return hipErrorInvalidValue;
    if (work_bytes < stream_work_bytes(len)) return hipErrorInvalidValue;
    if (start == len) {
        k_sd_empty<<<1, 1, 0, stream>>>(res, start);
        return hipGetLastError();
    }
    const uint64_t base = start & ~15ull;
    SParams P{buf + base, len - base, base, (uint32_t)(start - base), proto, legacy};
    // one tile more when len is a multiple of the tile: position len is a terminal the chain
    // must be able to land on
    const uint32_t tiles = (uint32_t)n_tiles_of(P.len + 1);
    const uint32_t groups = (tiles + kGT - 1) / kGT;
    const Layout L = layout_of(len);
    char* w = (char*)work;
    Work W{(uint8_t*)(w + L.cmap), (uint8_t*)(w + L.tconv), (uint8_t*)(w + L.tmap), (uint8_t*)(w + L.tent),
           (uint8_t*)(w + L.gmap), (uint8_t*)(w + L.gent), (uint32_t*)(w + L.tcnt),
           (uint32_t*)(w + L.tpre), (uint32_t*)(w + L.btot), (uint32_t*)(w + L.boff),
           (uint32_t*)(w + L.ticket), (uint2*)(w + L.cinfo), (uint64_t*)(w + L.stop)};
    const hipError_t r = hipMemsetAsync(w + L.ticket, 0, 4, stream);
    if (r != hipSuccess) return r;
    Outs O{outs.ar, outs.ar_cap, outs.prep, outs.prep_cap, outs.var, outs.var_cap, outs.oth,
           outs.oth_cap};
    k_sd_tile_maps<<<tiles, kTL, 0, stream>>>(P, W);
    k_sd_group_maps<<<groups, kParts * kE, 0, stream>>>(W, tiles);
    k_sd_walk<<<1, kParts * kE, 0, stream>>>(P, W, tiles, groups, res);
    k_sd_tile_entries<<<groups, kParts * kE, 0, stream>>>(W, tiles);
    k_sd_count<<<tiles, kTL, 0, stream>>>(P, W);
#if MPX_SD_TENT && MPX_SD_TCNT
    k_sd_count_conv<<<tiles, kWave, 0, stream>>>(P, W);
#endif
    k_sd_scan<<<(tiles + kScanT - 1) / kScanT, kScanT, 0, stream>>>(W, tiles);
    k_sd_emit<<<tiles, kTL, 0, stream>>>(P, W, O, tiles, res);
    return hipGetLastError();
}

}  // namespace mpx
