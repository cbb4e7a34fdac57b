// apply_small.hip — mpx_apply for replica-sized calls (at most 16384 commands: up to three
// drained MAX_BATCH batches).
//
// Reference: executeCommands (src/bareminpaxos/bareminpaxos.go:1066-1098) drains one committed
// batch (MAX_BATCH = 5000 commands, :22) and runs (*state.Command).Execute (src/state/state.go:
// 77-103) on each in log order; conf_prev[i] = state.Conflict (state.go:53-60) of command i with
// the previous command on the same key in the call. The replica shim calls mpx_apply once per
// drained batch, so the call's cost is its latency, not its bandwidth. Three launches, a thread
// per command (the call's scattered table accesses spread over many CUs' memory pipelines):
//   1. k_small_probe: PUTs find or claim their slot in the engine's table (kvtab.hpp, 64-bit
//      CAS), the other commands look theirs up; every command's default result goes out (PUT its
//      value, GET the table value at call start, the rest NIL); a command with a slot pushes its
//      position onto the slot's command list (one atomicExch on a per-slot head word tagged with
//      the call, the previous head and the command's PUT bit into its link word).
//   2. k_small_reprobe: the lookups that met a free slot probe again from there (a PUT of the
//      call may have claimed it since) and join the list; a key with no slot is final (NIL, no
//      conflict).
//   3. k_small_walk: each command walks its slot's list (every command of the call on its key,
//      in no particular order): the nearest earlier command gives conf, the nearest earlier PUT a
//      GET's result, and the PUT with no later PUT commits the key's value (and present bit).
//      Lists of a replica batch over a large key space hold one or two commands; a walk longer
//      than kWalkMax marks the command LONG instead.
//   4. the walk kernel's last workgroup returns at once unless a command is LONG; then it
//      resolves the LONG commands (all of every long list) in LDS: each slot gets a dense group id
//      (LDS open addressing), the (id, position) pairs are sorted by id, stably (a counting rank
//      for up to 1024 entries, else two 7-bit LSD passes with bit-sliced ballot ranks and one
//      2048-entry scan), and over the sorted groups the previous command on the key is the left
//      neighbour (conf), the last PUT before a command a segmented exclusive max-scan of PUT
//      positions (GET results), and each group's last PUT is committed.
// The call epoch is neither read nor advanced: conflicts never reach across calls (orc_apply),
// and the tags other pipelines compare stay older than their next epoch.
#include "common.hpp"
#include "kernels.hpp"
#include "kvtab.hpp"

namespace mpx {

// Diagnostic build only (-DMPX_SMALL_STAMP=1, tools/stamp_small.py): thread 0 adds the
// s_memrealtime (100 MHz) delta of each phase to a global accumulator.
#ifndef MPX_SMALL_STAMP
#define MPX_SMALL_STAMP 0
#endif
#if MPX_SMALL_STAMP
__device__ unsigned long long mpx_small_stamp[16];
#define SM_STAMP(k)                                                              \
    do {                                                                         \
        if (threadIdx.x == 0) {                                                  \
            const unsigned long long _n = __builtin_amdgcn_s_memrealtime();       \
            atomicAdd(&mpx_small_stamp[k], _n - _sm_prev);                       \
            _sm_prev = _n;                                                       \
        }                                                                        \
    } while (0)
#else
#define SM_STAMP(k) \
    do {            \
    } while (0)
#endif

namespace {
constexpr int kSmT = 1024;                 // threads of the workgroup
constexpr int kSmWaves = kSmT / kWave;     // 16
constexpr int kSmPer = 16;                 // commands per thread
constexpr int kSmMax = kSmT * kSmPer;      // 16384 = MPX_APPLY_SMALL_MAX
// LDS id table of the LONG slots: a LONG list holds more than kWalkMax commands, so a call has
// at most kSmMax / (kWalkMax + 1) = 963 LONG slots (load <= 0.47)
constexpr int kSmHash = 2048;
constexpr uint32_t kNoId = kSmHash - 1;    // reserved: commands without a slot sort last
constexpr int kPosBits = 14;
constexpr uint32_t kPosMask = (1u << kPosBits) - 1;
constexpr int kDigit = 6;                  // radix digit bits (2 passes cover the 11-bit id)
constexpr int kDigits = 1 << kDigit;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr uint32_t kShared = 0x80000000u;  // tab: a second command joined the slot
constexpr uint8_t kOpPresent = 0x80;       // LDS op byte: the key was present at call start
static_assert(kSmMax == MPX_APPLY_SMALL_MAX, "small apply capacity");
// command lists (steps 1-3): lhead[slot] = tag << 14 | position of the last command pushed;
// probe[kLinkOff + p] = the position pushed before p (kLinkEnd: none) | kLinkPut if p is a PUT
constexpr uint32_t kLinkEnd = 0xFFFFu;
constexpr uint32_t kLinkPut = 1u << 16;
constexpr uint32_t kLongBit = 0x80000000u;  // probe[p] after the walk: p's list is long
constexpr int kWalkMax = 16;                // longest list a walk resolves
constexpr uint32_t kLinkOff = 2 * kSmMax;
constexpr uint32_t kCtlOff = kSmallCtl;     // probe[kCtlOff]: LONG commands, [+1]: last call's tag
static_assert(kCtlOff == 3 * kSmMax && kCtlOff + 3 <= kSmallKeyOff, "small apply scratch");
static_assert(kSmMax <= (1 << kPosBits) && (kSmallTagMax << kPosBits) == 0, "tagged list head");

struct SmallLds {
    uint32_t tab[kSmHash];          // group id -> slot + 1 (0 = free)             8 KB
    uint32_t buf[2][kSmMax];        // (id << 14 | position), radix ping-pong     128 KB
    uint32_t cnt[kSmWaves][kDigits];  // per wave and digit: counts, then offsets  4 KB
    uint8_t op[kSmMax];             // op by position                              16 KB
    uint32_t wsum[kSmWaves];        // block scan: wave totals
    int32_t wv[kSmWaves];           // segmented scan: wave values
    uint32_t wf[kSmWaves];          //                 and head flags
    uint32_t n_new;                 // slots that became present
};

__device__ __forceinline__ uint32_t hash_slot(uint32_t s) {
    s ^= s >> 16;
    s *= 0x7feb352dU;
    s ^= s >> 15;
    s *= 0x846ca68bU;
    s ^= s >> 16;
    return s;
}

// exclusive prefix sum of v over the workgroup (thread order); all threads call
__device__ __forceinline__ uint32_t block_excl_sum(SmallLds& S, uint32_t v) {
    const int l = lane_id(), w = threadIdx.x / kWave;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (l >= d) x += y;
    }
    if (l == kWave - 1) S.wsum[w] = x;
    __syncthreads();
    uint32_t before = 0;
    for (int i = 0; i < w; ++i) before += S.wsum[i];
    __syncthreads();  // wsum is reused by the next call
    return before + x - v;
}
}  // namespace

// ---- 1. probe: one command per thread, spread over many CUs ---------------------------------
// A PUT finds or claims its key's slot (linear probe in the key's bucket, 64-bit CAS,
// kvtab.hpp); another command stops at its key or at the first free slot (a PUT of the same call
// may claim the key there later: k_small_reprobe probes those again from the position recorded
// here). Every command's default result goes out now: PUT its value, GET the value at call start
// (present ? value : NIL), the rest NIL; a slot's state word is kept for the commits.
// probe[p] = slot | kMissBit (resume position) | kNoSlot; probe[kSmMax + p] = state word.
constexpr uint32_t kMissBit = 0x80000000u;
constexpr int kProbeBlock = 256;
// MPX_SMALL_FOLD=1 (A/B builds): the re-probe runs at the start of the walk kernel, its
// workgroups then meet at a grid barrier (all of them are resident: at most 16, one per CU)
// before the walks, so a call is two launches; 0 (the default): three launches. Same-box A/B
// (5000 / 16000 commands, events): 14.0-14.2 / 14.4-14.5 us folded vs 13.7-13.9 / 14.0-14.1 us
// - the grid barrier costs what the launch it saves does
#ifndef MPX_SMALL_FOLD
#define MPX_SMALL_FOLD 0
#endif

// push command p onto its slot's list of this call
__device__ __forceinline__ uint32_t call_tag(const KvTable& t) { return t.probe[kCtlOff + 1] + 1u; }
__device__ __forceinline__ void list_push(const KvTable& t, uint32_t tag, uint32_t slot, uint32_t p,
                                          bool put) {
    const uint32_t old = atomicExch(&t.lhead[slot], (tag << kPosBits) | p);
    const uint32_t nx = (old >> kPosBits) == tag ? (old & kPosMask) : kLinkEnd;
    // (at the device's coherence point: a re-probe's push is walked by other workgroups of the
    // same kernel)
    __hip_atomic_store(&t.probe[kLinkOff + p], nx | (put ? kLinkPut : 0u), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// command p's probe (k_small_probe, and the one-launch form's first phase)
__device__ __forceinline__ void probe_cmd(const KvTable& t, uint32_t tag, uint8_t o, int64_t k,
                                          int64_t v, uint32_t p, int64_t* __restrict__ ret,
                                          uint32_t* err) {
    const bool put = o == MPX_OP_PUT;
    if (put) ret[p] = v;  // a PUT returns its value
    uint32_t slot = kNoSlot;
    if (k == kSentinel) {
        slot = (uint32_t)t.cap;  // the sentinel key lives in the side slot
    } else {
        const uint64_t h = hash64((uint64_t)k);
        const uint32_t base = bucket_of(h, t.lgnb) << kLgSB;
        uint32_t sp = home_of(h);
        for (int step = 0; step < kSB; ++step, sp = (sp + 1) & (kSB - 1)) {
            unsigned long long* a = reinterpret_cast<unsigned long long*>(t.keys + base + sp);
            unsigned long long cur = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == (unsigned long long)kSentinel) {
                if (!put) {  // not in the table (yet)
                    slot = kMissBit | (base + sp);
                    break;
                }
                cur = atomicCAS(a, (unsigned long long)kSentinel, (unsigned long long)k);
                if (cur == (unsigned long long)kSentinel) {
                    slot = base + sp;  // claimed
                    break;
                }
            }
            if ((int64_t)cur == k) {
                slot = base + sp;
                break;
            }
        }
        // a PUT that finds its bucket full fails the call; a lookup that walks a full bucket
        // without its key is absent (NIL, no table change), as on the other pipelines
        // (a plain read-modify-write: err may live in host memory, where device atomics are not
        // available; the threads of this kernel only ever add the same bit)
        if (slot == kNoSlot && put && err) *(volatile uint32_t*)err |= kErrKvFull;
    }
    uint32_t st = 0;
    if (!(slot & kMissBit)) {  // (kNoSlot has the bit too)
        // the slot's state and value at call start are loaded before the push (they do not
        // depend on it): one round trip for the three instead of three
        st = t.state[slot];
        const int64_t v0 = t.vals[slot];
        list_push(t, tag, slot, p, put);
        if (!put) ret[p] = (o == MPX_OP_GET && (st & kPresent)) ? v0 : 0;
    } else if (!put) {
        ret[p] = 0;  // absent at call start: NIL (a PUT of this call cannot precede a miss)
    }
    t.probe[p] = slot;
    t.probe[kSmMax + p] = st;
}

__global__ __launch_bounds__(kProbeBlock) void k_small_probe(KvTable t, const uint8_t* __restrict__ op,
                                                       const int64_t* __restrict__ key,
                                                       const int64_t* __restrict__ val, uint32_t m,
                                                       int64_t* __restrict__ ret, uint32_t* err,
                                                       bool host_out) {
    const uint32_t p = blockIdx.x * kProbeBlock + threadIdx.x;
    if (p >= m) return;
    const uint32_t tag = call_tag(t);
    const uint8_t o = op[p];
    const int64_t k = key[p];
    const int64_t v = val[p];
    // the later kernels read the commands from here (device memory)
    reinterpret_cast<int64_t*>(t.probe + kSmallKeyOff)[p] = k;
    reinterpret_cast<int64_t*>(t.probe + kSmallValOff)[p] = v;
    reinterpret_cast<uint8_t*>(t.probe + kSmallOpOff)[p] = o;
    probe_cmd(t, tag, o, k, v, p, ret, err);
    // host-mapped results: performed at system scope before the kernel ends, so the walk kernel's
    // completion flag (stored after its own results) can never overtake them
    if (host_out) __threadfence_system();
}

// ---- 2. the lookups that met a free slot, again now that every claim of the call is in --------
// (the slots before the recorded position hold other keys for good); a key found now was claimed
// by this call: not present at call start, state word 0 (as recorded)
__device__ __forceinline__ void reprobe_one(const KvTable& t, const int64_t* __restrict__ key,
                                            uint32_t m, uint32_t p) {
    if (p >= m) return;
    const uint32_t s = t.probe[p];
    if (s == kNoSlot || !(s & kMissBit)) return;
    const int64_t k = key[p];
    uint32_t pos = s & ~kMissBit, slot = kNoSlot;
    for (int step = 0; step < kSB; ++step) {
        const unsigned long long c = __hip_atomic_load(
            reinterpret_cast<unsigned long long*>(t.keys + pos), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT);
        if ((int64_t)c == k) {
            slot = pos;
            break;
        }
        if (c == (unsigned long long)kSentinel) break;  // absent, and no PUT of this call
        pos = (pos & ~(uint32_t)(kSB - 1)) | ((pos + 1) & (kSB - 1));
    }
    if (slot != kNoSlot) list_push(t, call_tag(t), slot, p, false);  // (a miss is never a PUT)
    // (read by the LONG phase, maybe in another workgroup of the same kernel)
    __hip_atomic_store(&t.probe[p], slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kProbeBlock) void k_small_reprobe(KvTable t,
                                                         const int64_t* __restrict__ key,
                                                         uint32_t m) {
    reprobe_one(t, key, m, blockIdx.x * kProbeBlock + threadIdx.x);
}

// every workgroup of the grid here before any goes on (all are resident: the walk grid is at most
// kSmMax / kSmT = 16 one-per-CU workgroups). Each thread's agent-scope stores are performed before
// its workgroup arrives. A bounded wait: past ~0.2 s the call fails (kErrInval) instead of hanging.
constexpr uint32_t kGridCtr = kCtlOff + 3;  // the arrivals (reset by the call's last workgroup)
__device__ __forceinline__ void grid_barrier(const KvTable& t, uint32_t* err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t* ctr = &t.probe[kGridCtr];
        (void)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins == (1u << 22)) {
                if (err) *(volatile uint32_t*)err |= kErrInval;
                break;
            }
        }
    }
    __syncthreads();
}

// ---- 3. the list walks ----------------------------------------------------------------------
// Command p's list holds every command of the call on its key. The nearest earlier one decides
// conf (state.Conflict: either is a PUT), the nearest earlier PUT a GET's result, and the PUT
// with no later PUT is the key's value after the call. A list longer than kWalkMax is left to the
// LONG phase (its commands marked LONG, counted in probe[kCtlOff]). Returns the commands it made
// present / marked LONG through fresh / lng.
__device__ __forceinline__ void walk_one(const KvTable& t, const uint8_t* __restrict__ op,
                                         const int64_t* __restrict__ val, uint32_t m, uint32_t p,
                                         int64_t* __restrict__ ret, uint8_t* __restrict__ conf,
                                         bool& fresh, bool& lng) {
    const bool v = p < m;
    const uint32_t pc = v ? p : 0u;  // (every load issued at once, clamped, before any use)
    const uint32_t slot0 = t.probe[pc];
    const uint8_t o0 = op[pc];
    const uint32_t mine = __hip_atomic_load(&t.probe[kLinkOff + pc], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t st = t.probe[kSmMax + pc];
    const uint32_t slot = v ? slot0 : kNoSlot;
    const uint8_t o = v ? o0 : (uint8_t)MPX_OP_NONE;
    fresh = false;
    lng = false;
    if (slot != kNoSlot) {
        // (tagged with this call: p is on the list; agent scope: pushes of this kernel)
        uint32_t q = __hip_atomic_load(&t.lhead[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
                     kPosMask;
        int32_t prev = -1, last_put = -1;
        bool prev_put = false, later_put = false;
        int n = 0;
        for (; q != kLinkEnd; ++n) {
            if (n == kWalkMax) {
                lng = true;
                break;
            }
            const uint32_t w = q == p ? mine
                                      : __hip_atomic_load(&t.probe[kLinkOff + q], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
            const bool put_q = (w & kLinkPut) != 0;
            if (q < p) {
                if ((int32_t)q > prev) {
                    prev = (int32_t)q;
                    prev_put = put_q;
                }
                if (put_q && (int32_t)q > last_put) last_put = (int32_t)q;
            } else if (q > p) {
                later_put |= put_q;
            }
            q = w & kLinkEnd;
        }
        if (lng) {
            // read by the grid's last workgroup (the LONG phase), maybe on another XCD: stored
            // at the device's coherence point
            __hip_atomic_store(&t.probe[p], slot | kLongBit, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const bool put = (mine & kLinkPut) != 0;
            if (conf) conf[p] = (prev >= 0 && (put || prev_put)) ? 1 : 0;
            if (put) {
                if (!later_put) {  // the key's value after the call
                    t.vals[slot] = val[p];
                    if (!(st & kPresent)) {
                        t.state[slot] = st | kPresent;
                        fresh = true;
                    }
                }
            } else if (o == MPX_OP_GET && last_put >= 0) {
                ret[p] = val[last_put];  // the last PUT before it (other ops return NIL)
            }
        }
    } else if (v && conf) {
        conf[p] = 0;  // nothing precedes it on a PUT-less key
    }
}

// ---- 4. the LONG lists: the walk kernel's last workgroup ----------------------------------------
// The call's last workgroup also closes it: the LONG count and the ticket back to 0 and the next
// call's tag; after the call with the last tag every list head is cleared and the tags restart at
// 1 (once per 2^18 - 1 calls: one workgroup's pass over the heads). All threads call it.
// the host form's completion flag: every result of the call is visible to the host before it
__device__ __forceinline__ void signal_done(uint32_t* done, uint32_t seq) {
    if (!done) return;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void end_of_call(const KvTable& t, uint32_t tag) {
    __syncthreads();  // every thread has read the control words
    const bool wrap = tag + 1u >= kSmallTagMax;
    if (wrap) {
        for (uint64_t i = threadIdx.x; i <= t.cap; i += blockDim.x) t.lhead[i] = 0u;
    }
    if (threadIdx.x == 0) {
        (void)atomic_take(&t.probe[kCtlOff]);
        (void)atomic_take(&t.probe[kGridCtr]);
        t.probe[kCtlOff + 1] = wrap ? 0u : tag;
    }
}

// The walks (a thread per command, kSmT per workgroup: a replica batch takes a few CUs; the
// workgroups carry the LONG phase's LDS, so one runs per CU), then the LONG phase in the grid's
// last workgroup: its LONG marks and counts reach the device's coherence point (agent-scope atomic
// stores, awaited atomic adds) before its ticket, and the last workgroup reads them the same way.
// The LONG lists (commands marked LONG by the walks; own != nullptr: only the positions whose
// bit is set, the calling workgroup's partition), resolved by the calling workgroup in LDS. All
// threads call it.
__device__ void long_lists(SmallLds& S, const KvTable& t, const uint8_t* __restrict__ op,
                           const int64_t* __restrict__ val, uint32_t m, int64_t* __restrict__ ret,
                           uint8_t* __restrict__ conf, const uint32_t* own) {
#if MPX_SMALL_STAMP
    unsigned long long _sm_prev = __builtin_amdgcn_s_memrealtime();
    const unsigned long long _sm_rt0 = _sm_prev, _sm_clk0 = __builtin_amdgcn_s_memtime();
#endif
    const int tid = threadIdx.x, l = lane_id(), w = tid / kWave;
    const uint64_t below = lanes_below(l);
    for (int i = tid; i < kSmHash; i += kSmT) S.tab[i] = 0;
    if (tid == 0) S.n_new = 0;

    uint8_t o8[kSmPer];
    uint32_t slot[kSmPer];     // kNoSlot: finished by k_small_walk (or no slot at all)
    bool pres[kSmPer];
    const uint32_t p0 = (uint32_t)(w * (kSmPer * kWave) + l);  // position of k: p0 + 64 k
    {
        uint32_t st[kSmPer];
#pragma unroll
        for (int k = 0; k < kSmPer; ++k) {  // every load in flight before the first use
            const uint32_t p = p0 + k * kWave;
            const bool v = p < m;
            o8[k] = v ? op[p] : (uint8_t)MPX_OP_NONE;
            const uint32_t s = v ? __hip_atomic_load(&t.probe[p], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)
                                 : kNoSlot;
            slot[k] = s != kNoSlot && (s & kLongBit) && (!own || ((own[p >> 5] >> (p & 31)) & 1u))
                          ? s & ~kLongBit
                          : kNoSlot;
            st[k] = v ? t.probe[kSmMax + p] : 0u;
        }
        SM_STAMP(0);
        SM_STAMP(1);
#pragma unroll
        for (int k = 0; k < kSmPer; ++k) {
            const uint32_t p = p0 + k * kWave;
            pres[k] = (st[k] & kPresent) != 0;
            if (p >= m) continue;
            S.op[p] = (uint8_t)(o8[k] | (pres[k] ? kOpPresent : 0));  // op + present at call start
        }
    }
    SM_STAMP(2);
    SM_STAMP(3);
    // ---- 4a. group ids, the stable sort by id ------------------------------------------------
    // Each slot gets a dense id (LDS open addressing: tab[id] = slot + 1, bit 31 set once a
    // second command of the call joins the slot); the LONG commands are sorted and scanned,
    // compacted in log order.
    __syncthreads();  // tab cleared
    uint32_t id[kSmPer];
#pragma unroll
    for (int k = 0; k < kSmPer; ++k) {
        const uint32_t p = p0 + k * kWave;
        id[k] = kNoId;
        if (p >= m || slot[k] == kNoSlot) continue;
        const uint32_t want = slot[k] + 1u;
        uint32_t h = hash_slot(want) & (kSmHash - 1);
        for (;;) {
            if (h == kNoId) h = 0;
            const uint32_t cur = atomicCAS(&S.tab[h], 0u, want);
            if (cur == 0u) break;
            if ((cur & ~kShared) == want) {
                if (!(cur & kShared)) atomicOr(&S.tab[h], kShared);
                break;
            }
            h = (h + 1) & (kSmHash - 1);
        }
        id[k] = h;
    }
    __syncthreads();
    // every command here is LONG, i.e. on a list of more than kWalkMax commands, so none is alone
    // on its key: each gets its rank in log order (wave w holds positions [1024 w, 1024 w + 1024),
    // round k of it the 64 positions 1024 w + 64 k + lane)
    uint32_t m2, rank[kSmPer];
    bool shared[kSmPer];
    uint32_t n_new = 0;
    {
        uint32_t before = 0;
#pragma unroll
        for (int k = 0; k < kSmPer; ++k) {
            shared[k] = id[k] != kNoId;
            const uint64_t b = __ballot(shared[k]);
            rank[k] = before + (uint32_t)popc(b & below);
            before += (uint32_t)popc(b);
        }
        if (l == 0) S.wsum[w] = before;
        __syncthreads();
        uint32_t off = 0;
        m2 = 0;
        for (int i = 0; i < kSmWaves; ++i) {
            off += i < w ? S.wsum[i] : 0u;
            m2 += S.wsum[i];
        }
#pragma unroll
        for (int k = 0; k < kSmPer; ++k) {
            if (shared[k]) S.buf[0][off + rank[k]] = (id[k] << kPosBits) | (p0 + k * kWave);
        }
    }
    SM_STAMP(4);
    // the shared commands' (id, position) pairs, stably by id: two 7-bit LSD passes; entry j of
    // a pass is held by thread (j / 512) * 64 + j % 64, like the positions above
#ifndef MPX_SMALL_RANK
#define MPX_SMALL_RANK 1
#endif
    if (MPX_SMALL_RANK && m2 <= (uint32_t)kSmT) {
        // few shared commands (a batch over a large key space): each entry's rank is the count
        // of smaller entries (id << 14 | position is unique, so the order is stable), one pass
        // of broadcast LDS reads instead of the two radix passes' dozen barriers
        __syncthreads();  // every shared command's entry is in buf[0]
        const uint32_t e = (uint32_t)tid < m2 ? S.buf[0][tid] : 0u;
        uint32_t r = 0;
        if ((uint32_t)tid < m2) {
            const uint4* b4 = reinterpret_cast<const uint4*>(S.buf[0]);
            const uint32_t n4 = m2 / 4;
            for (uint32_t i = 0; i < n4; ++i) {
                const uint4 q = b4[i];
                r += (q.x < e) + (q.y < e) + (q.z < e) + (q.w < e);
            }
            for (uint32_t i = n4 * 4; i < m2; ++i) r += S.buf[0][i] < e;
        }
        __syncthreads();
        if ((uint32_t)tid < m2) S.buf[0][r] = e;
    } else
    for (int pass = 0; pass < 2; ++pass) {
        const uint32_t* src = S.buf[pass];
        uint32_t* dst = S.buf[pass ^ 1];
        for (int i = tid; i < kDigits * kSmWaves; i += kSmT) (&S.cnt[0][0])[i] = 0;
        __syncthreads();
        uint32_t e[kSmPer], rk[kSmPer], dg[kSmPer];
        // wave w ranks its 512 positions in order, 64 at a time: lanes with the same digit by
        // bit-sliced ballots, the wave's running count per digit in its own cnt row
#pragma unroll
        for (int k = 0; k < kSmPer; ++k) {
            const uint32_t p = p0 + k * kWave;
            const bool v = p < m2;
            e[k] = v ? src[p] : 0xFFFFFFFFu;
            const uint32_t d = (e[k] >> (kPosBits + kDigit * pass)) & (kDigits - 1);
            dg[k] = d;
            uint64_t peers = __ballot(v);
#pragma unroll
            for (int b = 0; b < kDigit; ++b) {
                const uint64_t mb = __ballot((d >> b) & 1u);
                peers &= ((d >> b) & 1u) ? mb : ~mb;
            }
            const uint32_t run = S.cnt[w][d];
            rk[k] = run + (uint32_t)popc(peers & below);
            if (v && !(peers >> l >> 1))  // the group's last lane
                S.cnt[w][d] = run + (uint32_t)popc(peers);
        }
        __syncthreads();
        // offsets: exclusive scan of the counts in (digit, wave) order, one entry per thread
        static_assert(kDigits * kSmWaves == kSmT, "one (digit, wave) count per thread");
        {
            const uint32_t d = (uint32_t)tid / kSmWaves, w0 = (uint32_t)tid % kSmWaves;
            const uint32_t a = S.cnt[w0][d];
            const uint32_t ex = block_excl_sum(S, a);
            S.cnt[w0][d] = ex;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kSmPer; ++k)
            if (p0 + k * kWave < m2) dst[S.cnt[w][dg[k]] + rk[k]] = e[k];
        __syncthreads();
    }
    SM_STAMP(5);
    // ---- 4b. per group, in log order ---------------------------------------------------------
    // thread tid takes sorted entries q = 8 tid + j (blocked, two 16-byte LDS reads); groups of
    // kNoId (no slot) come last. The default results' stores are complete before any rewrite.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint32_t* srt = S.buf[0];
    const uint32_t q0 = (uint32_t)tid * kSmPer;
    uint32_t e[kSmPer];
#pragma unroll
    for (int v = 0; v < kSmPer / 4; ++v) {
        const uint4 a = reinterpret_cast<const uint4*>(srt)[(kSmPer / 4) * tid + v];
        e[4 * v] = a.x;
        e[4 * v + 1] = a.y;
        e[4 * v + 2] = a.z;
        e[4 * v + 3] = a.w;
    }
    const uint32_t e_prev = q0 > 0 && q0 - 1 < m2 ? srt[q0 - 1] : 0xFFFFFFFFu;
    const uint32_t e_next = q0 + kSmPer < m2 ? srt[q0 + kSmPer] : 0xFFFFFFFFu;
    uint8_t o[kSmPer];
#pragma unroll
    for (int j = 0; j < kSmPer; ++j) o[j] = q0 + j < m2 ? S.op[e[j] & kPosMask] : (uint8_t)0;
    const uint8_t o_prev =
        q0 > 0 && q0 - 1 < m2 ? (uint8_t)(S.op[e_prev & kPosMask] & ~kOpPresent) : (uint8_t)0;
    bool tpres[kSmPer];  // the key was present at call start
#pragma unroll
    for (int j = 0; j < kSmPer; ++j) {
        tpres[j] = (o[j] & kOpPresent) != 0;
        o[j] &= (uint8_t)~kOpPresent;
    }
    bool hd[kSmPer];
    int32_t ex[kSmPer];
    bool seen = false;  // a group starts in this thread at or before j
    int32_t run = -1;
#pragma unroll
    for (int j = 0; j < kSmPer; ++j) {
        const bool v = q0 + j < m2;
        const uint32_t before = j ? e[j - 1] : e_prev;
        hd[j] = v && (q0 + j == 0 || (before >> kPosBits) != (e[j] >> kPosBits));
        if (hd[j]) {
            run = -1;
            seen = true;
        }
        ex[j] = run;  // last PUT before it in the group, within this thread
        if (v && o[j] == MPX_OP_PUT) run = (int32_t)(e[j] & kPosMask);
    }
    // carry of the last PUT from earlier threads into this thread's open group: segmented scan
    // of (group starts in thread, last PUT) over the threads
    uint32_t f = seen ? 1u : 0u;
    int32_t x = run;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t fu = __shfl_up(f, d);
        const int32_t xu = __shfl_up(x, d);
        if (l >= d && !f) x = x > xu ? x : xu;
        if (l >= d) f |= fu;
    }
    if (l == kWave - 1) {
        S.wf[w] = f;
        S.wv[w] = x;
    }
    __syncthreads();
    int32_t cin = -1;  // inclusive scan of the earlier waves
    for (int i = 0; i < w; ++i) {
        if (S.wf[i]) cin = S.wv[i];
        else cin = cin > S.wv[i] ? cin : S.wv[i];
    }
    {  // exclusive value for this thread: the previous lane's inclusive, else the waves'
        const uint32_t fp = __shfl_up(f, 1);
        const int32_t xp = __shfl_up(x, 1);
        if (l > 0) cin = fp ? xp : (cin > xp ? cin : xp);
    }
    uint32_t cslot[kSmPer];  // commits: slot, or kNoSlot
    bool before_head = true;  // no group starts in this thread at or before j
#pragma unroll
    for (int j = 0; j < kSmPer; ++j) {
        cslot[j] = kNoSlot;
        before_head &= !hd[j];
        const uint32_t q = q0 + j;
        const uint32_t id = e[j] >> kPosBits, p = e[j] & kPosMask;
        if (q >= m2 || id == kNoId) continue;
        const int32_t pp = before_head ? (ex[j] > cin ? ex[j] : cin) : ex[j];
        if (conf) {
            const uint8_t ob = j ? o[j - 1] : o_prev;
            conf[p] = (!hd[j] && (ob == MPX_OP_PUT || o[j] == MPX_OP_PUT)) ? 1 : 0;
        }
        if (o[j] == MPX_OP_GET && pp >= 0) ret[p] = val[pp];  // the last PUT before it
        const uint32_t after = j + 1 < kSmPer ? e[j + 1] : e_next;
        const bool tail = q + 1 == m2 || (after >> kPosBits) != id;
        const int32_t lp = o[j] == MPX_OP_PUT ? (int32_t)p : pp;
        if (tail && lp >= 0) {  // the group's last PUT: the key's value after the call
            cslot[j] = (S.tab[id] & ~kShared) - 1u;
            t.vals[cslot[j]] = val[lp];
            if (!tpres[j]) {  // present from now on (the state word was read in step 1)
                atomicOr(&t.state[cslot[j]], kPresent);
                ++n_new;
            }
        }
    }
    if (n_new) atomicAdd(&S.n_new, n_new);
    __syncthreads();
    if (tid == 0 && S.n_new) atomicAdd(t.n_present, (unsigned long long)S.n_new);
    SM_STAMP(6);
#if MPX_SMALL_STAMP
    if (threadIdx.x == 0) {  // shader clock ticks and 100 MHz ticks of the LONG phase
        atomicAdd(&mpx_small_stamp[8], __builtin_amdgcn_s_memtime() - _sm_clk0);
        atomicAdd(&mpx_small_stamp[9], __builtin_amdgcn_s_memrealtime() - _sm_rt0);
    }
#endif
}

__global__ __launch_bounds__(kSmT) void k_small_walk(KvTable t, const uint8_t* __restrict__ op,
                                                     const int64_t* __restrict__ val, uint32_t m,
                                                     int64_t* __restrict__ ret,
                                                     uint8_t* __restrict__ conf, uint32_t* done,
                                                     uint32_t seq, const int64_t* __restrict__ key,
                                                     uint32_t* err) {
    __shared__ SmallLds S;
    if (MPX_SMALL_FOLD) {  // the re-probes, then every push of the call is in
        reprobe_one(t, key, m, blockIdx.x * kSmT + threadIdx.x);
        grid_barrier(t, err);
    }
    {
        bool fresh, lng;
        walk_one(t, op, val, m, blockIdx.x * kSmT + threadIdx.x, ret, conf, fresh, lng);
        const uint64_t bf = __ballot(fresh), bl = __ballot(lng);
        if (lane_id() == 0) {
            if (bf) atomicAdd(t.n_present, (unsigned long long)popc(bf));
            if (bl) atomic_add_done(&t.probe[kCtlOff], (uint32_t)popc(bl));
        }
    }
    if (done) __threadfence_system();  // this workgroup's host-mapped results, before its ticket
    if (!last_workgroup(&t.probe[kCtlOff + 2])) return;
    const uint32_t n_long = __hip_atomic_load(&t.probe[kCtlOff], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t tag = call_tag(t);
    if (n_long) long_lists(S, t, op, val, m, ret, conf, nullptr);  // (else every list was walked)
    end_of_call(t, tag);
    signal_done(done, seq);
}

// ---- the one-launch form (device-resident commands: mpx_apply_dev) -----------------------------
// Every workgroup reads every key and keeps the commands whose key hashes into its partition (the
// high 32 bits of hash64 scaled to the grid). All commands on a key are then in one workgroup,
// so steps 1-3 (probe, re-probe, walk) meet at workgroup barriers instead of kernel boundaries
// and the LONG lists of a partition are resolved by its own workgroup: one launch per call. (On
// MI355X an empty launch alone spans ~6 us between two events and each further one ~1.6 us,
// tools/launch_floor.hip; the three-launch form above keeps the host forms, whose commands sit in
// pinned host memory every workgroup would read over the link.) The grid's last workgroup
// (ticket) closes the call. Table slots are shared between partitions only as probe positions in
// a bucket: claims are device-scope CAS as in step 1, a key is probed and listed by one
// workgroup only.
#ifndef MPX_SMALL_PART
#define MPX_SMALL_PART 1
#endif
#ifndef MPX_SMALL_PART_CMDS
// commands per partition (the grid: the power of two >= m / this, at most kPartMax). Same-box
// A/B, 5000 / 16000 commands: 64 -> 9.9 / 14.2 us, 128 -> 9.3-9.6 / 13.1-13.3, 256 -> 9.7-10.0 /
// 13.7, 512 -> 10.4-10.6 / 15.2 (more partitions: fewer commands each, but every workgroup
// loads and hashes every key)
#define MPX_SMALL_PART_CMDS 128
#endif
constexpr uint32_t kPartMax = 256;  // one workgroup per CU (the LONG phase's LDS); a power of 2
#ifndef MPX_SMALL_FAST
#define MPX_SMALL_FAST 1  // 0 (A/B builds): every partition takes steps 1-4
#endif

// every store of the workgroup performed (list pushes, links, slots, state words), then a barrier
__device__ __forceinline__ void wg_barrier() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// Partition hash (phase 0 of the one-launch form): the key's two halves folded, a Fibonacci
// multiply, the top lgnp bits. Every workgroup hashes every key, so this stays one 32-bit
// multiply (hash64's two 64-bit ones cost ~4 us of VALU per workgroup at 16384 commands).
__device__ __forceinline__ uint32_t part_of(int64_t k, uint32_t lgnp) {
    const uint32_t x = ((uint32_t)k ^ (uint32_t)((uint64_t)k >> 32)) * 0x9E3779B1u;
    return lgnp ? x >> (32 - lgnp) : 0u;
}

// ---- the one-launch form's LDS resolve: a partition of at most kSmT commands, none of its keys
// on more than kWalkMax of them (the common case; anything else takes steps 1-4 above) ----------
// Command j of the partition is thread j. Its key goes into an LDS table of key hashes (hash64
// is a bijection, so equal hashes are equal keys; the sentinel key has an entry of its own) and
// gets a dense key id; the first thread to enter a key probes the engine's table for it once -
// its slot, state word and value at call start in one round trip from the home slot, a claim
// (64-bit CAS) when any command of the partition PUTs it - and every command then walks its
// key's LDS list (at most kWalkMax entries) for the nearest earlier command (conf), the nearest
// earlier PUT (a GET's result) and a later PUT (the last PUT commits). No list heads, links or
// re-probes in device memory: about four dependent round trips per call instead of ~11.
constexpr int kFTab = 2048;
constexpr uint32_t kFSent = kFTab - 1;              // the sentinel key's entry
constexpr uint64_t kHSent = 0x25c26ea579cea98aull;  // hash64(kSentinel): marks a free entry
struct PartFastLds {
    uint64_t th[kFTab];      // key hashes                                        16 KB
    int64_t v0[kSmT];        // per key id: the value at call start                8 KB
    int64_t cval[kSmT];      // per command: its value                             8 KB
    uint32_t slot[kSmT];     // per key id: its table slot (kNoSlot: absent)       4 KB
    uint32_t st[kSmT];       // per key id: its state word at call start           4 KB
    uint32_t head[kSmT];     // per key id: its list of commands (command + 1)     4 KB
    uint32_t cnt[kSmT];      // per key id: commands | PUTs << 16                  4 KB
    uint16_t id_of[kFTab];   // table entry -> key id                              4 KB
    uint16_t next[kSmT];     // per command: the next command on its key's list    2 KB
    uint8_t op[kSmT];        // per command: its op                                1 KB
    uint32_t nkeys, heavy;
};
static_assert(sizeof(PartFastLds) <= sizeof(uint32_t) * kSmMax, "overlays SmallLds::buf[0]");

// All threads call it; false (before any store to the table) when some key of the partition
// has more than kWalkMax commands. fresh: slots this thread made present.
__device__ bool part_fast(PartFastLds& F, const KvTable& t, const uint8_t* __restrict__ op,
                          const int64_t* __restrict__ key, const int64_t* __restrict__ val,
                          const uint32_t* lst, uint32_t no, int64_t* __restrict__ ret,
                          uint8_t* __restrict__ conf, uint32_t* err, uint32_t& fresh) {
    const uint32_t j = threadIdx.x;
    for (uint32_t i = j; i < (uint32_t)kFTab; i += kSmT) F.th[i] = kHSent;
    F.cnt[j] = 0u;
    F.head[j] = 0u;
    if (j == 0) {
        F.nkeys = 0u;
        F.heavy = 0u;
    }
    const bool act = j < no;
    const uint32_t p = act ? lst[j] : 0u;
    const uint8_t o = op[p];  // (p = 0 for the idle threads: every load unconditional)
    const int64_t k = key[p];
    const int64_t v = val[p];
    const bool put = act && o == MPX_OP_PUT;
    __syncthreads();  // table and counters cleared
    uint32_t e = 0;
    bool lead = false;
    uint64_t h = 0;
    if (act) {
        F.cval[j] = v;
        F.op[j] = o;
        if (k == kSentinel) {
            e = kFSent;
            lead = atomicCAS((unsigned long long*)&F.th[kFSent], (unsigned long long)kHSent, 0ull) ==
                   (unsigned long long)kHSent;
        } else {
            h = hash64((uint64_t)k);
            e = (uint32_t)(h >> 40) & (kFTab - 1);
            for (;;) {
                if (e == kFSent) e = 0;
                const unsigned long long cur =
                    atomicCAS((unsigned long long*)&F.th[e], (unsigned long long)kHSent,
                              (unsigned long long)h);
                if (cur == (unsigned long long)kHSent) {
                    lead = true;
                    break;
                }
                if (cur == (unsigned long long)h) break;
                e = (e + 1) & (kFTab - 1);
            }
        }
        if (lead) F.id_of[e] = (uint16_t)atomicAdd(&F.nkeys, 1u);
    }
    __syncthreads();  // every key has its id
    uint32_t id = 0;
    if (act) {
        id = F.id_of[e];
        const uint32_t c = atomicAdd(&F.cnt[id], 1u | (put ? 1u << 16 : 0u));
        if ((c & 0xFFFFu) == (uint32_t)kWalkMax) F.heavy = 1u;  // the list passes kWalkMax
        F.next[j] = (uint16_t)atomicExch(&F.head[id], j + 1u);
    }
    __syncthreads();  // counts and lists complete
    if (F.heavy) return false;
    if (lead) {  // the key's slot, state word and value at call start
        const bool anyput = (F.cnt[id] >> 16) != 0u;
        uint32_t slot = kNoSlot, st = 0u;
        int64_t v0 = 0;
        if (k == kSentinel) {
            slot = (uint32_t)t.cap;  // the side slot
            st = t.state[slot];
            v0 = t.vals[slot];
        } else {
            const uint32_t base = bucket_of(h, t.lgnb) << kLgSB;
            uint32_t sp = home_of(h);
            for (int step = 0; step < kSB; ++step, sp = (sp + 1) & (kSB - 1)) {
                unsigned long long* a = reinterpret_cast<unsigned long long*>(t.keys + base + sp);
                unsigned long long cur =
                    __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // (the slot's state and value in the same round trip: only this workgroup writes
                // them during the call, a claimed free slot's included)
                const uint32_t s1 = t.state[base + sp];
                const int64_t v1 = t.vals[base + sp];
                if (cur == (unsigned long long)kSentinel) {
                    if (!anyput) break;  // absent, and no PUT of the call
                    cur = atomicCAS(a, (unsigned long long)kSentinel, (unsigned long long)k);
                    if (cur == (unsigned long long)kSentinel) {
                        slot = base + sp;  // claimed
                        st = s1;
                        break;
                    }
                }
                if ((int64_t)cur == k) {
                    slot = base + sp;
                    st = s1;
                    v0 = v1;
                    break;
                }
            }
            if (slot == kNoSlot && anyput && err) *(volatile uint32_t*)err |= kErrKvFull;
        }
        F.slot[id] = slot;
        F.st[id] = st;
        F.v0[id] = v0;
    }
    __syncthreads();  // every key's slot
    fresh = 0u;
    if (act) {
        const uint32_t slot = F.slot[id], st = F.st[id];
        int32_t prev = -1, last_put = -1, lp_j = -1;
        bool prev_put = false, later_put = false;
        for (uint32_t q1 = F.head[id]; q1; q1 = F.next[q1 - 1]) {
            const uint32_t q = q1 - 1u;
            if (q == j) continue;
            const int32_t pq = (int32_t)lst[q];
            const bool put_q = F.op[q] == MPX_OP_PUT;
            if (pq < (int32_t)p) {
                if (pq > prev) {
                    prev = pq;
                    prev_put = put_q;
                }
                if (put_q && pq > last_put) {
                    last_put = pq;
                    lp_j = (int32_t)q;
                }
            } else {
                later_put |= put_q;
            }
        }
        int64_t r = 0;
        if (put) r = v;
        else if (o == MPX_OP_GET)
            r = lp_j >= 0 ? F.cval[lp_j] : (slot != kNoSlot && (st & kPresent)) ? F.v0[id] : 0;
        ret[p] = r;
        if (conf) conf[p] = (prev >= 0 && (put || prev_put)) ? 1 : 0;
        if (put && !later_put && slot != kNoSlot) {  // the key's value after the call
            t.vals[slot] = v;
            if (!(st & kPresent)) {
                t.state[slot] = st | kPresent;
                fresh = 1u;
            }
        }
    }
    return true;
}

__global__ __launch_bounds__(kSmT) void k_small_part(KvTable t, const uint8_t* __restrict__ op,
                                                     const int64_t* __restrict__ key,
                                                     const int64_t* __restrict__ val, uint32_t m,
                                                     int64_t* __restrict__ ret,
                                                     uint8_t* __restrict__ conf, uint32_t* err) {
    __shared__ SmallLds S;
    __shared__ uint32_t own[kSmMax / 32];  // bit p: command p is in this partition
    __shared__ uint32_t n_own, n_long, n_fresh;
    const int tid = threadIdx.x, l = lane_id();
    const uint64_t below = lanes_below(l);
    const uint32_t me = blockIdx.x, lgnp = 31u - (uint32_t)__builtin_clz(gridDim.x);
    const uint32_t tag = call_tag(t);
    if (tid == 0) {
        n_own = 0;
        n_long = 0;
        n_fresh = 0;
    }
    // ---- 0. the partition's positions: every key loaded at once (rounds of kSmT positions) ----
    int64_t kk[kSmPer];
#pragma unroll
    for (int i = 0; i < kSmPer; ++i) {
        const uint32_t p = (uint32_t)(i * kSmT + tid);
        if ((uint32_t)(i * kSmT) < m) kk[i] = key[p < m ? p : m - 1];
    }
    __syncthreads();  // counters zeroed
    uint32_t* lst = S.buf[1];  // this partition's positions, in no particular order
#pragma unroll
    for (int i = 0; i < kSmPer; ++i) {
        if ((uint32_t)(i * kSmT) >= m) break;
        const uint32_t p = (uint32_t)(i * kSmT + tid);
        const bool mine = p < m && part_of(kk[i], lgnp) == me;
        const uint64_t b = __ballot(mine);
        if ((l & 31) == 0 && p < m) own[p >> 5] = (uint32_t)(b >> (l & 32));
        if (b) {
            uint32_t base = 0;
            if (l == 0) base = atomicAdd(&n_own, (uint32_t)popc(b));
            base = (uint32_t)__shfl((int)base, 0);
            if (mine) lst[base + (uint32_t)popc(b & below)] = p;
        }
    }
    __syncthreads();
    const uint32_t no = n_own;
    if (MPX_SMALL_FAST && no <= (uint32_t)kSmT) {
        uint32_t fresh = 0;
        if (part_fast(*reinterpret_cast<PartFastLds*>(S.buf[0]), t, op, key, val, lst, no, ret,
                      conf, err, fresh)) {
            const uint64_t bf = __ballot(fresh != 0u);
            if (l == 0 && bf) atomicAdd(&n_fresh, (uint32_t)popc(bf));
            __syncthreads();
            if (tid == 0 && n_fresh) atomicAdd(t.n_present, (unsigned long long)n_fresh);
            if (last_workgroup(&t.probe[kCtlOff + 2])) end_of_call(t, tag);
            return;
        }
    }
    // ---- 1. probes -----------------------------------------------------------------------------
    for (uint32_t j = tid; j < no; j += kSmT) {
        const uint32_t p = lst[j];
        probe_cmd(t, tag, op[p], key[p], val[p], p, ret, err);
    }
    wg_barrier();
    // ---- 2. the lookups that met a free slot -----------------------------------------------------
    for (uint32_t j = tid; j < no; j += kSmT) reprobe_one(t, key, m, lst[j]);
    wg_barrier();
    // ---- 3. the walks --------------------------------------------------------------------------
    {
        uint32_t nf = 0, nl = 0;
        for (uint32_t j = tid; j < no; j += kSmT) {
            bool fresh, lng;
            walk_one(t, op, val, m, lst[j], ret, conf, fresh, lng);
            nf += fresh ? 1u : 0u;
            nl += lng ? 1u : 0u;
        }
        if (nf) atomicAdd(&n_fresh, nf);
        if (nl) atomicAdd(&n_long, nl);
    }
    wg_barrier();
    if (tid == 0 && n_fresh) atomicAdd(t.n_present, (unsigned long long)n_fresh);
    // ---- 4. this partition's LONG lists ----------------------------------------------------------
    if (n_long) long_lists(S, t, op, val, m, ret, conf, own);
    if (last_workgroup(&t.probe[kCtlOff + 2])) end_of_call(t, tag);
}

#if MPX_SMALL_STAMP
extern "C" int mpx_debug_small_stamps(unsigned long long* out16, int reset) {
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(mpx_small_stamp), 16 * sizeof(unsigned long long)) !=
        hipSuccess)
        return -3;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(mpx_small_stamp), z, sizeof(z)) != hipSuccess) return -3;
    }
    return 0;
}
#endif

hipError_t launch_apply_small(KvTable& t, const uint8_t* op, const int64_t* key, const int64_t* val,
                              uint64_t m, int64_t* ret, uint8_t* conf, uint32_t* err,
                              hipStream_t stream, uint32_t* done, uint32_t seq, bool host_io) {
    if (!m) return hipSuccess;
    if (m > (uint64_t)kSmMax || t.cap >= 0x7FFFFFFEull) return hipErrorInvalidValue;
    if (MPX_SMALL_PART && !host_io && !done) {
        // a power of two of partitions, about MPX_SMALL_PART_CMDS commands each
        unsigned np = 1;
        while (np < kPartMax && (uint64_t)np * MPX_SMALL_PART_CMDS < m) np <<= 1;
        k_small_part<<<np, kSmT, 0, stream>>>(t, op, key, val, (uint32_t)m, ret, conf, err);
        return hipGetLastError();
    }
    const unsigned g = (unsigned)((m + kProbeBlock - 1) / kProbeBlock);
    const int64_t* d_key = reinterpret_cast<const int64_t*>(t.probe + kSmallKeyOff);
    const int64_t* d_val = reinterpret_cast<const int64_t*>(t.probe + kSmallValOff);
    const uint8_t* d_op = reinterpret_cast<const uint8_t*>(t.probe + kSmallOpOff);
    k_small_probe<<<g, kProbeBlock, 0, stream>>>(t, op, key, val, (uint32_t)m, ret, err,
                                                 done != nullptr);
    if (!MPX_SMALL_FOLD) k_small_reprobe<<<g, kProbeBlock, 0, stream>>>(t, d_key, (uint32_t)m);
    k_small_walk<<<(unsigned)((m + kSmT - 1) / kSmT), kSmT, 0, stream>>>(
        t, d_op, d_val, (uint32_t)m, ret, conf, done, seq, d_key, err);
    return hipGetLastError();
}

}  // namespace mpx
