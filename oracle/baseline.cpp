// oracle/baseline.cpp — TEST/BENCH INFRASTRUCTURE ONLY: the CPU baseline that bench.py times
// beside the GPU ("cpu_baseline", kind "port").
//
// "Reference-faithful" restatement of the Go data structures on the hot path:
//   - instanceSpace []*Instance with a heap *LeaderBookkeeping per instance
//     (src/bareminpaxos/bareminpaxos.go:41,95 ; src/minpaxosproto/minpaxosproto.go:17-29)
//   - one sequential loop per reply, as the single run() goroutine does (bareminpaxos.go:344-349)
//   - state.State.Store as a hash map, one Execute per command in log order, as the single
//     executeCommands goroutine does (bareminpaxos.go:1066-1098, state.go:77-103)
// Only the per-reply / per-command loop is timed. The Go channel receive, unmarshal and
// per-message allocation that precede each handler call in the reference are NOT modelled,
// so this baseline is faster than the reference would be.
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../include/mpx.h"

namespace {

struct LeaderBookkeeping {  // minpaxosproto.go:24-29
    int32_t max_recv_ballot;
    int32_t accept_oks;
    int32_t nacks;
    void* client_proposals;
};
struct Instance {  // minpaxosproto.go:17-22
    int32_t ballot;
    int32_t status;
    LeaderBookkeeping* lb;
    void* cmds;
};

inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

struct Space {
    std::vector<Instance*> inst;
    explicit Space(const mpx_inst_state* st, size_t n) : inst(n) {
        for (size_t i = 0; i < n; ++i) {
            inst[i] = new Instance{0, st[i].status,
                                   new LeaderBookkeeping{st[i].max_recv_ballot, st[i].accept_oks,
                                                         st[i].nacks, nullptr},
                                   nullptr};
        }
    }
    ~Space() {
        for (auto* p : inst) { delete p->lb; delete p; }
    }
    void store(mpx_inst_state* st) const {
        for (size_t i = 0; i < inst.size(); ++i)
            st[i] = {inst[i]->status, inst[i]->lb->accept_oks, inst[i]->lb->nacks,
                     inst[i]->lb->max_recv_ballot};
    }
};

// the timed reply loop (MIN bareminpaxos.go:1014-1064 / CLASSIC paxos.go:631-673)
void reply_loop(int N, int mode, const mpx_accept_reply* recs, size_t n, Space& sp, int32_t base,
                int32_t* cu, int32_t* peer) {
    const int32_t half = (int32_t)N >> 1;
    for (size_t p = 0; p < n; ++p) {
        const mpx_accept_reply& a = recs[p];
        Instance* inst = sp.inst[a.instance - base];
        if (mode == MPX_MODE_MIN) {
            if (a.ok == 1) {
                inst->lb->accept_oks++;
                if (inst->lb->accept_oks + 1 > half) {
                    if (inst->lb->accept_oks == half) {
                        inst->status = MPX_COMMITTED;
                        *cu = a.instance;
                    }
                    peer[a.id] = a.instance - 1;
                }
            }
        } else {
            if (inst->status != MPX_PREPARED && inst->status != MPX_ACCEPTED) continue;
            if (a.ok == 1) {
                inst->lb->accept_oks++;
                if (inst->lb->accept_oks + 1 > half) {
                    inst->status = MPX_COMMITTED;
                    for (;;) {  // updateCommittedUpTo
                        int64_t nx = (int64_t)*cu + 1 - base;
                        if (nx < 0 || (size_t)nx >= sp.inst.size()) break;
                        if (sp.inst[nx]->status != MPX_COMMITTED) break;
                        *cu += 1;
                    }
                }
            } else {
                inst->lb->nacks++;
                if (a.ballot > inst->lb->max_recv_ballot) inst->lb->max_recv_ballot = a.ballot;
            }
        }
    }
}

inline int64_t execute(std::unordered_map<int64_t, int64_t>& s, uint8_t op, int64_t k, int64_t v) {
    if (op == MPX_OP_PUT) { s[k] = v; return v; }
    if (op == MPX_OP_GET) {
        auto it = s.find(k);
        if (it != s.end()) return it->second;
    }
    return 0;
}

}  // namespace

extern "C" {

// accept tally, one core. Returns elapsed ns of the reply loop; writes results back.
int64_t orc_bench_accept(int N, int mode, const mpx_accept_reply* recs, size_t n,
                         mpx_inst_state* st, size_t n_inst, int32_t base, int32_t* cu,
                         int32_t* peer) {
    Space sp(st, n_inst);
    int64_t t0 = now_ns();
    reply_loop(N, mode, recs, n, sp, base, cu, peer);
    int64_t t1 = now_ns();
    sp.store(st);
    return t1 - t0;
}

// KV apply, one core: Execute per command in log order on a hash map. Returns elapsed ns.
int64_t orc_bench_apply(const int64_t* init_keys, const int64_t* init_vals, size_t n_init,
                        const uint8_t* op, const int64_t* key, const int64_t* val, size_t m,
                        int64_t* ret) {
    std::unordered_map<int64_t, int64_t> s;
    s.reserve(n_init * 2 + 1024);
    for (size_t i = 0; i < n_init; ++i) s[init_keys[i]] = init_vals[i];
    int64_t t0 = now_ns();
    for (size_t i = 0; i < m; ++i) ret[i] = execute(s, op[i], key[i], val[i]);
    return now_ns() - t0;
}

// end-to-end per-group step (tally + executeCommands), groups sharded over `threads` host
// threads (threads = 1: one core, as one replica's goroutines). Returns elapsed ns of the
// timed region; outputs written like orc_group_step (committed/executed/ret only).
int64_t orc_bench_group_step(int N, int mode, const mpx_group_batch* b, uint32_t kv_per_group,
                             int threads) {
    const uint32_t G = b->n_groups, ipg = b->ipg;
    std::vector<Space*> spaces(G);
    std::vector<std::unordered_map<int64_t, int64_t>> stores(G);
    for (uint32_t g = 0; g < G; ++g) {
        spaces[g] = new Space(b->st_in + (size_t)g * ipg, ipg);
        auto& s = stores[g];
        for (uint32_t e = 0; e < b->kv_cnt_in[g]; ++e)
            s[b->kv_key_in[(size_t)g * kv_per_group + e]] = b->kv_val_in[(size_t)g * kv_per_group + e];
    }
    if (threads < 1) threads = 1;
    auto work = [&](uint32_t g0, uint32_t g1) {
        std::vector<int32_t> pc(N);
        for (uint32_t g = g0; g < g1; ++g) {
            int32_t cu = b->committed_in[g];
            for (int j = 0; j < N; ++j) pc[j] = b->peer_in[(size_t)g * N + j];
            reply_loop(N, mode, b->recs + b->grp_rec_off[g],
                       b->grp_rec_off[g + 1] - b->grp_rec_off[g], *spaces[g], 0, &cu, pc.data());
            int32_t i = b->executed_in[g] + 1;
            auto& s = stores[g];
            while (i <= cu && i >= 0 && (uint32_t)i < ipg) {
                size_t gi = (size_t)g * ipg + i;
                if (b->has_cmds && !b->has_cmds[gi]) break;
                for (uint32_t c = b->cmd_off[gi]; c < b->cmd_off[gi + 1]; ++c)
                    b->ret[c] = execute(s, b->op[c], b->key[c], b->val[c]);
                ++i;
            }
            b->committed_out[g] = cu;
            b->executed_out[g] = i - 1;
            for (int j = 0; j < N; ++j) b->peer_out[(size_t)g * N + j] = pc[j];
        }
    };
    int64_t t0 = now_ns();
    if (threads == 1) {
        work(0, G);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) {
            uint32_t g0 = (uint32_t)((uint64_t)G * t / threads);
            uint32_t g1 = (uint32_t)((uint64_t)G * (t + 1) / threads);
            th.emplace_back(work, g0, g1);
        }
        for (auto& x : th) x.join();
    }
    int64_t t1 = now_ns();
    for (auto* s : spaces) delete s;
    return t1 - t0;
}

}  // extern "C"
