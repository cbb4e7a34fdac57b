// oracle/oracle.cpp — TEST INFRASTRUCTURE ONLY. CPU restatement of the MinPaxos hot path.
//
// This file is the parity checker for the HIP engine (minpaxos_amd/csrc). Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it (liboracle.so); the
// product never links or calls it.
//
// Every function is a literal, record-at-a-time restatement of the cited Go text of
// arobertlin/MinPaxos (read as text at /root/reference; no Go toolchain exists in this image,
// so the reference itself cannot be run). Parity pinning: the reference ships no tests or
// golden vectors for this path, so the restatement is pinned by the
// hand-traced known-answer tests of SURVEY §8c (tests/test_oracle_kat.py) and by committed
// fixtures it generates (tests/golden/). See DESIGN.md "Parity".
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "../include/mpx.h"

namespace {

const uint8_t TRUE_ = 1;  // bareminpaxos.go:19 / paxos.go  `const TRUE = uint8(1)`

inline bool in_window(int64_t idx, size_t n) { return idx >= 0 && (uint64_t)idx < n; }

// paxos.(*Replica).updateCommittedUpTo  src/paxos/paxos.go:259-264 (same text as
// bareminpaxos.go:387-392): advance while instanceSpace[cu+1] != nil && status == COMMITTED.
// Instances outside [base, base+n_inst) are nil.
void update_committed_upto(const mpx_inst_state* st, size_t n_inst, int32_t base, int32_t* cu) {
    for (;;) {
        int64_t nxt = (int64_t)*cu + 1 - base;
        if (!in_window(nxt, n_inst)) break;
        if (st[nxt].status == MPX_STATUS_NIL) break;
        if (st[nxt].status != MPX_COMMITTED) break;
        *cu += 1;
    }
}

}  // namespace

extern "C" {

int orc_abi_version(void) { return MPX_ABI_VERSION; }

// ---- A1 / A2 ----------------------------------------------------------------------------
// MIN:     bareminpaxos.(*Replica).handleAcceptReply  src/bareminpaxos/bareminpaxos.go:1014-1064
// CLASSIC: paxos.(*Replica).handleAcceptReply         src/paxos/paxos.go:631-673
int orc_accept_tally(int N, int mode, const mpx_accept_reply* recs, size_t n, mpx_inst_state* st,
                     size_t n_inst, int32_t base, int32_t* committed_upto, int32_t* peer_commits,
                     uint8_t* decided_out) {
    if (N < 1 || N > MPX_MAX_REPLICAS) return MPX_E_INVAL;
    const int32_t half = (int32_t)N >> 1;  // int32(r.N)>>1
    // Where the reference panics the batch is refused (outputs then unspecified):
    //  - every record must name an instance inside the window (instanceSpace index);
    //  - a nil instance is dereferenced by CLASSIC for every reply (paxos.go:634) but by MIN
    //    only for OK replies (inst.Lb.AcceptOKs++, bareminpaxos.go:1024);
    //  - peerCommits[areply.Id] (bareminpaxos.go:1050) is checked where it is indexed.
    for (size_t p = 0; p < n; ++p) {
        int64_t idx = (int64_t)recs[p].instance - base;
        if (!in_window(idx, n_inst)) return MPX_E_NIL_INSTANCE;
        if (st[idx].status == MPX_STATUS_NIL && (mode == MPX_MODE_CLASSIC || recs[p].ok == TRUE_))
            return MPX_E_NIL_INSTANCE;
    }
    if (decided_out) memset(decided_out, 0, n_inst);
    for (size_t p = 0; p < n; ++p) {
        const mpx_accept_reply& a = recs[p];
        mpx_inst_state& inst = st[a.instance - base];  // inst := r.instanceSpace[areply.Instance]
        if (mode == MPX_MODE_MIN) {
            // bareminpaxos.go:1023-1053 (no status check, NACKs ignored, ballot ignored)
            if (a.ok == TRUE_) {
                inst.accept_oks++;                       // :1024
                if (inst.accept_oks + 1 > half) {        // :1025
                    if (inst.accept_oks == half) {       // :1026
                        inst.status = MPX_COMMITTED;     // :1028
                        *committed_upto = a.instance;    // :1048 (assignment, not max)
                        if (decided_out) decided_out[a.instance - base] = 1;
                    }
                    if (a.id < 0 || a.id >= N) return MPX_E_BAD_ID;  // index out of range
                    peer_commits[a.id] = a.instance - 1; // :1050
                }
            }
        } else {
            // paxos.go:634-637
            if (inst.status != MPX_PREPARED && inst.status != MPX_ACCEPTED) continue;
            if (a.ok == TRUE_) {
                inst.accept_oks++;                       // :640
                if (inst.accept_oks + 1 > half) {        // :641
                    inst.status = MPX_COMMITTED;         // :643
                    if (decided_out) decided_out[a.instance - base] = 1;
                    update_committed_upto(st, n_inst, base, committed_upto);  // :659
                }
            } else {
                inst.nacks++;                                                  // :665
                if (a.ballot > inst.max_recv_ballot) inst.max_recv_ballot = a.ballot;  // :666-668
            }
        }
    }
    return MPX_OK;
}

int orc_committed_prefix(const mpx_inst_state* st, size_t n_inst, int32_t base,
                         int32_t* committed_upto) {
    update_committed_upto(st, n_inst, base, committed_upto);
    return MPX_OK;
}

// ---- A4: CLASSIC prepare  paxos.(*Replica).handlePrepareReply  src/paxos/paxos.go:577-629 --
int orc_prepare_classic(int N, const mpx_prepare_reply* recs, size_t n, mpx_prep_state* st,
                        size_t n_inst, int32_t base, int32_t* default_ballot,
                        uint8_t* prepared_out) {
    if (N < 1 || N > MPX_MAX_REPLICAS) return MPX_E_INVAL;
    const int32_t half = (int32_t)N >> 1;  // r.N>>1
    for (size_t p = 0; p < n; ++p) {
        int64_t idx = (int64_t)recs[p].instance - base;
        if (!in_window(idx, n_inst) || st[idx].status == MPX_STATUS_NIL) return MPX_E_NIL_INSTANCE;
    }
    if (prepared_out) memset(prepared_out, 0, n_inst);
    for (size_t p = 0; p < n; ++p) {
        const mpx_prepare_reply& r = recs[p];
        mpx_prep_state& inst = st[r.instance - base];
        // per-call event flags describe this call, on every instance that has replies
        if (p == 0 || recs[p - 1].instance != r.instance)
            inst.flags &= ~(MPX_PF_REQUEUED | MPX_PF_PREPARED_NOW);
        if (inst.status != MPX_PREPARING) continue;                 // :580-584
        if (r.ok == TRUE_) {
            inst.prepare_oks++;                                      // :587
            if (r.ballot > inst.max_recv_ballot) {                   // :589 (strict)
                inst.value_id = r.value_id;                          // :590
                inst.max_recv_ballot = r.ballot;                     // :591
                if (inst.flags & MPX_PF_HAS_PROPOSALS) {             // :592-600
                    inst.flags &= ~MPX_PF_HAS_PROPOSALS;
                    inst.flags |= MPX_PF_REQUEUED;
                }
            }
            if (inst.prepare_oks + 1 > half) {                       // :603
                inst.status = MPX_PREPARED;                          // :604
                inst.nacks = 0;                                      // :605
                if (inst.ballot > *default_ballot) *default_ballot = inst.ballot;  // :606-608
                inst.flags |= MPX_PF_PREPARED_NOW;                   // :611 bcastAccept (host)
                if (prepared_out) prepared_out[r.instance - base] = 1;
            }
        } else {
            inst.nacks++;                                            // :615
            if (r.ballot > inst.max_recv_ballot) inst.max_recv_ballot = r.ballot;  // :616-618
            if (inst.nacks >= half) {                                // :619
                if (inst.flags & MPX_PF_HAS_PROPOSALS) {             // :620-626
                    inst.flags &= ~MPX_PF_HAS_PROPOSALS;
                    inst.flags |= MPX_PF_REQUEUED;
                }
            }
        }
    }
    return MPX_OK;
}

// ---- A3: MIN prepare  bareminpaxos.(*Replica).handlePrepareReply  bareminpaxos.go:912-966 --
int orc_prepare_min(int N, const mpx_prepare_reply_min* recs, size_t n, const uint64_t* off,
                    mpx_group_prep_state* gst, size_t G, int32_t* peer_commits,
                    mpx_prepare_effect* eff) {
    if (N < 1 || N > MPX_MAX_REPLICAS) return MPX_E_INVAL;
    const int32_t half = (int32_t)N >> 1;
    if (off[0] != 0 || off[G] != n) return MPX_E_INVAL;
    for (size_t g = 0; g < G; ++g) {
        if (off[g + 1] < off[g]) return MPX_E_INVAL;
        for (uint64_t p = off[g]; p < off[g + 1]; ++p)
            if (recs[p].ballot == gst[g].default_ballot && (recs[p].id < 0 || recs[p].id >= N))
                return MPX_E_BAD_ID;
    }
    for (size_t g = 0; g < G; ++g) {
        mpx_group_prep_state& b = gst[g];
        int32_t* pc = peer_commits + g * (size_t)N;
        for (uint64_t p = off[g]; p < off[g + 1]; ++p) {
            const mpx_prepare_reply_min& r = recs[p];
            uint32_t fl = 0;
            int32_t from = -1;
            if (b.default_ballot > r.ballot) {                       // :916-918
                if (eff) eff[p] = {fl, from};
                continue;
            }
            if (b.default_ballot == r.ballot) {                      // :921 (OK not checked)
                fl |= MPX_EF_COUNTED;
                b.prepare_oks++;                                     // :922
                pc[r.id] = r.last_committed;                         // :923
                if (r.instance > b.highest_instance ||
                    (r.instance == b.highest_instance && r.ballot > b.max_recv_ballot)) {  // :925
                    b.value_id = r.value_id;                         // :927
                    b.max_recv_ballot = r.ballot;                    // :928
                    b.highest_instance = r.instance;                 // :930
                    fl |= MPX_EF_SELECTED;
                }
                if (b.committed_upto <= r.last_committed) {          // :934
                    from = b.committed_upto + 1;                     // :936-938 (host copies)
                    fl |= MPX_EF_CATCHUP;
                    b.committed_upto = r.last_committed;             // :939
                }
                if (b.prepare_oks == half && b.highest_instance > b.committed_upto) {  // :945
                    b.committed_upto = b.highest_instance;           // :954
                    b.triggered++;
                    fl |= MPX_EF_TRIGGER;                            // :948-958 (host)
                }
            }
            if (eff) eff[p] = {fl, from};
        }
    }
    return MPX_OK;
}

// ---- A5 / A6: state.Command.Execute / Conflict ---------------------------------------------
struct OrcKV {
    std::unordered_map<int64_t, int64_t> store;  // state.State.Store map[Key]Value
};

void* orc_kv_new(void) { return new OrcKV(); }
void orc_kv_free(void* kv) { delete (OrcKV*)kv; }
size_t orc_kv_size(void* kv) { return ((OrcKV*)kv)->store.size(); }
// export sorted by key (deterministic)
size_t orc_kv_export(void* kv, int64_t* keys, int64_t* vals, size_t cap) {
    auto& s = ((OrcKV*)kv)->store;
    std::vector<std::pair<int64_t, int64_t>> v(s.begin(), s.end());
    std::sort(v.begin(), v.end());
    size_t k = std::min(cap, v.size());
    for (size_t i = 0; i < k; ++i) { keys[i] = v[i].first; vals[i] = v[i].second; }
    return v.size();
}
void orc_kv_import(void* kv, const int64_t* keys, const int64_t* vals, size_t n) {
    auto& s = ((OrcKV*)kv)->store;
    for (size_t i = 0; i < n; ++i) s[keys[i]] = vals[i];
}

// state.Conflict  src/state/state.go:53-60
static inline bool conflict(uint8_t op_g, int64_t k_g, uint8_t op_d, int64_t k_d) {
    if (k_g == k_d) {
        if (op_g == MPX_OP_PUT || op_d == MPX_OP_PUT) return true;
    }
    return false;
}

// (*Command).Execute  src/state/state.go:77-103
static inline int64_t execute(std::unordered_map<int64_t, int64_t>& store, uint8_t op, int64_t k,
                              int64_t v) {
    switch (op) {
        case MPX_OP_PUT:
            store[k] = v;  // :93
            return v;      // :94
        case MPX_OP_GET: {
            auto it = store.find(k);  // :97
            if (it != store.end()) return it->second;
            break;
        }
    }
    return 0;  // NIL :102
}

// executeCommands' inner loop (bareminpaxos.go:1074-1075) over a log slice, plus the
// per-command Conflict with the previous command on the same key in this slice.
int orc_apply(void* kv, const uint8_t* op, const int64_t* key, const int64_t* val, size_t m,
              int64_t* ret, uint8_t* conf_prev) {
    auto& store = ((OrcKV*)kv)->store;
    std::unordered_map<int64_t, uint8_t> last_op;
    for (size_t i = 0; i < m; ++i) {
        if (conf_prev) {
            auto it = last_op.find(key[i]);
            conf_prev[i] = (it != last_op.end()) && conflict(it->second, key[i], op[i], key[i]);
            last_op[key[i]] = op[i];
        }
        ret[i] = execute(store, op[i], key[i], val[i]);
    }
    return MPX_OK;
}

// state.ConflictBatch  src/state/state.go:62-71, for each consecutive instance pair
int orc_conflict_batch(const uint8_t* op, const int64_t* key, const uint64_t* inst_off,
                       size_t n_inst, uint8_t* out) {
    for (size_t i = 0; i + 1 < n_inst; ++i) {
        uint8_t r = 0;
        for (uint64_t a = inst_off[i]; a < inst_off[i + 1] && !r; ++a)
            for (uint64_t b = inst_off[i + 1]; b < inst_off[i + 2]; ++b)
                if (conflict(op[a], key[a], op[b], key[b])) { r = 1; break; }
        out[i] = r;
    }
    return MPX_OK;
}

// ---- fused per-group step: handleAcceptReply batch + executeCommands per replica ----------
// executeCommands  src/bareminpaxos/bareminpaxos.go:1066-1098 (CLASSIC paxos.go:675-706):
// i from executed+1 while i <= committedUpTo and instanceSpace[i].Cmds != nil.
// Group KV tables are compact arrays: existing entries keep their slot, keys first PUT in
// this step are appended in order of their first PUT.
int orc_group_step(int N, int mode, const mpx_group_batch* b, uint32_t kv_per_group) {
    const uint32_t G = b->n_groups, ipg = b->ipg;
    for (uint32_t g = 0; g < G; ++g) {
        const uint64_t r0 = b->grp_rec_off[g], r1 = b->grp_rec_off[g + 1];
        std::vector<mpx_inst_state> st(b->st_in + (size_t)g * ipg, b->st_in + (size_t)(g + 1) * ipg);
        int32_t cu = b->committed_in[g];
        std::vector<int32_t> pc(b->peer_in + (size_t)g * N, b->peer_in + (size_t)(g + 1) * N);
        std::vector<uint8_t> dec(ipg, 0);
        int rc = orc_accept_tally(N, mode, b->recs + r0, r1 - r0, st.data(), ipg, 0, &cu,
                                  pc.data(), dec.data());
        if (rc) return rc;
        // only instances with records are written to st_out (the kernel contract)
        for (uint64_t p = r0; p < r1; ++p) {
            int32_t i = b->recs[p].instance;
            b->st_out[(size_t)g * ipg + i] = st[i];
        }
        if (b->decided)
            for (uint32_t i = 0; i < ipg; ++i) b->decided[(size_t)g * ipg + i] = dec[i];
        if (b->n_decided) {
            uint32_t nd = 0;
            for (uint32_t i = 0; i < ipg; ++i) nd += dec[i];
            b->n_decided[g] = nd;
        }
        b->committed_out[g] = cu;
        for (int j = 0; j < N; ++j) b->peer_out[(size_t)g * N + j] = pc[j];

        // KV table of this group
        uint32_t cnt = b->kv_cnt_in[g];
        if (cnt > kv_per_group) return MPX_E_INVAL;
        std::vector<int64_t> tk(b->kv_key_in + (size_t)g * kv_per_group,
                                b->kv_key_in + (size_t)g * kv_per_group + cnt);
        std::vector<int64_t> tv(b->kv_val_in + (size_t)g * kv_per_group,
                                b->kv_val_in + (size_t)g * kv_per_group + cnt);
        std::unordered_map<int64_t, int64_t> store;
        std::unordered_map<int64_t, uint32_t> slot;
        for (uint32_t e = 0; e < cnt; ++e) { store[tk[e]] = tv[e]; slot[tk[e]] = e; }
        std::unordered_map<int64_t, uint8_t> last_op;
        int32_t ex = b->executed_in[g];
        for (;;) {
            int32_t i = ex + 1;
            if (i > cu) break;                                    // for i <= r.committedUpTo
            if (i < 0 || (uint32_t)i >= ipg) break;               // outside the instance space
            size_t gi = (size_t)g * ipg + i;
            if (st[i].status == MPX_STATUS_NIL) break;            // nil instance
            if (b->has_cmds && !b->has_cmds[gi]) break;           // Cmds == nil
            for (uint32_t c = b->cmd_off[gi]; c < b->cmd_off[gi + 1]; ++c) {
                uint8_t o = b->op[c];
                int64_t k = b->key[c];
                if (b->conf_prev) {
                    auto it = last_op.find(k);
                    b->conf_prev[c] = (it != last_op.end()) && conflict(it->second, k, o, k);
                    last_op[k] = o;
                }
                if (o == MPX_OP_PUT && !store.count(k)) {
                    if (tk.size() >= kv_per_group) return MPX_E_KV_FULL;
                    slot[k] = (uint32_t)tk.size();
                    tk.push_back(k);
                    tv.push_back(0);
                }
                b->ret[c] = execute(store, o, k, b->val[c]);
            }
            ex = i;
        }
        b->executed_out[g] = ex;
        for (auto& kvp : store) tv[slot[kvp.first]] = kvp.second;
        b->kv_cnt_out[g] = (uint32_t)tk.size();
        for (size_t e = 0; e < tk.size(); ++e) {
            b->kv_key_out[(size_t)g * kv_per_group + e] = tk[e];
            b->kv_val_out[(size_t)g * kv_per_group + e] = tv[e];
        }
    }
    return MPX_OK;
}

}  // extern "C"
