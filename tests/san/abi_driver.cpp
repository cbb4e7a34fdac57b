// tests/san/abi_driver.cpp — TEST INFRASTRUCTURE ONLY: drives every host entry point of
// include/mpx.h over the stub runtime (hip_stub.cpp) with invalid and valid arguments, under
// ASan + UBSan. Checks return codes and that every failure on a live handle explains itself
// (mpx_last_error). Exit status 0 = all checks passed.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "mpx.h"

static int failures = 0;
#define CHECK(cond)                                                        \
    do {                                                                   \
        if (!(cond)) {                                                     \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                    \
        }                                                                  \
    } while (0)
// a failure on a live handle names its reason
#define FAILS(e, call, code)                                   \
    do {                                                       \
        mpx_last_error(e);                                     \
        const int _rc = (call);                                \
        CHECK(_rc == (code));                                  \
        CHECK(strlen(mpx_last_error(e)) > 0);                  \
    } while (0)

int main() {
    CHECK(mpx_abi_version() == MPX_ABI_VERSION);
    int n = -1;
    CHECK(mpx_device_count(&n) == MPX_OK && n == 1);
    mpx_config bad{0, MPX_MODE_MIN, 0, 0, 0, 0};
    mpx_engine* e = nullptr;
    CHECK(mpx_open(0, &bad, &e) == MPX_E_INVAL && !e);
    bad.n_replicas = 17;
    CHECK(mpx_open(0, &bad, &e) == MPX_E_INVAL);
    bad.n_replicas = 5;
    bad.mode = 7;
    CHECK(mpx_open(0, &bad, &e) == MPX_E_INVAL);
    bad.mode = MPX_MODE_MIN;
    bad.kv_per_group = 2048;
    CHECK(mpx_open(0, &bad, &e) == MPX_E_UNSUPPORTED);
    CHECK(mpx_open(3, &bad, &e) == MPX_E_NODEV);
    mpx_config cfg{5, MPX_MODE_MIN, 1 << 10, 64, 0, 16};
    CHECK(mpx_open(0, &cfg, &e) == MPX_OK && e);
    CHECK(mpx_stream(e) != nullptr);

    // A1/A2
    std::vector<mpx_accept_reply> ar(8);
    for (int i = 0; i < 8; ++i) ar[i] = mpx_accept_reply{i / 4, 16, 1 + i % 4, 1, {0, 0, 0}};
    std::vector<mpx_inst_state> st(2, mpx_inst_state{MPX_PREPARED, 0, 0, 0});
    int32_t cu = -1, pc[5] = {0};
    std::vector<uint8_t> dec(2);
    FAILS(e, mpx_accept_tally(e, nullptr, 8, st.data(), 2, 0, &cu, pc, dec.data()), MPX_E_INVAL);
    FAILS(e, mpx_accept_tally(e, ar.data(), 8, st.data(), 2, 0, nullptr, pc, dec.data()), MPX_E_INVAL);
    CHECK(mpx_accept_tally(e, ar.data(), 8, st.data(), 2, 0, &cu, pc, dec.data()) == MPX_OK);
    CHECK(mpx_accept_tally(e, ar.data(), 0, st.data(), 2, 0, &cu, pc, nullptr) == MPX_OK);
    FAILS(e, mpx_accept_tally_dev(e, ar.data(), 8, nullptr, nullptr, 2, 0, pc, nullptr, nullptr), MPX_E_INVAL);
    CHECK(mpx_committed_prefix(e, st.data(), 2, 0, &cu) == MPX_OK);
    FAILS(e, mpx_committed_prefix(e, nullptr, 2, 0, &cu), MPX_E_INVAL);

    // A4 / A3
    std::vector<mpx_prepare_reply> pr(8, mpx_prepare_reply{0, 16, 1, 3});
    std::vector<mpx_prep_state> ps(2);
    int32_t db = -1;
    CHECK(mpx_prepare_select(e, pr.data(), 8, ps.data(), 2, 0, &db, dec.data()) == MPX_OK);
    FAILS(e, mpx_prepare_select(e, pr.data(), 8, ps.data(), 2, 0, nullptr, nullptr), MPX_E_INVAL);
    std::vector<mpx_prepare_reply_min> pm(4);
    std::vector<mpx_group_prep_state> gs(2);
    std::vector<int32_t> gpc(10);
    std::vector<mpx_prepare_effect> eff(4);
    uint64_t off_ok[3] = {0, 2, 4}, off_bad0[3] = {1, 2, 4}, off_dec[3] = {0, 3, 2};
    CHECK(mpx_prepare_select_min(e, pm.data(), 4, off_ok, gs.data(), 2, gpc.data(), eff.data()) == MPX_OK);
    FAILS(e, mpx_prepare_select_min(e, pm.data(), 4, off_bad0, gs.data(), 2, gpc.data(), nullptr), MPX_E_INVAL);
    FAILS(e, mpx_prepare_select_min(e, pm.data(), 4, off_dec, gs.data(), 2, gpc.data(), nullptr), MPX_E_INVAL);

    // A5/A6
    const size_t m = 100;
    std::vector<uint8_t> op(m, MPX_OP_PUT), conf(m);
    std::vector<int64_t> key(m), val(m), ret(m);
    for (size_t i = 0; i < m; ++i) key[i] = (int64_t)(i % 7), val[i] = (int64_t)i;
    CHECK(mpx_apply(e, op.data(), key.data(), val.data(), m, ret.data(), conf.data()) == MPX_OK);
    FAILS(e, mpx_apply(e, op.data(), nullptr, val.data(), m, ret.data(), nullptr), MPX_E_INVAL);
    FAILS(e, mpx_apply_dev(e, op.data(), key.data(), val.data(), 1u << 20, ret.data(), nullptr, nullptr), MPX_E_INVAL);
    CHECK(mpx_apply_reserve(e, m) == MPX_OK);
    mpx_apply_io aio{};
    CHECK(mpx_apply_buffers(e, m, &aio) == MPX_OK && aio.cap >= m && aio.op && aio.conf);
    for (size_t i = 0; i < m; ++i) aio.op[i] = op[i], aio.key[i] = key[i], aio.val[i] = val[i];
    CHECK(mpx_apply_staged(e, m) == MPX_OK);
    FAILS(e, mpx_apply_staged(e, aio.cap + 1), MPX_E_INVAL);
    FAILS(e, mpx_apply_buffers(e, 0, &aio), MPX_E_INVAL);
    FAILS(e, mpx_apply_buffers(e, MPX_APPLY_SMALL_MAX + 1, &aio), MPX_E_INVAL);
    size_t nk = 9;
    CHECK(mpx_kv_size(e, &nk) == MPX_OK);
    int64_t kk[4], kv[4];
    CHECK(mpx_kv_export(e, kk, kv, 4, &nk) == MPX_OK);
    CHECK(mpx_kv_import(e, key.data(), val.data(), 7) == MPX_OK);
    CHECK(mpx_kv_clear(e) == MPX_OK);
    uint64_t io[4] = {0, 30, 60, 100}, io_bad[4] = {0, 60, 30, 100};
    std::vector<uint8_t> cb(3);
    CHECK(mpx_conflict_batch(e, op.data(), key.data(), io, 3, cb.data()) == MPX_OK);
    FAILS(e, mpx_conflict_batch(e, op.data(), key.data(), io_bad, 3, cb.data()), MPX_E_INVAL);
    CHECK(mpx_conflict_batch_dev(e, op.data(), key.data(), io, 1, cb.data(), nullptr) == MPX_OK);

    // fused group step: offsets validated on the host
    const uint32_t G = 2, ipg = 4;
    std::vector<mpx_accept_reply> grec(G * ipg * 4);
    for (size_t i = 0; i < grec.size(); ++i)
        grec[i] = mpx_accept_reply{(int32_t)((i / 4) % ipg), 16, 1 + (int32_t)(i % 4), 1, {0, 0, 0}};
    uint64_t groff[3] = {0, 16, 32};
    std::vector<mpx_inst_state> gst(G * ipg, mpx_inst_state{MPX_PREPARED, 0, 0, 0});
    int32_t ci[2] = {-1, -1}, co[2], ei[2] = {-1, -1}, eo[2];
    std::vector<int32_t> pin(G * 5), pout(G * 5);
    std::vector<uint32_t> coff(G * ipg + 1);
    for (size_t i = 0; i < coff.size(); ++i) coff[i] = (uint32_t)(i * 2);
    std::vector<uint8_t> gop(16, MPX_OP_GET), gconf(16);
    std::vector<int64_t> gkey(16, 3), gval(16, 4), gret(16);
    std::vector<uint32_t> kc(G), kc2(G), nd(G);
    std::vector<int64_t> kk2(G * 64), kv2(G * 64), kk3(G * 64), kv3(G * 64);
    mpx_group_batch gb{G, ipg, grec.data(), groff, gst.data(), gst.data(), ci, co, ei, eo,
                       pin.data(), pout.data(), gop.data(), gkey.data(), gval.data(), coff.data(),
                       nullptr, gret.data(), gconf.data(), kc.data(), kk2.data(), kv2.data(),
                       kc2.data(), kk3.data(), kv3.data(), nullptr, nd.data()};
    CHECK(mpx_group_step(e, &gb) == MPX_OK);
    groff[1] = 40;  // not sorted
    FAILS(e, mpx_group_step(e, &gb), MPX_E_INVAL);
    groff[1] = 16;
    coff[3] = 0;  // not sorted
    FAILS(e, mpx_group_step(e, &gb), MPX_E_INVAL);
    coff[3] = 6;
    gb.ipg = 9000;
    FAILS(e, mpx_group_step_dev(e, &gb, nullptr), MPX_E_UNSUPPORTED);
    gb.ipg = ipg;
    gb.n_groups = 100;  // beyond max_groups (16)
    FAILS(e, mpx_group_step_dev(e, &gb, nullptr), MPX_E_INVAL);
    gb.n_groups = G;
    int64_t tot[3];
    CHECK(mpx_step_totals_dev(e, &gb, tot, nullptr) == MPX_OK);
    gb.n_decided = nullptr;
    FAILS(e, mpx_step_totals_dev(e, &gb, tot, nullptr), MPX_E_INVAL);

    // collectives
    int32_t wm[4] = {1, 2, 3, 4};
    FAILS(e, mpx_watermarks_allreduce(e, wm, wm + 2, 2), MPX_E_INVAL);  // no communicator yet
    unsigned char uid[128];
    CHECK(mpx_comm_unique_id(uid) == MPX_OK);
    CHECK(mpx_comm_init(e, 1, 0, uid) == MPX_OK);
    CHECK(mpx_comm_init(e, 2, 5, uid) == MPX_E_INVAL);
    CHECK(mpx_watermarks_allreduce(e, wm, wm + 2, 2) == MPX_OK);
    CHECK(mpx_step_allreduce_dev(e, wm, 2, tot, 3, nullptr) == MPX_OK);
    FAILS(e, mpx_step_allreduce_dev(e, nullptr, 2, tot, 3, nullptr), MPX_E_INVAL);

    // peer streams
    std::vector<uint8_t> buf(300, 13);
    std::vector<mpx_accept_reply> dar(40);
    std::vector<mpx_peer_frame> doth(40);
    mpx_decode_result dres;
    CHECK(mpx_decode_peer_stream(e, buf.data(), buf.size(), dar.data(), 40, doth.data(), 40, &dres) == MPX_OK);
    FAILS(e, mpx_decode_peer_stream(e, nullptr, 10, dar.data(), 40, doth.data(), 40, &dres), MPX_E_INVAL);
    std::vector<mpx_prepare_reply_min> dpr(40);
    std::vector<mpx_var_frame> dvar(40);
    mpx_decode_out out{dar.data(), 40, dpr.data(), 40, dvar.data(), 40, doth.data(), 40};
    mpx_stream_result sres;
    CHECK(mpx_decode_stream(e, buf.data(), buf.size(), &out, &sres) == MPX_OK);
    CHECK(mpx_decode_stream(e, buf.data(), 0, &out, &sres) == MPX_OK);
    mpx_decode_out out_bad = out;
    out_bad.var = nullptr;
    FAILS(e, mpx_decode_stream(e, buf.data(), buf.size(), &out_bad, &sres), MPX_E_INVAL);
    FAILS(e, mpx_decode_stream_dev(e, buf.data() + 1, 10, 0, &out, &sres, nullptr), MPX_E_INVAL);
    FAILS(e, mpx_decode_stream_dev(e, buf.data(), 10, 11, &out, &sres, nullptr), MPX_E_INVAL);
    CHECK(mpx_decode_stream_reserve(e, buf.size()) == MPX_OK);

    // fan-out, logs, replay
    std::vector<mpx_reply_rec> rr(10, mpx_reply_rec{1, 2, 3, 1});
    std::vector<uint8_t> rout(250);
    std::vector<uint64_t> roff(4);
    CHECK(mpx_encode_replies(e, rr.data(), 10, 3, 1, 0, rout.data(), roff.data()) == MPX_OK);
    CHECK(mpx_encode_replies(e, rr.data(), 10, 0, 1, 0, rout.data(), roff.data()) == MPX_E_INVAL);
    std::vector<mpx_log_rec> lr(3, mpx_log_rec{16, MPX_COMMITTED, 0, 0});
    uint64_t loff[4] = {0, 2, 4, 6}, loff_bad[4] = {0, 4, 2, 6};
    std::vector<uint8_t> lout(mpx_encode_log_bound(3, 6));
    std::vector<uint64_t> lro(4);
    CHECK(mpx_encode_log(e, MPX_LOG_CATCHUP, lr.data(), 3, loff, op.data(), key.data(), val.data(), 6, lout.data(), lout.size(), lro.data()) == MPX_OK);
    FAILS(e, mpx_encode_log(e, MPX_LOG_DURABLE, lr.data(), 3, loff_bad, op.data(), key.data(), val.data(), 6, lout.data(), lout.size(), lro.data()), MPX_E_INVAL);
    FAILS(e, mpx_encode_log(e, 5, lr.data(), 3, loff, op.data(), key.data(), val.data(), 6, lout.data(), lout.size(), lro.data()), MPX_E_INVAL);
    std::vector<uint8_t> log(29 * 4);
    std::vector<mpx_log_rec> rrec(4);
    std::vector<int32_t> last(8, -1);
    int32_t sc[2] = {0, -1};
    CHECK(mpx_replay_durable(e, log.data(), log.size(), 8, 0, rrec.data(), op.data(), key.data(), val.data(), last.data(), sc) == MPX_OK);
    FAILS(e, mpx_replay_durable(e, log.data(), log.size() - 1, 8, 0, rrec.data(), op.data(), key.data(), val.data(), last.data(), sc), MPX_E_INVAL);
    FAILS(e, mpx_replay_durable(e, log.data(), log.size(), 0, 0, rrec.data(), op.data(), key.data(), val.data(), last.data(), sc), MPX_E_NIL_INSTANCE);
    FAILS(e, mpx_replay_durable(e, log.data(), log.size(), 8, -1, rrec.data(), op.data(), key.data(), val.data(), last.data(), sc), MPX_E_INVAL);
    FAILS(e, mpx_replay_durable(e, log.data(), log.size(), 8, INT32_MAX - 2, rrec.data(), op.data(), key.data(), val.data(), last.data(), sc), MPX_E_UNSUPPORTED);
    FAILS(e, mpx_replay_durable_dev(e, log.data(), log.size(), 0, 0, rrec.data(), op.data(), key.data(), val.data(), last.data(), sc, nullptr), MPX_E_NIL_INSTANCE);

    // device utilities
    void* d = nullptr;
    CHECK(mpx_dev_alloc(e, 64, &d) == MPX_OK && d);
    CHECK(mpx_memset_async(e, d, 0xFF, 64, nullptr) == MPX_OK);
    CHECK(mpx_memcpy_async(e, d, buf.data(), 64, MPX_COPY_H2D, nullptr) == MPX_OK);
    FAILS(e, mpx_memcpy_async(e, d, buf.data(), 64, 9, nullptr), MPX_E_INVAL);
    void *s = nullptr, *ev0 = nullptr, *ev1 = nullptr;
    CHECK(mpx_stream_create(e, &s) == MPX_OK);
    CHECK(mpx_event_create(e, 1, &ev0) == MPX_OK && mpx_event_create(e, 0, &ev1) == MPX_OK);
    CHECK(mpx_event_record(e, ev0, s) == MPX_OK && mpx_stream_wait_event(e, nullptr, ev0) == MPX_OK);
    float ms = -1;
    CHECK(mpx_event_elapsed_ms(e, ev0, ev1, &ms) == MPX_OK);
    FAILS(e, mpx_stream_destroy(e, mpx_stream(e)), MPX_E_INVAL);
    CHECK(mpx_stream_destroy(e, s) == MPX_OK);
    CHECK(mpx_event_destroy(e, ev0) == MPX_OK && mpx_event_destroy(e, ev1) == MPX_OK);
    CHECK(mpx_dev_free(e, d) == MPX_OK && mpx_dev_free(e, nullptr) == MPX_OK);
    char info[8];
    const int full = mpx_runtime_info(info, sizeof(info));
    CHECK(full > 8 && strlen(info) == 7);
    CHECK(mpx_runtime_info(nullptr, 0) == full);

    CHECK(mpx_synchronize(e) == MPX_OK);
    CHECK(mpx_close(e) == MPX_OK);
    CHECK(mpx_close(nullptr) == MPX_E_INVAL);
    if (failures) fprintf(stderr, "%d check(s) failed\n", failures);
    else printf("abi_driver: all checks passed\n");
    return failures ? 1 : 0;
}
