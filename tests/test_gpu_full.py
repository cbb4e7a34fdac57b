"""BASELINE.json configurations at FULL size on the GPU, bit-exact against the CPU oracle.

Every output the engine produces is compared (instance states, watermarks, peerCommits, decided
flags and counts, Execute results, conflicts, the KV tables):
  config 2  accept tally, 2^24 instances x 4 AcceptReplies, MIN and CLASSIC
  config 3  CLASSIC prepare selection, 2^24 instances x 4 PrepareReplies
            (+ the MIN variant, one PrepareBookkeeping per group, 65,536 groups)
  config 4  batched KV apply, 2^26 PUT/GET over 2^20 keys, uniform and Zipf(2, 1): a first call
            on the empty table and a second on the table it left (the bench's steady state)
  config 5  the fused group step of one GPU's share, 65,536 groups x 256 instances x 4 replies
            + 4 commands, two consecutive steps (the second from the tables the first produced)
  config 1  the shape stock MinPaxos runs (bareminpaxos.go:22,634-651): ONE group, 20 instances
            of MAX_BATCH = 5000 commands (100k PUT/GET, 50 % writes, keys Zipf(s=2, v=1) over
            [0, 100000) as client.go:45-46,93 draws them), N = 3 — the work-list kernel
  config 5 at N = 7 (6 replies per instance: past the fast path's 1024-reply image)
Reduced-size and edge-case parity lives in test_gpu_parity.py.
"""
import numpy as np
import pytest

from oracle_lib import Oracle
from minpaxos_amd import records as R
from minpaxos_amd import synth

pytestmark = pytest.mark.gpu


def eq_struct(a, b, what):
    assert a.dtype == b.dtype
    for f in a.dtype.names:
        if f == "pad":
            continue
        bad = np.nonzero(a[f] != b[f])[0]
        assert len(bad) == 0, f"{what}.{f} differs at {bad[:8]}"


def eq(a, b, what):
    bad = np.nonzero(np.asarray(a) != np.asarray(b))[0]
    assert len(bad) == 0, f"{what} differs at {bad[:8]} ({len(bad)} entries)"


@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC], ids=["min", "classic"])
def test_config2_accept_tally_full(mk_engine, mode):
    I = 1 << 24
    rec, st = synth.accept_replies(I, 5, 0.7, seed=42)
    e, o = mk_engine(5, mode), Oracle(5, mode)
    got = e.accept_tally(rec, st, 0, -1, np.zeros(5, np.int32))
    want = o.accept_tally(rec, st, 0, -1, np.zeros(5, np.int32))
    eq_struct(got[0], want[0], "st")
    assert got[1] == want[1]
    eq(got[2], want[2], "peerCommits")
    eq(got[3], want[3], "decided")


def test_config3_prepare_full(mk_engine):
    I = 1 << 24
    rec, st = synth.prepare_replies(I, 5, 0.8, seed=43)
    e, o = mk_engine(5, R.MODE_CLASSIC), Oracle(5, R.MODE_CLASSIC)
    got = e.prepare_select(rec, st, 0, -1)
    want = o.prepare_select(rec, st, 0, -1)
    eq_struct(got[0], want[0], "st")
    assert got[1] == want[1]
    eq(got[2], want[2], "prepared")


def test_config3_prepare_min_full(mk_engine):
    G = 65536
    rec, off, gst = synth.prepare_replies_min(G, 5, seed=46)
    pc = np.zeros(G * 5, np.int32)
    e, o = mk_engine(5, R.MODE_MIN), Oracle(5, R.MODE_MIN)
    got = e.prepare_select_min(rec, off, gst, pc)
    want = o.prepare_select_min(rec, off, gst, pc)
    eq_struct(got[0], want[0], "gst")
    eq(got[1], want[1], "peerCommits")
    eq_struct(got[2], want[2], "effects")


@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_config4_apply_full(mk_engine, dist):
    M, K = 1 << 26, 1 << 20
    op, key, val = synth.commands(M, K, 0.5, dist, seed=44)
    e, o = mk_engine(5, R.MODE_MIN, kv_capacity=2 * K), Oracle(5, R.MODE_MIN)
    for call in range(2):  # empty table, then the table the first call left
        gr, gc = e.apply(op, key, val)
        wr, wc = o.apply(op, key, val)
        eq(gr, wr, f"ret (call {call})")
        eq(gc, wc, f"conf_prev (call {call})")
        gk, gv = e.kv_export()
        wk, wv = o.kv_export()
        eq(gk, wk, "table keys")
        eq(gv, wv, "table values")


def _cmp_group(got, want, G, K):
    for f in ("committed_out", "executed_out", "peer_out", "ret", "conf_prev", "kv_cnt",
              "decided", "n_decided"):
        eq(got[f], want[f], f)
    eq_struct(got["st_out"], want["st_out"], "st_out")
    cnt = want["kv_cnt"].astype(np.int64)
    mask = (np.arange(K)[None, :] < cnt[:, None]).reshape(-1)  # live table entries only
    eq(got["kv_key"][mask], want["kv_key"][mask], "kv_key")
    eq(got["kv_val"][mask], want["kv_val"][mask], "kv_val")


# kv_per_group 256 is the bench's shape (bench.py --kv-per-group default): the FastBase variant
# the headline times; 512 runs FastKeys (step.hip fast_variant)
@pytest.mark.parametrize("K", [256, 512], ids=["K256_fastbase", "K512_fastkeys"])
@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC], ids=["min", "classic"])
def test_config5_group_step_full(mk_engine, mode, K):
    G, ipg = 65536, 256
    b = synth.group_batch(G, ipg, 5, 4, 256, seed=45)
    e, o = mk_engine(5, mode, kv_per_group=K), Oracle(5, mode, kv_per_group=K)
    got = e.group_step(b)
    want = o.group_step(b)
    _cmp_group(got, want, G, K)
    # the bench's steady state: the same batch against the tables the first step produced
    got2 = e.group_step(b, want["kv_cnt"], want["kv_key"], want["kv_val"])
    want2 = o.group_step(b, want["kv_cnt"], want["kv_key"], want["kv_val"])
    _cmp_group(got2, want2, G, K)
    assert int(want2["n_decided"].sum()) > 0.9 * G * ipg * 0.8  # p_ok 0.7 at N = 5: ~92 %


@pytest.mark.parametrize("K", [256, 512], ids=["K256_fastrecs", "K512_fastwide"])
def test_config5_n7_full(mk_engine, K):
    """N = 7: 6 replies x 256 instances = 1536 records per group, beyond FastBase's reply image:
    FastRecs at kv_per_group 256 (the bench's step_n7 line), FastWide at 512"""
    G, ipg = 65536, 256
    b = synth.group_batch(G, ipg, 7, 4, 256, seed=47)
    e, o = mk_engine(7, R.MODE_MIN, kv_per_group=K), Oracle(7, R.MODE_MIN, kv_per_group=K)
    _cmp_group(e.group_step(b), o.group_step(b), G, K)


def config1_batch(n_inst=20, batch=5000, n_keys=100000, seed=48):
    """one group as stock MinPaxos runs it: instances of MAX_BATCH commands, N = 3"""
    b = synth.group_batch(1, n_inst, 3, batch, 1, p_ok=0.7, seed=seed)
    op, key, val = synth.commands(n_inst * batch, n_keys, 0.5, "zipf", seed=seed)
    b.update(op=op, key=key, val=val)
    return b


@pytest.mark.parametrize("mode", [R.MODE_MIN, R.MODE_CLASSIC], ids=["min", "classic"])
def test_config1_shape_one_group_max_batch(mk_engine, mode):
    K = 1024
    b = config1_batch()
    e, o = mk_engine(3, mode, kv_per_group=K), Oracle(3, mode, kv_per_group=K)
    want = o.group_step(b)
    assert want["executed_out"][0] >= 0 and int(want["kv_cnt"][0]) > 100
    _cmp_group(e.group_step(b), want, 1, K)
    # and again from the table it left, as executeCommands continues on the same State
    b2 = config1_batch(seed=49)
    b2["committed_in"] = want["committed_out"]
    b2["executed_in"] = np.full(1, -1, np.int32)
    got2 = e.group_step(b2, want["kv_cnt"], want["kv_key"], want["kv_val"])
    want2 = o.group_step(b2, want["kv_cnt"], want["kv_key"], want["kv_val"])
    _cmp_group(got2, want2, 1, K)
