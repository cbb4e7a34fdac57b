"""Adversarial random inputs for parity tests (seeded numpy; sizes the oracle finishes fast)."""
import numpy as np

from minpaxos_amd import records as R


def ragged_accept(rng, n_inst, n_replicas, max_r=8, long_every=0, long_len=300, p_ok=0.6,
                  gaps=True, base=0, random_state=True, bad_ids=False):
    """Replies grouped by instance in ascending order, 0..max_r replies per instance (some
    instances have none), occasional very long instances, random ids / oks / ballots and random
    initial bookkeeping (oks, nacks, maxRecvBallot, status)."""
    counts = rng.integers(0 if gaps else 1, max_r + 1, n_inst)
    if long_every:
        counts[::long_every] = long_len
    n = int(counts.sum())
    rec = np.zeros(n, R.ACCEPT_REPLY)
    rec["instance"] = np.repeat(np.arange(base, base + n_inst, dtype=np.int32), counts)
    hi = n_replicas + (2 if bad_ids else 0)
    rec["id"] = rng.integers(0, hi, n)
    rec["ok"] = np.where(rng.random(n) < p_ok, 1, np.where(rng.random(n) < 0.1, 2, 0))
    rec["ballot"] = rng.integers(-5, 300, n)
    st = np.zeros(n_inst, R.INST_STATE)
    if random_state:
        st["status"] = rng.choice([R.PREPARING, R.PREPARED, R.ACCEPTED, R.COMMITTED], n_inst,
                                  p=[0.1, 0.5, 0.3, 0.1])
        st["accept_oks"] = rng.integers(0, 4, n_inst)
        st["nacks"] = rng.integers(0, 3, n_inst)
        st["max_recv_ballot"] = rng.integers(-2, 200, n_inst)
    else:
        st["status"] = R.PREPARED
    return rec, st


def ragged_prepare(rng, n_inst, n_replicas, max_r=8, long_every=0, long_len=300, p_ok=0.7,
                   base=0):
    counts = rng.integers(0, max_r + 1, n_inst)
    if long_every:
        counts[::long_every] = long_len
    n = int(counts.sum())
    rec = np.zeros(n, R.PREPARE_REPLY)
    rec["instance"] = np.repeat(np.arange(base, base + n_inst, dtype=np.int32), counts)
    rec["ok"] = np.where(rng.random(n) < p_ok, 1, 0)
    rec["ballot"] = rng.integers(-1, 12, n) * 16 + rng.integers(0, 5, n)
    rec["ballot"][rng.random(n) < 0.05] = -1
    rec["value_id"] = rng.integers(0, 1 << 31, n)
    st = np.zeros(n_inst, R.PREP_STATE)
    st["ballot"] = rng.integers(0, 20, n_inst) * 16
    st["status"] = rng.choice([R.PREPARING, R.PREPARED, R.COMMITTED], n_inst, p=[0.8, 0.1, 0.1])
    st["prepare_oks"] = rng.integers(0, 3, n_inst)
    st["nacks"] = rng.integers(0, 3, n_inst)
    st["max_recv_ballot"] = rng.integers(-1, 100, n_inst)
    st["value_id"] = rng.integers(0, 1 << 31, n_inst)
    st["flags"] = rng.integers(0, 8, n_inst)
    return rec, st


def commands_mixed(rng, m, n_keys, p_put=0.4, p_other=0.15, neg_keys=True):
    op = np.where(rng.random(m) < p_put, R.OP_PUT, R.OP_GET).astype(np.uint8)
    other = rng.random(m) < p_other
    op[other] = rng.choice([R.OP_NONE, R.OP_DELETE, R.OP_RLOCK, R.OP_WLOCK], int(other.sum()))
    key = rng.integers(0, n_keys, m).astype(np.int64)
    if neg_keys:
        # exercise the full int64 range, including the table's sentinel INT64_MIN and 0
        special = np.array([np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1], np.int64)
        pick = rng.random(m) < 0.02
        key[pick] = special[rng.integers(0, 4, int(pick.sum()))]
    val = rng.integers(-(1 << 62), 1 << 62, m).astype(np.int64)
    return op, key, val
