"""Committed golden fixtures (tests/golden/, made by make_golden.py from the oracle).

CPU: the fixtures are intact (sha256) and the oracle still reproduces every one bit for bit.
GPU: the HIP engine reproduces every one bit for bit.
"""
import glob
import hashlib
import os

import numpy as np
import pytest

from golden.make_golden import run_case
from oracle_lib import Oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    kind = str(z["meta_kind"])
    p = {k[6:]: z[k].item() for k in z.files if k.startswith("param_")}
    x = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    y = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return kind, p, x, y


def check(got, want):
    assert set(want) <= set(got), (set(want), set(got))
    for k, w in want.items():
        g = np.asarray(got[k])
        if w.dtype.names:
            g = g.view(np.uint8)
            w = w.view(np.uint8)
        assert np.array_equal(g.reshape(-1), w.reshape(-1)), k


def test_manifest():
    lines = open(os.path.join(GOLDEN, "MANIFEST.sha256")).read().split("\n")
    listed = {}
    for ln in lines:
        if ln.strip():
            h, name = ln.split()
            listed[name] = h
    assert sorted(listed) == sorted(os.path.basename(f) for f in FILES)
    for f in FILES:
        assert hashlib.sha256(open(f, "rb").read()).hexdigest() == listed[os.path.basename(f)], f


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_golden(path):
    kind, p, x, y = load(path)
    got = run_case(kind, p, x, lambda n, mode, **kw: Oracle(n, mode, **kw))
    check(got, y)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_engine_reproduces_golden(path, mk_engine):
    kind, p, x, y = load(path)
    got = run_case(kind, p, x, mk_engine)
    check(got, y)
