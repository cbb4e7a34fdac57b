"""CPU-side checks of the boundary: libmpx.so loads and exports exactly the C ABI that
include/mpx.h declares; record layouts agree between the header, numpy and ctypes."""
import ctypes as C
import os
import re
import subprocess

import numpy as np

from minpaxos_amd import _lib
from minpaxos_amd import records as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mpx.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mpx_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_bound_symbols():
    assert header_functions() == sorted(_lib.SIGNATURES)


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mpx_[a-z0-9_]+)", out))
    assert set(header_functions()) <= exported
    assert lib.mpx_abi_version() == 8


def test_no_device_calls_fail_cleanly():
    lib = _lib.load()
    c = C.c_int(-1)
    assert lib.mpx_device_count(C.byref(c)) == 0 and c.value >= 0
    assert lib.mpx_close(None) == R.E_INVAL
    assert lib.mpx_accept_tally(None, None, 0, None, 0, 0, None, None, None) == R.E_INVAL
    if c.value == 0:  # this container: opening fails loudly with E_NODEV, never a CPU fallback
        cfg = _lib.MpxConfig(5, 0, 0, 0, 0, 0)
        h = C.c_void_p()
        assert lib.mpx_open(0, C.byref(cfg), C.byref(h)) == R.E_NODEV


def test_struct_sizes_match_header():
    # compile a tiny C program against the header and compare sizeof / offsetof
    src = r"""
    #include <stdio.h>
    #include <stddef.h>
    #include "mpx.h"
    int main(void) {
      printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(mpx_accept_reply),
        sizeof(mpx_inst_state), sizeof(mpx_prepare_reply), sizeof(mpx_prep_state),
        sizeof(mpx_prepare_reply_min), sizeof(mpx_group_prep_state), sizeof(mpx_prepare_effect),
        sizeof(mpx_config), sizeof(mpx_group_batch));
      printf("%zu %zu %zu %zu\n", offsetof(mpx_accept_reply, ok), offsetof(mpx_prep_state, flags),
        offsetof(mpx_group_batch, decided), offsetof(mpx_group_batch, n_decided));
      return 0;
    }"""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        exe = os.path.join(d, "t")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    sizes = [int(x) for x in lines[0].split()]
    offs = [int(x) for x in lines[1].split()]
    assert sizes[:7] == [R.ACCEPT_REPLY.itemsize, R.INST_STATE.itemsize, R.PREPARE_REPLY.itemsize,
                         R.PREP_STATE.itemsize, R.PREPARE_REPLY_MIN.itemsize,
                         R.GROUP_PREP_STATE.itemsize, R.PREPARE_EFFECT.itemsize]
    assert sizes[7] == C.sizeof(_lib.MpxConfig)
    assert sizes[8] == C.sizeof(_lib.MpxGroupBatch)
    assert offs[0] == R.ACCEPT_REPLY.fields["ok"][1]
    assert offs[1] == R.PREP_STATE.fields["flags"][1]
    assert offs[2] == _lib.MpxGroupBatch.decided.offset
    assert offs[3] == _lib.MpxGroupBatch.n_decided.offset


def test_runtime_info_names_the_bound_runtimes():
    """libmpx.so reports the HIP / RCCL it is bound to (bench.py records it in its JSON line)"""
    info = _lib.runtime_info()
    assert info["hip_runtime"] > 0 and info["rccl"] > 0
    assert "libamdhip64" in info["hip_path"] and "librccl" in info["rccl_path"]


def test_no_device_utilities_fail_cleanly():
    lib = _lib.load()
    p = C.c_void_p()
    assert lib.mpx_dev_alloc(None, 16, C.byref(p)) == R.E_INVAL
    assert lib.mpx_stream_create(None, C.byref(p)) == R.E_INVAL
    assert lib.mpx_step_allreduce_dev(None, None, 0, None, 0, None) == R.E_INVAL
    assert lib.mpx_replay_durable(None, None, 0, 0, 0, None, None, None, None, None, None) == \
        R.E_INVAL


def test_product_does_not_reference_oracle():
    """the shipped library and package never link or import the oracle"""
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    pkg = os.path.join(ROOT, "minpaxos_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", "Makefile")):
                assert "oracle" not in open(os.path.join(dp, f)).read().lower() or \
                    f == "__init__.py", f
