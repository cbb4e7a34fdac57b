import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: larger parity sizes")
    # Build the oracle (g++) and, where hipcc exists, the engine (incremental make), then load
    # libmpx.so BEFORE any test module imports torch: the engine binds /opt/rocm's HIP and RCCL
    # (the runtime bench.py measures on too), not the copies torch bundles.
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if os.environ.get("MPX_TESTS_NO_ENGINE"):  # oracle-only runs (the sanitizer subprocess)
        return
    if os.path.exists("/opt/rocm/bin/hipcc"):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "minpaxos_amd")], check=True)
    from minpaxos_amd import _lib
    _lib.load()


def pytest_report_header(config):
    if os.environ.get("MPX_TESTS_NO_ENGINE"):
        return "oracle only"
    from minpaxos_amd import _lib
    return f"libmpx.so runtime: {_lib.runtime_info()}"


@pytest.fixture(scope="session")
def have_gpu():
    from minpaxos_amd import engine
    return engine.device_count() > 0


@pytest.fixture
def mk_oracle():
    from oracle_lib import Oracle

    def mk(n, mode, **kw):
        return Oracle(n_replicas=n, mode=mode, **kw)
    return mk


@pytest.fixture
def mk_engine():
    from minpaxos_amd.engine import Engine, device_count
    if device_count() < 1:
        pytest.fail("GPU test collected but no HIP device is visible")
    made = []

    def mk(n, mode, **kw):
        e = Engine(0, n_replicas=n, mode=mode, **kw)
        made.append(e)
        return e
    yield mk
    for e in made:
        e.close()


@pytest.fixture(scope="session")
def stub_lib():
    """libmpx_stub.so: engine.cpp (the real C ABI host code) over tests/san/hip_stub.cpp built
    with MPX_STUB_ORACLE=1 — host-memory "devices", the group step through the CPU oracle and
    RCCL all-reduces that really reduce across processes (shared memory). TEST INFRASTRUCTURE:
    lets the multi-rank path of bench.py / engine.cpp run on a CPU; never shipped."""
    out_dir = os.path.join(TESTS, "san", "_build")
    os.makedirs(out_dir, exist_ok=True)
    so = os.path.join(out_dir, "libmpx_stub.so")
    srcs = [os.path.join(ROOT, "minpaxos_amd", "csrc", "engine.cpp"),
            os.path.join(TESTS, "san", "hip_stub.cpp"), os.path.join(ROOT, "oracle", "oracle.cpp")]
    deps = srcs + [os.path.join(ROOT, "include", "mpx.h"),
                   os.path.join(ROOT, "minpaxos_amd", "csrc", "kernels.hpp")]
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(d) for d in deps):
        subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fPIC", "-shared",
                        "-D__HIP_PLATFORM_AMD__", "-DMPX_STUB_ORACLE=1", "-I/opt/rocm/include",
                        "-I" + os.path.join(ROOT, "include"), *srcs, "-ldl", "-lrt", "-o", so],
                       check=True)
    return so
