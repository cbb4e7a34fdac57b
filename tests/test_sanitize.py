"""CPU hygiene: the host code under AddressSanitizer + UndefinedBehaviorSanitizer.

- the C ABI's host side (engine.cpp: argument validation, staging, the decode loop, error
  reporting) built with g++ -fsanitize=address,undefined over a host-memory stand-in for the
  HIP / RCCL runtime (tests/san/hip_stub.cpp) and driven through every entry point by
  tests/san/abi_driver.cpp, leak checking on;
- the CPU oracle (oracle/liboracle_san.so) under the oracle-facing CPU tests, in a subprocess
  with the ASan runtime preloaded.
Device code is not instrumented (GPU sanitizers are not available on this pool).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "san")


def _libasan():
    p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


@pytest.fixture(scope="module")
def asan():
    lib = _libasan()
    if not lib:
        pytest.skip("gcc's libasan is not installed")
    return lib


def test_abi_host_paths_asan_ubsan(tmp_path, asan):
    exe = str(tmp_path / "abi_driver")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           "-I" + os.path.join(ROOT, "include"), "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", os.path.join(ROOT, "minpaxos_amd", "csrc", "engine.cpp"),
           os.path.join(SAN, "hip_stub.cpp"), os.path.join(SAN, "abi_driver.cpp"), "-ldl", "-o", exe]
    subprocess.run(cmd, check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_oracle_cpu_tests_asan_ubsan(asan):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle_san.so"],
                   check=True)
    env = dict(os.environ, LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", MPX_TESTS_NO_ENGINE="1",
               MPX_ORACLE_SO=os.path.join(ROOT, "oracle", "liboracle_san.so"))
    tests = [os.path.join(ROOT, "tests", t) for t in
             ("test_oracle_kat.py", "test_golden.py", "test_stream_decode.py", "test_replay.py",
              "test_decode.py", "test_fanout.py", "test_logenc.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p",
                        "no:cacheprovider", *tests], capture_output=True, text=True, env=env,
                       timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "passed" in r.stdout
