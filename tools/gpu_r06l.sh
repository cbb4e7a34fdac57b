#!/bin/bash
# round 6: run-by-run fan-out write-out: parity, then A/B against the per-slot write-out
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_fan2 PYTEST_FILES="tests/test_fanout.py tests/test_gpu_fuzz.py tests/test_golden.py" PYTEST_K="fan or reply or encode" LIBS="main minpaxos_amd/ab/libmpx_fanold.so minpaxos_amd/ab/libmpx_fanrabl1.so minpaxos_amd/ab/libmpx_fanrabl8.so" ARGS="--workload fanout --steps 10 --warmup 2" bash tools/gpu_ab.sh
