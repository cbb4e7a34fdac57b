#!/bin/bash
# round 6: the resolve's loop-top wait (no vmcnt(0) for the previous batch's result stores)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_apply5 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_fuzz.py tests/test_golden.py" PYTEST_K="apply" bash tools/gpu_ab.sh || exit $?
TAG=r06_aptrace5 PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_head.so" bash tools/gpu_apply_ab.sh
