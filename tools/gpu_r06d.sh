#!/bin/bash
# round 6: apply parity + traces (marks with register positions vs per-record expansion); conflict staging sizes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_apply3 PYTEST_FILES="tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fuzz.py tests/test_gpu_full.py" PYTEST_K="apply or conflict" bash tools/gpu_ab.sh || exit $?
TAG=r06_aptrace3 PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_r06a.so" bash tools/gpu_apply_ab.sh || exit $?
TAG=r06_conf4 LIBS="main minpaxos_amd/ab/libmpx_confs1534.so minpaxos_amd/ab/libmpx_confs1790.so" ARGS="--workload conflict --steps 20 --warmup 3" bash tools/gpu_ab.sh
