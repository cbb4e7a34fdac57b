#!/bin/bash
# round 6: conflict parity + A/B; apply parity; per-kernel traces of the apply pipelines (new vs old);
# fan-out ablations
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_conf PYTEST_K="conflict or events_destroyed" LIBS="main minpaxos_amd/ab/libmpx_confold.so" ARGS="--workload conflict --steps 20 --warmup 3" bash tools/gpu_ab.sh || exit $?
TAG=r06_apply PYTEST_FILES="tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fuzz.py tests/test_gpu_full.py" PYTEST_K="apply" bash tools/gpu_ab.sh || exit $?
TAG=r06_aptrace PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_resp.so minpaxos_amd/ab/libmpx_apold.so" bash tools/gpu_apply_ab.sh || exit $?
TAG=r06_fan LIBS="main minpaxos_amd/ab/libmpx_fanabl1.so minpaxos_amd/ab/libmpx_fanabl2.so minpaxos_amd/ab/libmpx_fanabl8.so" ARGS="--workload fanout --steps 5 --warmup 1" bash tools/gpu_ab.sh
