#!/bin/bash
# round 6: leaner framing DP (parity + traces vs the round-start build) and per-phase stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_sd11 PYTEST_FILES="tests/test_stream_decode.py tests/test_gpu_fuzz.py tests/test_golden.py" PYTEST_K="stream" MODES="min classic" PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_sdlds0.so" bash tools/gpu_stream_ab.sh || exit $?
MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_sdstamp.so timeout -k 10 300 python bench.py --workload stream --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r06_sd11/stamp.log 2>&1
rc=$?; echo "stamp rc=$rc"; grep SD_STAMP gpurun_out/r06_sd11/stamp.log | head -30
