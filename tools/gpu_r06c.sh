#!/bin/bash
# round 6: apply parity; per-kernel traces (marks vs per-record expansion vs round 5); stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_apply2 PYTEST_FILES="tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fuzz.py tests/test_gpu_full.py" PYTEST_K="apply" bash tools/gpu_ab.sh || exit $?
TAG=r06_aptrace2 PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_r06a.so minpaxos_amd/ab/libmpx_apold.so" bash tools/gpu_apply_ab.sh || exit $?
OUT=gpurun_out/r06_stamp2; mkdir -p $OUT
for d in uniform zipf; do
  MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_rlstamp.so timeout -k 10 300 python bench.py --workload apply --dist $d --steps 2 --warmup 0 --no-cpu-baseline > $OUT/rlstamp_$d.log 2>&1
  rc=$?; echo "rlstamp $d rc=$rc"; grep RL_STAMP $OUT/rlstamp_$d.log | tail -2; [ $rc = 0 ] || exit $rc
done
