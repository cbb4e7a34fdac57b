#!/bin/bash
# round 6: XCD-contiguous resolve bins: apply parity, traces (xcd / no xcd / partition-order
# results + xcd), FETCH/WRITE passes of each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_apply4 PYTEST_FILES="tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_fuzz.py" PYTEST_K="apply" bash tools/gpu_ab.sh || exit $?
TAG=r06_aptrace4 PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_noxcd.so minpaxos_amd/ab/libmpx_respxcd.so" DISTS=uniform bash tools/gpu_apply_ab.sh || exit $?
for lib in main noxcd respxcd; do
  mkdir -p gpurun_out/pmc_r06_$lib
  [ $lib = main ] && export MPX_LIB=$PWD/minpaxos_amd/libmpx.so || export MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_$lib.so
  timeout -k 10 400 python tools/pmc_collect.py --out gpurun_out/pmc_r06_$lib/traffic.json "--workload apply --dist uniform" || exit $?
done
