#!/bin/bash
# round 6: conflict parity + A/B (32-bit key planes); resolve phase stamps, new vs old pipeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_conf2 PYTEST_K="conflict" LIBS="main minpaxos_amd/ab/libmpx_confold.so" ARGS="--workload conflict --steps 20 --warmup 3" bash tools/gpu_ab.sh || exit $?
OUT=gpurun_out/r06_stamp; mkdir -p $OUT
for lib in rlstamp oldstamp; do
  for d in uniform zipf; do
    MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_$lib.so timeout -k 10 300 python bench.py --workload apply --dist $d --steps 2 --warmup 0 --no-cpu-baseline > $OUT/${lib}_$d.log 2>&1
    rc=$?; echo "$lib $d rc=$rc"; grep RL_STAMP $OUT/${lib}_$d.log | tail -3; [ $rc = 0 ] || exit $rc
  done
done
