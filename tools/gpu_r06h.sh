#!/bin/bash
# round 6: FastBase key slots 512 vs 448 vs 384 (7 workgroups per CU): step parity of the 384
# build, then P = 1 and the P = 8 / P = 4 per-rank shapes (graph replay)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_fb
MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_fb384.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -k "group_step or config5 or step" > gpurun_out/r06_fb/pytest384.log 2>&1
rc=$?; echo "pytest384 rc=$rc"; tail -2 gpurun_out/r06_fb/pytest384.log; [ $rc = 0 ] || exit $rc
TAG=r06_fb LIBS="main minpaxos_amd/ab/libmpx_fb448.so minpaxos_amd/ab/libmpx_fb384.so" ARGS="--steps 40 --warmup 3;--emulate-world 8 --graph on --steps 100 --warmup 3;--emulate-world 4 --graph on --steps 100 --warmup 3" bash tools/gpu_ab.sh
