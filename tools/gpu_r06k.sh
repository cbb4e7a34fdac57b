#!/bin/bash
# round 6: the resolve's result stores as one 16-byte record at image positions, or nontemporal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_res16img.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread -k "apply" > gpurun_out/r06_res16_pytest.log 2>&1
rc=$?; echo "pytest res16img rc=$rc"; tail -1 gpurun_out/r06_res16_pytest.log; [ $rc = 0 ] || exit $rc
TAG=r06_aptrace6 PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_res16img.so minpaxos_amd/ab/libmpx_rlnt.so" bash tools/gpu_apply_ab.sh
