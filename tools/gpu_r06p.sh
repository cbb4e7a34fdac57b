#!/bin/bash
# round 6: bit-6 variable-message marker (fewer VALU ops per dword) + TileEnt scratch in the row
# padding: parity (default and forced-unconverged builds), then traces against the previous build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06_sd21; mkdir -p $OUT
F="tests/test_stream_decode.py tests/test_decode.py tests/test_gpu_fuzz.py tests/test_golden.py"
timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or decode" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
MPX_FUZZ_EXT=400 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz_ext.py -m gpu -x -q --timeout 300 --timeout-method thread -k stream > $OUT/fuzz_ext.log 2>&1
rc=$?; echo "fuzz_ext rc=$rc"; tail -1 $OUT/fuzz_ext.log; [ $rc = 0 ] || exit $rc
MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_sdtentnc.so timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or decode" > $OUT/pytest_nc.log 2>&1
rc=$?; echo "pytest noconv rc=$rc"; tail -1 $OUT/pytest_nc.log; [ $rc = 0 ] || exit $rc
TAG=r06_sd21 MODES="min classic" PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_sdwpe4.so minpaxos_amd/ab/libmpx_sdprev.so" bash tools/gpu_stream_ab.sh
