#!/bin/bash
# round 6: TileEnt (converged tiles skip the chunk maps): parity of the default build and of a
# build forcing every tile down the unconverged path, then traces against the chunk-map build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06_sd13; mkdir -p $OUT
F="tests/test_stream_decode.py tests/test_decode.py tests/test_gpu_fuzz.py tests/test_golden.py"
timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or decode" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
MPX_FUZZ_EXT=200 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz_ext.py -m gpu -x -q --timeout 300 --timeout-method thread -k stream > $OUT/fuzz_ext.log 2>&1
rc=$?; echo "fuzz_ext rc=$rc"; tail -1 $OUT/fuzz_ext.log; [ $rc = 0 ] || exit $rc
MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_sdtentnc.so timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or decode" > $OUT/pytest_nc.log 2>&1
rc=$?; echo "pytest noconv rc=$rc"; tail -1 $OUT/pytest_nc.log; [ $rc = 0 ] || exit $rc
MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_sdtentnc.so MPX_FUZZ_EXT=100 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz_ext.py -m gpu -x -q --timeout 300 --timeout-method thread -k stream > $OUT/fuzz_ext_nc.log 2>&1
rc=$?; echo "fuzz_ext noconv rc=$rc"; tail -1 $OUT/fuzz_ext_nc.log; [ $rc = 0 ] || exit $rc
TAG=r06_sd13 MODES="min classic" PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_sdtent0.so" bash tools/gpu_stream_ab.sh
