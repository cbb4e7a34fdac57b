#!/bin/bash
# round 6: stream decoder after the framing-DP / TileEnt work: parity (default + forced
# unconverged build), the two stream config lines under rocprofv3, then their FETCH/WRITE passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06_sd14; mkdir -p $OUT
F="tests/test_stream_decode.py tests/test_decode.py tests/test_gpu_fuzz.py tests/test_golden.py"
timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or decode" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
MPX_FUZZ_EXT=400 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz_ext.py -m gpu -x -q --timeout 300 --timeout-method thread -k stream > $OUT/fuzz_ext.log 2>&1
rc=$?; echo "fuzz_ext rc=$rc"; tail -1 $OUT/fuzz_ext.log; [ $rc = 0 ] || exit $rc
MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_sdtentnc.so timeout -k 10 600 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or decode" > $OUT/pytest_nc.log 2>&1
rc=$?; echo "pytest noconv rc=$rc"; tail -1 $OUT/pytest_nc.log; [ $rc = 0 ] || exit $rc
TAG=r06s WORKLOADS="stream_min stream_classic" bash tools/gpu_prof_configs.sh || exit $?
TAG=r06 TRAFFIC_SETS="--workload stream --steps 3 --warmup 1;--workload stream --mode classic --prepare-every 1 --instances 4194304 --steps 3 --warmup 1" bash tools/gpu_counters.sh
