#!/bin/bash
# GPU-box A/B of stream-decoder builds (round 6): parity tests (PYTEST_K, empty = skip), per-call
# kernel traces of every build in PROF_LIBS for the modes in MODES, then ms per call of every
# build in LIBS (ab_libs.sh). Output gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-stream_ab}; mkdir -p $OUT
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests/test_stream_decode.py tests/test_gpu_fuzz.py tests/test_golden.py} -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $OUT/pytest.log | tail -3; [ $rc = 0 ] || exit $rc
fi
for m in ${MODES:-min}; do
  for lib in ${PROF_LIBS:-}; do
    n=$(basename $lib .so)_$m
    MPX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o t -- python3 bench.py --workload stream --mode $m --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_$n.log 2>&1
    rc=$?; echo "prof $n rc=$rc"; [ $rc = 0 ] || exit $rc
    python3 tools/trace_calls.py $OUT/prof_$n/t_kernel_trace.csv k_sd | tail -9
  done
done
if [ -n "${LIBS:-}" ]; then
  A=""
  for m in ${MODES:-min}; do A="$A;--workload stream --mode $m --steps 10 --warmup 2"; done
  TAG=${TAG:-stream_ab} ARGS="${A#;}" timeout -k 10 900 bash tools/ab_libs.sh
fi
