#!/bin/bash
# GPU-box A/B of apply builds (round 5): parity tests on libmpx.so (PYTEST_K, empty = skip),
# phase stamps of a -DMPX_RL_STAMP=1 build (STAMP_LIB), per-call kernel traces (PROF_LIBS), then
# ms per call of every build in LIBS (ab_libs.sh) for the dists in DISTS. Output gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-apply_ab}; mkdir -p $OUT
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_golden.py tests/test_gpu_fuzz.py -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $OUT/pytest.log | tail -3; [ $rc = 0 ] || exit $rc
fi
for d in ${DISTS:-uniform zipf}; do
  if [ -n "${STAMP_LIB:-}" ]; then
    MPX_LIB=$PWD/$STAMP_LIB timeout -k 10 300 python bench.py --workload apply --dist $d --steps 2 --warmup 0 --no-cpu-baseline > $OUT/stamp_$d.log 2>&1
    rc=$?; echo "stamp $d rc=$rc"; grep _STAMP $OUT/stamp_$d.log | tail -3; [ $rc = 0 ] || exit $rc
  fi
  for lib in ${PROF_LIBS:-}; do
    n=$(basename $lib .so)_$d
    MPX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o t -- python3 bench.py --workload apply --dist $d --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_$n.log 2>&1
    rc=$?; echo "prof $n rc=$rc"; [ $rc = 0 ] || exit $rc
    python3 tools/trace_calls.py $OUT/prof_$n/t_kernel_trace.csv k_ap | tail -6
  done
done
if [ -n "${LIBS:-}" ]; then
  A=""
  for d in ${DISTS:-uniform zipf}; do A="$A;--workload apply --dist $d --steps 5 --warmup 1"; done
  TAG=${TAG:-apply_ab} ARGS="${A#;}" timeout -k 10 900 bash tools/ab_libs.sh
fi
