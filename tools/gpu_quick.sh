#!/bin/bash
# GPU-box run: a few named -m gpu tests (K=pytest -k expression) and bench lines (B=";"-separated
# bench.py argument lists). Each step under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/quick_${TAG:-x}
mkdir -p $OUT
if [ -n "${K:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
fi
i=0
IFS=';' read -ra BS <<< "${B:-}"
for args in "${BS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $args > $OUT/bench_$i.log 2>&1
  rc=$?; echo "bench $i ($args) rc=$rc"
  grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"frac": [0-9.]*\|"bit_exact": [a-z]*' $OUT/bench_$i.log | tr '\n' ' '; echo
  [ $rc = 0 ] || exit $rc
done
