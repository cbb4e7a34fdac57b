#!/bin/bash
# GPU-box: a subset of the GPU tests (PYTEST_K, a pytest -k expression; empty = skip), then bench
# lines, one per ';'-separated argument set in BENCHES, into gpurun_out/quick_${TAG}/.
# Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/quick_${TAG:-r04}; mkdir -p $OUT
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$PYTEST_K" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $OUT/pytest.log | tail -3; [ $rc = 0 ] || exit $rc
fi
i=0
IFS=';' read -ra SETS <<< "${BENCHES:-}"
for args in "${SETS[@]}"; do
  [ -z "${args// }" ] && continue
  i=$((i+1))
  timeout -k 10 ${BT:-300} python bench.py $args > $OUT/b$i.log 2>&1
  rc=$?; echo "b$i [$args] rc=$rc"; grep '^{' $OUT/b$i.log | tail -1 | cut -c1-160; [ $rc = 0 ] || exit $rc
done
