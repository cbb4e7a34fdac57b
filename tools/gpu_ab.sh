#!/bin/bash
# GPU-box round-6 A/B: parity tests (PYTEST_K over PYTEST_FILES, empty K = skip), then
# tools/ab_libs.sh over LIBS with ARGS (';'-separated bench.py argument sets). Output gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $OUT/pytest.log | tail -3; [ $rc = 0 ] || exit $rc
fi
if [ -n "${LIBS:-}" ]; then
  TAG=${TAG:-ab} timeout -k 10 900 bash tools/ab_libs.sh
fi
