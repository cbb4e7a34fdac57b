#!/bin/bash
# GPU-box check: parity tests, smoke, short bench. Stops at the first fault-class exit status
# (timeout 124/137, abort 134, segfault 139); plain test failures (1) do not stop the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fault() { case $1 in 0|1) ;; *) echo "fault-class exit $1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; stop_if_fault $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log; stop_if_fault $rc smoke
if [ "${SKIP_BENCH:-0}" = "0" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -20 gpurun_out/bench.log; stop_if_fault $rc bench
fi
