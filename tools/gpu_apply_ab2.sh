#!/bin/bash
# GPU-box: apply parity (reduced + full config 4) on libmpx.so, then the interleaved config-4
# A/B of tools/ab_apply.sh (LIBS, default libmpx_old.so libmpx.so) and per-kernel stats of the
# new build under rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/apply_ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -m gpu -x -q -k "config4" --timeout 300 --timeout-method thread > gpurun_out/apply_ab/pytest_full.log 2>&1
rc=$?; echo "pytest full rc=$rc"; tail -3 gpurun_out/apply_ab/pytest_full.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_apply.sh || exit $?
for d in uniform zipf; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/apply_ab/prof_$d -o p -- python3 bench.py --workload apply --dist $d --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/apply_ab/prof_$d.log 2>&1
  rc=$?; echo "prof $d rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
