#!/bin/bash
# GPU-box: apply parity (reduced + full config 4), old/new config-4 A/B (tools/ab_apply.sh),
# replica-batch apply lines (5000 commands: one-launch kernel vs the sort-based pipeline) and
# their rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/apply_check; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -v -k "apply or config4" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
if [ "${AB:-1}" = 1 ]; then bash tools/ab_apply.sh || exit $?; fi
for p in auto sorted; do
  timeout -k 10 300 python bench.py --workload apply --commands 5000 --apply-path $p --steps 200 --warmup 20 > $OUT/small_$p.log 2>&1
  rc=$?; echo "small $p rc=$rc"; grep '^{' $OUT/small_$p.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_small_$p -o p -- python3 bench.py --workload apply --commands 5000 --apply-path $p --steps 200 --warmup 20 --no-cpu-baseline > $OUT/prof_small_$p.log 2>&1
  rc=$?; echo "prof small $p rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
