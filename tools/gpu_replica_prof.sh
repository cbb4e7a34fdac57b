#!/bin/bash
# replica-batch apply (5000 / 16000 commands): bench lines (both host forms reported) and a
# rocprofv3 kernel trace of the same command (one kernel per device-pointer call)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/replica_${TAG:-r05}; mkdir -p $OUT
for m in 5000 16000; do
  timeout -k 10 200 python bench.py --workload apply --commands $m --steps 50 --warmup 5 > $OUT/apply$m.log 2>&1
  rc=$?; echo "apply$m rc=$rc"; grep '^{' $OUT/apply$m.log | cut -c1-200; [ $rc = 0 ] || exit $rc
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$m -o trace -- python3 bench.py --workload apply --commands $m --steps 50 --warmup 5 --no-cpu-baseline > $OUT/trace$m.log 2>&1
  rc=$?; echo "trace$m rc=$rc"; [ $rc = 0 ] || exit $rc
done
