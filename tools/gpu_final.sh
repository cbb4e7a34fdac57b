#!/bin/bash
# GPU-box: the round's closing evidence in one call — the GPU suite + smoke (tools/gpu_check.sh,
# no bench), the headline line and its rocprofv3 kernel trace (gpurun_out/head_${TAG}/), and
# the counter passes of tools/gpu_counters.sh for $TRAFFIC_SETS / $INSTR_SETS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  SKIP_BENCH=1 bash tools/gpu_check.sh > gpurun_out/check_$TAG.txt 2>&1
  rc=$?; grep -E "rc=|passed|failed" gpurun_out/check_$TAG.txt | tail -5; [ $rc = 0 ] || exit $rc
  grep -q "smoke rc=0" gpurun_out/check_$TAG.txt || exit 1
fi
OUT=gpurun_out/head_$TAG; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $OUT/bench.log | cut -c1-400; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc = 0 ] || exit $rc
bash tools/gpu_counters.sh
