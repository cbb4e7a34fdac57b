#!/bin/bash
# round 6 closing evidence after the stream-decoder work: the GPU suite + smoke, the headline
# line, the two stream config lines under rocprofv3 and their FETCH/WRITE passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SKIP_BENCH=1 bash tools/gpu_check.sh > gpurun_out/check_r06c.txt 2>&1
rc=$?; grep -E "rc=|passed|failed" gpurun_out/check_r06c.txt | tail -5; [ $rc = 0 ] || exit $rc
grep -q "smoke rc=0" gpurun_out/check_r06c.txt || exit 1
grep -qE "[0-9]+ failed" gpurun_out/pytest_gpu.log && exit 1
OUT=gpurun_out/head_r06c; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $OUT/bench.log | cut -c1-300; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
