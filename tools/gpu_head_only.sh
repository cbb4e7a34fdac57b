#!/bin/bash
# the headline bench line (with its CPU baseline) + a rocprofv3 kernel trace of the same command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/head_${TAG:-r05}
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $OUT/bench.log | cut -c1-300; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
