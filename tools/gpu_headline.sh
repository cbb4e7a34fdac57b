#!/bin/bash
# GPU-box run for the headline (BASELINE config 5): the default bench line (with the CPU
# baseline), rocprofv3 kernel stats of the same command, and the FETCH_SIZE / WRITE_SIZE passes
# of k_group_fast, laid out for tools/traffic.py:
#   gpurun_out/headline_${TAG}/{bench.log, trace/, pmc_FETCH_SIZE/, pmc_WRITE_SIZE/}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/headline_${TAG:-r02}
mkdir -p $OUT
ARGS=${ARGS:---steps 20 --warmup 3}
timeout -k 10 400 python bench.py $ARGS > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-600; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py $ARGS --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc = 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o pmc -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/pmc_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc = 0 ] || exit $rc
done
