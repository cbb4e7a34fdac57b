#!/bin/bash
# GPU-box profiling: bench, rocprofv3 kernel trace + stats, and separate PMC passes for the
# HBM byte counters (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${ARGS:---steps 10 --warmup 2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
stop_if_fault() { case $1 in 0) ;; *) echo "exit $1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 400 python bench.py $ARGS > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.log; stop_if_fault $rc bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py $ARGS --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; stop_if_fault $rc trace
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${PMC_ARGS:-} > $OUT/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; stop_if_fault $rc pmc_$c
done
find $OUT -name "*.csv" | head -20
