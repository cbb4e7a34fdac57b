#!/bin/bash
# Generic GPU-box run: an optional pytest selection, then bench lines, each optionally under
# rocprofv3 --kernel-trace --stats. Stops at the first failing GPU step.
#   TESTS="tally or prepare"    pytest -m gpu -k expression (empty: no tests; "all": every gpu test)
#   BENCHES="--workload tally --mode min;--workload prepare"   bench.py argument sets, ';'-separated
#   PROF=1                      also run each bench under rocprofv3 (kernel stats csv)
#   TAG=name                    output directory gpurun_out/$TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  sel=(); [ "$TESTS" != "all" ] && sel=(-k "$TESTS")
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 \
      --timeout-method thread "${sel[@]}" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $OUT/pytest.log | tail -3
  [ $rc = 0 ] || { tail -60 $OUT/pytest.log; exit $rc; }
fi
i=0
IFS=';' read -ra SETS <<< "${BENCHES:-}"
for args in "${SETS[@]}"; do
  [ -z "$args" ] && continue
  i=$((i+1))
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $args > $OUT/bench_$i.json 2> $OUT/bench_$i.err
  rc=$?; echo "bench $i ($args) rc=$rc"; tail -c 700 $OUT/bench_$i.json; echo
  [ $rc = 0 ] || { tail -20 $OUT/bench_$i.err; exit $rc; }
  if [ "${PROF:-0}" = "1" ]; then
    timeout -k 10 ${BENCH_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv \
        -d $OUT/prof_$i -o trace -- python3 bench.py $args --no-cpu-baseline > $OUT/prof_$i.log 2>&1
    rc=$?; echo "prof $i rc=$rc"; [ $rc = 0 ] || { tail -20 $OUT/prof_$i.log; exit $rc; }
    f=$(find $OUT/prof_$i -name "*kernel_stats.csv" | head -1)
    [ -n "$f" ] && cut -d, -f1-4 "$f" | head -12
  fi
done
exit 0
