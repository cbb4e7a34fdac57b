#!/bin/bash
# GPU-box run: rocprofv3 kernel stats of one bench.py command line (A="..."), into
# gpurun_out/prof_${TAG}/ ; optional FETCH_SIZE / WRITE_SIZE passes (PMC=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-x}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o trace -- python3 bench.py $A > $OUT/stats.log 2>&1
rc=$?; echo "stats rc=$rc"; [ $rc = 0 ] || exit $rc
f=$(ls $OUT/stats/*/trace_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | head -25
if [ "${PMC:-0}" = "1" ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- python3 bench.py $A > $OUT/fetch.log 2>&1
  rc=$?; echo "fetch rc=$rc"; [ $rc = 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- python3 bench.py $A > $OUT/write.log 2>&1
  rc=$?; echo "write rc=$rc"; [ $rc = 0 ] || exit $rc
fi
