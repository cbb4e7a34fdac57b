#!/bin/bash
# GPU-box: fan-out parity tests, the logenc bench line, and its rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/logenc_${TAG:-r01}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_logenc.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload log --steps 10 --warmup 2 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $OUT/bench.log | tail -1; [ $rc -eq 0 ] || { tail -20 $OUT/bench.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- python3 bench.py --workload log --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - $OUT/prof/p_kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print(f"{float(r['AverageNs'])/1e3:9.1f}us x{r['Calls']:>4}  {r['Name'][:100]}")
PY
