#!/bin/bash
# round 6: replay's binned maximum from chunk-sorted runs (MPX_REPLAY_SORTCHUNK=1, the default
# build) vs the count / scan / scatter form (ab/libmpx_rpold.so): parity, then per-kernel traces
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_replay}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_replay.py tests/test_golden.py tests/test_gpu_full.py -m gpu -x -v --timeout 300 --timeout-method thread -k "replay or durable" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
i=0
for d in "" "--replay-dups"; do
  for lib in minpaxos_amd/libmpx.so ${OLD:-minpaxos_amd/ab/libmpx_rpold.so} minpaxos_amd/libmpx.so ${OLD:-minpaxos_amd/ab/libmpx_rpold.so}; do
    i=$((i+1)); n=$(basename $lib .so)${d:+_dups}_$i
    MPX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o t -- python3 bench.py --workload replay $d --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_$n.log 2>&1
    rc=$?; echo "prof $n rc=$rc"; [ $rc = 0 ] || exit $rc
    python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$OUT/prof_$n/t_kernel_stats.csv')))
tot=0
for r in rows:
    if 'k_r' in r['Name'] or 'k_scan' in r['Name']:
        a=float(r['AverageNs'])/1e3; tot+=a; print('  %-40s %8.1f' % (r['Name'].split('(')[0][-40:], a))
print('  sum %.1f us' % tot)"
    tail -1 $OUT/prof_$n.log | cut -c1-160
  done
done
