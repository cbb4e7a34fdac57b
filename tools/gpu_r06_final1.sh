#!/bin/bash
# round 6 closing evidence, part 1: the GPU suite + smoke, the headline line and its rocprofv3
# kernel trace (gpurun_out/head_r06/), the counter passes of the headline and the rebuilt rows
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SKIP_BENCH=1 bash tools/gpu_check.sh > gpurun_out/check_r06.txt 2>&1
rc=$?; grep -E "rc=|passed|failed" gpurun_out/check_r06.txt | tail -5; [ $rc = 0 ] || exit $rc
grep -q "smoke rc=0" gpurun_out/check_r06.txt || exit 1
OUT=gpurun_out/head_r06; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $OUT/bench.log | cut -c1-300; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc = 0 ] || exit $rc
mkdir -p gpurun_out/pmc_r06final
cp profiles/traffic_r06.json gpurun_out/pmc_r06final/traffic.json
timeout -k 10 900 python tools/pmc_collect.py --out gpurun_out/pmc_r06final/traffic.json "" "--workload apply --dist uniform" "--workload apply --dist zipf" "--workload conflict"
rc=$?; echo "pmc rc=$rc"; exit $rc
