#!/bin/bash
# GPU-box profile of the headline (BASELINE config 5) and the group-step variants:
#   gpurun_out/head_${TAG}/trace/     rocprofv3 --kernel-trace --stats of the default bench line
#   gpurun_out/head_${TAG}/bench.log  the bench line itself (with the CPU baseline)
#   gpurun_out/pmc_${TAG}/traffic.json  FETCH_SIZE / WRITE_SIZE per exact configuration
#                                        (tools/pmc_collect.py; copy to profiles/traffic_r03.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/head_$TAG
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $OUT/bench.log | cut -c1-300; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 900 python tools/pmc_collect.py --out gpurun_out/pmc_$TAG/traffic.json "$@"
rc=$?; echo "pmc rc=$rc"; exit $rc
