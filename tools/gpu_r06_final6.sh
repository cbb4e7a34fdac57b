#!/bin/bash
# round 6 closing check after the replay changes (4-byte instNo): the GPU suite + smoke, the headline line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SKIP_BENCH=1 bash tools/gpu_check.sh > gpurun_out/check_r06g.txt 2>&1
rc=$?; grep -E "rc=|passed|failed" gpurun_out/check_r06g.txt | tail -4; [ $rc = 0 ] || exit $rc
grep -q "smoke rc=0" gpurun_out/check_r06g.txt || exit 1
grep -qE "[0-9]+ failed" gpurun_out/pytest_gpu.log && exit 1
mkdir -p gpurun_out/r06_f7
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r06_f7/headline.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r06_f7/headline.log | cut -c1-200; exit $rc
