#!/bin/bash
# round 6 closing check after the count fold: the GPU suite + smoke, the extended stream sweep
# (default and forced-unconverged builds), the headline line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SKIP_BENCH=1 bash tools/gpu_check.sh > gpurun_out/check_r06e.txt 2>&1
rc=$?; grep -E "rc=|passed|failed" gpurun_out/check_r06e.txt | tail -4; [ $rc = 0 ] || exit $rc
grep -q "smoke rc=0" gpurun_out/check_r06e.txt || exit 1
grep -qE "[0-9]+ failed" gpurun_out/pytest_gpu.log && exit 1
mkdir -p gpurun_out/r06_fz2
MPX_FUZZ_EXT=1000 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz_ext.py -m gpu -x -q --timeout 300 --timeout-method thread -k stream > gpurun_out/r06_fz2/stream_ext_1000.log 2>&1
rc=$?; echo "ext rc=$rc"; tail -1 gpurun_out/r06_fz2/stream_ext_1000.log; [ $rc = 0 ] || exit $rc
MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_sdtentnc.so MPX_FUZZ_EXT=400 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz_ext.py -m gpu -x -q --timeout 300 --timeout-method thread -k stream > gpurun_out/r06_fz2/stream_ext_nc_400.log 2>&1
rc=$?; echo "ext nc rc=$rc"; tail -1 gpurun_out/r06_fz2/stream_ext_nc_400.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r06_fz2/headline.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r06_fz2/headline.log | cut -c1-200; exit $rc
