#!/bin/bash
# round 6: the fixed-frame decoder's emit image padded per chunk: parity, then A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06_dec1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_decode.py tests/test_gpu_fuzz.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread -k "decode or peer" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
for lib in minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_decpad0.so; do
  n=$(basename $lib .so)
  MPX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o t -- python3 bench.py --workload decode --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_$n.log 2>&1
  rc=$?; echo "prof $n rc=$rc"; [ $rc = 0 ] || exit $rc
  python3 tools/trace_calls.py $OUT/prof_$n/t_kernel_trace.csv k_dec | tail -8
done
