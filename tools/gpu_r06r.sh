#!/bin/bash
# round 6: PrepareReply mark in the landing table (MPX_SD_PRMARK=1, ab/libmpx_prmark.so):
# stream parity on the variant, then per-call traces MIN / CLASSIC against the default build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06_prmark; mkdir -p $OUT
MPX_LIB=$PWD/minpaxos_amd/ab/libmpx_prmark.so MPX_FUZZ_EXT=200 timeout -k 10 600 python -u -m pytest tests/test_stream_decode.py tests/test_gpu_fuzz.py tests/test_gpu_fuzz_ext.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or peer" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
i=0
for m in min classic; do
  for lib in minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_prmark.so minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_prmark.so; do
    i=$((i+1)); n=$(basename $lib .so)_${m}_$i
    MPX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o t -- python3 bench.py --workload stream --mode $m --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_$n.log 2>&1
    rc=$?; echo "prof $n rc=$rc"; [ $rc = 0 ] || exit $rc
    python3 tools/trace_calls.py $OUT/prof_$n/t_kernel_trace.csv k_sd | tail -9
  done
done
