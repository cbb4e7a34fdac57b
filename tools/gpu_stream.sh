#!/bin/bash
# GPU-box run: the stream decoder's parity tests, the legacy decode tests, and decode benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/stream_${TAG:-r02}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_stream_decode.py tests/test_decode.py -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 $OUT/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
run() {
  name=$1; shift
  timeout -k 10 ${BT:-400} python bench.py "$@" > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-600
  case $rc in 0) ;; *) exit $rc;; esac
}
run decode_legacy --workload decode --steps 10 --warmup 2 --no-cpu-baseline
run stream_min_ar --workload stream --mode min --prepare-every 0 --steps 10 --warmup 2 --no-cpu-baseline
run stream_min --workload stream --mode min --steps 10 --warmup 2 --no-cpu-baseline
run stream_classic --workload stream --mode classic --prepare-every 1 --instances 4194304 --steps 10 --warmup 2 --no-cpu-baseline
if [ "${PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o trace -- python3 bench.py --workload stream --mode min --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_legacy -o trace -- python3 bench.py --workload decode --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_legacy.log 2>&1
  rc=$?; echo "prof legacy rc=$rc"
fi
