#!/bin/bash
# GPU-box: one rank's share of P-rank strong scaling (bench.py --emulate-world P), with and
# without the hipGraph replay, into gpurun_out/emu_${TAG}/; P=8 also under rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/emu_${TAG:-r04}; mkdir -p $OUT
run() {
  name=$1; shift
  timeout -k 10 ${BT:-300} python bench.py "$@" > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; grep '^{' $OUT/$name.log | tail -1 | cut -c1-200
  [ $rc = 0 ] || exit $rc
}
for P in ${PS:-1 2 4 8}; do
  run p${P} --emulate-world $P --graph off --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline ${XARGS:-}
  run p${P}_graph --emulate-world $P --graph on --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline ${XARGS:-}
done
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_p8 -o trace -- python3 bench.py --emulate-world 8 --graph off --steps 40 --warmup 3 --no-cpu-baseline > $OUT/trace_p8.log 2>&1
  rc=$?; echo "trace_p8 rc=$rc"; [ $rc = 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_p8g -o trace -- python3 bench.py --emulate-world 8 --graph on --steps 40 --warmup 3 --no-cpu-baseline > $OUT/trace_p8g.log 2>&1
  rc=$?; echo "trace_p8g rc=$rc"; [ $rc = 0 ] || exit $rc
fi
