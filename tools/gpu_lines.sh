#!/bin/bash
# GPU-box: bench lines (no profiler) for the workloads in WORKLOADS, into gpurun_out/lines_${TAG}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lines_${TAG:-r03}; mkdir -p $OUT
run() {
  name=$1; shift
  timeout -k 10 ${BT:-300} python bench.py "$@" > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; grep '^{' $OUT/$name.log | tail -1 | cut -c1-160
  [ $rc = 0 ] || exit $rc
}
for w in ${WORKLOADS:-decode stream_min stream_classic fanout log_catchup log_durable conflict}; do
  case $w in
    decode) run $w --workload decode --steps 10 --warmup 2;;
    stream_min) run $w --workload stream --steps 5 --warmup 1;;
    stream_classic) run $w --workload stream --mode classic --prepare-every 1 --instances 4194304 --steps 5 --warmup 1;;
    fanout) run $w --workload fanout --steps 10 --warmup 2;;
    log_catchup) run $w --workload log --log-format catchup --steps 10 --warmup 2;;
    log_durable) run $w --workload log --log-format durable --steps 10 --warmup 2;;
    conflict) run $w --workload conflict --steps 5 --warmup 1;;
    tally_min) run $w --workload tally --mode min --steps 10 --warmup 2;;
    tally_classic) run $w --workload tally --mode classic --steps 10 --warmup 2;;
    apply_small) run $w --workload apply --commands 5000 --steps 200 --warmup 20;;
  esac
done
