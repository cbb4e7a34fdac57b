#!/bin/bash
# GPU-box rocprofv3 kernel stats + bench lines (with CPU baselines) for the single-path
# workloads: BASELINE configs 2-4 and the SURVEY 8(f) rows (decode, fanout, log).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/profcfg_${TAG:-r01}
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -k 10 ${BT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o $name -- python3 bench.py "$@" > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; grep '^{' $OUT/$name.log | tail -1 | cut -c1-400
  case $rc in 0) ;; *) exit $rc;; esac
}
for w in ${WORKLOADS:-tally_min tally_classic prepare prepare_min apply_uniform apply_zipf conflict decode stream_min stream_classic fanout log_catchup log_durable replay replay_dups step_keys1024 step_n7 step_ipg512 step_strong}; do
  case $w in
    tally_min) run $w --workload tally --mode min --steps 10 --warmup 2 ${XARGS:-};;
    tally_classic) run $w --workload tally --mode classic --steps 10 --warmup 2 ${XARGS:-};;
    prepare) run $w --workload prepare --steps 10 --warmup 2 ${XARGS:-};;
    apply_uniform) run $w --workload apply --dist uniform --steps 5 --warmup 1 ${XARGS:-};;
    apply_zipf) run $w --workload apply --dist zipf --steps 5 --warmup 1 ${XARGS:-};;
    decode) run $w --workload decode --steps 10 --warmup 2 ${XARGS:-};;
    fanout) run $w --workload fanout --steps 10 --warmup 2 ${XARGS:-};;
    log_catchup) run $w --workload log --log-format catchup --steps 10 --warmup 2 ${XARGS:-};;
    log_durable) run $w --workload log --log-format durable --steps 10 --warmup 2 ${XARGS:-};;
    prepare_min) run $w --workload prepare_min --steps 10 --warmup 2 ${XARGS:-};;
    conflict) run $w --workload conflict --steps 5 --warmup 1 ${XARGS:-};;
    stream_min) run $w --workload stream --steps 5 --warmup 1 ${XARGS:-};;
    stream_classic) run $w --workload stream --mode classic --prepare-every 1 --instances 4194304 --steps 5 --warmup 1 ${XARGS:-};;
    replay) run $w --workload replay --steps 10 --warmup 2 ${XARGS:-};;
    replay_dups) run $w --workload replay --replay-dups --steps 10 --warmup 2 ${XARGS:-};;
    step_keys1024) run $w --keys 1024 --kv-per-group 1024 --steps 10 --warmup 2 --no-cpu-baseline ${XARGS:-};;
    step_n7) run $w --replicas 7 --steps 10 --warmup 2 --no-cpu-baseline ${XARGS:-};;
    step_ipg512) run $w --ipg 512 --groups 32768 --steps 10 --warmup 2 --no-cpu-baseline ${XARGS:-};;
    step_strong) run $w --scaling strong --steps 20 --warmup 3 --no-cpu-baseline ${XARGS:-};;
  esac
done
