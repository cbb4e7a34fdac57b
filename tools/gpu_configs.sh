#!/bin/bash
# GPU-box run of the single-kernel configurations (BASELINE configs 2-4) through bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/configs_${TAG:-r01}
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -k 10 ${BT:-400} python bench.py "$@" > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log
  case $rc in 0) ;; *) exit $rc;; esac
}
run tally_min --workload tally --mode min --steps 10 --warmup 2 ${XARGS:-}
run tally_classic --workload tally --mode classic --steps 10 --warmup 2 ${XARGS:-}
run prepare --workload prepare --steps 10 --warmup 2 ${XARGS:-}
run apply_uniform --workload apply --dist uniform --steps 5 --warmup 1 ${XARGS:-}
run apply_zipf --workload apply --dist zipf --steps 5 --warmup 1 ${XARGS:-}
