#!/bin/bash
# GPU-box run: group-step variants that leave the fast path (general kernel), and the kernel
# benches of rows without a line yet (MIN prepare, ConflictBatch). One JSON line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/variants_${TAG:-r02}
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -k 10 ${BT:-300} python bench.py "$@" > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300
  grep -o '"kernel_ms_avg": [0-9.]*\|"frac": [0-9.]*\|"bit_exact": [a-z]*' $OUT/$name.log | tr '\n' ' '; echo
  case $rc in 0) ;; *) exit $rc;; esac
}
run step_keys1024 --keys 1024 --kv-per-group 1024 --steps 10 --warmup 2 --no-cpu-baseline ${XARGS:-}
run step_n7 --replicas 7 --steps 10 --warmup 2 --no-cpu-baseline ${XARGS:-}
run step_ipg512 --ipg 512 --groups 32768 --steps 10 --warmup 2 --no-cpu-baseline ${XARGS:-}
run prepare_min --workload prepare_min --steps 10 --warmup 2 ${XARGS:-}
run conflict --workload conflict --steps 5 --warmup 1 ${XARGS:-}
if [ "${PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  for v in "keys1024 --keys 1024 --kv-per-group 1024" "n7 --replicas 7" "ipg512 --ipg 512 --groups 32768"; do
    set -- $v; n=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o trace -- python3 bench.py "$@" --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_$n.log 2>&1
    rc=$?; echo "prof $n rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  done
fi
