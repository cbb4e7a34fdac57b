#!/bin/bash
# GPU-box: FETCH/WRITE traffic passes (tools/pmc_collect.py) for the single-path workloads and
# SQ instruction passes for the issue-bound rows, into gpurun_out/pmc_r03/traffic.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r03
[ -f gpurun_out/pmc_r03/traffic.json ] || cp profiles/traffic_r03.json gpurun_out/pmc_r03/traffic.json
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 1000 python tools/pmc_collect.py --out gpurun_out/pmc_r03/traffic.json \
  "--workload apply --dist uniform" "--workload apply --dist zipf" "--workload conflict" \
  "--keys 1024 --kv-per-group 1024" "--workload prepare_min" "--workload replay" \
  "--workload log --log-format catchup" "--workload log --log-format durable"
else
timeout -k 10 1000 python tools/pmc_collect.py --out gpurun_out/pmc_r03/traffic.json \
  "--workload decode" "--workload stream" "--workload stream --mode classic --prepare-every 1 --instances 4194304" "--workload fanout" || exit $?
timeout -k 10 600 python tools/pmc_collect.py --out gpurun_out/pmc_r03/traffic.json --instr SQ_INSTS_VALU,SQ_INSTS_LDS \
  "--workload decode" "--workload stream" "--workload stream --mode classic --prepare-every 1 --instances 4194304" "--workload fanout"
fi
