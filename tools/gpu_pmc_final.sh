#!/bin/bash
# GPU-box: FETCH/WRITE + SQ instruction passes for the kernels changed late in round 3, into
# gpurun_out/pmc_r03/traffic.json (seeded from profiles/traffic_r03.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r03
cp profiles/traffic_r03.json gpurun_out/pmc_r03/traffic.json
timeout -k 10 900 python tools/pmc_collect.py --out gpurun_out/pmc_r03/traffic.json "--workload log --log-format catchup" "--workload log --log-format durable" "--workload conflict" "--workload decode" "--workload stream" "--workload stream --mode classic --prepare-every 1 --instances 4194304" || exit $?
timeout -k 10 600 python tools/pmc_collect.py --out gpurun_out/pmc_r03/traffic.json --instr SQ_INSTS_VALU,SQ_INSTS_LDS "--workload decode" "--workload stream" "--workload stream --mode classic --prepare-every 1 --instances 4194304"
