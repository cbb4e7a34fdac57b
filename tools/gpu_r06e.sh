#!/bin/bash
# round 6: tally tile / occupancy A/B; FETCH/WRITE passes + kernel stats of the rebuilt apply and
# conflict kernels (into gpurun_out/pmc_r06/traffic.json, seeded from profiles/traffic_r06.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_tally LIBS="main minpaxos_amd/ab/libmpx_t512.so minpaxos_amd/ab/libmpx_t512w5.so minpaxos_amd/ab/libmpx_t1024w5.so" ARGS="--workload tally --mode min --steps 20 --warmup 3;--workload tally --mode classic --steps 20 --warmup 3" bash tools/gpu_ab.sh || exit $?
mkdir -p gpurun_out/pmc_r06
cp profiles/traffic_r06.json gpurun_out/pmc_r06/traffic.json
timeout -k 10 900 python tools/pmc_collect.py --out gpurun_out/pmc_r06/traffic.json "--workload apply --dist uniform" "--workload apply --dist zipf" "--workload conflict" || exit $?
TAG=r06 WORKLOADS="apply_uniform apply_zipf conflict" bash tools/gpu_prof_configs.sh
