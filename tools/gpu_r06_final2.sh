#!/bin/bash
# round 6 closing evidence, part 2: kernel stats + lines of the rebuilt rows and the step, and an
# SQ pass of the rebuilt apply kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06final WORKLOADS="apply_uniform apply_zipf conflict step_strong" bash tools/gpu_prof_configs.sh || exit $?
mkdir -p gpurun_out/sq_r06
timeout -k 10 600 python tools/pmc_sq.py --out gpurun_out/sq_r06/apply_uniform.json --match k_ap_ "--workload apply --dist uniform --steps 3 --warmup 1"
rc=$?; echo "sq rc=$rc"; exit $rc
