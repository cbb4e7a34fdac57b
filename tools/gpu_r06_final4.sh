#!/bin/bash
# round 6: config lines + FETCH/WRITE passes of the padded-image stream and decode builds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06s4 WORKLOADS="stream_min stream_classic" bash tools/gpu_prof_configs.sh || exit $?
TAG=r06 TRAFFIC_SETS="--workload stream --steps 3 --warmup 1;--workload stream --mode classic --prepare-every 1 --instances 4194304 --steps 3 --warmup 1" INSTR_SETS="--workload stream --steps 3 --warmup 1" bash tools/gpu_counters.sh
