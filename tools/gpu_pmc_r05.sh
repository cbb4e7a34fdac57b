#!/bin/bash
# GPU-box: FETCH_SIZE / WRITE_SIZE passes (tools/pmc_collect.py) for the configurations whose
# kernels changed in round 5, into gpurun_out/pmc_r05/traffic.json, seeded from the tracked
# profiles/traffic_r05.json (gpurun_out/ does not travel to the box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r05
cp profiles/traffic_r05.json gpurun_out/pmc_r05/traffic.json
timeout -k 10 1000 python tools/pmc_collect.py --out gpurun_out/pmc_r05/traffic.json "$@"
