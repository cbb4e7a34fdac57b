#!/bin/bash
# round 6: the replay extended sweep (chunk-sorted binned maximum)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_fz3
MPX_FUZZ_EXT=${EXT:-400} timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz_ext.py -m gpu -x -q --timeout 300 --timeout-method thread -k replay > gpurun_out/r06_fz3/replay_ext_${EXT:-400}.log 2>&1
rc=$?; echo "ext rc=$rc"; tail -3 gpurun_out/r06_fz3/replay_ext_${EXT:-400}.log; exit $rc
