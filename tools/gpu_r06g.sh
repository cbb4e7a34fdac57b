#!/bin/bash
# round 6: per-workgroup spans of the group step at the P = 8 per-rank shape (and P = 1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_span
timeout -k 10 300 python tools/stamp_span.py --groups 8192 --json gpurun_out/r06_span/p8.json > gpurun_out/r06_span/p8.log 2>&1; rc=$?; echo "p8 rc=$rc"; tail -2 gpurun_out/r06_span/p8.log | cut -c1-1500; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/stamp_span.py --groups 65536 --reps 2 --json gpurun_out/r06_span/p1.json > gpurun_out/r06_span/p1.log 2>&1; rc=$?; echo "p1 rc=$rc"; tail -1 gpurun_out/r06_span/p1.log | cut -c1-600
