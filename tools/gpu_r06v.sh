#!/bin/bash
# round 6: replay with 4-byte instNos from the record pass (the sort reads 4 B per record):
# parity, 100 sweep seeds, A/B against the 8-byte-pair build (ab/libmpx_rphead.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
EXT=400 bash tools/gpu_r06u.sh || exit $?
TAG=${T2:-r06_replay2} OLD=${OLD:-minpaxos_amd/ab/libmpx_rphead.so} bash tools/gpu_r06s.sh
