#!/bin/bash
# round 6: price the resolve's phases (diagnostic ablations: no result stores, one list-walk step)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_rsabl PROF_LIBS="minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_rsabl2.so minpaxos_amd/ab/libmpx_rsabl4.so minpaxos_amd/ab/libmpx_rsabl6.so" DISTS=uniform bash tools/gpu_apply_ab.sh
