#!/bin/bash
# GPU-box: k_ap_resolve per-phase stamps (MPX_RS_STAMP builds in LIBS) on config-4 apply
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/stamp
for d in ${DISTS:-uniform}; do
  for lib in ${LIBS:-libmpx_oldst.so libmpx_newst.so}; do
    MPX_LIB=$PWD/minpaxos_amd/$lib timeout -k 10 300 python bench.py --workload apply --dist $d --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/stamp/${d}_$lib.log 2>&1
    rc=$?; echo "== $d $lib rc=$rc"; grep RS_STAMP gpurun_out/stamp/${d}_$lib.log | tail -2; [ $rc -eq 0 ] || exit $rc
  done
done
