#!/bin/bash
# GPU-box: FETCH_SIZE and WRITE_SIZE passes (separate runs) over the config-4 apply, per kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/apply_pmc_${DIST:-uniform}
mkdir -p $OUT
A="--workload apply --dist ${DIST:-uniform} --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- python3 bench.py $A > $OUT/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- python3 bench.py $A > $OUT/write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc = 0 ] || exit $rc
python3 tools/apply_pmc.py $OUT
