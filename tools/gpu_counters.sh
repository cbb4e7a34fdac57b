#!/bin/bash
# GPU-box: the counter database's passes for one round into gpurun_out/pmc_${TAG}/traffic.json
# (seeded from profiles/traffic_${TAG}.json): FETCH/WRITE passes for $TRAFFIC_SETS, then one SQ
# pass (8 SQ + 1 GRBM counters, within one pass's limits) for $INSTR_SETS. Sets are ';'-separated
# bench.py argument strings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r04}; OUT=gpurun_out/pmc_$T; mkdir -p $OUT
cp profiles/traffic_$T.json $OUT/traffic.json
IFS=';' read -ra TS <<< "${TRAFFIC_SETS:-}"
IFS=';' read -ra IS <<< "${INSTR_SETS:-}"
if [ ${#TS[@]} -gt 0 ]; then
  timeout -k 10 ${TT:-600} python tools/pmc_collect.py --out $OUT/traffic.json "${TS[@]}" > $OUT/traffic.log 2>&1
  rc=$?; echo "traffic rc=$rc"; tail -3 $OUT/traffic.log | cut -c1-300; [ $rc = 0 ] || exit $rc
fi
if [ ${#IS[@]} -gt 0 ]; then
  timeout -k 10 ${TI:-500} python tools/pmc_collect.py --out $OUT/traffic.json \
    --instr "SQ_WAVES+SQ_WAVE_CYCLES+SQ_WAIT_ANY+SQ_WAIT_INST_ANY+SQ_ACTIVE_INST_ANY+SQ_INSTS_VALU+SQ_INSTS_LDS+SQ_BUSY_CYCLES+GRBM_GUI_ACTIVE" \
    "${IS[@]}" > $OUT/instr.log 2>&1
  rc=$?; echo "instr rc=$rc"; tail -4 $OUT/instr.log | cut -c1-400; [ $rc = 0 ] || exit $rc
fi
