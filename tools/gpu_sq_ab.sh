#!/bin/bash
# SQ counter passes for each given engine build, driving tools/ab_step.py (one lib per run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sqab
mkdir -p $OUT
for lib in "$@"; do
  n=$(basename $lib .so)
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
             "SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex group_fast --output-format csv -d $OUT/${n}_p$i -o pmc -- python3 tools/ab_step.py $lib --rounds 1 --iters 2 > $OUT/${n}_p$i.log 2>&1
    rc=$?; echo "$n pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/${n}_p$i.log; exit $rc; }
  done
done
