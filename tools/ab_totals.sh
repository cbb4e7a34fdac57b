#!/bin/bash
# GPU-box: interleaved A/B of the headline step, totals fused into the step kernels vs their own
# launch (bench.py --separate-totals), same library and box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_totals
for rep in 1 2 3; do
  for v in fused separate; do
    x=""; [ $v = separate ] && x="--separate-totals"
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $x ${BARGS:-} > gpurun_out/ab_totals/${v}_$rep.log 2>&1 || exit $?
    grep '^{' gpurun_out/ab_totals/${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', '%.4f ms/step  kernel avg %.4f min %.4f  decided %d' % (d['ms_per_step'], r['kernel_ms_avg'], r['kernel_ms_min'], d['decided_instances_per_step']))"
  done
done
