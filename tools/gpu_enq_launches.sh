#!/bin/bash
# Enqueued (no graph) group step at emulated P ranks: one vs two launches per step, twice each
# (the multi-process line has no graph; which form is faster there?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-enq_launches}
mkdir -p $OUT
for rep in 1 2; do
  for P in ${PS:-8 4 2}; do
    for L in 2 1; do
      name=P${P}_L${L}_r$rep
      timeout -k 10 300 python bench.py --emulate-world $P --graph off --step-launches $L --steps 200 --warmup 20 --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err
      rc=$?; [ $rc = 0 ] || { echo "$name rc=$rc"; tail -5 $OUT/$name.err; exit $rc; }
      python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', 'step %.4f ms' % d['ms_per_step'], 'kernel %.4f' % r['kernel_ms_median'], 'launches', r['launches_per_step'], 'enq %.4f' % d['enqueue_ms_per_step'])"
    done
  done
done
