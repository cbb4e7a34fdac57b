#!/bin/bash
# one- vs two-launch group step, same box: the config-5 line at P=1 and the emulated P=8 share
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-step1}
mkdir -p $OUT
for rep in 1 2; do
  for sl in 1 2; do
    for emu in 0 8; do
      name=sl${sl}_emu${emu}_r$rep
      timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 10 --step-launches $sl --emulate-world $emu --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', 'step %.4f ms' % d['ms_per_step'], 'kernel %.4f ms' % r['kernel_ms_avg'], 'frac %.3f' % r['frac'], 'launches', r.get('launches_per_step'), 'parity', d['parity'].get('bit_exact', d['parity']))"
    done
  done
done
