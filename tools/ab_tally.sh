#!/bin/bash
# GPU-box: interleaved A/B of bench.py kernel timings between libmpx_nt0.so (default access
# policy) and libmpx.so; WORKLOADS lists bench.py --workload argument strings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS=';' read -ra WL <<< "${WORKLOADS:-tally --mode min;tally --mode classic;prepare}"
for w in "${WL[@]}"; do
  for rep in 1 2; do
    for lib in ${LIBS:-libmpx_nt0.so libmpx.so}; do
      r=$(MPX_LIB=$PWD/minpaxos_amd/$lib timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print('%.4f' % d['roofline']['kernel_ms_avg'], d['parity']['bit_exact'])")
      echo "$w $lib $r"
    done
  done
done
