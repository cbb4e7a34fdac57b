#!/bin/bash
# GPU-box: apply tests (reduced) + replica-batch stamps and bench line, then the fused-totals
# A/B of the headline step (tools/ab_totals.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03b
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "apply or fused" --timeout 120 --timeout-method thread > gpurun_out/r03b/pt.log 2>&1
rc=$?; tail -2 gpurun_out/r03b/pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/stamp_small.py minpaxos_amd/ab/libmpx_sstamp.so --commands 5000 || exit $?
timeout -k 10 300 python bench.py --workload apply --commands 5000 --steps 200 --warmup 20 > gpurun_out/r03b/small.log 2>&1 || exit $?
grep '^{' gpurun_out/r03b/small.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('small', d['ms_per_step']*1e3, r['kernel_ms_avg']*1e3, d.get('host_call'), d['parity'])"
bash tools/ab_totals.sh
