#!/bin/bash
# GPU-box: apply parity tests on libmpx.so, then interleaved ms/step A/B of config-4 apply
# between LIBS (default libmpx_old.so = previous build, libmpx.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/apply_ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "apply or kat" --timeout 120 --timeout-method thread > gpurun_out/apply_ab/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/apply_ab/pytest.log; [ $rc -eq 0 ] || exit $rc
for d in ${DISTS:-uniform zipf}; do
  for rep in 1 2; do
    for lib in ${LIBS:-libmpx_old.so libmpx.so}; do
      r=$(MPX_LIB=$PWD/minpaxos_amd/$lib timeout -k 10 300 python bench.py --workload apply --dist $d --steps 5 --warmup 1 --no-cpu-baseline ${BARGS:-} 2>gpurun_out/apply_ab/err.log | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print('%.3f' % d['ms_per_step'], d['parity'])")
      rc=$?; [ $rc -eq 0 ] || { echo "bench $d $lib rc=$rc"; tail -5 gpurun_out/apply_ab/err.log; exit $rc; }
      echo "$d $lib $r"
    done
  done
done
