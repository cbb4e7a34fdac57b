#!/bin/bash
# GPU-box: apply parity tests, then config-4 bench across apply chunk sizes (MPX_APPLY_CHUNK).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/apply_ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "apply or kat" --timeout 120 --timeout-method thread > gpurun_out/apply_ab/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/apply_ab/pytest.log; [ $rc -eq 0 ] || exit $rc
for d in ${DISTS:-uniform zipf}; do
  for c in ${CHUNKS:-1048576 2097152 4194304 8388608 67108864}; do
    MPX_APPLY_CHUNK=$c timeout -k 10 300 python bench.py --workload apply --dist $d --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/apply_ab/${d}_$c.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $d $c rc=$rc"; tail -5 gpurun_out/apply_ab/${d}_$c.log; exit $rc; }
    python - gpurun_out/apply_ab/${d}_$c.log $d $c <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l)
print(sys.argv[2], sys.argv[3], "ms/step %.3f" % d["ms_per_step"], "frac %.3f" % d["roofline"]["frac"], "parity", d.get("parity"))
PY
  done
done
