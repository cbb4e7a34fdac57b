#!/bin/bash
# GPU-box: rocprofv3 kernel stats of the config-4 apply pipeline at given chunk sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/apply_prof
mkdir -p $OUT
for d in ${DISTS:-uniform}; do
  for c in ${CHUNKS:-4194304 67108864}; do
    MPX_APPLY_CHUNK=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${d}_$c -o p -- python3 bench.py --workload apply --dist $d --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${d}_$c.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "prof $d $c rc=$rc"; exit $rc; }
    python3 - $OUT/${d}_$c/p_kernel_stats.csv $d $c <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
print("==", sys.argv[2], sys.argv[3])
for r in rows[:12]: print(f"{float(r['TotalDurationNs'])/1e6:8.2f}ms tot {float(r['AverageNs'])/1e3:9.1f}us x{r['Calls']:>5}  {r['Name'][:90]}")
PY
  done
done
