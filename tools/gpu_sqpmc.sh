#!/bin/bash
# GPU-box run: one rocprofv3 SQ counter pass (C="SQ_A SQ_B ...", at most 8 SQ counters) over a
# bench.py command line (A="..."), summarised per kernel into gpurun_out/sq_${TAG}/summary.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sq_${TAG:-x}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc -o pmc -- python3 bench.py $A > $OUT/run.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc = 0 ] || { tail -5 $OUT/run.log; exit $rc; }
python3 - $OUT <<'PY' > $OUT/summary.txt
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
cat $OUT/summary.txt
