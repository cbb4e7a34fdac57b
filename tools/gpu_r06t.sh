#!/bin/bash
# round 6: the replay rows after the chunk-sorted binned maximum: FETCH/WRITE passes merged into
# the counter database (a copy comes back as gpurun_out/r06_rp/traffic_r06.json), then the two
# config lines with their CPU baselines and kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06_rp; mkdir -p $OUT
timeout -k 10 500 python tools/pmc_collect.py --out $OUT/traffic_new.json "--workload replay" "--workload replay --replay-dups" > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 $OUT/pmc.log; [ $rc = 0 ] || exit $rc
python3 - <<'PY' || exit 1
import json
db = json.load(open("profiles/traffic_r06.json"))
new = json.load(open("gpurun_out/r06_rp/traffic_new.json"))["entries"]
keys = [e["key"] for e in new]
db["entries"] = [e for e in db["entries"] if e["key"] not in keys] + new
json.dump(db, open("profiles/traffic_r06.json", "w"), indent=1)
json.dump(db, open("gpurun_out/r06_rp/traffic_r06.json", "w"), indent=1)
for e in new: print(e["key"], e["bytes_per_launch"], e["ratio_to_alg"])
PY
TAG=r06_rp WORKLOADS="replay replay_dups" bash tools/gpu_prof_configs.sh
