#!/bin/bash
# apply (config 4): new partitioned pipeline, uniform + zipf, the sort-based fallback beside it,
# then rocprofv3 kernel stats of the uniform run
set -e
cd /root/repo
mkdir -p gpurun_out/apply
export TMPDIR=/tmp
for d in ${DISTS:-uniform zipf}; do
  timeout -k 10 300 python bench.py --workload apply --dist $d --steps 10 --warmup 3 > gpurun_out/apply/bench_$d.json 2> gpurun_out/apply/bench_$d.err
  tail -1 gpurun_out/apply/bench_$d.json | cut -c1-330
done
[ -n "$FB" ] && MPX_APPLY_FALLBACK=1 timeout -k 10 300 python bench.py --workload apply --dist uniform --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/apply/bench_uniform_fallback.json 2> gpurun_out/apply/fb.err || true
[ -n "$FB" ] && tail -1 gpurun_out/apply/bench_uniform_fallback.json || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/apply/prof_u -o run -- python bench.py --workload apply --dist uniform --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/apply/prof_u.log 2>&1
find gpurun_out/apply/prof_u -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/apply/uniform_kernel_stats.csv
python3 tools/kstats.py gpurun_out/apply/uniform_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/apply/prof_z -o run -- python bench.py --workload apply --dist zipf --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/apply/prof_z.log 2>&1
find gpurun_out/apply/prof_z -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/apply/zipf_kernel_stats.csv
python3 tools/kstats.py gpurun_out/apply/zipf_kernel_stats.csv
if [ -n "$CAP1" ]; then
  timeout -k 10 300 python bench.py --workload apply --dist uniform --steps 10 --warmup 3 --no-cpu-baseline --kv-capacity 1048576 > gpurun_out/apply/bench_uniform_cap1m.json 2>&1
  tail -1 gpurun_out/apply/bench_uniform_cap1m.json | cut -c1-330
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/apply/prof_u1 -o run -- python bench.py --workload apply --dist uniform --steps 5 --warmup 2 --no-cpu-baseline --kv-capacity 1048576 > gpurun_out/apply/prof_u1.log 2>&1
  python3 tools/kstats.py gpurun_out/apply/prof_u1/run_kernel_stats.csv
fi
