#!/bin/bash
# resolve ablations: kernel stats of the config-4 uniform apply with each variant library
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for v in main ${VARIANTS:-a1 a2 a5}; do
  lib=minpaxos_amd/libmpx.so; [ $v != main ] && lib=minpaxos_amd/ab/libmpx_$v.so
  MPX_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/$v -o run -- python bench.py --workload apply --dist ${DIST:-uniform} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abl/$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/abl/$v.log; exit 1; }
  echo "== $v"; grep '^{' gpurun_out/abl/$v.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['parity'])"
  python3 tools/kstats.py gpurun_out/abl/$v/run_kernel_stats.csv | grep "k_ap_"
done
