set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=ab_ovr LIBS="main minpaxos_amd/ab/libmpx_ovr.so" ARGS="--workload tally --mode min --steps 10 --warmup 2;--workload tally --mode classic --steps 10 --warmup 2;--workload prepare --steps 10 --warmup 2" timeout -k 10 400 bash tools/ab_libs.sh > gpurun_out/ab_ovr.txt 2>&1
rc=$?; cat gpurun_out/ab_ovr.txt; [ $rc = 0 ] || exit $rc
MPX_LIB=minpaxos_amd/ab/libmpx_ovr.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tally or prepare or accept" > gpurun_out/t_ovr.log 2>&1
rc=$?; tail -2 gpurun_out/t_ovr.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/pmc_sq.py --out gpurun_out/sq_r04/tally.json --match k_accept_tile "--workload tally --mode min --steps 3 --warmup 1" > gpurun_out/sq_tally.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc = 0 ] || exit $rc
TAG=r04 BT=300 WORKLOADS='fanout log_catchup log_durable replay replay_dups step_keys1024 step_n7 step_ipg512 step_strong' bash tools/gpu_prof_configs.sh
rc=$?; [ $rc = 0 ] || exit $rc
cp profiles/traffic_r04.json gpurun_out/pmc_r04_replay.json && timeout -k 10 300 python tools/pmc_collect.py --out gpurun_out/pmc_r04_replay.json "--workload replay" "--workload replay --replay-dups" > gpurun_out/pmc_replay.log 2>&1
rc=$?; echo "pmc replay rc=$rc"; tail -2 gpurun_out/pmc_replay.log | cut -c1-200; exit $rc
