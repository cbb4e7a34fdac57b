set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r05_step1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "group_step or config5 or config1" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
for G in 65536 8192; do
  timeout -k 10 300 python tools/ab_step.py minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_pm.so --groups $G --kv 256 --totals --rounds 7 --iters 20 > $OUT/ab_step_$G.txt 2>&1
  rc=$?; echo "ab_step G=$G rc=$rc"; tail -2 $OUT/ab_step_$G.txt; [ $rc = 0 ] || exit $rc
done
for v in "" "--no-overlap"; do
  for lib in minpaxos_amd/libmpx.so minpaxos_amd/ab/libmpx_pm.so; do
    n=p8$(echo $v | tr -d ' -')_$(basename $lib .so)
    MPX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --emulate-world 8 --graph on --steps 64 --warmup 3 --no-cpu-baseline $v > $OUT/$n.log 2>&1
    rc=$?; [ $rc = 0 ] || { echo "$n rc=$rc"; exit $rc; }
    python3 -c "import json; d=[json.loads(l) for l in open('$OUT/$n.log') if l.startswith('{')][-1]; print('$n', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_median'],4))"
  done
done
