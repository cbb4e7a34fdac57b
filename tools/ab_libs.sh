#!/bin/bash
# Same-box A/B of engine builds: for every library in $LIBS (space-separated paths; "main" =
# minpaxos_amd/libmpx.so) run bench.py $ARGS (';'-separated sets) and print ms/launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
IFS=';' read -ra SETS <<< "$ARGS"
for rep in 1 2; do
  for lib in $LIBS; do
    path=$lib; [ "$lib" = main ] && path=minpaxos_amd/libmpx.so
    j=0
    for args in "${SETS[@]}"; do
      j=$((j+1))
      name=$(basename $path .so)_${j}_r$rep
      MPX_LIB=$path timeout -k 10 300 python bench.py $args --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err
      rc=$?
      [ $rc = 0 ] || { echo "$name rc=$rc"; tail -5 $OUT/$name.err; exit $rc; }
      python3 -c "import json,sys; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', '%.4f ms' % r['kernel_ms_avg'], 'step %.4f ms' % d['ms_per_step'], 'frac %s' % (r['frac'] if r['frac'] is None else round(r['frac'], 3)), 'exact', d['parity']['bit_exact'])"
    done
  done
done
