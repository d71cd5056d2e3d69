#!/bin/bash
# Bench the product library and every build/variants/*.so (same bench, DIRT_MI355X_LIB override).
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for lib in $R/dirt_amd/libdirt_mi355x.so $R/build/variants/*.so; do
  n=$(basename $lib .so)
  DIRT_MI355X_LIB=$lib timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/var_$n.json 2> $R/gpurun_out/var_$n.err
  rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -3 $R/gpurun_out/var_$n.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-24s %8.1f Mpix/s  %s' % (sys.argv[2], d['value'], ' '.join('%s=%.1f'%(k[:6],v) for k,v in d['kernels_us'].items())))" $R/gpurun_out/var_$n.json $n
done
