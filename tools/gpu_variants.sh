#!/bin/bash
# Bench the product library and every build/variants/*.so (same bench, DIRT_MI355X_LIB override),
# interleaved over REPS rounds (A B A B ...) so that box drift hits every variant alike.
# usage: tools/gpu_variants.sh [REPS]
R=$GRAFT_REPO_ROOT
REPS=${1:-1}
mkdir -p $R/gpurun_out
for rep in $(seq 1 $REPS); do
for lib in $R/dirt_amd/libdirt_mi355x.so $R/build/variants/*.so; do
  n=$(basename $lib .so)
  DIRT_MI355X_LIB=$lib timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --rotate 0 --no-api-leg --no-recompute-leg > $R/gpurun_out/var_${n}_$rep.json 2> $R/gpurun_out/var_${n}_$rep.err
  rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -3 $R/gpurun_out/var_${n}_$rep.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-24s %8.1f Mpix/s  %s' % (sys.argv[2], d['value'], ' '.join('%s=%.1f'%(k[:6],v) for k,v in d['kernels_us'].items())))" $R/gpurun_out/var_${n}_$rep.json "$n#$rep"
done
done
