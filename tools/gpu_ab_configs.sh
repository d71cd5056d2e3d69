#!/bin/bash
# A/B of the product library and every build/variants/*.so on selected bench_configs configs.
# usage: tools/gpu_ab_configs.sh REPS config-substring...
R=$GRAFT_REPO_ROOT
REPS=$1; shift
mkdir -p $R/gpurun_out
for rep in $(seq 1 $REPS); do
for lib in $R/dirt_amd/libdirt_mi355x.so $R/build/variants/*.so; do
  n=$(basename $lib .so)
  DIRT_NO_CPU=1 DIRT_MI355X_LIB=$lib timeout -k 10 300 python3 $R/tools/bench_configs.py "$@" > $R/gpurun_out/abc_${n}_$rep.jsonl 2> $R/gpurun_out/abc_${n}_$rep.err
  rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -3 $R/gpurun_out/abc_${n}_$rep.err; exit $rc; }
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print('%-20s %-34s %8.1f Mpix/s  %s' % (sys.argv[2], d['config'], d['Mpixels_per_s_fwd_bwd'], ' '.join('%s=%.1f'%(k[:6],v) for k,v in d['kernels_us'].items())))" $R/gpurun_out/abc_${n}_$rep.jsonl "$n#$rep"
done
done
