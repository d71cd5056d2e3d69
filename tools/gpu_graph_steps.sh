#!/bin/bash
R=$GRAFT_REPO_ROOT
for rep in 1 2 3; do
for gs in 10 50 100 200; do
for st in 20 200; do
  timeout -k 10 200 python3 $R/bench.py --steps $st --warmup 5 --graph-steps $gs --no-cpu-baseline > $R/gpurun_out/gs_${gs}_${st}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('gs %s steps %s rep %s: %.1f Mpix/s' % (sys.argv[2], sys.argv[3], sys.argv[4], d['value']))" $R/gpurun_out/gs_${gs}_${st}_$rep.json $gs $st $rep
done; done; done
