#!/bin/bash
# The driver's bench command (--steps 20 --warmup 5) with and without the untimed clock warm-up, against
# the default 200-step run, interleaved on one box.  usage: tools/gpu_driver_flags.sh [REPS]
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/drv; mkdir -p $out
REPS=${1:-3}
for k in $(seq 1 $REPS); do
  timeout -k 10 200 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --min-warm-ms 0 --no-cpu-baseline --rotate 0 --no-api-leg > $out/k20_nowarm_$k.json 2> $out/k20_nowarm_$k.err || exit 1
  timeout -k 10 200 python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --rotate 0 --no-api-leg > $out/k20_$k.json 2> $out/k20_$k.err || exit 1
  timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --rotate 0 --no-api-leg > $out/k200_$k.json 2> $out/k200_$k.err || exit 1
done
for f in $out/k*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], d.get('clock_warm'), d['kernels_us'])" $f; done
