#!/bin/bash
# A/B of an environment knob (read at call time) on bench_configs configs, interleaved rounds, one process per run.
# usage: tools/gpu_ab_env.sh tag VAR "val_a val_b" rounds config-substrings...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=$1; var=$2; vals=$3; rounds=$4; shift 4
for r in $(seq 1 $rounds); do
  for v in $vals; do
    env DIRT_NO_CPU=1 $var=$v timeout -k 10 300 python3 tools/bench_configs.py "$@" > gpurun_out/${tag}_${v}_r$r.jsonl 2>> gpurun_out/${tag}.err || exit $?
    echo "== $var=$v round $r"; python3 -c "
import json
for l in open('gpurun_out/${tag}_${v}_r$r.jsonl'):
    d=json.loads(l); print(d['config'][:40], d.get('Mpixels_per_s_fwd_bwd'), d.get('kernels_us'), d.get('ms_per_step_graph'))"
  done
done
