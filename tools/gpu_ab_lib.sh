#!/bin/bash
# A/B of a variant library against the product on bench_configs configs, interleaved rounds.
# usage: tools/gpu_ab_lib.sh tag variant_name rounds config-substrings...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=$1; var=$2; rounds=$3; shift 3
for r in $(seq 1 $rounds); do
  for lib in product $var; do
    if [ $lib = product ]; then L=$GRAFT_REPO_ROOT/dirt_amd/libdirt_mi355x.so; else L=$GRAFT_REPO_ROOT/build/variants/$lib.so; fi
    DIRT_NO_CPU=1 DIRT_MI355X_LIB=$L timeout -k 10 300 python3 tools/bench_configs.py "$@" > gpurun_out/${tag}_${lib}_r$r.jsonl 2>> gpurun_out/${tag}.err || exit $?
    echo "== $lib round $r"; python3 -c "
import json
for l in open('gpurun_out/${tag}_${lib}_r$r.jsonl'):
    d=json.loads(l); print(d['config'][:40], d.get('Mpixels_per_s_fwd_bwd'), d.get('kernels_us'), d.get('ms_per_step_graph'))"
  done
done
