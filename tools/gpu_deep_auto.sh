#!/bin/bash
# automatic deep culling: full GPU suite, then bench_configs c3 / c5 / stress with the rule on and off (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=${1:-deep}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 0 1; do
  for a in 1 0; do
    DIRT_NO_CPU=1 DIRT_DEEP_CULL_AUTO=$a timeout -k 10 300 python3 tools/bench_configs.py c3_random c5_batch c3_stress > gpurun_out/${tag}_cfg_auto${a}_r${r}.jsonl 2>> gpurun_out/${tag}_cfg.err || exit $?
    echo "auto=$a round=$r"; python3 -c "
import json,sys
for l in open('gpurun_out/${tag}_cfg_auto${a}_r${r}.jsonl'):
    d=json.loads(l); print(d['config'], d['Mpixels_per_s_fwd_bwd'], d['kernels_us'])"
  done
done
