#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/share
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_shared_geometry.py -x -q --timeout 120 --timeout-method thread > gpurun_out/share/tests_new.log 2>&1
rc=$?; tail -3 gpurun_out/share/tests_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/share/tests_all.log 2>&1
rc=$?; tail -3 gpurun_out/share/tests_all.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for sh in 1 0; do
    DIRT_NO_CPU=1 DIRT_SHARE_GEOMETRY=$sh timeout -k 10 300 python3 tools/bench_configs.py c4 > gpurun_out/share/chain_share${sh}_r$r.jsonl 2>gpurun_out/share/chain_share${sh}_r$r.err || { echo "bench_configs rc=$?"; tail -3 gpurun_out/share/chain_share${sh}_r$r.err; exit 1; }
    echo "share=$sh round $r"; python3 -c "
import json
for l in open('gpurun_out/share/chain_share${sh}_r$r.jsonl'):
    d=json.loads(l); print('  ', d['config'][:60], d.get('Mpixels_per_s_fwd_bwd'), d.get('ms_per_step_graph'), d.get('ms_per_step_eager'))"
  done
done
