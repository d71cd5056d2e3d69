#!/bin/bash
# scratch GPU command: -m gpu suite with the default backward tile choice and with 16x16 forced, then c3 / c4 with
# the backward tile height forced to 16 and 8 (interleaved, 2 rounds)
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/th; mkdir -p $out; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $out/pytest_default.log 2>&1
rc=$?; tail -2 $out/pytest_default.log; [ $rc -eq 0 ] || exit $rc
DIRT_GRAD_TILE_H=16 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $out/pytest_th16.log 2>&1
rc=$?; tail -2 $out/pytest_th16.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for th in 16 8; do
  DIRT_GRAD_TILE_H=$th timeout -k 10 300 python3 tools/bench_configs.py c3_random c4_deferred20k > $out/cfg_th${th}_$rep.jsonl 2> $out/cfg_th${th}_$rep.err || { tail -3 $out/cfg_th${th}_$rep.err; exit 1; }
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['config'][:24], d.get('Mpixels_per_s_fwd_bwd'), d.get('kernels_us'))
" $out/cfg_th${th}_$rep.jsonl "th=$th#$rep"
done; done
