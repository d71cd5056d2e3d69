#!/bin/bash
# scratch GPU command: widened parity sweeps on the current tree (5000 fuzz scenes, frame-size sweep, dense tiles)
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/sweep; mkdir -p $out; cd $R
DIRT_FUZZ_SEEDS=5000 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k fuzz > $out/fuzz5000.log 2>&1
rc=$?; tail -2 $out/fuzz5000.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/debug/size_sweep.py > $out/size_sweep.txt 2>&1 || { tail -5 $out/size_sweep.txt; exit 1; }
tail -3 $out/size_sweep.txt
timeout -k 10 300 python3 tools/debug/dense_tiles.py > $out/dense_tiles.txt 2>&1 || { tail -5 $out/dense_tiles.txt; exit 1; }
tail -3 $out/dense_tiles.txt
