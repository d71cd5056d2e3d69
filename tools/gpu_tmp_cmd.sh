#!/bin/bash
# scratch GPU command: the fused small-scene fuzz widened to 20000 scenes
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/fuzz4; mkdir -p $out; cd $R
DIRT_FUSED_FUZZ_SEEDS=20000 timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k fused_small_scene_forward > $out/fused20000.log 2>&1
rc=$?; tail -4 $out/fused20000.log; exit $rc
