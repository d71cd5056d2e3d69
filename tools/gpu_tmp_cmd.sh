#!/bin/bash
# scratch GPU command: hill (no depth test) over 3000 adversarial scenes
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/hill; mkdir -p $out; cd $R
DIRT_HILL_FUZZ_SEEDS=3000 timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_oceanic.py -k hill_adversarial > $out/hill3000.log 2>&1
rc=$?; tail -3 $out/hill3000.log; exit $rc
