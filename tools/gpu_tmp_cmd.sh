#!/bin/bash
# scratch GPU command: fuzz seeds 40000..99999
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/fuzz3; mkdir -p $out; cd $R
DIRT_FUZZ_FIRST=40000 DIRT_FUZZ_SEEDS=100000 timeout -k 10 1000 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k fuzz > $out/fuzz_40k_100k.log 2>&1
rc=$?; tail -4 $out/fuzz_40k_100k.log; exit $rc
