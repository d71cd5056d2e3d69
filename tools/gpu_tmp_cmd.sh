#!/bin/bash
# scratch GPU command: the G-buffer outputs over 5000 adversarial fuzz scenes
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/fuzz5; mkdir -p $out; cd $R
DIRT_GBUF_FUZZ_SEEDS=5000 timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_gbuffer_deferred.py -k adversarial_fuzz > $out/gbuf5000.log 2>&1
rc=$?; tail -4 $out/gbuf5000.log; exit $rc
