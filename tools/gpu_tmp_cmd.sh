#!/bin/bash
# scratch GPU command: config 3 at full size over 8 seeds x {affine, perspective}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
DIRT_FULL_SEEDS=8 timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "full_size" > gpurun_out/full_seeds.log 2>&1; rc=$?; tail -20 gpurun_out/full_seeds.log; exit $rc
