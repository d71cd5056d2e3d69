#!/bin/bash
# scratch GPU command: 20000 fuzz scenes + the full-size scenes against a 10x tighter gradient tolerance (measurement)
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/tight; mkdir -p $out; cd $R
DIRT_GRAD_RTOL=1e-5 DIRT_GRAD_ATOL_REL=1e-6 DIRT_FUZZ_SEEDS=20000 DIRT_FULL_SEEDS=8 timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fuzz_adversarial or full_size" > $out/tight.log 2>&1
rc=$?; tail -3 $out/tight.log; grep -c FAILED $out/tight.log; exit 0
