#!/bin/bash
# After the R5 vertex cap: the GPU suite, then 100,000 near-w0 clipping scenes.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests_cap.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/gpu_tests_cap.log; [ $rc -eq 0 ] || exit $rc
DIRT_W0_A=16000 DIRT_W0_B=66000 DIRT_W0_N=50000 bash $R/tools/gpu_fuzz_w0.sh
