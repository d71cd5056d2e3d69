#!/bin/bash
# After the R5 sub-vertex clamp: the regression seed, the full GPU suite, then the fresh-seed fuzz campaigns.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests_clamp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/gpu_tests_clamp.log; [ $rc -eq 0 ] || exit $rc
bash $R/tools/gpu_fuzz_final.sh
