#!/bin/bash
# One A/B call: the GPU parity suites on the product library, then the bench over the product and every
# build/variants/*.so interleaved (tools/gpu_variants.sh), then optionally the LDS PMC pass over the ablations.
#   tools/gpu_ab.sh TAG [REPS] [pmc]
tag=${1:-ab}; reps=${2:-3}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_recompute_bwd.py tests/test_gpu_gbuffer_deferred.py tests/test_gpu_rasterise_tests.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_variants.sh $reps || exit $?
if [ "$3" = "pmc" ]; then
  bash tools/gpu_pmc_ablate.sh $tag c3 > gpurun_out/pmc_ablate_$tag.txt 2>&1; echo "pmc rc=$?"
fi
exit 0
