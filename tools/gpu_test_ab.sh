#!/bin/bash
# One GPU session for a kernel change: the whole -m gpu suite on the working tree (parity first), then the
# A/B of the product library against every build/variants/*.so (tools/gpu_variants.sh, REPS rounds).
# usage: tools/gpu_test_ab.sh tag [REPS]
tag=${1:-ab}; REPS=${2:-3}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_variants.sh $REPS
