#!/bin/bash
# shared-vertex flush merge: full GPU suite (the auto rule puts every mesh test on the merged flush), then the
# interleaved A/B (tools/ab_merge.py)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=${1:-merge}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u tools/ab_merge.py ${2:-3} > gpurun_out/${tag}_ab.jsonl 2> gpurun_out/${tag}_ab.err
rc=$?; tail -c 2500 gpurun_out/${tag}_ab.jsonl; exit $rc
