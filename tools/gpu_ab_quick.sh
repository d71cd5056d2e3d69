#!/bin/bash
# Quick A/B: parity core on the product library, c3 A/B (2 rounds) and selected configs (1 round).
# usage: tools/gpu_ab_quick.sh tag [config-substrings...]
tag=${1:-ab}; shift
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_recompute_bwd.py -m gpu -q -rf -x --timeout 300 --timeout-method thread > $out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/gpu_tests_$tag.log
ok_rc $rc || exit $rc
bash $R/tools/gpu_variants.sh 2 || exit $?
[ $# -gt 0 ] && { bash $R/tools/gpu_ab_configs.sh 1 "$@" || exit $?; }
exit 0
