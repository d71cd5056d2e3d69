#!/bin/bash
# GPU suite, c3 A/B (product vs build/variants), config A/B (stress, clustered, c4), deferred chain.
tag=${1:-r04b}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $out/gpu_tests_$tag.log
ok_rc $rc || exit $rc
bash $R/tools/gpu_variants.sh 2 || exit $?
bash $R/tools/gpu_ab_configs.sh 2 stress clustered c4_ || exit $?
DIRT_NO_CPU=1 timeout -k 10 300 python3 $R/tools/bench_configs.py c4_deferred_chain > $out/chain_$tag.jsonl 2> $out/chain_$tag.err
rc=$?; echo "chain rc=$rc"; cat $out/chain_$tag.jsonl; tail -3 $out/chain_$tag.err
exit $rc
