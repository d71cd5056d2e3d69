#!/bin/bash
# GPU suite, then the deferred chain timed and under rocprofv3 kernel stats.  usage: tools/gpu_chain_prof.sh tag
tag=${1:-chain}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $out/gpu_tests_$tag.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
DIRT_NO_CPU=1 timeout -k 10 300 python3 $R/tools/bench_configs.py c4_deferred_chain > $out/chain_$tag.jsonl 2> $out/chain_$tag.err
rc=$?; echo "chain rc=$rc"; cat $out/chain_$tag.jsonl
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_chain_$tag -o run --output-format csv -- python3 $R/tools/bench_configs.py c4_deferred_chain > $out/prof_chain_$tag.log 2>&1
rc=$?; echo "rocprof chain rc=$rc"
exit $rc
