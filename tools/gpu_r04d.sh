#!/bin/bash
# GPU suite, stress rows with / without deep cull, the deferred chain under rocprof, the bench.
tag=${1:-r04d}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $out/gpu_tests_$tag.log
ok_rc $rc || exit $rc
DIRT_NO_CPU=1 timeout -k 10 300 python3 $R/tools/bench_configs.py stress c4_deferred20k > $out/configs_$tag.jsonl 2> $out/configs_$tag.err
rc=$?; echo "configs rc=$rc"; cut -c1-300 $out/configs_$tag.jsonl
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
DIRT_NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_chain_$tag -o run --output-format csv -- python3 $R/tools/bench_configs.py c4_deferred_chain > $out/prof_chain_$tag.log 2>&1
rc=$?; echo "rocprof chain rc=$rc"; tail -3 $out/prof_chain_$tag.log
[ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --cpu-budget 8 > $out/bench_$tag.json 2> $out/bench_$tag.err
rc=$?; echo "bench rc=$rc"; cut -c1-1500 $out/bench_$tag.json; tail -3 $out/bench_$tag.err
exit $rc
