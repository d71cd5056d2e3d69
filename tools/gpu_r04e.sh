#!/bin/bash
# Round-end evidence: GPU suite, deferred chain (eager / graph / profiled), bench (default and the driver's
# command), bench under rocprofv3 kernel stats, HBM traffic passes.
tag=${1:-r04e}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $out/gpu_tests_$tag.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$tag.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $out/smoke_$tag.log
[ $rc -eq 0 ] || exit $rc
DIRT_NO_CPU=1 timeout -k 10 300 python3 $R/tools/bench_configs.py c4_deferred_chain > $out/chain_$tag.jsonl 2> $out/chain_$tag.err
rc=$?; echo "chain rc=$rc"; cat $out/chain_$tag.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $out/bench_default_$tag.json 2> $out/bench_default_$tag.err
rc=$?; echo "bench default rc=$rc"; cut -c1-700 $out/bench_default_$tag.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench_driver_$tag.json 2> $out/bench_driver_$tag.err
rc=$?; echo "bench driver rc=$rc"; cut -c1-400 $out/bench_driver_$tag.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_bench_$tag -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $out/prof_bench_$tag.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; tail -c 600 $out/prof_bench_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_chain_$tag -o run --output-format csv -- python3 $R/tools/bench_configs.py c4_deferred_chain > $out/prof_chain_$tag.log 2>&1
rc=$?; echo "rocprof chain rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R
bash tools/gpu_traffic.sh $tag
