#!/bin/bash
# Quick GPU iteration: parity tests (optionally filtered) + bench without CPU baseline.
# usage: tools/gpu_quick.sh tag [pytest -k expr]
tag=${1:-q}
out=gpurun_out; mkdir -p $out
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ -n "$2" ]; then K="-k $2"; else K=""; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread $K > $out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 $out/gpu_tests_$tag.log
[ $rc -eq 1 ] && echo "!!!!!!!! GPU TESTS FAILED !!!!!!!!"
ok_rc $rc || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $out/bench_$tag.json 2> $out/bench_$tag.err
rc=$?; echo "bench rc=$rc"; cat $out/bench_$tag.json; tail -5 $out/bench_$tag.err
exit $rc
