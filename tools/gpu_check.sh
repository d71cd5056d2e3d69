#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace profile.  Stops at the first GPU fault/timeout.
# usage: tools/gpu_check.sh [tag]
tag=${1:-r01}
out=gpurun_out
mkdir -p $out
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = ordinary test failure, anything else = stop
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > $out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 $out/gpu_tests_$tag.log
ok_rc $rc || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-budget 8 > $out/bench_$tag.json 2> $out/bench_$tag.err
rc=$?; echo "bench rc=$rc"; cat $out/bench_$tag.json; tail -5 $out/bench_$tag.err
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_$tag -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-graph --rotate 0 --no-api-leg > $GRAFT_REPO_ROOT/$out/prof_$tag.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -5 $GRAFT_REPO_ROOT/$out/prof_$tag.log
exit $rc
