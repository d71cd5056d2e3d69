#!/bin/bash
# Round-4 GPU session: full GPU suite on the product library, the parity core on each variant library,
# interleaved A/B of the variants, then the full bench.  Stops at the first GPU fault / timeout.
# usage: tools/gpu_r04.sh tag [reps]
tag=${1:-r04}
reps=${2:-3}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = ordinary test failure, anything else = stop
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $out/gpu_tests_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $out/gpu_tests_$tag.log
ok_rc $rc || exit $rc
for lib in $R/build/variants/*.so; do
  n=$(basename $lib .so)
  DIRT_MI355X_LIB=$lib DIRT_TORCH_EXT=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_recompute_bwd.py -m gpu -q -rf -x --timeout 300 --timeout-method thread > $out/gpu_tests_${tag}_$n.log 2>&1
  rc=$?; echo "variant $n pytest rc=$rc"; tail -3 $out/gpu_tests_${tag}_$n.log
  ok_rc $rc || exit $rc
done
bash $R/tools/gpu_variants.sh $reps || exit $?
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --cpu-budget 8 > $out/bench_$tag.json 2> $out/bench_$tag.err
rc=$?; echo "bench rc=$rc"; cat $out/bench_$tag.json; tail -3 $out/bench_$tag.err
exit $rc
