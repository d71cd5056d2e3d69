#!/bin/bash
# Fuzz campaigns on the end-of-round build with seeds never run before: the full backward (50,000 adversarial
# scenes), the partial-gradient backward (5,000) and the recompute backward (5,000).
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
run() {  # name, env..., -- pytest -k expression, file
  local name=$1; shift
  timeout -k 10 540 env "$@" > $out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 $out/$name.log; return $rc
}
run fz_full_150k DIRT_FUZZ_FIRST=150000 DIRT_FUZZ_SEEDS=200000 python -u -m pytest tests/test_gpu_parity.py \
    -k test_fuzz_adversarial_scenes -q -x --timeout 300 --timeout-method thread || exit $?
run fz_gm DIRT_GM_FUZZ_FIRST=20000 DIRT_GM_FUZZ_SEEDS=25000 python -u -m pytest tests/test_gpu_parity.py \
    -k test_backward_partial_gradients_fuzz -q -x --timeout 300 --timeout-method thread || exit $?
run fz_rc DIRT_RC_FUZZ_FIRST=30000 DIRT_RC_FUZZ_SEEDS=35000 python -u -m pytest tests/test_gpu_recompute_bwd.py \
    -k test_recompute_fuzz_adversarial_scenes -q -x --timeout 300 --timeout-method thread
