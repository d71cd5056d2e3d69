#!/bin/bash
# Wide fresh-seed fuzz on the final build: 100,000 more adversarial scenes (two steps), 100,000 fused small
# scenes, 20,000 G-buffer scenes, 8,000 hill and 4,800 procedural-program scenes, 10,000 partial-gradient and
# 10,000 recompute-backward scenes -- every range past the ones run before.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
run() {  # name, then env assignments and the pytest command
  local name=$1; shift
  timeout -k 10 540 env "$@" > $out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 $out/$name.log; return $rc
}
P="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
run w_full_a DIRT_FUZZ_FIRST=200000 DIRT_FUZZ_SEEDS=250000 $P tests/test_gpu_parity.py -k test_fuzz_adversarial_scenes || exit $?
run w_full_b DIRT_FUZZ_FIRST=250000 DIRT_FUZZ_SEEDS=300000 $P tests/test_gpu_parity.py -k test_fuzz_adversarial_scenes || exit $?
run w_fused DIRT_FUSED_FUZZ_FIRST=20000 DIRT_FUSED_FUZZ_SEEDS=120000 $P tests/test_gpu_parity.py -k test_fused_small_scene_forward || exit $?
run w_gbuf DIRT_GBUF_FUZZ_FIRST=5000 DIRT_GBUF_FUZZ_SEEDS=25000 $P tests/test_gpu_gbuffer_deferred.py -k test_gbuffer_outputs_adversarial_fuzz || exit $?
run w_proc DIRT_HILL_FUZZ_FIRST=3000 DIRT_HILL_FUZZ_SEEDS=11000 DIRT_PROC_FUZZ_FIRST=1200 DIRT_PROC_FUZZ_SEEDS=6000 $P tests/test_gpu_oceanic.py -k fuzz || exit $?
run w_gm DIRT_GM_FUZZ_FIRST=25000 DIRT_GM_FUZZ_SEEDS=35000 $P tests/test_gpu_parity.py -k test_backward_partial_gradients_fuzz || exit $?
run w_rc DIRT_RC_FUZZ_FIRST=35000 DIRT_RC_FUZZ_SEEDS=45000 $P tests/test_gpu_recompute_bwd.py -k test_recompute_fuzz_adversarial_scenes
