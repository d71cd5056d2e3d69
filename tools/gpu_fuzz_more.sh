#!/bin/bash
# More fresh ranges on the final tree: 50,000 adversarial scenes and 66,000 near-w0 scenes.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
timeout -k 10 540 env DIRT_FUZZ_FIRST=300000 DIRT_FUZZ_SEEDS=350000 python -u -m pytest -q -x --timeout 300 \
    --timeout-method thread tests/test_gpu_parity.py -k test_fuzz_adversarial_scenes > $out/m_full.log 2>&1
rc=$?; echo "m_full rc=$rc"; tail -1 $out/m_full.log; [ $rc -eq 0 ] || exit $rc
DIRT_W0_A=0 DIRT_W0_B=116000 DIRT_W0_N=16000 bash $R/tools/gpu_fuzz_w0.sh || exit $?
DIRT_W0_A=132000 DIRT_W0_B=166000 DIRT_W0_N=34000 bash $R/tools/gpu_fuzz_w0.sh
