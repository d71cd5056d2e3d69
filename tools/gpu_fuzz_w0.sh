#!/bin/bash
# Clipping stress around w = 0 (scenes.near_w0_scene): scenes in two steps (DIRT_W0_A, DIRT_W0_B: first seeds, default 0 and 8000; N each, default 8000).
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
P="python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k test_fuzz_near_w0_clipping"
timeout -k 10 540 env DIRT_W0_FUZZ_FIRST=${A:=${DIRT_W0_A:-0}} DIRT_W0_FUZZ_SEEDS=$((A + ${DIRT_W0_N:-8000})) $P > $out/w0_a.log 2>&1
rc=$?; echo "w0_a rc=$rc"; tail -1 $out/w0_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 540 env DIRT_W0_FUZZ_FIRST=${B:=${DIRT_W0_B:-8000}} DIRT_W0_FUZZ_SEEDS=$((B + ${DIRT_W0_N:-8000})) $P > $out/w0_b.log 2>&1
rc=$?; echo "w0_b rc=$rc"; tail -1 $out/w0_b.log; exit $rc
