#!/bin/bash
# Round-4 fuzz campaigns on the final kernels: fused small scenes, hill, procedural programs, full-size c3 seeds.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out; mkdir -p $out
DIRT_FUSED_FUZZ_SEEDS=20000 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k test_fused_small_scene_forward -q -x --timeout 300 --timeout-method thread > $out/fz_fused.log 2>&1
rc=$?; echo "fused rc=$rc"; tail -1 $out/fz_fused.log; [ $rc -eq 0 ] || exit $rc
DIRT_HILL_FUZZ_SEEDS=3000 DIRT_PROC_FUZZ_SEEDS=1200 timeout -k 10 600 python -u -m pytest tests/test_gpu_oceanic.py -k fuzz -q -x --timeout 300 --timeout-method thread > $out/fz_proc.log 2>&1
rc=$?; echo "procedural rc=$rc"; tail -1 $out/fz_proc.log; [ $rc -eq 0 ] || exit $rc
DIRT_FULL_SEEDS=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k test_full_size_c3_more_seeds -q -x --timeout 300 --timeout-method thread > $out/fz_full.log 2>&1
rc=$?; echo "full-size rc=$rc"; tail -1 $out/fz_full.log; exit $rc
