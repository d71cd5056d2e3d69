#!/bin/bash
# round-5 first GPU session: the ADVICE r4 fixes' tests, then the steady-state per-frame kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch_multigpu.py tests/test_gpu_lighting.py "tests/test_gpu_parity.py::test_r5_deviation_counters" "tests/test_gpu_parity.py::test_deep_cull_flag_bit_exact" "tests/test_gpu_parity.py::test_fused_small_scene_forward" tests/test_abi.py > gpurun_out/g1_tests.log 2>&1
rc=$?; tail -5 gpurun_out/g1_tests.log; [ $rc -ne 0 ] && exit $rc
DIRT_NO_CPU=1 timeout -k 10 300 python3 tools/bench_configs.py c3_random c3x8 c5_batch > gpurun_out/g1_configs.jsonl 2> gpurun_out/g1_configs.err
