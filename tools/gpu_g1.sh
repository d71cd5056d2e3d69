#!/bin/bash
# round-5 GPU session: the tests touched this round, then the bench (legs: recompute with the stash, api eager)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_batch_multigpu.py tests/test_gpu_lighting.py "tests/test_gpu_parity.py::test_r5_deviation_counters" "tests/test_gpu_parity.py::test_deep_cull_flag_bit_exact" "tests/test_gpu_parity.py::test_fused_small_scene_forward" tests/test_abi.py tests/test_gpu_recompute_bwd.py tests/test_gpu_gbuffer_deferred.py > gpurun_out/g1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g1_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 > gpurun_out/g1_bench.json 2> gpurun_out/g1_bench.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/g1_bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('gpurun_out/g1_bench.json'))
print('value', d['value'], 'kernels', d['kernels_us'])
for k,v in d['legs'].items(): print(k, {a:b for a,b in v.items() if a!='what'})
"
