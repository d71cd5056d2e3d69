#!/bin/bash
# round-5 first GPU session: the ADVICE r4 fixes' tests, the persistent backward's parity, then an A/B of
# the persistent backward (DIRT_GRAD_PERSIST workgroups per CU) against the product grid
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_batch_multigpu.py tests/test_gpu_lighting.py "tests/test_gpu_parity.py::test_r5_deviation_counters" "tests/test_gpu_parity.py::test_deep_cull_flag_bit_exact" "tests/test_gpu_parity.py::test_fused_small_scene_forward" tests/test_abi.py tests/test_gpu_recompute_bwd.py -k "not two_graphs" > gpurun_out/g1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g1_tests.log; [ $rc -ne 0 ] && exit $rc
for P in 1 4; do
DIRT_GRAD_PERSIST=$P timeout -k 10 300 $T tests/test_gpu_parity.py -k "full_size or batch or config4 or dense or shared_vertex or golden or backward_accumulate or partial" tests/test_gpu_recompute_bwd.py > gpurun_out/g1_persist$P.log 2>&1
rc=$?; tail -3 gpurun_out/g1_persist$P.log; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do for P in 0 4 2 5; do
DIRT_GRAD_PERSIST=$P DIRT_NO_CPU=1 timeout -k 10 300 python3 tools/bench_configs.py c3_random c3x8 > gpurun_out/g1_ab_P${P}_$rep.jsonl 2> gpurun_out/g1_ab_P${P}_$rep.err
rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/g1_ab_P${P}_$rep.err; exit $rc; }
python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print('P=%s#%s %-36s %8.1f Mpix/s  %s' % (sys.argv[2], sys.argv[3], d['config'], d['Mpixels_per_s_fwd_bwd'], ' '.join('%s=%.1f'%(k[:6],v) for k,v in d['kernels_us'].items())))" gpurun_out/g1_ab_P${P}_$rep.jsonl $P $rep
done; done
bash tools/gpu_repro.sh
