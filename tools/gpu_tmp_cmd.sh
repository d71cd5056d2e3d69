#!/bin/bash
# scratch GPU command: the -m gpu suite, the formerly failing fuzz seed, then 40000 fuzz seeds
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/fuzz2; mkdir -p $out; cd $R
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/debug/fuzz_seed.py 37851 > $out/seed37851.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/seed37851.txt
DIRT_FUZZ_SEEDS=40000 timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k fuzz > $out/fuzz40000.log 2>&1
rc=$?; tail -2 $out/fuzz40000.log; exit $rc
