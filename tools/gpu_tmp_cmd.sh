#!/bin/bash
# scratch GPU command: the procedural programs over 1200 adversarial scenes
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/proc; mkdir -p $out; cd $R
DIRT_PROC_FUZZ_SEEDS=1200 timeout -k 10 700 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_oceanic.py -k procedural_programs_adversarial > $out/proc1200.log 2>&1
rc=$?; tail -3 $out/proc1200.log; exit $rc
