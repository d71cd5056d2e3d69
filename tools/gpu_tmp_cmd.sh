#!/bin/bash
# scratch GPU command: the RCCL / sharding GPU tests
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_batch_multigpu.py > gpurun_out/rccl.log 2>&1; rc=$?; tail -12 gpurun_out/rccl.log; exit $rc
