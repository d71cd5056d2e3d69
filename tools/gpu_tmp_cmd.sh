#!/bin/bash
# scratch GPU command: the default -m gpu suite on the final tree
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/final3_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/final3_pytest.log; exit $rc
