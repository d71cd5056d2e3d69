#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ablate.py c3 > gpurun_out/ablate_c3.txt 2>&1; echo rc=$?; grep grad gpurun_out/ablate_c3.txt
timeout -k 10 300 python3 tools/ablate.py c4 > gpurun_out/ablate_c4.txt 2>&1; echo rc=$?; grep grad gpurun_out/ablate_c4.txt
exit 0
