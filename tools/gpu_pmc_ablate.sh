#!/bin/bash
# Dynamic instruction counts per ablation variant of grad/raster (one rocprofv3 --pmc pass over ablate.py).
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_ablate; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $out/p1 -o run --output-format csv -- python3 $R/tools/ablate.py > $out/p1.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
