#!/bin/bash
# scratch GPU command: bench.py's N-rank path on one GPU (gloo rehearsal) with the gather legs
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_multirank.sh r03d || exit 1
