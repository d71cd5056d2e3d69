#!/bin/bash
# scratch GPU command: final evidence of the round (suite, smoke, bench, rocprof, PMC) and the N-rank rehearsal
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_evidence.sh r03c || exit 1
bash tools/gpu_multirank.sh r03c || exit 1
