#!/bin/bash
# Round evidence in one GPU session: parity tests, bench (with CPU baseline), kernel-trace stats,
# PMC traffic.  usage: tools/gpu_round.sh tag   (outputs under gpurun_out/, copy to profiles/)
tag=${1:-r01}
bash $GRAFT_REPO_ROOT/tools/gpu_check.sh $tag && bash $GRAFT_REPO_ROOT/tools/gpu_traffic.sh $tag
