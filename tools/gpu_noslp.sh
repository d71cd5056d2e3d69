#!/bin/bash
# A/B of the product against build/variants/*.so: configs (3 rounds) and the backward by requested gradients.
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_ab_configs.sh 3 c3_random c4_deferred20k c5_batch8 || exit $?
for lib in $R/dirt_amd/libdirt_mi355x.so $R/build/variants/*.so; do
  echo "# $(basename $lib)"
  DIRT_MI355X_LIB=$lib timeout -k 10 120 python3 $R/tools/bwd_gm_timing.py || exit $?
done
