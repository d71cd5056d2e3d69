#!/bin/bash
# GPU tests of the partial-gradient backward, then its kernel times for the product and build/variants/*.so.
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "partial or without_background" -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
for lib in $R/dirt_amd/libdirt_mi355x.so $R/build/variants/*.so; do
  echo "# $(basename $lib)"
  DIRT_MI355X_LIB=$lib timeout -k 10 120 python3 $R/tools/bwd_gm_timing.py || exit $?
done
