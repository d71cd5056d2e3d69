#!/bin/bash
# HBM traffic per kernel (rocprofv3 --pmc, one counter per pass, kernel-trace only) for the bench and
# for the FETCH_SIZE width calibration.  usage: tools/gpu_traffic.sh tag
tag=${1:-t}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/traffic_$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/cal -o run --output-format csv -- python3 $R/tools/pmc_calibrate.py > $out/cal.log 2>&1 || { echo "calibration rc=$?"; tail -5 $out/cal.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $c -d $out/$c -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-graph --profile-steps 2 --rotate 0 --no-api-leg > $out/$c.log 2>&1 || { echo "$c rc=$?"; tail -5 $out/$c.log; exit 1; }
done
echo traffic passes done
