#!/bin/bash
# Kernel timeline of the graph-replayed bench step (rocprofv3 --kernel-trace), for gap analysis.
tag=${1:-tl}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/timeline_$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $out -o run --output-format csv -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline --profile-steps 1 > $out/bench.log 2>&1
rc=$?; echo "timeline rc=$rc"; tail -2 $out/bench.log; exit $rc
