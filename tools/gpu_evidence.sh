#!/bin/bash
# Round evidence in one GPU session: -m gpu suite, smoke(), bench.py (default line), rocprofv3 kernel-trace
# stats of the bench's main loop, and the PMC traffic passes.  usage: tools/gpu_evidence.sh tag
tag=${1:-r03}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/ev_$tag; mkdir -p $out
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cut -c1-400 $out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-graph --rotate 0 --no-api-leg > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $out/prof.log; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -8'
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/cal -o run --output-format csv -- python3 $R/tools/pmc_calibrate.py > $out/cal.log 2>&1 || { echo "calibration failed"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $c -d $out/$c -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-graph --profile-steps 2 --rotate 0 --no-api-leg > $out/$c.log 2>&1 || { echo "$c failed"; tail -5 $out/$c.log; exit 1; }
done
echo evidence done
