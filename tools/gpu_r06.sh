#!/bin/bash
# Round-6 evidence run: GPU tests, smoke, the driver's bench command, a rocprofv3 kernel-trace summary of the bench,
# and (last, since one variant is expected to crash the host process) the capture_end control experiment.
#   tools/gpu_r06.sh TAG [control]
tag=${1:-v1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_$tag; mkdir -p $O
cd $R
echo "== pytest -m gpu"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== smoke"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "== bench (driver command)"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { echo "bench rc=$?"; tail -5 $O/bench_driver.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_driver.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['avg_us'], r['avg_us_events'], d['kernels_us'], d['legs'].get('api_autograd',{}).get('eager_mpix_s'))"
echo "== rocprofv3 kernel trace of the bench (200 steps)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rotate 0 --no-api-leg --no-recompute-leg > $O/bench_prof.json 2> $O/bench_prof.err || { echo "rocprof rc=$?"; tail -5 $O/bench_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -6 $O/kernel_stats.csv | cut -c1-200
cd $R
if [ "$2" = "control" ]; then
  echo "== capture_end control (the crash-expected variant last)"
  for v in "ext released" "py released" "torch released" "torch kept"; do
    n=$(echo "$v" | tr ' ' '_')
    timeout -k 10 120 python3 tools/debug/capture_control.py $v > $O/control_$n.log 2>&1
    rc=$?; echo "$v rc=$rc: $(grep -v '^ ' $O/control_$n.log | grep -E 'ok|warnings|Fatal|Error' | tr '\n' ' ' | cut -c1-300)"
    [ $rc -eq 0 ] || exit 0
  done
fi
exit 0
