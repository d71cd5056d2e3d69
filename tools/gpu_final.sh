#!/bin/bash
# Evidence run of a tree: GPU tests, smoke, the driver's bench command, a 200-step bench, rocprofv3 kernel stats of
# the bench, and the HBM traffic passes (FETCH_SIZE calibration + one --pmc pass per counter) -> traffic.json tagged
# with the tree.   tools/gpu_final.sh TAG TREE_SHA
tag=${1:-final}; tree=${2:-unknown}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_$tag; mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { echo "bench rc=$?"; tail -5 $O/bench_driver.err; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench200 rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "
import json
for f in ('$O/bench_driver.json','$O/bench.json'):
    d=json.load(open(f)); r=d['roofline']; l=d['legs']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], 'frac', r['frac'], 'avg_us', r['avg_us'], 'ev', r['avg_us_events'], d['kernels_us'], 'api', l.get('api_autograd',{}).get('eager_mpix_s'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
cd /tmp && export TMPDIR=/tmp
# (the driver's command under rocprofv3; tools/trace_summary.py then takes the single-frame launches out of the trace)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || { echo "rocprof rc=$?"; tail -5 $O/bench_prof.err; exit 1; }
python3 $R/tools/trace_summary.py $O/prof/run_kernel_trace.csv $O/bench_driver.json > $O/trace_summary.txt && cat $O/trace_summary.txt
T=$O/traffic
mkdir -p $T
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $T/cal -o run --output-format csv -- python3 $R/tools/pmc_calibrate.py > $T/cal.log 2>&1 || { echo "calibration rc=$?"; tail -5 $T/cal.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $c -d $T/$c -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-graph --profile-steps 2 --rotate 0 --no-api-leg --no-recompute-leg > $T/$c.log 2>&1 || { echo "$c rc=$?"; tail -5 $T/$c.log; exit 1; }
done
cd $R
python3 tools/pmc_traffic.py $T $O/traffic.json $tree
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    print('%-50s %6s %9.2f us' % (r['Name'][:50].replace('void (anonymous namespace)::',''), r['Calls'], float(r['AverageNs'])/1e3))" | head -5
exit 0
