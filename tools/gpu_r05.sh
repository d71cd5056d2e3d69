#!/bin/bash
# round-5 evidence run: full GPU suite, smoke, default bench, the N-rank rehearsal (shared GPU, gloo)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=${1:-r05}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/${tag}_smoke.log; exit 1; }
timeout -k 10 500 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo bench failed; tail -5 gpurun_out/${tag}_bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_driver.json 2> gpurun_out/${tag}_bench_driver.err || { echo bench20 failed; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/${tag}_bench.json','gpurun_out/${tag}_bench_driver.json'):
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'], d['kernels_us'], d['roofline'].get('frac'), d.get('r5_clip_stats'))
d=json.load(open('gpurun_out/${tag}_bench.json'))
for k,v in d['legs'].items(): print(k, {a:b for a,b in v.items() if a!='what'})
"
bash tools/gpu_multirank.sh $tag > gpurun_out/${tag}_multirank_console.txt 2>&1; echo "multirank rc=$?"; tail -c 3000 gpurun_out/multirank_$tag.txt
