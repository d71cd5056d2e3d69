mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/ext_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ext_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/profile_api.py > gpurun_out/profile_api.txt 2>&1 || exit 1
head -8 gpurun_out/profile_api.txt
timeout -k 10 200 python tools/launch_overhead.py > gpurun_out/launch_overhead.txt 2>&1 || exit 1
cat gpurun_out/launch_overhead.txt
DIRT_NO_CPU=1 timeout -k 10 200 python tools/bench_configs.py c4_deferred_chain > gpurun_out/chain.jsonl 2>&1; tail -2 gpurun_out/chain.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ext_bench.json 2>gpurun_out/ext_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/ext_bench.json')); print(d['value'], d['kernels_us'], json.dumps(d['legs']))"
bash tools/gpu_multirank.sh r03 || exit 1
