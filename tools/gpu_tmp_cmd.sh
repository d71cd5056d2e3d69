#!/bin/bash
# scratch GPU command: the driver's exact bench command, then every BASELINE config (tools/bench_configs.py)
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/cfg; mkdir -p $out; cd $R
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/driver_cmd.json 2> $out/driver_cmd.err || { tail -5 $out/driver_cmd.err; exit 1; }
cut -c1-300 $out/driver_cmd.json
timeout -k 10 500 python3 tools/bench_configs.py > $out/configs.jsonl 2> $out/configs.err || { tail -5 $out/configs.err; exit 1; }
cut -c1-250 $out/configs.jsonl
