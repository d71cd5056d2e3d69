#!/bin/bash
# scratch GPU command: bench with the in-graph pass timing (the driver's command)
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/gp; mkdir -p $out; cd $R
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['roofline']), d['parity_vs_oracle']['grad_vertices_within_tol'])" $out/bench.json
grep -v amdgpu.ids $out/bench.err | tail -3
