#!/bin/bash
# The public op's eager leg across repeated bench runs on one box: the driver's command twice, the default
# (200-step) command, the driver's command again.   tools/api_variance.sh
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/apix; mkdir -p $O; cd $R
for k in d1 d2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/$k.json 2>$O/$k.err || exit 1; done
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/full.json 2>$O/full.err || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/d3.json 2>$O/d3.err || exit 1
python3 - <<'PY'
import json, os
O = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out", "apix")
for f in ("d1", "d2", "full", "d3"):
    d = json.load(open(os.path.join(O, f + ".json")))
    a = d["legs"]["api_autograd"]
    print(f, d["value"], a["eager_mpix_s"], a["eager_chunks_mpix_s"], a["eager_shared_geometry_mpix_s"], a["graph20_mpix_s"])
PY
