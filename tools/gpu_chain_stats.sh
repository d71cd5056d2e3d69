#!/bin/bash
# the deferred chain (c4) timed, then under rocprofv3 kernel stats (ours vs torch glue per step)
set -o pipefail
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out; mkdir -p $out; tag=${1:-chain}
DIRT_NO_CPU=1 timeout -k 10 300 python3 $R/tools/bench_configs.py c4_deferred_chain > $out/chain_$tag.jsonl 2> $out/chain_$tag.err || exit $?
cat $out/chain_$tag.jsonl
cd /tmp && export TMPDIR=/tmp
DIRT_NO_CPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_chain_$tag -o run --output-format csv -- python3 $R/tools/bench_configs.py c4_deferred_chain > $out/prof_chain_$tag.log 2>&1
