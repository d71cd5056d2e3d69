#!/bin/bash
# Rehearsal of bench.py's N-rank path on one MI355X (DIRT_BENCH_SHARED_GPU=1: ranks share cuda:0, collectives
# over gloo).  usage: tools/gpu_multirank.sh tag   -> gpurun_out/multirank_<tag>.txt
tag=${1:-r03}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/multirank_$tag.txt
: > $out
for n in 2 4; do
  echo "# torchrun --nproc-per-node $n ... bench.py --gpus $n --steps 50 --warmup 5 (DIRT_BENCH_SHARED_GPU=1)" >> $out
  DIRT_BENCH_SHARED_GPU=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) $R/bench.py --gpus $n --steps 50 --warmup 5 \
      --rotate 0 --no-api-leg >> $out 2>$R/gpurun_out/multirank_${tag}_$n.err || { echo "n=$n failed"; tail -5 $R/gpurun_out/multirank_${tag}_$n.err; exit 1; }
done
grep -v "^\[Gloo\]" $out | cut -c1-600
