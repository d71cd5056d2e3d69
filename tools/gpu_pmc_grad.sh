#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group, --kernel-trace only) over the c3 bench loop,
# for the per-kernel bottleneck study.  usage: tools/gpu_pmc_grad.sh tag "GROUP1" "GROUP2" ...
tag=$1; shift
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-graph --profile-steps 2 --rotate 0 --no-api-leg > $out/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; exit $rc; fi
done
python3 $R/tools/pmc_summary.py $out > $out/summary.txt 2>&1; head -80 $out/summary.txt
exit 0
