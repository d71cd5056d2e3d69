#!/bin/bash
# PMC counter passes over the bench (one counter group per rocprofv3 run, --kernel-trace only).
# usage: tools/gpu_pmc.sh tag "GROUP1" "GROUP2" ...   (each group: space-separated counter names)
tag=$1; shift
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $out/counters_list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-graph --profile-steps 2 --rotate 0 --no-api-leg > $out/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $out/p$i.log; exit $rc; fi
  [ $rc -eq 1 ] && tail -3 $out/p$i.log
done
exit 0
