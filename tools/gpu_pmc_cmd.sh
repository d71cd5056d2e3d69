#!/bin/bash
# PMC counter passes over an arbitrary python script (one group per rocprofv3 run, --kernel-trace only).
# usage: tools/gpu_pmc_cmd.sh tag "script.py args" "GROUP1" "GROUP2" ...
tag=$1; shift; cmd=$1; shift
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv -- python3 $R/$cmd > $out/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $out/p$i.log; exit $rc; }
done
exit 0
