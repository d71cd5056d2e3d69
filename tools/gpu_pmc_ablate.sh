#!/bin/bash
# LDS counters per ablation variant of grad/raster (tools/ablate.py: each variant is its own kernel instantiation,
# so rocprofv3 attributes the counters per variant): bank-conflict cycles against LDS-active cycles, LDS and VALU
# instruction counts.  One rocprofv3 --pmc pass per counter group, kernel-trace only.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_ablate_${1:-a}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv -- python3 $R/tools/ablate.py ${2:-c3} > $out/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out/p$i.log; exit $rc; }
done
python3 $R/tools/pmc_summary.py $out > $out/summary.txt 2>&1
grep -A9 "grad_kernel" $out/summary.txt | head -150
exit 0
