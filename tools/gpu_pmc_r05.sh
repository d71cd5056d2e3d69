#!/bin/bash
# Round 5: PMC passes over the bench at c3 (one frame per launch) and c3x8 (eight frames per launch: the steady
# state), for the backward's bound.  One rocprofv3 --pmc run per group, kernel-trace only.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for cfg in c3 c3x8; do
  out=$R/gpurun_out/pmc5_$cfg; mkdir -p $out
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-graph --profile-steps 2 --rotate 0 --no-api-leg --no-recompute-leg --min-warm-ms 50 > $out/p$i.log 2>&1
    rc=$?; echo "$cfg pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; exit $rc; fi
  done
  python3 $R/tools/pmc_summary.py $out > $out/summary.txt 2>&1; grep -A40 "grad_kernel" $out/summary.txt | head -32
done
exit 0
