#!/bin/bash
# One measurement session: graph-replay timeline, per-phase timestamps of the three kernels, SQ counters.
# usage: tools/gpu_measure.sh tag     (outputs under gpurun_out/meas_<tag>/)
tag=${1:-m}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/meas_$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/phase_ts.py > $out/phase_grad.txt 2>&1 || { echo "phase_ts rc=$?"; tail -5 $out/phase_grad.txt; exit 1; }
timeout -k 10 120 python3 $R/tools/raster_ts.py > $out/phase_raster.txt 2>&1 || { echo "raster_ts rc=$?"; tail -5 $out/phase_raster.txt; exit 1; }
timeout -k 10 120 python3 $R/tools/setup_ts.py > $out/phase_setup.txt 2>&1 || { echo "setup_ts rc=$?"; tail -5 $out/phase_setup.txt; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace -d $out/tl -o run --output-format csv -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline --profile-steps 1 > $out/tl.log 2>&1 || { echo "timeline rc=$?"; tail -5 $out/tl.log; exit 1; }
python3 $R/tools/timeline.py $out/tl > $out/timeline.txt 2>&1
timeout -k 10 60 rocprofv3 -L > $out/counters_list.txt 2>&1
i=0
for grp in "$@"; do :; done
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-graph --profile-steps 2 > $out/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && tail -3 $out/p$i.log
  [ $rc -ge 124 ] && exit $rc
done
cat $out/timeline.txt | tail -12
exit 0
