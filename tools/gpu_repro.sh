#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for args in "py 000 one" "py 000 one keep_saved" "py 000 one scratch"; do
  n=$(echo "$args" | tr ' ' '_'); echo "== $args"; timeout -k 10 120 python3 tools/debug/capture_repro3.py $args > gpurun_out/repro3_$n.log 2>&1; echo "rc=$?"; grep -E "^replay|intact|scratch P|Error" gpurun_out/repro3_$n.log | head -12
done
echo; env | grep -i -E "alloc_conf|PYTORCH" ; exit 0
