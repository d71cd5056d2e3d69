#!/bin/bash
# Round-3 check in one GPU session: the whole -m gpu suite, smoke(), then bench.py (default N=1 line).
# usage: tools/gpu_r3_check.sh tag   (outputs under gpurun_out/<tag>_*)
tag=${1:-r03}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out || exit 1
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
tail -c 3000 gpurun_out/${tag}_bench.json
