#!/bin/bash
# scratch GPU command: -m gpu suite, then c3 / c4 / c5 with the setup workgroup size chosen by grid size (product)
# against HEAD (base), 2 interleaved rounds
R=$GRAFT_REPO_ROOT; out=$R/gpurun_out/st; mkdir -p $out; cd $R
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in $R/dirt_amd/libdirt_mi355x.so $R/build/variants/base.so; do
  n=$(basename $lib .so)
  DIRT_MI355X_LIB=$lib timeout -k 10 300 python3 tools/bench_configs.py c4_deferred20k c3_random c5_batch > $out/${n}_$rep.jsonl 2> $out/${n}_$rep.err || { tail -3 $out/${n}_$rep.err; exit 1; }
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['config'][:24], d.get('Mpixels_per_s_fwd_bwd'), d.get('kernels_us'))
" $out/${n}_$rep.jsonl "$n#$rep"
done; done
