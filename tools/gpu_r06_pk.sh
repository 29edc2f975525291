#!/bin/bash
# Round 6: the affine output layer as packed FMAs (libnfx_pk.so) against the shipped libnfx.so —
# parity of the variant on the affine / chain / log_prob suites, then cfg2 at 1M and at the
# 125k shard, alternating the two libraries on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06pk; mkdir -p $O; cd $R
PK=$R/normalizing-flows-study_amd/nfs_amd/libnfx_pk.so
NFX_LIB=$PK timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_chain.py tests/test_gpu_logprob.py > $O/tests_pk.log 2>&1 || { tail -30 $O/tests_pk.log; exit 1; }
tail -2 $O/tests_pk.log
for rep in 1 2 3; do
  for lib in main pk; do
    if [ $lib = pk ]; then export NFX_LIB=$PK; else unset NFX_LIB; fi
    for b in 1048576 125000; do
      timeout -k 10 200 python bench.py --config cfg2 --batch $b --steps 50 --warmup 10 --no-cpu --no-secondary \
        > $O/${lib}_${b}_$rep.json 2> $O/${lib}_${b}_$rep.err || exit $?
      python -c "
import json; d=json.loads(open('$O/${lib}_${b}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$lib', $b, $rep, round(d['ms_per_step']*1e3,1), 'us/step', round(r['mean_launch_ms']*1e3,1), 'us kernel frac', round(r['frac'],3))"
    done
  done
done
