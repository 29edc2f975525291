#!/bin/bash
# Round 6: affine layer 2 on bf16x3-split MFMAs (libnfx_bf.so) against the shipped libnfx.so —
# cfg2 at 1M and at the 125k shard alternating the two libraries on one box, then the variant's
# parity on the affine / chain / log_prob / training / sampling suites.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06bf; mkdir -p $O; cd $R
PK=$R/normalizing-flows-study_amd/nfs_amd/libnfx_bf.so
for rep in 1 2; do
  for lib in main bf; do
    if [ $lib = bf ]; then export NFX_LIB=$PK; else unset NFX_LIB; fi
    for b in 1048576 125000; do
      timeout -k 10 200 python bench.py --config cfg2 --batch $b --steps 50 --warmup 10 --no-cpu --no-secondary \
        > $O/${lib}_${b}_$rep.json 2> $O/${lib}_${b}_$rep.err || exit $?
      python -c "
import json; d=json.loads(open('$O/${lib}_${b}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$lib', $b, $rep, round(d['ms_per_step']*1e3,1), 'us/step', round(r['mean_launch_ms']*1e3,1), 'us kernel frac', round(r['frac'],3))"
    done
  done
done
NFX_LIB=$PK timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_affine.py tests/test_gpu_chain.py tests/test_gpu_logprob.py tests/test_gpu_affine_train.py tests/test_gpu_sample.py > $O/tests_bf.log 2>&1 || { tail -40 $O/tests_bf.log; exit 1; }
tail -2 $O/tests_bf.log
