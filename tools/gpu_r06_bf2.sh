#!/bin/bash
# Round 6: affine layer 2 on bf16x3-split MFMAs (truncated activation pieces, round-to-nearest weight pieces), hi/lo accumulators —
# libnfx_bf.so against the shipped libnfx.so: precision vs the fp32
# small-batch kernel, cfg2 at 1M and at the 125k shard, then the variants' affine suites.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06bf4; mkdir -p $O; cd $R
NL=$R/normalizing-flows-study_amd/nfs_amd
for lib in libnfx libnfx_bf; do
  NFX_LIB=$NL/$lib.so timeout -k 10 200 python tools/split_precision.py >> $O/precision.jsonl 2> $O/precision_$lib.err || exit $?
done
cat $O/precision.jsonl
for rep in 1 2; do
  for lib in libnfx libnfx_bf; do
    for b in 1048576 125000; do
      NFX_LIB=$NL/$lib.so timeout -k 10 200 python bench.py --config cfg2 --batch $b --steps 50 --warmup 10 --no-cpu --no-secondary \
        > $O/${lib}_${b}_$rep.json 2> $O/${lib}_${b}_$rep.err || exit $?
      python -c "
import json; d=json.loads(open('$O/${lib}_${b}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$lib', $b, $rep, round(d['ms_per_step']*1e3,1), 'us/step', round(r['mean_launch_ms']*1e3,1), 'us kernel frac', round(r['frac'],3))"
    done
  done
done
for lib in libnfx_bf; do
  NFX_LIB=$NL/$lib.so timeout -k 10 500 python -u -m pytest -q --maxfail=8 --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_affine.py tests/test_gpu_chain.py tests/test_gpu_logprob.py tests/test_gpu_affine_train.py \
    tests/test_gpu_sample.py tests/test_gpu_relational.py > $O/tests_$lib.log 2>&1
  rc=$?
  echo "$lib tests rc=$rc"; grep -E "^FAILED|passed|failed" $O/tests_$lib.log | tail -12
  [ $rc -le 1 ] || exit $rc
done
