#!/bin/bash
# Round 6: push-kernel (cfg5i 1 Ki shard) chain ablations — timing only, wrong results by design
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06i; mkdir -p $O; cd $R
L=$R/normalizing-flows-study_amd/nfs_amd
for v in main sum aff chain all3 nearall main; do
  if [ $v = main ]; then lib=$L/libnfx.so; else lib=$L/libnfx_$v.so; fi
  NFX_LIB=$lib timeout -k 10 120 python -u tools/seq_batch_sweep.py 1024 > $O/$v.jsonl 2>&1 || exit $?
  echo "$v $(grep '^{' $O/$v.jsonl)"
done
