#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: 2 ranks share cuda:0 over gloo
# (NFX_BENCH_REHEARSE=1). Checks the code path end to end, not scaling.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-rehearse}; mkdir -p $O
cd $R
export NFX_BENCH_REHEARSE=1
for c in cfg2 cfg4t cfg5i; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --config $c --steps 5 --warmup 2 --no-cpu > $O/r2_$c.json 2> $O/r2_$c.err || exit $?
  echo "rehearsed $c"
done
