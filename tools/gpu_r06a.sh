#!/bin/bash
# Round 6, first GPU call: the full GPU suite + smoke on the ABI-3 build, bench.py --gpus 2 with no
# launcher (2 ranks sharing cuda:0 over gloo), and the cfg2 profile with the MFMA-busy pass.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06a; mkdir -p $O
cd $R
bash tools/gpu_suite.sh r06a || exit $?
NFX_BENCH_REHEARSE=1 timeout -k 10 300 python3 bench.py --gpus 2 --config cfg2 --steps 5 --warmup 2 --no-cpu \
  > $O/gpus2_cfg2.json 2> $O/gpus2_cfg2.err || exit $?
echo "gpus2 ok"; tail -c 600 $O/gpus2_cfg2.json
bash tools/profile_bench.sh r06a --pmc cfg2 cfg4 cfg5i:1024 || exit $?
