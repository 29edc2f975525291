#!/bin/bash
# Affine-coupling parity tests + cfg2 bench (run on the GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_affine.py tests/test_gpu_logprob.py tests/test_gpu_relational.py tests/test_gpu_graph_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_affine.log 2>&1 || { tail -30 gpurun_out/t_affine.log; exit 1; }
tail -2 gpurun_out/t_affine.log
timeout -k 10 300 python -u bench.py > gpurun_out/b_cfg2.json 2> gpurun_out/b_cfg2.err || exit 1
cat gpurun_out/b_cfg2.json
