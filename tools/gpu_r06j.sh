#!/bin/bash
# Round 6: fused draw in the spline chain — sampling + spline chain tests
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06j; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_sample.py tests/test_gpu_spline_chain.py tests/test_gpu_spline.py tests/test_gpu_logprob.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
