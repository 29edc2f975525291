#!/bin/bash
# Round 6 rebuild (split-MFMA affine layer 2): the GPU suite + smoke, the eval profiles
# (trace + FETCH/WRITE + MFMA-busy)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_suite.sh r06final3 || exit $?
bash tools/profile_bench.sh r06final3 --pmc cfg2 cfg3 cfg4 || exit $?
