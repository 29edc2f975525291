#!/bin/bash
# Round 6 final build: the GPU suite + smoke, then the eval profiles (trace + FETCH/WRITE + MFMA-busy)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_suite.sh r06final || exit $?
bash tools/profile_bench.sh r06final --pmc cfg2 cfg3 cfg4 || exit $?
