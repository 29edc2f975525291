#!/bin/bash
# Round 6: the suite on the fetch_add + clean-tag logp_commit build, then the eval profiles
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_suite.sh r06b || exit $?
bash tools/profile_bench.sh r06b --pmc cfg2 cfg5i:1024 cfg3 cfg5i || exit $?
