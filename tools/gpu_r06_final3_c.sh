#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/profile_bench.sh r06final3 --pmc cfg4t+graph cfg2t+graph cfg3t+graph sample4k_maf sample4k_iaf || exit $?
