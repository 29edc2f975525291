#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/profile_bench.sh r06final3 --pmc cfg5f cfg5i cfg5i:1024 cfg2:125000 cfg3:125000 || exit $?
