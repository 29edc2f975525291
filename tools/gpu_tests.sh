#!/bin/bash
# GPU test suite only (optionally a -k filter): bash tools/gpu_tests.sh <tag> [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd $R
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --maxfail=25 --timeout 300 --timeout-method thread -s "${K[@]}" > $O/t_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/t_gpu.log | tail -3
exit $rc
