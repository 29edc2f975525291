#!/bin/bash
# Round-2 GPU check: full GPU test suite (no -x: collect every failure), then the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r02a}; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --maxfail=25 --timeout 300 --timeout-method thread -s > $O/t_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/t_gpu.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "bench done"
exit $rc
