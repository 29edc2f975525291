#!/bin/bash
# Spline GPU tests and the cfg3 / cfg3t bench lines (run on the GPU box): bash tools/gpu_spline_check.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "spline or arqs or rqs or poison or wide" > $O/t_spline.log 2>&1
rc=$?
tail -2 $O/t_spline.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg3 > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg3t > $O/bench_cfg3t.json 2> $O/bench_cfg3t.err || exit $?
echo ok
