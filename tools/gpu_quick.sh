#!/bin/bash
# Quick GPU iteration: a pytest -k filter, then bench lines for the given configs.
#   bash tools/gpu_quick.sh <tag> "<pytest -k expr or ''>" cfg3 [cfg5i ...]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd $R
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rs --maxfail=10 --timeout 300 --timeout-method thread -k "$2" > $O/t_gpu.log 2>&1
  rc=$?; tail -3 $O/t_gpu.log; [ $rc -le 1 ] || exit $rc
fi
shift 2
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-secondary > $O/b_$c.json 2> $O/b_$c.err || exit $?
  python3 -c "import json,sys; j=json.load(open('$O/b_$c.json')); r=j['roofline']; print('$c', round(j['value']/1e6,1), 'M/s frac', round(r['frac'],3), 'kernel ms', round(r['mean_launch_ms'],4))"
done
