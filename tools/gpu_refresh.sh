#!/bin/bash
# Full GPU test suite, then one bench line per eval/sampling config (run on the GPU box).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/refresh; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_gpu.log 2>&1 || { tail -30 $O/t_gpu.log; exit 1; }
tail -2 $O/t_gpu.log
for c in cfg2 cfg3 cfg4 cfg5f cfg5i; do
  timeout -k 10 300 python -u bench.py --config $c > $O/b_$c.json 2> $O/b_$c.err || exit 1
  echo "done $c"
done
for c in sample4k sample4k_spline sample4k_maf sample4k_iaf; do
  timeout -k 10 120 python bench.py --config $c --steps 200 --warmup 20 --graph --no-cpu > $O/b_${c}_graph.json 2>$O/b_${c}_graph.err || exit 1
  echo "done $c"
done
