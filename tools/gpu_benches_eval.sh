#!/bin/bash
# Eval-path benches (bench.py JSON line per config) into gpurun_out/ (run on the GPU box).
set -e
cd $GRAFT_REPO_ROOT
for c in ${*:-cfg2 cfg3 cfg4 cfg5f cfg5i}; do
  timeout -k 10 300 python -u bench.py --config $c > gpurun_out/b_$c.json 2> gpurun_out/b_$c.err
  echo "done $c"
done
