#!/bin/bash
# Round-2 bench lines: every config (eval + training + sampling) into gpurun_out/<tag>/, then
# rocprofv3 kernel stats of the training configs.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r02_benches}; mkdir -p $O
cd $R
for c in cfg2 cfg3 cfg4 cfg5f cfg5i cfg2t cfg3t cfg4t; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 > $O/b_$c.json 2> $O/b_$c.err || exit $?
  echo "done $c"
done
timeout -k 10 240 python -u bench.py --config train5k --graph --steps 50 --warmup 5 > $O/b_train5k_graph.json 2> $O/b_train5k_graph.err || exit $?
timeout -k 10 240 python -u bench.py --config sample4k --steps 50 --warmup 5 > $O/b_sample4k.json 2> $O/b_sample4k.err || exit $?
export TMPDIR=/tmp
for c in cfg2t cfg3t cfg4t; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -- \
     python3 $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu > $O/prof_$c.log 2>&1) || exit $?
  echo "profiled $c"
done
