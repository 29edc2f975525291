#!/bin/bash
# Sequential MADE kernel check on the GPU box: batch sweep of the cfg5i kernel
# (tools/seq_batch_sweep.py), the MADE/relational/LDS-poison GPU tests and the cfg5i bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/seq_batch_sweep.py > $O/sweep.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "made or iaf or maf or relational or poison or logprob or seq" > $O/t_made.log 2>&1
rc=$?
tail -3 $O/t_made.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg5i > $O/bench_cfg5i.json 2> $O/bench_cfg5i.err || exit $?
echo ok
