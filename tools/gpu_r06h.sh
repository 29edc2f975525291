#!/bin/bash
# Round 6: layer-1 statistics from the input moments — train-mode parity, cfg2t A/B, relational seeds A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06h; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_affine_train.py tests/test_gpu_fig_models.py tests/test_gpu_graph_train.py tests/test_gpu_grad_fixtures.py tests/test_gpu_generic_coupling.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in moments pass moments pass; do
  if [ $v = pass ]; then export NFX_TRAIN_STATS1=pass; else unset NFX_TRAIN_STATS1; fi
  timeout -k 10 300 python bench.py --config cfg2t --steps 20 --warmup 5 --no-cpu --graph > $O/cfg2t_$v.json 2> $O/cfg2t_$v.err || exit $?
  python -c "
import json; d=json.loads(open('$O/cfg2t_$v.json').read().strip().splitlines()[-1])
print('$v', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,1), 'M/s')"
done
unset NFX_TRAIN_STATS1
timeout -k 10 400 python -u tools/relational_seeds.py > $O/moments_keep1.jsonl 2>&1 || exit $?
NFX_TRAIN_KEEP=0 timeout -k 10 400 python -u tools/relational_seeds.py > $O/moments_keep0.jsonl 2>&1 || exit $?
grep realnvp $O/moments_keep1.jsonl $O/moments_keep0.jsonl
