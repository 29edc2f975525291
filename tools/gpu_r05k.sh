#!/bin/bash
# round 5: kept layer-2 pre-activations, per-net BWD2K, OUTK, per-stage LDS image of the train-mode coupling passes
out=gpurun_out/r05k4; mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_affine_train.py tests/test_gpu_grad_fixtures.py tests/test_gpu_graph_train.py tests/test_gpu_fig_models.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for v in default both; do
lib=$PWD/normalizing-flows-study_amd/nfs_amd/libnfx.so; [ $v != default ] && lib=$PWD/normalizing-flows-study_amd/nfs_amd/libnfx_$v.so
NFX_LIB=$lib timeout -k 10 300 python bench.py --config cfg2t --graph --steps 10 --warmup 3 --no-cpu > $out/bench_$v.json 2> $out/bench_$v.err || exit $?
python -c "import json; d=json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg2t --graph --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || exit $?
f=$(ls $GRAFT_REPO_ROOT/$out/prof/*/*_kernel_stats.csv | head -1); python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows[:12]:
    print(r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:70])
"
