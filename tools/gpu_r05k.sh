#!/bin/bash
# round 5: kept / g_y1 tiles as 16-byte lane vectors (variant x4) against the default layout
out=gpurun_out/r05k6; mkdir -p $out
X4=$PWD/normalizing-flows-study_amd/nfs_amd/libnfx_x4.so
NFX_LIB=$X4 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_affine_train.py tests/test_gpu_grad_fixtures.py tests/test_gpu_graph_train.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for v in default x4; do
lib=$PWD/normalizing-flows-study_amd/nfs_amd/libnfx.so; [ $v = x4 ] && lib=$X4
NFX_LIB=$lib timeout -k 10 300 python bench.py --config cfg2t --graph --steps 10 --warmup 3 --no-cpu > $out/bench_$v.json 2> $out/bench_$v.err || exit $?
python -c "import json; d=json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp && NFX_LIB=$X4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg2t --graph --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || exit $?
f=$(ls $GRAFT_REPO_ROOT/$out/prof/*/*_kernel_stats.csv | head -1); python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows[:8]:
    print(r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:70])
"
