#!/bin/bash
# Round 6: made_wgrad_kernel variants on one box (cfg4t, graph): old (round 5), 1 tile/task single
# buffer (default build), 1 tile/task double buffer, 2 tiles/task single buffer
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06e; mkdir -p $O; cd $R
L=$R/normalizing-flows-study_amd/nfs_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_made_backward.py tests/test_gpu_grad_fixtures.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in wold main t1db t2s wold main; do
  if [ $v = main ]; then lib=$L/libnfx.so; else lib=$L/libnfx_$v.so; fi
  NFX_LIB=$lib timeout -k 10 300 python bench.py --config cfg4t --steps 10 --warmup 3 --no-cpu --graph > $O/cfg4t_$v.json 2> $O/cfg4t_$v.err || exit $?
  python -c "
import json; d=json.loads(open('$O/cfg4t_$v.json').read().strip().splitlines()[-1]); w=d['roofline'].get('wgrad',{})
print('$v', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,1), 'M/s', 'bwd', round(d['roofline']['mean_launch_ms']*1e3,1), 'us', 'wgrad', round(w.get('mean_launch_ms',0)*1e3,1), 'us')"
done
