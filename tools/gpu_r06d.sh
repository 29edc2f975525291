#!/bin/bash
# Round 6: MADE weight-gradient pairs + masked-tile skip — parity, then cfg4t single vs double buffer
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06d; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_made_backward.py tests/test_gpu_grad_fixtures.py tests/test_gpu_fig_models.py tests/test_gpu_relational.py tests/test_gpu_options.py tests/test_gpu_generic.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config cfg4t --steps 10 --warmup 3 --no-cpu --graph > $O/cfg4t_single.json 2> $O/cfg4t_single.err || exit $?
NFX_LIB=$R/normalizing-flows-study_amd/nfs_amd/libnfx_wgdb.so timeout -k 10 300 python bench.py --config cfg4t --steps 10 --warmup 3 --no-cpu --graph > $O/cfg4t_double.json 2> $O/cfg4t_double.err || exit $?
for f in single double; do python -c "
import json,sys; d=json.loads(open('$O/cfg4t_$f.json').read().strip().splitlines()[-1]); w=d['roofline'].get('wgrad',{})
print('$f', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,1), 'M/s', 'bwd', round(d['roofline']['mean_launch_ms']*1e3,1), 'us', 'wgrad', round(w.get('mean_launch_ms',0)*1e3,1), 'us')"; done
