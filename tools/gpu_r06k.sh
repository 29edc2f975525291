#!/bin/bash
# Round 6: the fused-draw sampling lines next to the plain sampling lines
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06k; mkdir -p $O; cd $R
for c in sample4k sample4k_fused sample4k_spline sample4k_spline_fused; do
  timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 > $O/$c.json 2> $O/$c.err || exit $?
  python -c "
import json; d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$c', round(d['ms_per_step']*1e3,1), 'us/step', round(d['value']/1e6,2), 'M/s', 'vs_baseline', round(d['vs_baseline'],1), r['kernel'], round(r['mean_launch_ms']*1e3,1), 'us kernel', d['config']['launch'])"
done
