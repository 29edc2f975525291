#!/bin/bash
# Round 6 rebuild: the default bench line (as the driver runs it) and the --gpus 2 launcher rehearsal
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06final3_bench; mkdir -p $O; cd $R
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/default.json 2> $O/default.err || exit $?
NFX_BENCH_REHEARSE=1 timeout -k 10 300 python3 bench.py --gpus 2 --config cfg2 --steps 10 --warmup 3 --no-cpu > $O/gpus2_rehearse.json 2> $O/gpus2_rehearse.err || exit $?
timeout -k 10 300 python3 bench.py --config cfg5i --batch 1024 --steps 20 --warmup 5 --no-cpu > $O/cfg5i_1024.json 2> $O/cfg5i_1024.err || exit $?
timeout -k 10 300 python3 bench.py --config cfg2t --graph --steps 20 --warmup 5 > $O/cfg2t.json 2> $O/cfg2t.err || exit $?
python3 - <<PY
import json
for f in ("default", "gpus2_rehearse", "cfg5i_1024", "cfg2t"):
    d = json.loads(open("$O/%s.json" % f).read().strip().splitlines()[-1])
    rp = d["roofline"].get("rocprof") or {}
    print(f, d["n_gpus"], d.get("world_size"), round(d["value"] / 1e6, 2), "M/s", round(d["roofline"]["frac"], 3),
          "busy", rp.get("mfma_busy_frac"), "stale", rp.get("stale"))
PY
for c in sample4k sample4k_fused sample4k_spline sample4k_spline_fused sample4k_maf sample4k_iaf; do
  timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 > $O/$c.json 2> $O/$c.err || exit $?
  python -c "
import json; d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$c', round(d['ms_per_step']*1e3,1), 'us/step', round(d['value']/1e6,2), 'M/s', 'vs_baseline', round(d['vs_baseline'],1), r['kernel'], round(r['mean_launch_ms']*1e3,1), 'us kernel')"
done
