#!/bin/bash
# Round 6: per-kernel rocprof of the cfg4t step, round-5 wgrad (wold) vs the new build (main) vs 2 tiles/task
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06f; mkdir -p $O; cd $R
L=$R/normalizing-flows-study_amd/nfs_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_made_backward.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for v in wold main t2s; do
  if [ $v = main ]; then lib=$L/libnfx.so; else lib=$L/libnfx_$v.so; fi
  cd /tmp
  NFX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -- python3 $R/bench.py --config cfg4t --steps 10 --warmup 3 --no-cpu --graph > $O/$v.json 2> $O/$v.err || exit $?
  cd $R
  python - <<PY
import csv, glob
f = sorted(glob.glob("$O/$v/*/*_kernel_stats.csv"))[-1]
for r in csv.DictReader(open(f)):
    if "wgrad" in r["Name"] or "sum_finish" in r["Name"] or "made_bwd" in r["Name"]:
        print("$v", r["Calls"], round(float(r["AverageNs"])/1e3, 1), "us", r["Name"][:70])
PY
done
