#!/bin/bash
# Full GPU suite, default bench line, cfg5i bench line + rocprofv3 kernel stats and the
# sequential-kernel PMC passes (run on the GPU box): bash tools/gpu_r02_final.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --maxfail=25 --timeout 300 --timeout-method thread > $O/t_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $O/t_gpu.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 300 python -u bench.py --config cfg5i > $O/bench_cfg5i.json 2> $O/bench_cfg5i.err || exit $?
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg5i -- \
  python3 $R/bench.py --config cfg5i --steps 20 --warmup 3 --no-cpu --no-secondary > $O/prof_cfg5i.log 2>&1 || exit $?
bash $R/tools/seqs_pmc.sh > $O/seqs_pmc.log 2>&1 || exit $?
echo done
