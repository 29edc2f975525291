set -o pipefail
out=gpurun_out/r05aa; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spline_chain.py tests/test_gpu_spline.py tests/test_gpu_logprob.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for spec in "cfg3" "cfg3" "cfg3 --batch 125000"; do
  n=$(echo $spec | tr ' ' '_')
  timeout -k 10 300 python bench.py --config $spec --steps 50 --warmup 10 --no-cpu > $out/b_$n.json 2> $out/b_$n.err || exit $?
  python -c "
import json; d=json.loads(open('$out/b_$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', round(d['value']/1e6,1), round(d['ms_per_step']*1e3,1), r['kernel'], round(r['mean_launch_ms']*1e3,1), round(r['frac'],3))"
done
