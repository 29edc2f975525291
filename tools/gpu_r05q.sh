set -o pipefail
out=gpurun_out/r05q; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_made_backward.py tests/test_gpu_grad_fixtures.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config cfg4t --graph --steps 20 --warmup 5 --no-cpu > $out/bench_cfg4t.json 2> $out/bench_cfg4t.err || exit $?
python -c "
import json; d=json.loads(open('$out/bench_cfg4t.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['mean_launch_ms'], r.get('wgrad'))"
timeout -k 10 300 python bench.py --config cfg2t --graph --steps 10 --warmup 3 --no-cpu > $out/bench_cfg2t.json 2> $out/bench_cfg2t.err || exit $?
python -c "
import json; d=json.loads(open('$out/bench_cfg2t.json').read().strip().splitlines()[-1]); print('cfg2t', d['value'], d['ms_per_step'])"
