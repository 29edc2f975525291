set -o pipefail
out=gpurun_out/r05v; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "train or backward or grad or fig or options or step" > $out/tests.log 2>&1
rc=$?; tail -15 $out/tests.log | grep -v "^$"
for c in cfg4t cfg2t; do
timeout -k 10 300 python bench.py --config $c --graph --steps 10 --warmup 3 --no-cpu > $out/bench_$c.json 2> $out/bench_$c.err || exit $?
python -c "
import json; d=json.loads(open('$out/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'])"
done
exit $rc
