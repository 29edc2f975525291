set -o pipefail
out=gpurun_out/r05x; mkdir -p $out
for spec in "cfg2 --batch 125000" "cfg2 --batch 125000 --eager" "cfg3 --batch 125000" "cfg3 --batch 125000 --eager" "cfg2" "cfg2 --eager" "cfg5i --batch 1024" "cfg5i --batch 1024 --eager"; do
  n=$(echo $spec | tr ' ' '_')
  timeout -k 10 300 python bench.py --config $spec --steps 50 --warmup 10 --no-cpu --no-secondary > $out/b_$n.json 2> $out/b_$n.err || exit $?
  python -c "
import json; d=json.loads(open('$out/b_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), d['config']['launch'])"
done
