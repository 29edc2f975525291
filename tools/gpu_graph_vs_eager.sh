set -o pipefail
R=gpurun_out/r04_ge; mkdir -p $R
for spec in "cfg2 125000" "cfg3 125000" "cfg5i 1024" "cfg2 1000000"; do
  set -- $spec
  timeout -k 10 200 python -u bench.py --config $1 --batch $2 --steps 50 --warmup 10 --no-cpu --no-secondary > $R/${1}_${2}_graph.json 2>/dev/null || exit $?
  timeout -k 10 200 python -u bench.py --config $1 --batch $2 --eager --steps 50 --warmup 10 --no-cpu --no-secondary > $R/${1}_${2}_eager.json 2>/dev/null || exit $?
done
