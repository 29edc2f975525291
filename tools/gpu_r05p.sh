set -o pipefail
out=gpurun_out/r05p; mkdir -p $out
bash tools/gpu_suite.sh r05p || exit $?
for spec in "cfg3" "cfg3 --batch 125000" "cfg5i --batch 1024"; do
  n=$(echo $spec | tr ' ' '_')
  timeout -k 10 300 python bench.py --config $spec --steps 20 --warmup 5 --no-cpu > $out/bench_$n.json 2> $out/bench_$n.err || exit $?
  tail -1 $out/bench_$n.json | cut -c1-400
done
bash tools/profile_bench.sh r05p --pmc cfg3
