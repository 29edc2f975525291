set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r1; mkdir -p $O
export TMPDIR=/tmp
cd $R
for c in sample4k sample4k_spline sample4k_maf sample4k_iaf; do
  timeout -k 10 120 python bench.py --config $c --steps 200 --warmup 20 > $O/bench_${c}_eager.json 2>$O/bench_${c}_eager.err || exit 1
  timeout -k 10 120 python bench.py --config $c --steps 200 --warmup 20 --graph --no-cpu > $O/bench_${c}_graph.json 2>$O/bench_${c}_graph.err || exit 1
  echo "done $c"
done
cd /tmp
for c in sample4k cfg4t; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -- python3 $R/bench.py --config $c --steps 20 --warmup 5 --no-cpu > $O/prof_$c.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_arqs -- python3 $R/tools/arqs_bench.py 10 1000000 > $O/prof_arqs.log 2>&1 || exit 1
echo ok
