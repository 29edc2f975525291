set -e
cd $GRAFT_REPO_ROOT
for c in cfg2t cfg4t; do
  timeout -k 10 240 python -u bench.py --config $c --steps 10 --warmup 3 > gpurun_out/b_$c.json 2> gpurun_out/b_$c.err
done
timeout -k 10 240 python -u bench.py --config train5k --graph --steps 50 --warmup 5 > gpurun_out/b_train5k_graph.json 2> gpurun_out/b_train5k_graph.err
