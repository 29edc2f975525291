set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_made.py tests/test_gpu_logprob.py tests/test_gpu_relational.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_made.log 2>&1 || { tail -30 gpurun_out/t_made.log; exit 1; }
tail -3 gpurun_out/t_made.log
timeout -k 10 300 python -u bench.py --config cfg5i > gpurun_out/b_cfg5i.json 2> gpurun_out/b_cfg5i.err || exit 1
cat gpurun_out/b_cfg5i.json
