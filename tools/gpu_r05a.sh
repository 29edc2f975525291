set -o pipefail
mkdir -p gpurun_out/r05a
timeout -k 10 600 python -u -m pytest tests/test_gpu_made.py -x -q -k "push" --timeout 120 --timeout-method thread > gpurun_out/r05a/tests.log 2>&1
rc=$?
tail -30 gpurun_out/r05a/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/seq_batch_sweep.py 256 1024 2048 4096 8192 > gpurun_out/r05a/sweep.jsonl 2>&1
rc=$?
cat gpurun_out/r05a/sweep.jsonl
exit $rc
