set -o pipefail
out=gpurun_out/r05y; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_made.py tests/test_gpu_logprob.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/seqp_debug.py > $out/debug.txt 2>&1 || exit $?; grep badz $out/debug.txt
timeout -k 10 300 python -u tools/seq_batch_sweep.py 256 1024 2048 4096 8192 > $out/sweep.jsonl 2>&1 || exit $?
grep push $out/sweep.jsonl
