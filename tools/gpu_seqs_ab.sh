set -o pipefail
R=gpurun_out/${1:-seqs_ab}; mkdir -p $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_made.py > $R/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/seq_batch_sweep.py 1024 8192 16384 > $R/sweep.jsonl 2>&1 || exit $?
NFX_LIB=$PWD/normalizing-flows-study_amd/nfs_amd/libnfx_timing.so timeout -k 10 200 python -u tools/seqs_timing.py 8192 > $R/timing.jsonl 2>&1 || exit $?
NFX_LIB=$PWD/normalizing-flows-study_amd/nfs_amd/libnfx_timing.so timeout -k 10 120 python -u tools/seqw_timing.py 1024 > $R/seqw_timing.jsonl 2>&1
