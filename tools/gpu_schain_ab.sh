# A/B of the streaming chains' wave count (CFG=cfg2|cfg3, WAVES="0 8 12") (run on the GPU box via gpurun):
#   bash tools/gpu_schain_ab.sh <tag>  -> gpurun_out/<tag>/{tests.log,*.json}
set -o pipefail
R=gpurun_out/${1:-schain_ab}; mkdir -p $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_spline.py tests/test_gpu_spline_chain.py > $R/tests.log 2>&1 || exit $?
for w in ${WAVES:-0 8 12}; do
  NFX_SCHAIN_WAVES=$w timeout -k 10 200 python -u bench.py --config ${CFG:-cfg3} --batch 125000 --graph --steps 50 --warmup 10 --no-cpu --no-secondary > $R/${CFG:-cfg3}_125k_w$w.json 2> $R/err_125k_$w.log || exit $?
  NFX_SCHAIN_WAVES=$w timeout -k 10 200 python -u bench.py --config ${CFG:-cfg3} --steps 20 --warmup 5 --no-cpu --no-secondary > $R/${CFG:-cfg3}_w$w.json 2> $R/err_1m_$w.log || exit $?
done
