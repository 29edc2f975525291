set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/${1:-gemmprof}
mkdir -p $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/trace -- python3 $GRAFT_REPO_ROOT/tools/generic_bench.py --gemm-only > $R/bench.jsonl 2> $R/trace.err || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $R/pmc1 -- python3 $GRAFT_REPO_ROOT/tools/generic_bench.py --gemm-only --steps 2 > $R/pmc1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA TA_BUSY_avr --output-format csv -d $R/pmc2 -- python3 $GRAFT_REPO_ROOT/tools/generic_bench.py --gemm-only --steps 2 > $R/pmc2.log 2>&1
echo done
