set -o pipefail
root=$PWD
out=$root/gpurun_out/r05r2; mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $out/pmc1 -- python3 $root/bench.py --config cfg4t --steps 2 --warmup 1 --no-cpu > $out/pmc1.log 2>&1; echo "pmc1 rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/pmc2 -- python3 $root/bench.py --config cfg4t --steps 2 --warmup 1 --no-cpu > $out/pmc2.log 2>&1; echo "pmc2 rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d $out/pmc3 -- python3 $root/bench.py --config cfg4t --steps 2 --warmup 1 --no-cpu > $out/pmc3.log 2>&1; echo "pmc3 rc=$?"
