set -o pipefail
root=$PWD
out=$root/gpurun_out/r05z; mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU --output-format csv -d $out/pmc1 -- python3 $root/bench.py --config cfg2t --steps 2 --warmup 1 --no-cpu > $out/pmc1.log 2>&1; echo "pmc1 rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $out/pmc2 -- python3 $root/bench.py --config cfg2t --steps 2 --warmup 1 --no-cpu > $out/pmc2.log 2>&1; echo "pmc2 rc=$?"
