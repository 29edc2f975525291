set -o pipefail
out=gpurun_out/r05b; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 env NFX_LIB=$PWD/normalizing-flows-study_amd/nfs_amd/libnfx_timing.so python -u tools/seqp_timing.py 1024 > $out/timing_1024.json 2>&1 || exit $?
timeout -k 10 120 env NFX_LIB=$PWD/normalizing-flows-study_amd/nfs_amd/libnfx_timing.so python -u tools/seqp_timing.py 256 > $out/timing_256.json 2>&1 || exit $?
cat $out/timing_*.json
root=$PWD
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $root/$out/pmc_push -- python3 $root/tools/seqp_probe.py push 1024 10 > $root/$out/pmc_push.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $root/$out/pmc_wave -- python3 $root/tools/seqp_probe.py wave 1024 10 > $root/$out/pmc_wave.log 2>&1 || exit $?
echo done
