#!/bin/bash
# PMC passes over tools/seqs_probe.py (run on the GPU box); CSVs into gpurun_out/seqs_pmc/<pass>.
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
out="$root/gpurun_out/seqs_pmc"
mkdir -p "$out"
cd /tmp || exit 1
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d "$out/p$i" -- \
    python3 "$root/tools/seqs_probe.py" > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; exit 1; }
done
echo done
