#!/usr/bin/env bash
# Stall-breakdown counters of bench.py per config (one --pmc pass, kernel trace only).
#   bash tools/profile_stalls.sh <tag> [cfg...]
set -o pipefail
tag="$1"; shift
cfgs="${*:-cfg2 cfg3 cfg4}"
root="${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
out="$root/gpurun_out/stall_$tag"
mkdir -p "$out"
cd /tmp || exit 1
for c in $cfgs; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$out/$c" -- \
    python3 "$root/bench.py" --config "$c" --steps 3 --warmup 1 --no-cpu > "$out/$c.log" 2>&1 || exit $?
  echo "stalls $c"
done
