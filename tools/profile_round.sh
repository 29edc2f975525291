#!/usr/bin/env bash
# Kernel-trace + PMC profiles of bench.py per config (run on the GPU box via gpurun).
#   bash tools/profile_round.sh <tag> [cfg2 cfg3 cfg4]
# Writes gpurun_out/prof_<tag>/<cfg>/{trace,fetch,write,sq}/... (CSV). Counter passes are
# separate runs with --kernel-trace only (FETCH_SIZE and WRITE_SIZE do not fit one pass).
set -o pipefail
tag="$1"; shift
cfgs="${*:-cfg2 cfg3 cfg4}"
root="${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
out="$root/gpurun_out/prof_$tag"
mkdir -p "$out"
cd /tmp || exit 1
for c in $cfgs; do
  d="$out/$c"
  mkdir -p "$d"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/trace" -- \
    python3 "$root/bench.py" --config "$c" --steps 10 --warmup 3 --no-cpu --no-secondary > "$d/trace.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$d/fetch" -- \
    python3 "$root/bench.py" --config "$c" --steps 3 --warmup 1 --no-cpu --no-secondary > "$d/fetch.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$d/write" -- \
    python3 "$root/bench.py" --config "$c" --steps 3 --warmup 1 --no-cpu --no-secondary > "$d/write.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$d/sq" -- \
    python3 "$root/bench.py" --config "$c" --steps 3 --warmup 1 --no-cpu --no-secondary > "$d/sq.log" 2>&1 || exit $?
  echo "profiled $c"
done
