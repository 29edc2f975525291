#!/usr/bin/env bash
# rocprofv3 around bench.py ITSELF (no launcher hop), one config per run, so the kernel trace and
# the bench line's ms_per_step come from one process and one clock (run on the GPU box via gpurun):
#   bash tools/profile_bench.sh <tag> [--pmc] <cfg>[:<batch>][+graph] ...
# Writes gpurun_out/prof_<tag>/<cfg>[_<batch>]/{trace/,bench.json,fetch/,write/,mfma/}. The PMC passes
# (FETCH_SIZE, WRITE_SIZE: they do not fit one pass; the MFMA-busy / instruction-mix / clock pass)
# are separate runs with --kernel-trace only.
# Reconcile afterwards on the CPU: python tools/reconcile_profile.py gpurun_out/prof_<tag> <round tag>
set -o pipefail
tag="$1"; shift
pmc=0
if [ "$1" = "--pmc" ]; then pmc=1; shift; fi
root="${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
out="$root/gpurun_out/prof_$tag"
mkdir -p "$out"
cd /tmp || exit 1
for spec0 in "$@"; do
  spec="${spec0%+graph}"   # a trailing +graph: replay the captured training step (--graph)
  c="${spec%%:*}"
  b=""
  name="$c"
  if [ "$spec" != "$c" ]; then b="${spec#*:}"; name="${c}_$b"; fi
  extra=()
  if [ -n "$b" ]; then extra=(--batch "$b"); fi
  if [ "$spec0" != "$spec" ]; then extra+=(--graph); fi
  d="$out/$name"
  rm -rf "$d"
  mkdir -p "$d"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/trace" -- \
    python3 "$root/bench.py" --config "$c" "${extra[@]}" --steps 20 --warmup 5 --no-cpu --no-secondary \
    > "$d/bench.json" 2> "$d/trace.err" || exit $?
  if [ "$pmc" = 1 ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$d/fetch" -- \
      python3 "$root/bench.py" --config "$c" "${extra[@]}" --steps 3 --warmup 1 --no-cpu --no-secondary \
      > "$d/fetch.log" 2>&1 || exit $?
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$d/write" -- \
      python3 "$root/bench.py" --config "$c" "${extra[@]}" --steps 3 --warmup 1 --no-cpu --no-secondary \
      > "$d/write.log" 2>&1 || exit $?
    # MFMA pipe busy cycles, instruction mix and the clock (GRBM_GUI_ACTIVE over the 8 XCDs)
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE \
      --output-format csv -d "$d/mfma" -- \
      python3 "$root/bench.py" --config "$c" "${extra[@]}" --steps 3 --warmup 1 --no-cpu --no-secondary \
      > "$d/mfma.log" 2>&1 || exit $?
  fi
  echo "profiled $name"
done
