#!/usr/bin/env bash
# Single-GPU proxies of the 8-way strong-scaling curve (run on the GPU box via gpurun):
# bench.py at each config's full batch and at its per-rank shard of an 8-GPU split, each under
# rocprofv3 --kernel-trace --stats (the kernel time per shard), no CPU baseline.
#   bash tools/gpu_r03_scaling.sh <tag>
# Writes gpurun_out/scal_<tag>/<cfg>_<B>.json (+ rocprof stats dirs).
set -o pipefail
tag="$1"
root="${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
out="$root/gpurun_out/scal_$tag"
mkdir -p "$out"
cd /tmp || exit 1
run() {  # cfg batch (a trailing x in the batch: one-launch coupling chain forced, NFX_CHAIN_MAX_B)
  local c="$1" b="${2%x}" tagb="$2"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${c}_${tagb}_prof" -- \
    python3 "$root/bench.py" --config "$c" --batch "$b" --steps 20 --warmup 5 --no-cpu --no-secondary \
    > "$out/${c}_${tagb}.json" 2> "$out/${c}_${tagb}.err" || return $?
  echo "done $c $tagb"
}
run_chain() { NFX_CHAIN_MAX_B=10000000 run "$@"; }
run cfg2 1000000 && run cfg2 125000 && run_chain cfg2 125000x && run cfg4 4000000 && run cfg4 500000 && \
run cfg5f 524288 && run cfg5f 65536 && run cfg5i 8192 && run cfg5i 1024 && run cfg3 1000000 && run cfg3 125000
