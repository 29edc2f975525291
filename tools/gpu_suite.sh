#!/usr/bin/env bash
# The whole GPU test suite in one process, then smoke (run on the GPU box via gpurun):
#   bash tools/gpu_suite.sh <tag>   -> gpurun_out/<tag>/{tests.log,smoke.txt}
set -o pipefail
tag="$1"
root="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$root/gpurun_out/$tag"
mkdir -p "$out"
cd "$root" || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
rc=$?
tail -3 "$out/tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1
rc=$?
cat "$out/smoke.txt"
exit $rc
