set -o pipefail
root="${GRAFT_REPO_ROOT:-$(pwd)}"; out="$root/gpurun_out/w5"; mkdir -p "$out"
timeout -k 10 400 python3 -u -m pytest "$root/tests/test_gpu_made.py" "$root/tests/test_gpu_logprob.py" "$root/tests/test_gpu_relational.py" "$root/tests/test_gpu_lds_poison.py" -q --timeout 300 --timeout-method thread > "$out/t.log" 2>&1 || exit $?
echo tests done
for b in 65536 524288 131072; do
  timeout -k 10 200 python3 "$root/bench.py" --config cfg5f --batch $b --no-cpu --steps 30 --warmup 5 > "$out/cfg5f_$b.json" 2> "$out/cfg5f_$b.err" || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof64k" -- python3 "$root/bench.py" --config cfg5f --batch 65536 --no-cpu --steps 20 --warmup 5 > "$out/prof64k.log" 2>&1 || exit $?
echo done
