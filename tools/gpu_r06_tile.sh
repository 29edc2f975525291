#!/bin/bash
# Round 6: small-batch MADE — the tile kernel spread over more CUs (libnfx_tile1.so: weights
# staged in LDS, libnfx_tile0.so: read from L2) against the shipped libnfx.so, MADE parity on the
# variant, and the sequential policies over d on the shipped library.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06tile; mkdir -p $O; cd $R
NL=$R/normalizing-flows-study_amd/nfs_amd
NFX_LIB=$NL/libnfx_tile0.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_made.py > $O/tests_tile0.log 2>&1 || { tail -30 $O/tests_tile0.log; exit 1; }
tail -1 $O/tests_tile0.log
for rep in 1 2; do
  for lib in libnfx libnfx_tile1 libnfx_tile0; do
    NFX_LIB=$NL/$lib.so timeout -k 10 200 python tools/made_small_sweep.py --par >> $O/par.jsonl 2> $O/par_$lib.err || exit $?
  done
done
timeout -k 10 400 python tools/made_small_sweep.py --seq > $O/seq.jsonl 2> $O/seq.err || exit $?
for lib in libnfx libnfx_tile0; do
  NFX_LIB=$NL/$lib.so timeout -k 10 200 python tools/made_sample_timing.py > $O/sample_$lib.jsonl 2>&1 || exit $?
done
python - <<'PY'
import json, collections
O = "gpurun_out/r06tile"
par = collections.defaultdict(list)
for l in open(f"{O}/par.jsonl"):
    r = json.loads(l); par[(r["d"], r["B"], r["lib"])].append(r["us"])
for (d, B, lib), v in sorted(par.items()):
    print("par", d, B, lib, min(v))
seq = [json.loads(l) for l in open(f"{O}/seq.jsonl")]
for r in seq:
    print("seq", r["d"], r["B"], r["policy"], r["us"])
PY
