#!/bin/bash
# Round 6: fused on-device base draw in the sampling chain — tests, then sample4k timing
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06g; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_sample.py tests/test_gpu_logprob.py tests/test_gpu_chain.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python - > $O/sample_timing.txt 2>&1 <<'PY'
import sys, torch
sys.path.insert(0, "normalizing-flows-study_amd"); sys.path.insert(0, ".")
import nfs_amd
from bench import perturb
torch.manual_seed(3); m = nfs_amd.RealNVP(2, 10, 128); perturb(m, 0.1, 4); m = m.cuda().eval()
n = 4000
with torch.no_grad():
    for mode in ("fused", "normal_+chain"):
        if mode == "fused":
            f = lambda: m.sample_fused(n)
        else:
            z = torch.empty(n, 2, device="cuda")
            f = lambda: m.forward(z.normal_())
        for _ in range(20): f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200): f()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 200 * 1e3
        print(f"{mode}: {us:.1f} us per {n}-sample draw+forward, {n / us:.1f} M samples/s")
    g = nfs_amd.GraphedFlow(m, torch.empty(n, 2, device="cuda"), mode="sample")
    for _ in range(20): g()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(200): g()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 200 * 1e3
    print(f"graph (fused_draw={g.fused_draw}, {g.launches} launch): {us:.1f} us, {n / us:.1f} M samples/s")
PY
rc=$?; cat $O/sample_timing.txt; exit $rc
