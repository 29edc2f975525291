"""Throughput of the any-shape path (csrc/nfx_generic.hip) on layers beyond the fused families.

    python tools/generic_bench.py [--steps N] > profiles/<tag>_generic_bench.jsonl

One JSON line per case: ms per call (HIP events on torch's current stream, which the path
launches on), samples/s, and for the GEMM cases the achieved fp32 TFLOP/s against the dense
fp32 MFMA peak (157.3 TF/s) and the streamed bytes against HBM (8 TB/s). Synthetic data; weights
random-init of the named shapes. Not the headline bench (bench.py): a measurement of the
coverage path.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import nfs_amd  # noqa: E402
from nfs_amd.flows import generic as G  # noqa: E402

PEAK_TF, PEAK_GBS = 157.3, 8000.0


def timed(fn, steps, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--gemm-only", action="store_true", help="only the GEMM cases (profiling runs)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    out = []

    # 1) the GEMM alone: one conditioner layer's forward, data gradient and weight gradient
    for M, K, N in ((262144, 512, 512), (1 << 20, 128, 128), (1 << 20, 2, 256)):
        lin = torch.nn.Linear(K, N).to(dev)
        x = torch.randn(M, K, device=dev)
        gy = torch.randn(M, N, device=dev)
        fl = 2.0 * M * K * N
        for name, fn, nbytes in (
                ("linear_forward", lambda: G.linear_forward(x, lin, relu=True), 4.0 * M * (K + N)),
                ("linear_backward_data", lambda: G.linear_backward_data(gy, lin), 4.0 * M * (K + N)),
                ("linear_backward_weight", lambda: G.linear_backward_weight(gy, x, lin), 4.0 * M * (K + N))):
            ms = timed(fn, a.steps)
            tf = fl / (ms * 1e-3) / 1e12
            gbs = nbytes / (ms * 1e-3) / 1e9
            out.append({"case": f"{name} M={M} K={K} N={N}", "ms": ms, "tflops": tf, "frac_mfma": tf / PEAK_TF,
                        "gbs_streamed": gbs, "frac_hbm": gbs / PEAK_GBS})

    # 2) whole layers beyond the fused families
    B = 262144
    cases = []
    if a.gemm_only:
        for o in out:
            print(json.dumps(o), flush=True)
        return
    m = nfs_amd.MaskedAutoregressiveFlow(63, 512).to(dev).eval()
    cases.append(("MAF(63,512) inverse (log-density direction), eval", m, B, -1, False))
    c = nfs_amd.CouplingLayer(2, 256, torch.tensor([1.0, 0.0])).to(dev).eval()
    cases.append(("CouplingLayer(2,256) inverse, eval", c, 1 << 20, -1, False))
    s = nfs_amd.SplineCouplingLayer(2, 128, torch.tensor([1.0, 0.0]), num_bins=10).to(dev).eval()
    cases.append(("SplineCouplingLayer(2,128,K=10) inverse + backward (training step body)", s, B, -1, True))
    s4 = nfs_amd.SplineCouplingLayer(4, 64, torch.tensor([1.0, 0.0, 1.0, 0.0]), num_bins=8).to(dev).eval()
    cases.append(("SplineCouplingLayer(4,64,K=8) inverse + backward (2 transformed dims)", s4, B, -1, True))
    for what, layer, n, direction, bwd in cases:
        x = torch.randn(n, layer.data_dim, device=dev)
        if bwd:
            def fn():
                xr = x.requires_grad_(True)
                y, ld = layer.inverse(xr) if direction < 0 else layer.forward(xr)
                (y.sum() + ld.sum()).backward()
        else:
            def fn():
                with torch.no_grad():
                    layer.inverse(x) if direction < 0 else layer.forward(x)
        nfs_amd.reset_stats()
        ms = timed(fn, a.steps)
        assert nfs_amd.STATS["torch"] == 0, nfs_amd.STATS
        out.append({"case": what, "batch": n, "ms": ms, "samples_per_s": n / (ms * 1e-3)})
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
