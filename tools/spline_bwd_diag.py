"""Diagnostics for the fused spline backward: per-tensor error of the HIP gradients and of the
reference's fp32 composite against float64 autograd, per element for dL/dx."""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-study_amd"), os.path.join(ROOT, "tests")]
import nfs_amd  # noqa: E402
from test_gpu_spline_backward import _grads, _layer  # noqa: E402

dev = torch.device("cuda:0")
for (d, H, K, mask, B, direction) in [(2, 64, 8, [1, 0], 4096, -1), (2, 32, 5, [1, 0], 777, -1),
                                      (2, 64, 8, [1, 0], 1, -1), (2, 64, 8, [1, 0], 4096, 1)]:
    f = _layer(d, H, K, mask, d * 1000 + H * 10 + K)
    f64 = copy.deepcopy(f).double()
    g = torch.Generator().manual_seed(B + K)
    x = 2.0 * torch.randn(B, d, generator=g)
    if B >= 8:
        x[:4] *= 4.0
    gy = torch.randn(B, d, generator=g)
    gld = torch.randn(B, generator=g)
    gx64, gp64, y64, l64 = _grads(f64, x.double(), gy.double(), gld.double(), direction)
    gx32, gp32, _, _ = _grads(f, x, gy, gld, direction)
    gx, gp, _, _ = _grads(copy.deepcopy(f).to(dev), x.to(dev), gy.to(dev), gld.to(dev), direction)
    print(f"== d={d} H={H} K={K} B={B} dir={direction}")
    for name, a, b, c in [("gx", gx, gx32, gx64)] + list(zip([n for n, _ in f.named_parameters()], gp, gp32, gp64)):
        a, b, c = a.double().cpu(), b.double(), c.double()
        ea, eb = (a - c).abs(), (b - c).abs()
        print(f"  {name:20s} |g64|max {c.abs().max():.3e}  hip max {ea.max():.3e} mean {ea.mean():.3e}   "
              f"fp32-ref max {eb.max():.3e} mean {eb.mean():.3e}")
    ea = (gx.double().cpu() - gx64).abs()
    eb = (gx32.double() - gx64).abs()
    i = int(ea.sum(1).argmax())
    print("  worst gx row", i, "x", x[i].tolist(), "gx64", gx64[i].tolist(), "hip", gx[i].tolist(), "f32", gx32[i].tolist())
    print("  y64", y64[i].tolist(), "ld64", float(l64[i]))
