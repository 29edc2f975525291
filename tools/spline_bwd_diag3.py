"""Row-error quantiles of dL/dx vs float64: HIP kernel, CPU fp32 composite, GPU fp32 composite."""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-study_amd"), os.path.join(ROOT, "tests")]
import nfs_amd  # noqa: E402
from test_gpu_spline_backward import _grads, _layer  # noqa: E402

dev = torch.device("cuda:0")


def comp_grads(f, x, gy, gld, direction):
    x = x.clone().requires_grad_(True)
    y, ld = f._torch_call(x, direction)
    ((y * gy).sum() + (ld * gld).sum()).backward()
    return x.grad


for (d, H, K, mask, B) in [(2, 64, 10, [0, 1], 1000), (2, 64, 8, [1, 0], 4096), (2, 32, 5, [1, 0], 777)]:
    for direction in (1, -1):
        f = _layer(d, H, K, mask, d * 1000 + H * 10 + K)
        f64 = copy.deepcopy(f).double()
        g = torch.Generator().manual_seed(B + K)
        x = 2.0 * torch.randn(B, d, generator=g)
        x[:4] *= 4.0
        gy = torch.randn(B, d, generator=g)
        gld = torch.randn(B, generator=g)
        gx64, _, _, _ = _grads(f64, x.double(), gy.double(), gld.double(), direction)
        gx32, _, _, _ = _grads(f, x, gy, gld, direction)
        fg = copy.deepcopy(f).to(dev)
        gx, _, _, _ = _grads(fg, x.to(dev), gy.to(dev), gld.to(dev), direction)
        gxc = comp_grads(fg, x.to(dev), gy.to(dev), gld.to(dev), direction)
        print(f"== d={d} H={H} K={K} B={B} dir={direction}")
        for name, a in (("cpu32", gx32), ("hip", gx), ("gpu-composite", gxc)):
            e = ((a.double().cpu() - gx64).abs() / (1 + gx64.abs())).max(1).values
            print(f"  {name:14s}" + " ".join(f"q{q}={e.quantile(q).item():.2e}" for q in (0.5, 0.9, 0.99, 1.0)))
