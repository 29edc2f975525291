"""Debug: train-mode CouplingLayer HIP gradients vs float64 autograd, every parameter."""
import copy
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_ROOT, "normalizing-flows-study_amd"), _ROOT, os.path.join(_ROOT, "tests")]
import torch  # noqa: E402
from test_gpu_affine_train import _perturbed_layer  # noqa: E402

dev = torch.device("cuda:0")
for d, H, B, direction in [(2, 64, 1000, 1), (2, 64, 64, -1), (2, 32, 64, -1)]:
    layer = _perturbed_layer(d, H, 100 + d * 7 + H, True)
    ref = copy.deepcopy(layer).double().train()
    gpu = layer.to(dev).train()
    gen = torch.Generator().manual_seed(B)
    x = torch.randn(B, d, generator=gen) * 1.3 + 0.2
    wy = torch.randn(B, d, generator=gen)
    wl = torch.randn(B, generator=gen)
    xr = x.double().requires_grad_(True)
    yr, ldr = ref.forward(xr) if direction > 0 else ref.inverse(xr)
    ((yr * wy.double()).sum() + (ldr * wl.double()).sum()).backward()
    xg = x.to(dev).requires_grad_(True)
    yg, ldg = gpu.forward(xg) if direction > 0 else gpu.inverse(xg)
    ((yg * wy.to(dev)).sum() + (ldg * wl.to(dev)).sum()).backward()
    print(f"d={d} H={H} B={B} dir={direction}: y {((yg.cpu().double()-yr).abs().max()):.2e} "
          f"gx {((xg.grad.cpu().double()-xr.grad).abs().max() / xr.grad.abs().max()):.2e}")
    for (k, pg), (_, pr) in zip(gpu.named_parameters(), ref.named_parameters()):
        e = (pg.grad.cpu().double() - pr.grad).abs().max().item()
        print(f"   {k:16s} err {e:.3e}  max|ref| {pr.grad.abs().max().item():.3e}  max|gpu| {pg.grad.abs().max().item():.3e}")
