"""Time the fused spline backward kernel alone (HIP events on the launch stream).

    NFX_LIB=expt/libnfx_1.so python tools/spline_bwd_bench.py [B] [K] [H] [dir]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-study_amd")]
import nfs_amd  # noqa: E402
from nfs_amd.flows import spline as sp  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
H = int(sys.argv[3]) if len(sys.argv) > 3 else 64
direction = int(sys.argv[4]) if len(sys.argv) > 4 else -1
dev = torch.device("cuda:0")
torch.manual_seed(0)
f = nfs_amd.SplineCouplingLayer(2, H, torch.tensor([1.0, 0.0]), num_bins=K)
with torch.no_grad():
    for p in f.parameters():
        p.add_(0.1 * torch.randn(p.shape))
f = f.to(dev)
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(B, 2, device=dev, generator=g)
gy = torch.randn(B, 2, device=dev, generator=g)
gld = torch.randn(B, device=dev, generator=g)
for _ in range(3):
    f._hip_backward(x, gy, gld, direction)
sp.BACKWARD_EVENTS = []
for _ in range(20):
    f._hip_backward(x, gy, gld, direction)
torch.cuda.synchronize()
ms = [a.elapsed_time(b) for _, a, b in sp.BACKWARD_EVENTS]
sp.BACKWARD_EVENTS = None
ms.sort()
print(f"{os.environ.get('NFX_LIB', 'libnfx.so')}: B={B} K={K} H={H} dir={direction} "
      f"median {ms[len(ms) // 2] * 1e3:.1f} us  min {ms[0] * 1e3:.1f} us")
