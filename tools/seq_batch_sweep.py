"""Sequential IAF(784, 64) inverse (cfg5i shape): kernel time per batch size, HIP events around
the layer call.   python tools/seq_batch_sweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import torch  # noqa: E402
import nfs_amd  # noqa: E402

d, H = 784, 64
torch.manual_seed(0)
f = nfs_amd.InverseAutoregressiveFlow(d, H)
with torch.no_grad():
    for p in f.parameters():
        p.add_(0.05 * torch.randn_like(p))
f = f.cuda().eval()
for B in (8192, 16384, 32768, 65536):
    x = torch.randn(B, d, device="cuda")
    with torch.no_grad():
        for _ in range(2):
            f.inverse(x)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f.inverse(x)
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"B={B} {ms:.3f} ms {B / ms / 1e3:.1f} M samples/s", flush=True)
