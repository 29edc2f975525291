"""Run only the sequential IAF(784, 64) inverse kernel (cfg5i shape) a few times, for PMC passes:
    rocprofv3 --kernel-trace --pmc <counters> -- python3 tools/seqs_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import torch  # noqa: E402
import nfs_amd  # noqa: E402

B = int(os.environ.get("PROBE_B", 8192))
d, H = int(os.environ.get("PROBE_D", 784)), int(os.environ.get("PROBE_H", 64))
torch.manual_seed(0)
f = nfs_amd.InverseAutoregressiveFlow(d, H)
with torch.no_grad():
    for p in f.parameters():
        p.add_(0.05 * torch.randn_like(p))
f = f.cuda().eval()
x = torch.randn(B, d, device="cuda")
with torch.no_grad():
    for _ in range(int(os.environ.get("PROBE_ITERS", 5))):
        z, ld = f.inverse(x)
torch.cuda.synchronize()
print("ok", float(ld.float().mean()))
