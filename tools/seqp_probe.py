"""IAF(784, 64) fused log_prob through one sequential-MADE kernel (nfx_made_seq_policy), repeated,
for rocprofv3 counter passes:  python tools/seqp_probe.py <policy: wave|segment|push> [B] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import torch  # noqa: E402
import nfs_amd  # noqa: E402
from nfs_amd import _lib  # noqa: E402

pol = {"wave": _lib.NFX_MADE_SEQ_WAVE, "segment": _lib.NFX_MADE_SEQ_SEGMENT, "push": _lib.NFX_MADE_SEQ_PUSH}[sys.argv[1]]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
d, H = 784, 64
torch.manual_seed(0)
f = nfs_amd.InverseAutoregressiveFlow(d, H)
with torch.no_grad():
    for p in f.parameters():
        p.add_(0.05 * torch.randn_like(p))
m = nfs_amd.NormalizingFlowModel([f]).cuda().eval()
_lib.lib().nfx_made_seq_policy(pol)
x = torch.randn(B, d, device="cuda")
with torch.no_grad():
    for _ in range(reps):
        m.log_prob(x, return_sums=True)
torch.cuda.synchronize()
print("done", sys.argv[1], B, reps)
