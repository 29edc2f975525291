"""Sequential IAF(784, 64) inverse (cfg5i shape) + fused Gaussian log_prob: kernel time per
batch size for each sequential-MADE kernel (nfx_made_seq_policy: wave-per-sample made_seqw_kernel
vs segment-parallel made_seqs_kernel vs push made_seqp_kernel), HIP events around the log_prob call.

    python tools/seq_batch_sweep.py [B ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import torch  # noqa: E402
import nfs_amd  # noqa: E402
from nfs_amd import _lib  # noqa: E402

d, H = 784, 64
torch.manual_seed(0)
f = nfs_amd.InverseAutoregressiveFlow(d, H)
with torch.no_grad():
    for p in f.parameters():
        p.add_(0.05 * torch.randn_like(p))
m = nfs_amd.NormalizingFlowModel([f]).cuda().eval()
L = _lib.lib()
batches = [int(b) for b in sys.argv[1:]] or [256, 512, 1024, 2048, 4096, 8192, 16384, 32768]
for B in batches:
    x = torch.randn(B, d, device="cuda")
    row = {"B": B}
    for name, pol in (("wave", _lib.NFX_MADE_SEQ_WAVE), ("segment", _lib.NFX_MADE_SEQ_SEGMENT),
                      ("push", _lib.NFX_MADE_SEQ_PUSH)):
        L.nfx_made_seq_policy(pol)
        with torch.no_grad():
            for _ in range(2):
                m.log_prob(x, return_sums=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                m.log_prob(x, return_sums=True)
            e1.record()
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        row[name + "_us"] = round(ms * 1e3, 1)
        row[name + "_Msps"] = round(B / ms / 1e3, 2)
    print(json.dumps(row), flush=True)
L.nfx_made_seq_policy(_lib.NFX_MADE_SEQ_AUTO)
