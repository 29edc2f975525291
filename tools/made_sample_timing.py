"""Per-layer kernels of the reference's MADE sampling figure models (6x IAF(2,64) forward =
parallel, 6x MAF(2,64) forward = sequential) at n = 4,000: kernel name and event-timed launch per
layer, per sequential policy for MAF.
    python tools/made_sample_timing.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import nfs_amd  # noqa: E402
from nfs_amd import _lib  # noqa: E402

n = 4000
for kind in ("iaf", "maf"):
    torch.manual_seed(7)
    cls = nfs_amd.InverseAutoregressiveFlow if kind == "iaf" else nfs_amd.MaskedAutoregressiveFlow
    m = nfs_amd.NormalizingFlowModel([cls(2, 64) for _ in range(6)]).cuda().eval()
    z = torch.randn(n, 2, device="cuda")
    pols = [("auto", _lib.NFX_MADE_SEQ_AUTO)] if kind == "iaf" else [
        ("auto", _lib.NFX_MADE_SEQ_AUTO), ("segment", _lib.NFX_MADE_SEQ_SEGMENT), ("wave", _lib.NFX_MADE_SEQ_WAVE),
        ("push", _lib.NFX_MADE_SEQ_PUSH)]
    for name, pol in pols:
        _lib.lib().nfx_made_seq_policy(pol)
        with torch.no_grad():
            for _ in range(5):
                m.forward(z)
            rec = []
            m.layer_events = rec
            for _ in range(20):
                m.forward(z)
            m.layer_events = None
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                m.forward(z)
            e1.record()
            torch.cuda.synchronize()
        ks = sorted({k for k, _, _ in rec})
        per = sum(a.elapsed_time(b) for _, a, b in rec) / len(rec) * 1e3
        print(json.dumps({"model": f"6x{kind.upper()}(2,64)", "policy": name, "kernels": ks, "layer_us": round(per, 1),
                          "forward_us": round(e0.elapsed_time(e1) / 50 * 1e3, 1)}), flush=True)
_lib.lib().nfx_made_seq_policy(_lib.NFX_MADE_SEQ_AUTO)
