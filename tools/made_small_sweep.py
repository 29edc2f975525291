"""Small-batch MADE layer timings, one JSON line each: the parallel direction (IAF forward, the
tile kernel for d <= 64) and the sequential direction (MAF forward) under each sequential policy,
over d and the batch. Event-timed mean of one layer's forward over 50 calls after 10 warm-ups.
The library is whatever NFX_LIB names (default: the in-tree libnfx.so).
    python tools/made_small_sweep.py [--seq] [--par]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import nfs_amd  # noqa: E402
from nfs_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seq", action="store_true")
ap.add_argument("--par", action="store_true")
ap.add_argument("--tag", default=os.path.basename(os.environ.get("NFX_LIB", "libnfx.so")))
a = ap.parse_args()


def timed(m, x, reps=50):
    with torch.no_grad():
        for _ in range(10):
            m(x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            m(x)
        e1.record()
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def emit(**kw):
    print(json.dumps(dict(lib=a.tag, **kw)), flush=True)


L = _lib.lib()
if a.par:
    for d in (2, 8, 32, 63):
        torch.manual_seed(d)
        m = nfs_amd.InverseAutoregressiveFlow(d, 64).cuda().eval()
        for B in (256, 1024, 4000, 16384, 65536):
            x = torch.randn(B, d, device="cuda")
            emit(kind="iaf_forward", d=d, B=B, us=round(timed(m, x), 2))
if a.seq:
    pols = (("segment", _lib.NFX_MADE_SEQ_SEGMENT), ("wave", _lib.NFX_MADE_SEQ_WAVE),
            ("push", _lib.NFX_MADE_SEQ_PUSH), ("auto", _lib.NFX_MADE_SEQ_AUTO))
    for d in (2, 4, 8, 16, 32, 63, 128, 256, 784):
        torch.manual_seed(d)
        m = nfs_amd.MaskedAutoregressiveFlow(d, 64).cuda().eval()
        for B in (256, 1024, 4000):
            x = torch.randn(B, d, device="cuda")
            for name, pol in pols:
                L.nfx_made_seq_policy(pol)
                emit(kind="maf_forward", d=d, B=B, policy=name, us=round(timed(m, x, 20 if d >= 256 else 50), 2))
    L.nfx_made_seq_policy(_lib.NFX_MADE_SEQ_AUTO)
