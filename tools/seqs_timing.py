"""Per-stage clock64 breakdown of the sequential MADE kernel (cfg5i shape, IAF(784, 64) inverse,
B = 8 Ki) from a timing build (-DNFX_SEQS_TIMING: workgroup 0's first lane writes its accumulated
stage cycles into sample 0's first outputs; results are otherwise unchanged).
    NFX_LIB=tools/expt_lib/libnfx_timing.so python tools/seqs_timing.py
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
names = ["chunk start + dot products + row reads", "affine map, poison ballot, step stores",
         "row broadcasts + rank-1 updates", "completion (layers 1-3)", "block: log-det sums + output rows",
         "block: vmcnt(0) + barrier", "block start: tile, block end, DMA + x issue"]
for B in (8192, 2048):
    x = torch.randn(B, d, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            z, _ = f.inverse(x)
        torch.cuda.synchronize()
    t = z[0, :7].double().cpu().tolist()
    tot = sum(t)
    print(f"B={B}: total {tot:.0f} clock64 ticks for workgroup 0's wave 0 ({tot / 65:.0f} per chunk over ~65 chunks)")
    for n, v in zip(names, t):
        print(f"  {n:42s} {v:10.0f}  {100 * v / max(tot, 1):5.1f} %")
