"""ARQS throughput: ARQS(d, 128, K=8) forward/inverse on the GPU kernel vs the CPU oracle.

    python tools/arqs_bench.py [d] [B]
"""
import os
import sys
import time

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_ROOT, "normalizing-flows-study_amd"))
sys.path.insert(0, _ROOT)
import torch
import nfs_amd
import oracle

d = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = nfs_amd.ARQS(d, 128, num_bins=8)
with torch.no_grad():
    for p in m.parameters():
        p.add_(0.3 * torch.randn(p.shape))
m = m.to(dev).eval()
x = torch.rand(B, d, device=dev)
H, R = 128, 23
flop = d * 2 * (2 * H * H + 32 * H)  # MFMA flops per sample (layers 2-3 + one 32-row output tile per step)
for name, fn in (("forward", m.forward), ("inverse", m.inverse)):
    with torch.no_grad():
        fn(x)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            fn(x)
        e.record()
        torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 5
    print(f"ARQS({d},128,K=8) {name} B={B}: {ms:.3f} ms, {B / ms / 1e3:.1f} M samples/s, "
          f"{flop * B / ms / 1e9:.1f} TFLOP/s MFMA-algorithmic", flush=True)
sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
torch.set_num_threads(16)
xs = x[:4000].cpu()
t0 = time.perf_counter()
with torch.no_grad():
    oracle.arqs(sd, "", xs, 1, K=8)
t = time.perf_counter() - t0
print(f"CPU oracle (16 threads) forward 4000 rows: {t:.3f} s = {4000 / t / 1e3:.1f} k samples/s", flush=True)
