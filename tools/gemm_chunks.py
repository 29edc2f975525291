"""Timing of the split-K sample GEMM (factors [M, B] x [N, B]^T) for several chunk sizes."""
import sys, time
sys.path.insert(0, "normalizing-flows-study_amd")
import torch
from nfs_amd.flows.autoregressive import _sample_gemm
dev = torch.device("cuda:0")
B = 500000
for M, N in ((126, 65), (64, 65), (64, 64)):
    a = torch.randn(M, B, device=dev); b = torch.randn(N, B, device=dev)
    ref = (a.double() @ b.double().t()).float()
    for chunk in (2048, 4096, 8192, 16384, 32768, 10**9):
        f = (lambda: a @ b.t()) if chunk == 10**9 else (lambda: _sample_gemm(a, b, chunk))
        for _ in range(3): f()
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(20): out = f()
        torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 20
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        print(f"M={M} N={N} chunk={chunk:>10} {dt*1e6:8.1f} us {2*M*N*B/dt/1e12:6.1f} TF err {err:.1e}")
