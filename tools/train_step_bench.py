"""Training-step timing of 5x MAF(63,64): fused HIP backward vs the composite (torch) backward."""
import sys, time
sys.path.insert(0, "normalizing-flows-study_amd"); sys.path.insert(0, ".")
import torch
import nfs_amd
from nfs_amd.flows import autoregressive as ar

dev = torch.device("cuda:0")
torch.manual_seed(0)
model = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(63, 64) for _ in range(5)]).to(dev).train()
opt = torch.optim.Adam(model.parameters(), lr=1e-4)
ar._MadeAffineFlow._orig_ok = ar._MadeAffineFlow._hip_backward_ok
for B in (65536, 500000):
    x = torch.randn(B, 63, device=dev)
    for mode in ("fused", "composite"):
        if mode == "composite":
            ar._MadeAffineFlow._hip_backward_ok = lambda self, x, d: False
        else:
            ar._MadeAffineFlow._hip_backward_ok = ar._MadeAffineFlow._orig_ok
        def step():
            opt.zero_grad(set_to_none=True)
            loss = -model.log_prob(x).mean()
            loss.backward()
            opt.step()
            return loss
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 10
        for _ in range(n):
            loss = step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        print(f"B={B} {mode:9s} {dt*1e3:8.2f} ms/step  {B/dt/1e6:8.2f} M samples/s  loss {loss.item():.4f}", flush=True)
