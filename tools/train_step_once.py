"""A few training steps of 5x MAF(63,64) at B=500k (for rocprofv3 kernel traces)."""
import sys
sys.path.insert(0, "normalizing-flows-study_amd"); sys.path.insert(0, ".")
import torch
import nfs_amd

dev = torch.device("cuda:0")
torch.manual_seed(0)
model = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(63, 64) for _ in range(5)]).to(dev).train()
opt = torch.optim.Adam(model.parameters(), lr=1e-4)
x = torch.randn(500000, 63, device=dev)
for _ in range(4):
    opt.zero_grad(set_to_none=True)
    loss = -model.log_prob(x).mean()
    loss.backward()
    opt.step()
torch.cuda.synchronize()
print("ok", loss.item())
