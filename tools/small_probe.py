"""One CouplingLayer(2, 128) forward at small batches, each affine kernel, event-timed (run under
rocprofv3 --kernel-trace --stats to see the kernel durations)."""
import sys

sys.path.insert(0, "normalizing-flows-study_amd")
import torch
import nfs_amd

dev = torch.device("cuda:0")
torch.manual_seed(0)
mask = torch.tensor([1.0, 0.0])
layer = nfs_amd.CouplingLayer(2, 128, mask).to(dev).eval()
f = nfs_amd._lib.lib().nfx_affine_small_batch_max
for B in [int(a) for a in (sys.argv[1:] or ["512", "4000"])]:
    x = torch.randn(B, 2, device=dev)
    for name, thr in (("small", 1 << 40), ("streaming", 0)):
        f(thr)
        with torch.no_grad():
            for _ in range(10):
                layer.forward(x)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(200):
                layer.forward(x)
            e.record()
            torch.cuda.synchronize()
        print(f"B={B} {name}: {1000 * s.elapsed_time(e) / 200:.1f} us/layer (eager, incl. host issue)", flush=True)
