"""Small-batch vs streaming affine kernel vs AUTO: graphed RealNVP(2,10,H) forward time per batch.

    python tools/affine_small_sweep.py [H]
"""
import sys

sys.path.insert(0, "normalizing-flows-study_amd")
import torch
import nfs_amd
from nfs_amd import _lib as L

BATCHES = [512, 2048, 4000, 8192, 12288, 16384, 24576, 32768, 49152, 65536, 98304, 131072, 262144]
POLICIES = (("streaming", L.NFX_AFFINE_STREAMING), ("small", L.NFX_AFFINE_SMALL), ("auto", L.NFX_AFFINE_AUTO))


def main():
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = nfs_amd.RealNVP(2, 10, H).to(dev).eval()
    print(f"RealNVP(2,10,{H}) graphed forward, us per 10 layers")
    print(f"{'B':>8} " + " ".join(f"{n:>10}" for n, _ in POLICIES))
    for B in BATCHES:
        x = torch.randn(B, 2, device=dev)
        row = []
        for _, pol in POLICIES:
            L.lib().nfx_affine_kernel_policy(pol)
            g = nfs_amd.GraphedFlow(m, x, mode="forward", strict=False)
            for _ in range(5):
                g()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50
            s.record()
            for _ in range(n):
                g()
            e.record()
            torch.cuda.synchronize()
            row.append(1000.0 * s.elapsed_time(e) / n)
        print(f"{B:>8} " + " ".join(f"{v:>10.1f}" for v in row), flush=True)
    L.lib().nfx_affine_kernel_policy(L.NFX_AFFINE_AUTO)


if __name__ == "__main__":
    main()
