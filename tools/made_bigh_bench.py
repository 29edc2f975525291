"""Time the wide-hidden MADE kernels (128 < H <= 256, nfx_made_big.hip) on cuda:0.

Prints one JSON line per (direction, d, H, B): mean ms per call (HIP events on the launch stream)
and algorithmic TFLOP/s (dense masked MADE flops: 2 B (d H + 2 H^2 + 2 d H); the sequential
directions are priced at ONE MADE evaluation per sample, like cfg5i).
    python tools/made_bigh_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "normalizing-flows-study_amd"))
import nfs_amd  # noqa: E402

CASES = [("maf", -1, 63, 256, 500_000), ("maf", -1, 63, 128, 500_000), ("iaf", 1, 784, 256, 65_536),
         ("iaf", -1, 784, 256, 8192), ("maf", 1, 63, 256, 65_536)]


def main():
    dev = torch.device("cuda:0")
    for kind, direction, d, H, B in CASES:
        torch.manual_seed(0)
        cls = nfs_amd.MaskedAutoregressiveFlow if kind == "maf" else nfs_amd.InverseAutoregressiveFlow
        f = cls(d, H)
        with torch.no_grad():
            for p in f.parameters():
                p.add_(0.02 * torch.randn_like(p))
        f = f.to(dev).eval()
        x = torch.randn(B, d, device=dev)
        fn = f.forward if direction > 0 else f.inverse
        with torch.no_grad():
            for _ in range(2):
                fn(x)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 5
            e0.record()
            for _ in range(n):
                fn(x)
            e1.record()
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        flops = 2.0 * B * (d * H + 2 * H * H + 2 * d * H)
        print(json.dumps({"kind": kind, "direction": direction, "d": d, "H": H, "B": B, "ms": round(ms, 4),
                          "tflops": round(flops / ms / 1e9, 2), "samples_per_s": round(B / ms * 1e3)}), flush=True)


if __name__ == "__main__":
    main()
