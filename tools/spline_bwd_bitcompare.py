"""Bit-for-bit comparison of the fused spline backward between two builds of libnfx.so.

    NFX_LIB=<lib A> python tools/spline_bwd_bitcompare.py dump a.pt
    NFX_LIB=<lib B> python tools/spline_bwd_bitcompare.py dump b.pt
    python tools/spline_bwd_bitcompare.py compare a.pt b.pt

Cases: K in {2, 3, 5, 8, 11}, both directions, H in {32, 64}, inputs partly outside the tail
bound, a lone dL/dy or dL/dld; every gradient tensor (dL/dx and the parameters) is saved.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-study_amd")]


def cases():
    for K in (2, 3, 5, 8, 11):
        for H in (32, 64):
            for direction in (1, -1):
                yield K, H, direction


def dump(path):
    import nfs_amd
    dev = torch.device("cuda:0")
    out = {}
    for K, H, direction in cases():
        torch.manual_seed(K * 100 + H + (direction > 0))
        f = nfs_amd.SplineCouplingLayer(3, H, torch.tensor([1.0, 0.0, 1.0]), num_bins=K)
        g = torch.Generator().manual_seed(7)
        with torch.no_grad():
            for p in f.parameters():
                p.add_(0.2 * torch.randn(p.shape, generator=g))
        f = f.to(dev)
        x = (2.0 * torch.randn(20000, 3, generator=g)).to(dev)
        gy = torch.randn(20000, 3, generator=g).to(dev)
        gl = torch.randn(20000, generator=g).to(dev)
        for mode in ("both", "y_only", "ld_only"):
            f.zero_grad(set_to_none=True)
            xr = x.clone().requires_grad_(True)
            y, ld = (f.forward if direction > 0 else f.inverse)(xr)
            loss = (0.0 if mode == "ld_only" else (y * gy).sum()) + (0.0 if mode == "y_only" else (ld * gl).sum())
            loss.backward()
            out[f"K{K}_H{H}_d{direction}_{mode}"] = [xr.grad.cpu()] + [p.grad.cpu() for p in f.parameters()]
    torch.save(out, path)
    print("dumped", len(out), "cases with", os.environ.get("NFX_LIB", "default lib"))


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = 0
    for k in A:
        for i, (u, v) in enumerate(zip(A[k], B[k])):
            same = torch.equal(u, v) or bool(((u == v) | (torch.isnan(u) & torch.isnan(v))).all())
            if not same:
                bad += 1
                print("DIFF", k, i, (u - v).abs().max().item())
    print("compared", len(A), "cases:", "bit-identical" if bad == 0 else f"{bad} tensors differ")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
