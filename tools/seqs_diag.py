"""Diagnose run-to-run differences of the sequential MADE kernel (made_seqs_kernel).

Runs one IAF(150, 64) layer's inverse (unfused and with the fused Gaussian term) repeatedly at
small batches on cuda:0 and reports, per call, which rows differ from the torch composite of the
same layer on the GPU (fp32, same math) and from the first call. Prints one line per finding.
    python tools/seqs_diag.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "normalizing-flows-study_amd"))
import nfs_amd  # noqa: E402
from nfs_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(7)
    layer = nfs_amd.InverseAutoregressiveFlow(150, 64)
    g = torch.Generator().manual_seed(9)
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.02 * torch.randn(p.shape, generator=g))
    layer = layer.to(dev).eval()
    for B in (77, 4099, 33, 200):
        x = (1.5 * torch.randn(B, 150, generator=torch.Generator().manual_seed(B))).to(dev)
        with torch.no_grad():
            zr, ldr = layer._torch_call(x, -1)
            ref = None
            for it in range(12):
                out = torch.empty_like(x)
                ld = torch.zeros(B, device=dev)
                if it % 2 == 0:
                    layer._hip_launch(x, out, ld, -1, accumulate=True)
                    lp = None
                else:
                    lp = torch.empty(B, device=dev)
                    sums = torch.zeros(2, device=dev, dtype=torch.float64)
                    ws = torch.empty(4096, device=dev, dtype=torch.float64)
                    assert layer._hip_launch_logprob(x, out, ld, lp, sums, ws, accumulate=True)
                torch.cuda.synchronize()
                rz = ((out - zr).abs().amax(dim=1))
                bad = (rz > 1e-3 * (1 + zr.abs().amax(dim=1))).nonzero().flatten().tolist()
                if ref is None:
                    ref = (out.clone(), ld.clone())
                diff = ((out != ref[0]).any(dim=1) | (ld != ref[1])).nonzero().flatten().tolist()
                print(f"B={B} it={it} fused={lp is not None} rows_vs_torch_bad={len(bad)} {bad[:12]} "
                      f"max_abs_vs_torch={rz.max().item():.3g} rows_vs_first={len(diff)} {diff[:12]}",
                      flush=True)
                if bad:
                    r = bad[0]
                    col = ((out[r] - zr[r]).abs() > 1e-3).nonzero().flatten().tolist()
                    print(f"   row {r}: first bad cols {col[:12]} of {len(col)}; ld {ld[r].item():.6g} "
                          f"vs torch {ldr[r].item():.6g}", flush=True)


if __name__ == "__main__":
    print("lib", _lib.lib()._name, flush=True)
    main()
