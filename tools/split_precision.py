"""Precision of the streaming affine path (layer 2 on split bf16 MFMAs) against the fp32
small-batch kernel and the reference's full-scale cfg2 NLL: RealNVP(2,8,64) with the G2 weights
on the G8 1M batch. One JSON line. The library is whatever NFX_LIB names.
    python tools/split_precision.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import nfs_amd  # noqa: E402
from nfs_amd import _lib  # noqa: E402
from conftest import load_golden, state_dict_from  # noqa: E402

g = load_golden("g2_realnvp.npz")
m = nfs_amd.RealNVP(2, 8, 64)
m.load_state_dict(state_dict_from(g, "", m))
m = m.cuda().eval()
torch.manual_seed(1234)
x = (torch.randn(1 << 20, 2) * 1.5).cuda()
L = _lib.lib()
out = {"lib": os.path.basename(os.environ.get("NFX_LIB", "libnfx.so"))}
res = {}
for name, pol in (("streaming", _lib.NFX_AFFINE_STREAMING), ("small", _lib.NFX_AFFINE_SMALL)):
    prev = L.nfx_affine_kernel_policy(pol)
    with torch.no_grad():
        z, ld = m.inverse(x)
        lp = m.log_prob(x)
    L.nfx_affine_kernel_policy(prev)
    res[name] = (z.double(), ld.double(), lp.double())
zs, lds, lps = res["streaming"]
zf, ldf, lpf = res["small"]
dz = (zs - zf).abs()
out["max_abs_dz"] = float(dz.max())
out["max_rel_dz"] = float((dz / (1 + zf.abs())).max())
out["p99_rel_dz"] = float(torch.quantile((dz / (1 + zf.abs())).flatten()[:1 << 22].float(), 0.99))
out["max_abs_dld"] = float((lds - ldf).abs().max())
out["mean_dlogp"] = float((lps - lpf).mean())
out["nll_streaming"] = float(-lps.mean())
out["nll_small"] = float(-lpf.mean())
print(json.dumps(out), flush=True)
