"""Stage clocks of the push-formulation sequential MADE kernel (made_seqp_kernel, IAF(784, 64)
inverse) from a timing build:
  NFX_BUILD_VARIANT=timing NFX_EXTRA_CFLAGS=-DNFX_SEQP_TIMING python normalizing-flows-study_amd/build.py
  NFX_LIB=.../libnfx_timing.so python tools/seqp_timing.py [B]
Workgroup 0 / wave 0 writes its accumulated clock64 ticks per stage into out[0, 0:8]."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import torch  # noqa: E402
import nfs_amd  # noqa: E402
from nfs_amd import _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
d, H = 784, 64
torch.manual_seed(0)
f = nfs_amd.InverseAutoregressiveFlow(d, H)
with torch.no_grad():
    for p in f.parameters():
        p.add_(0.05 * torch.randn_like(p))
f = f.cuda().eval()
_lib.lib().nfx_made_seq_policy(_lib.NFX_MADE_SEQ_PUSH)
x = torch.randn(B, d, device="cuda")
with torch.no_grad():
    for _ in range(3):
        z, _ = f.inverse(x)
    torch.cuda.synchronize()
t = z[0, :8].double().cpu().tolist()
names = ["push+entry", "column issue+affine", "W1 wait+layer-1 sum", "layers 1-3 chain", "rows issue+poison",
         "slot end", "stores", "-"]
tot = sum(t)
print(json.dumps({"B": B, "total_ticks": tot, **{n: round(v / tot, 3) for n, v in zip(names, t)},
                  "ticks": dict(zip(names, t))}))
