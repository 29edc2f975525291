"""Stage clocks of the segment-parallel sequential MADE kernel (made_seqs_kernel, IAF(784, 64)
inverse + fused log_prob, the cfg5i shape), from a timing build:
    NFX_BUILD_VARIANT=timing NFX_EXTRA_CFLAGS="-DNFX_SEQS_TIMING -DNFX_SEQW_TIMING" python normalizing-flows-study_amd/build.py
    NFX_LIB=.../libnfx_timing.so python tools/seqs_timing.py [B ...]
Workgroup 0's first lane writes its wave's accumulated clock64 ticks per stage into out[0, 0:7]
(stage names below, in NFX_TMARK order of csrc/nfx_made_seqs_kernel.h)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import torch  # noqa: E402
import nfs_amd  # noqa: E402
from nfs_amd import _lib  # noqa: E402

d, H = 784, 64
torch.manual_seed(0)
f = nfs_amd.InverseAutoregressiveFlow(d, H)
with torch.no_grad():
    for p in f.parameters():
        p.add_(0.05 * torch.randn_like(p))
f = f.cuda().eval()
_lib.lib().nfx_made_seq_policy(_lib.NFX_MADE_SEQ_SEGMENT)
names = ["chunk start + dot products + row reads", "affine map, poison ballot, step stores",
         "row broadcasts + rank-1 updates", "completion (layers 1-3)", "block: log-det sums + output rows",
         "block: vmcnt(0) + barrier", "block start: tile, block end, DMA + x issue"]
for B in [int(b) for b in sys.argv[1:]] or [8192, 2048]:
    x = torch.randn(B, d, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            z, _ = f.inverse(x)
        torch.cuda.synchronize()
    t = z[0, :7].double().cpu().tolist()
    tot = sum(t)
    print(json.dumps({"B": B, "total_ticks": tot, "per_chunk_65": tot / 65,
                      **{n: round(v / tot, 3) for n, v in zip(names, t)}, "ticks": dict(zip(names, t))}))
