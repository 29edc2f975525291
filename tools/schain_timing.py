"""Stage clocks of the streaming spline chain (cfg3: 8x SplineCouplingLayer(2, 64, K=8) inverse +
log_prob), from a timing build:
    NFX_BUILD_VARIANT=timing NFX_EXTRA_CFLAGS="-DNFX_SCHAIN_TIMING" python normalizing-flows-study_amd/build.py
    NFX_LIB=.../libnfx_timing.so python tools/schain_timing.py [B ...]
Workgroup 0's waves 0 and 4 write their accumulated clock64 ticks per stage into the first 12
outputs (stage names below, NFX_CMARK order of csrc/nfx_spline_schain_kernel.h). The timing build
assumes one transformed dim per layer (d = 2). The round-4 stagger experiment's numbers
(profiles/r04f_stage_clocks/) came from the same marks in that variant of the kernel."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
import torch  # noqa: E402
import nfs_amd  # noqa: E402

torch.manual_seed(0)
layers = []
for i in range(8):
    mask = torch.zeros(2)
    mask[i % 2] = 1
    layers.append(nfs_amd.SplineCouplingLayer(2, 64, mask, num_bins=8))
m = nfs_amd.NormalizingFlowModel(layers).cuda().eval()
names = ["barrier", "mfma part", "spline", "layer start + row io", "slice prologue", "slice epilogue"]
for B in [int(b) for b in sys.argv[1:]] or [125000, 1000000]:
    x = torch.randn(B, 2, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            lp = m.log_prob(x)
        torch.cuda.synchronize()
        z, _ = m.inverse(x)
        torch.cuda.synchronize()
    t = z.reshape(-1)[:12].double().cpu().tolist()
    for w, tt in ((0, t[:6]), (4, t[6:])):
        tot = sum(tt)
        print(json.dumps({"B": B, "wave": w, "total_ticks": tot, **{n: round(v / max(tot, 1), 3) for n, v in zip(names, tt)}}))
