import sys, os
sys.path.insert(0, os.path.join(os.getcwd(), "normalizing-flows-study_amd"))
import torch, numpy as np
import nfs_amd
from nfs_amd import _lib
L = _lib.lib()
for (d, H, B) in [(200, 64, 1500), (200, 64, 1024), (200, 64, 2100), (784, 64, 3000)]:
    torch.manual_seed(1)
    f = nfs_amd.InverseAutoregressiveFlow(d, H)
    with torch.no_grad():
        for p in f.parameters():
            p.add_(0.05 * torch.randn_like(p))
    f = f.cuda().eval()
    x = torch.randn(B, d).cuda()
    res = {}
    for name, pol in (("wave", _lib.NFX_MADE_SEQ_WAVE), ("push", _lib.NFX_MADE_SEQ_PUSH)):
        L.nfx_made_seq_policy(pol)
        with torch.no_grad():
            z, ld = f.inverse(x)
        torch.cuda.synchronize()
        res[name] = (z.cpu().numpy(), ld.cpu().numpy())
    dz = np.abs(res["wave"][0] - res["push"][0]).max(axis=1)
    dl = np.abs(res["wave"][1] - res["push"][1])
    badz = np.nonzero(dz > 1e-3)[0]; badl = np.nonzero(dl > 1e-3)[0]
    print(d, H, B, "badz", len(badz), badz[:10].tolist(), "badl", len(badl), badl[:20].tolist(), float(dl.max()))
