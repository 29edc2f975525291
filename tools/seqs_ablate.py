"""Same-box A/B timing of sequential-MADE kernel variants (cfg5i shape, IAF(784, 64) inverse,
B = 2 Ki .. 16 Ki): every library tools/expt_lib/libnfx_e*.so (libnfx.so relinked with a variant
of nfx_made.o: a git revision, or an ablation build with parts of made_seqs_kernel switched off)
is timed in its own child process, the list twice in alternation.
    python tools/seqs_ablate.py
"""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
    import torch
    import nfs_amd
    d, H = 784, 64
    torch.manual_seed(0)
    f = nfs_amd.InverseAutoregressiveFlow(d, H)
    with torch.no_grad():
        for p in f.parameters():
            p.add_(0.05 * torch.randn_like(p))
    f = f.cuda().eval()
    out = []
    for B in (2048, 4096, 8192, 16384):
        x = torch.randn(B, d, device="cuda")
        with torch.no_grad():
            for _ in range(3):
                f.inverse(x)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f.inverse(x)
            e1.record()
            torch.cuda.synchronize()
        out.append(f"B={B} {e0.elapsed_time(e1) / 10 * 1e3:.1f}us")
    print(os.path.basename(os.environ["NFX_LIB"]), " ".join(out), flush=True)


if __name__ == "__main__":
    if os.environ.get("NFX_LIB"):
        child()
    else:
        for lib in sorted(glob.glob(os.path.join(ROOT, "tools", "expt_lib", "libnfx_e*.so"))) * 2:
            env = dict(os.environ, NFX_LIB=lib)
            r = subprocess.run([sys.executable, "-u", __file__], env=env, timeout=180)
            if r.returncode != 0:
                sys.exit(r.returncode)
