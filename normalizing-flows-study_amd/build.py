"""Build libnfx.so (all HIP kernels + the C-ABI) in-tree for gfx950.

    python normalizing-flows-study_amd/build.py [--jobs N] [--force]

hipcc compiles each csrc/*.hip translation unit to an object in build/ (in parallel, skipping
objects newer than their sources and headers), then links nfs_amd/libnfx.so. Deliberately no
-ffast-math: the kernels reproduce torch's NaN/Inf guards and clamp semantics, and the NLL
target (|dNLL| <= 1e-5) needs the precise expf/logf/sqrtf.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# NFX_BUILD_VARIANT=<name> (with NFX_EXTRA_CFLAGS, e.g. -DNFX_SEQW_TIMING) builds a diagnostic
# variant into build-<name>/ and nfs_amd/libnfx_<name>.so (load it with NFX_LIB=...).
_VARIANT = os.environ.get("NFX_BUILD_VARIANT", "")
BUILD = os.path.join(HERE, "build" + (f"-{_VARIANT}" if _VARIANT else ""))
OUT = os.path.join(HERE, "nfs_amd", f"libnfx_{_VARIANT}.so" if _VARIANT else "libnfx.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
ARCH = os.environ.get("NFX_OFFLOAD_ARCH", "gfx950")

# -amdgpu-mfma-vgpr-form: keep MFMA accumulators in the (unified) VGPR file, so the ReLU /
# epilogue VALU ops read them directly instead of paying a v_accvgpr_read per element.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
          "-Wno-unused-function", f"-I{INCLUDE}", f"-I{CSRC}",
          "-mllvm", "-amdgpu-mfma-vgpr-form=1"]


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm 7.x required)")


def _stale(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(jobs=None, force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    cc = hipcc()
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _stale(o, [s] + headers):
            todo.append((s, o))

    def compile_one(so):
        s, o = so
        cmd = [cc] + CFLAGS + os.environ.get("NFX_EXTRA_CFLAGS", "").split() + ["-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {os.path.basename(s)}:\n{r.stderr[-4000:]}")
        return s

    jobs = jobs or min(16, os.cpu_count() or 4)
    if todo:
        if verbose:
            print(f"[nfx build] compiling {len(todo)} TU(s) with {jobs} job(s)", flush=True)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for s in ex.map(compile_one, todo):
                if verbose:
                    print(f"[nfx build]   {os.path.basename(s)}", flush=True)
    if force or todo or _stale(OUT, objs):
        cmd = [cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        if verbose:
            print(f"[nfx build] linked {OUT}", flush=True)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    try:
        build(a.jobs, a.force)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
