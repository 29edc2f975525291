"""Per-kernel register usage of one translation unit (hipcc -Rpass-analysis=kernel-resource-usage).
    python tools/kres.py normalizing-flows-study_amd/csrc/<file>.hip [extra hipcc flags]"""
import os
import re
import subprocess
import sys

here = os.path.dirname(os.path.abspath(__file__))
csrc = os.path.join(here, "..", "normalizing-flows-study_amd", "csrc")
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function",
       f"-I{os.path.join(here, '..', 'include')}", f"-I{csrc}", "-mllvm", "-amdgpu-mfma-vgpr-form=1",
       "-Rpass-analysis=kernel-resource-usage", "-c", sys.argv[1], "-o", "/tmp/kres.o"] + sys.argv[2:]
r = subprocess.run(cmd, capture_output=True, text=True)
cur = None
rows = []
for line in r.stderr.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k] = v
for c in rows:
    print(f"{c.get('VGPRs','?'):>4} vgpr {c.get('AGPRs','?'):>3} agpr spill {c.get('VGPRs Spill','?'):>3} occ {c.get('Occupancy [waves/SIMD]','?')}  {c['name'][:150]}")
if r.returncode:
    print(r.stderr[-3000:])
