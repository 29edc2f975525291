"""Per-kernel ISA statistics of a hipcc --save-temps .s file (VGPRs, spills, instruction mix).

    python tools/isa_stats.py file.s [name-substring]
"""
import re
import sys
from collections import Counter


def kernel_meta(s):
    meta = {}
    blk = s[s.find("amdhsa.kernels:"):]
    for ent in re.split(r"\n  - ", blk)[1:]:
        m = re.search(r"\.name:\s+(\S+)", ent)
        if not m:
            continue
        get = lambda k: (re.search(rf"\.{k}:\s+(\d+)", ent) or [None, None])[1]
        meta[m.group(1)] = {k: get(k) for k in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count",
                                                "sgpr_spill_count", "private_segment_fixed_size",
                                                "group_segment_fixed_size")}
    return meta


def main():
    s = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    meta = kernel_meta(s)
    for n in re.findall(r"^(_Z\S+):\s*(?:;.*)?$", s, re.M):
        if sub not in n or n not in meta:
            continue
        i = s.find(n + ":")
        j = s.find(".Lfunc_end", i)
        ins = [l.strip().split()[0] for l in s[i:j].split("\n") if l.startswith("\t") and not l.strip().startswith((".", ";"))]
        c = Counter(ins)
        mf = sum(v for k, v in c.items() if "mfma" in k)
        va = sum(v for k, v in c.items() if k.startswith("v_")) - mf
        print(f"{n[:70]:70s} vgpr {meta[n]['vgpr_count']} agpr {meta[n]['agpr_count']} spill {meta[n]['vgpr_spill_count']} "
              f"scratch {meta[n]['private_segment_fixed_size']} | mfma {mf} valu {va} br {sum(v for k, v in c.items() if 'cbranch' in k)}")


if __name__ == "__main__":
    main()
