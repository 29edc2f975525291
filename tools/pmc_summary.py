"""Summarise a tools/profile_round.sh output directory into per-kernel numbers.

    python tools/pmc_summary.py gpurun_out/prof_<tag> [--write-profiles profiles/<name>]

Per config and per hot kernel: mean dispatch duration (kernel trace), FETCH_SIZE / WRITE_SIZE
per dispatch (rocprofv3 reports KiB; converted to bytes), the gfx950 correction of
MI355X_MICROARCH.md §HBM (FETCH_SIZE reads exactly half of a wide coalesced stream: doubled),
SQ instruction mix and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration).
With --write-profiles it also writes <name>_<cfg>.json next to the committed stats CSVs and the
profiles/pmc_traffic_<cfg>.json that bench.py reads for roofline.traffic.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

HOT = ("affine_coupling_kernel", "spline_coupling_kernel", "made_parallel_kernel", "made_tile_kernel", "made_seq_kernel",
       "made_wide_kernel", "made_seqs_kernel", "made_seqw_kernel", "gauss_logprob_kernel", "rqs_unit_kernel",
       "affine_chain_kernel", "affine_small_kernel", "affine_trainw_kernel", "affine_train_kernel")


def rows(path_glob):
    out = []
    for p in glob.glob(path_glob):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def hot_name(name):
    for h in HOT:
        if h in name:
            return name.split("(")[0].replace("void ", "")
    return None


def summarise(cfg_dir):
    res = {}
    for r in rows(os.path.join(cfg_dir, "trace", "*", "*_kernel_trace.csv")):
        k = hot_name(r["Kernel_Name"])
        if k:
            res.setdefault(k, {"dur_ns": []})["dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for sub in ("fetch", "write", "sq"):
        for r in rows(os.path.join(cfg_dir, sub, "*", "*_counter_collection.csv")):
            k = hot_name(r["Kernel_Name"])
            if not k:
                continue
            e = res.setdefault(k, {"dur_ns": []})
            e.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                e.setdefault("sq_dur_ns", []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for k, e in res.items():
        s = {"dispatches": len(e["dur_ns"])}
        if e["dur_ns"]:
            s["mean_us"] = statistics.mean(e["dur_ns"]) / 1e3
        for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA",
                  "SQ_INSTS_LDS", "GRBM_GUI_ACTIVE"):
            if c in e:
                s[c] = statistics.mean(e[c])
        if "FETCH_SIZE" in e:
            s["pmc_dispatches"] = len(e["FETCH_SIZE"])
        if "FETCH_SIZE" in s:
            s["fetch_bytes_raw"] = s["FETCH_SIZE"] * 1024
            s["fetch_bytes_corrected"] = 2 * s["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in s:
            s["write_bytes"] = s["WRITE_SIZE"] * 1024
        if "fetch_bytes_corrected" in s and "write_bytes" in s:
            s["hbm_bytes_per_launch"] = s["fetch_bytes_corrected"] + s["write_bytes"]
        if "GRBM_GUI_ACTIVE" in s and e.get("sq_dur_ns"):
            s["eff_clock_ghz"] = s["GRBM_GUI_ACTIVE"] / 8 / statistics.mean(e["sq_dur_ns"])
        out[k] = s
    return out


def main():
    d = sys.argv[1]
    dest = None
    if "--write-profiles" in sys.argv:
        dest = sys.argv[sys.argv.index("--write-profiles") + 1]
    allres = {}
    for cfg_dir in sorted(glob.glob(os.path.join(d, "cfg*"))):
        cfg = os.path.basename(cfg_dir)
        allres[cfg] = summarise(cfg_dir)
    print(json.dumps(allres, indent=1))
    if dest:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        for cfg, res in allres.items():
            with open(f"{dest}_{cfg}.json", "w") as f:
                json.dump(res, f, indent=1)
            for p in glob.glob(os.path.join(d, cfg, "trace", "*", "*_kernel_stats.csv")):
                shutil.copy(p, f"{dest}_{cfg}_kernel_stats.csv")
            dom = {"affine_coupling_kernel": "cfg2", "spline_coupling_kernel": "cfg3", "made_tile_kernel": "cfg4",
                   "made_wide_kernel": "cfg5f", "made_seqs_kernel": "cfg5i"}
            for tag, c in dom.items():
                # every template instance of the dominant kernel (the last layer runs the fused
                # log_prob variant), weighted by dispatch count = the per-launch mean bench.py times
                inst = [(k, s) for k, s in res.items() if tag in k and c == cfg and "hbm_bytes_per_launch" in s]
                if not inst:
                    continue
                n = sum(s.get("pmc_dispatches", 1) for _, s in inst)
                avg = lambda f: sum(s[f] * s.get("pmc_dispatches", 1) for _, s in inst) / n
                spl = None
                for logname in ("fetch.log", "trace.log"):  # bench's JSON line: samples per launch
                    try:
                        with open(os.path.join(d, cfg, logname)) as lf:
                            lines = [ln for ln in lf if ln.startswith("{")]
                        spl = json.loads(lines[-1])["roofline"]["samples_per_launch"]
                        break
                    except (OSError, IndexError, KeyError, ValueError):
                        continue
                with open(os.path.join(root, "profiles", f"pmc_traffic_{cfg}.json"), "w") as f:
                    json.dump({"kernel": [k for k, _ in inst], "hbm_bytes_per_launch": avg("hbm_bytes_per_launch"),
                               "samples_per_launch": spl,
                               "fetch_bytes_raw": avg("fetch_bytes_raw"), "write_bytes": avg("write_bytes"),
                               "source": os.path.basename(dest) + f"_{cfg}.json",
                               "note": "dispatch-weighted over the kernel's template instances; FETCH_SIZE "
                                       "doubled per MI355X_MICROARCH.md §HBM (gfx950 reports half of a wide "
                                       "streaming read); WRITE_SIZE as reported"}, f, indent=1)

if __name__ == "__main__":
    main()
