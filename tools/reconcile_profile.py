"""Reconcile a rocprofv3 trace of bench.py with the bench line the same process printed.

    python tools/reconcile_profile.py gpurun_out/prof_<tag> <round tag, e.g. r04>

For every config directory written by tools/profile_bench.sh (bench.json = the bench line,
trace/ = rocprofv3 --kernel-trace --stats of that same process, optional fetch/ and write/ =
the FETCH_SIZE / WRITE_SIZE passes) this writes profiles/<round>_<cfg>.json with
  * the per-kernel dispatch counts and mean durations (kernel_stats.csv),
  * the hot kernel's launches per step (the bench's event pass: launches / steps),
  * rocprof_ms_per_step = the summed duration of every kernel dispatched inside the bench's timed
    window (bench.py prints it as timed_window_monotonic_ns, on the clock rocprofv3 stamps kernels
    with) / steps, and the hot kernel's mean over those dispatches only (no warm-up ramps),
  * the check rocprof_ms_per_step <= the bench's own ms_per_step (same process, same clock),
  * the rocprof frac (algorithmic flop per launch / rocprof mean / peak) next to the event frac,
  * with the PMC passes: HBM bytes per launch (FETCH_SIZE doubled per MI355X_MICROARCH.md, gfx950
    reports half of a wide streaming read; WRITE_SIZE as reported), dispatch-weighted.
and copies the kernel_stats.csv next to it (profiles/<round>_<cfg>_kernel_stats.csv).
bench.py quotes profiles/rocprof_<cfg>.json (the latest reconciled file per config).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 157.3

# hot-kernel name fragments per config family (template instances are summed)
HOT = {
    "cfg2": ("affine_coupling_kernel", "affine_schain_kernel", "affine_chain_kernel"),
    "cfg3": ("spline_coupling_kernel", "spline_schain_kernel"),
    "cfg4": ("made_tile_kernel",),
    "cfg5i": ("made_seqs_kernel", "made_seqw_kernel", "made_seqp_kernel"),
    "cfg5f": ("made_wide_kernel",),
    "sample4k": ("affine_chain_kernel", "affine_small_kernel", "affine_coupling_kernel"),
    "sample4k_spline": ("spline_coupling_kernel", "spline_schain_kernel"),
    "sample4k_maf": ("made_seqs_kernel", "made_seqw_kernel", "made_seqp_kernel", "made_seq_kernel"),
    "sample4k_iaf": ("made_tile_kernel",),
    "trainfig_iaf": ("made_seq_bwd_kernel", "made_seqw_bwd_kernel"),
    "trainfig_maf": ("made_bwd_kernel",),
    "trainfig_spline": ("spline_bwd_kernel",),
    "cfg4t": ("made_bwd_kernel",),
    "cfg2t": ("affine_train_kernel<2, 2, 3>", "affine_train_kernel<2, 2, 6>"),  # BWD2 / BWD2K (event-timed)
    "cfg3t": ("spline_bwd_kernel",),
}
PER_PASS = ("gauss_finish_kernel",)  # once per log_prob pass besides the layer kernels


def _newest(pattern):
    """The newest match (a re-profiled config leaves the previous run's pid-named files beside it)."""
    m = glob.glob(pattern)
    return max(m, key=os.path.getmtime) if m else None


def _kernel_stats(path):
    out = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = r["Name"].split("(")[0].replace("void ", "")
            out[name] = {"dispatches": int(r["Calls"]), "mean_us": float(r["AverageNs"]) / 1e3,
                         "total_us": float(r["TotalDurationNs"]) / 1e3}
    return out


def _counter(path, counter):
    """Per-dispatch counter values of counter_collection.csv: {kernel: [value, ...]}"""
    out = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            out.setdefault(name, []).append(float(r["Counter_Value"]))
    return out


N_SIMD = 256 * 4         # MI355X: 256 CUs x 4 SIMDs
MFMA_F32_CYCLES = 64     # v_mfma_f32_32x32x2_f32: 4,096 flop at 64 flop/clk/SIMD
PEAK_CLOCK_GHZ = 2.4     # the clock the 157.3 TFLOP/s peak is quoted at


def mfma_busy(counter_csv, trace_csv, hot):
    """The MFMA-busy pass: per dispatch of the hot kernel, SQ_VALU_MFMA_BUSY_CYCLES (cycles the
    matrix pipe was busy, summed over every SIMD), SQ_INSTS_MFMA / SQ_INSTS_VALU (wave
    instructions) and GRBM_GUI_ACTIVE (GPU-active cycles summed over the 8 XCDs). With the
    dispatch's duration (its kernel trace) they give
      clock_ghz      = GRBM_GUI_ACTIVE / 8 / duration           (MI355X_MICROARCH.md 'DVFS give-back')
      mfma_busy_frac = BUSY / (1,024 SIMDs x GRBM_GUI_ACTIVE / 8) (share of the SIMD-cycles the pipe ran)
    and the identity frac = mfma_busy_frac x clock / 2.4 GHz x (algorithmic / issued MFMA flop):
    the roofline frac is below the busy fraction by the clock and by any MFMA work beyond the
    algorithmic count, and the rest of the SIMD-cycles are VALU / waiting."""
    per = {}
    with open(counter_csv) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k not in hot:
                continue
            key = (k, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    dur = {}
    if trace_csv:
        with open(trace_csv) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                if k in hot:
                    dur[(k, r.get("Dispatch_Id") or r.get("Correlation_Id"))] = (
                        int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = [(v, dur.get(key)) for key, v in per.items()
            if all(c in v for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"))]
    if not rows:
        return {}
    n = len(rows)
    busy = sum(v["SQ_VALU_MFMA_BUSY_CYCLES"] for v, _ in rows) / n
    imfma = sum(v["SQ_INSTS_MFMA"] for v, _ in rows) / n
    ivalu = sum(v["SQ_INSTS_VALU"] for v, _ in rows) / n
    grbm = sum(v["GRBM_GUI_ACTIVE"] for v, _ in rows) / n
    cyc = grbm / 8
    out = {"pmc_mfma": {"dispatches": n, "SQ_VALU_MFMA_BUSY_CYCLES": busy, "SQ_INSTS_MFMA": imfma,
                        "SQ_INSTS_VALU": ivalu, "GRBM_GUI_ACTIVE": grbm,
                        "busy_cycles_per_mfma": busy / imfma if imfma else None,
                        "source": os.path.relpath(counter_csv, ROOT)},
           "mfma_busy_frac": busy / (N_SIMD * cyc) if cyc else None,
           "mfma_issue_frac": imfma * MFMA_F32_CYCLES / (N_SIMD * cyc) if cyc else None,
           "valu_insts_per_mfma": ivalu / imfma if imfma else None,
           # SQ_INSTS_VALU counts the MFMAs themselves too: the other vector instructions per MFMA
           "non_mfma_valu_per_mfma": (ivalu - imfma) / imfma if imfma else None,
           # VALU issue slots used, at 4 cycles per wave instruction (8 for transcendentals: a
           # lower bound) — the pipe of the kernels that issue no MFMA (cfg5i)
           "valu_issue_frac": (ivalu - imfma) * 4 / (N_SIMD * cyc) if cyc else None}
    ds = [d for _, d in rows if d]
    if ds:
        mean_ns = sum(ds) / len(ds)
        out["clock_ghz"] = cyc / mean_ns
        out["pmc_mfma"]["mean_duration_us"] = mean_ns / 1e3
    return out


def busy_identity(res, f_launch, spl):
    """The frac of the MFMA-busy pass's own dispatches (algorithmic flop / its duration / peak)
    and the same number rebuilt from the counters: busy x clock / 2.4 GHz / (issued / algorithmic
    MFMA flop) — equal by construction when BUSY counts 64 cycles per fp32 32x32x2 MFMA; the
    trace pass's frac differs from it only by the PMC pass running its kernels a little slower."""
    pm = res.get("pmc_mfma")
    if not pm or not pm.get("mean_duration_us") or not pm.get("SQ_INSTS_MFMA"):
        return
    alg = f_launch * spl
    issued = pm["SQ_INSTS_MFMA"] * 4096.0
    frac_pmc = alg / (pm["mean_duration_us"] * 1e-6) / 1e12 / PEAK
    res["mfma_identity"] = {
        "frac_pmc_pass": frac_pmc,
        "issued_over_algorithmic": issued / alg,
        "busy_x_clock_over_peak_clock": res["mfma_busy_frac"] * res["clock_ghz"] / PEAK_CLOCK_GHZ,
        "rebuilt_frac": res["mfma_busy_frac"] * res["clock_ghz"] / PEAK_CLOCK_GHZ * alg / issued,
        "note": "frac = busy x clock/2.4 GHz x algorithmic/issued; the rest of the SIMD-cycles are "
                "VALU (fp32 VALU and fp32 MFMA share the pipe) and waits"}


def reconcile(cdir, rtag):
    name = os.path.basename(cdir.rstrip("/"))
    cfg = "_".join(p for p in name.split("_") if not p.isdigit())  # cfg2_125000 -> cfg2
    with open(os.path.join(cdir, "bench.json")) as fh:
        bench = json.loads([ln for ln in fh.read().splitlines() if ln.startswith("{")][-1])
    ks_path = _newest(os.path.join(cdir, "trace", "*", "*_kernel_stats.csv"))
    ks = _kernel_stats(ks_path)
    frags = HOT.get(cfg, ())
    rf = bench["roofline"]
    win = bench.get("timed_window_monotonic_ns")
    tr = _newest(os.path.join(cdir, "trace", "*", "*_kernel_trace.csv"))
    if win and tr:
        # exactly the kernels of the timed steps: dispatches inside the bench's timed window
        # (bench.py stamps it with time.monotonic_ns, the clock rocprofv3 stamps kernels with)
        with open(tr) as fh:
            rows = [r for r in csv.DictReader(fh)
                    if int(r["Start_Timestamp"]) >= win[0] and int(r["End_Timestamp"]) <= win[1]]
        win_k = {}
        for r in rows:
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            e = win_k.setdefault(k, {"dispatches": 0, "total_us": 0.0})
            e["dispatches"] += 1
            e["total_us"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for e in win_k.values():
            e["mean_us"] = e["total_us"] / e["dispatches"]
        hot = {k: v for k, v in win_k.items() if any(f in k for f in frags)}
        n_hot = sum(v["dispatches"] for v in hot.values())
        lps = n_hot / bench["steps"]
        passes = bench["steps"]
        hot_ms = sum(v["total_us"] for v in hot.values()) / passes / 1e3
        extra_ms = (sum(v["total_us"] for v in win_k.values()) / passes / 1e3) - hot_ms  # every other kernel
        window = {"kernels_in_window": win_k, "span_ms": (win[1] - win[0]) / 1e6}
    else:
        # no window: every dispatch of the process (warm-up ramps included), per pass
        hot = {k: v for k, v in ks.items() if any(f in k for f in frags)}
        lps = rf["launches"] / bench["steps"]  # launches of the hot kernel per pass (event pass)
        n_hot = sum(v["dispatches"] for v in hot.values())
        passes = n_hot / lps
        hot_ms = sum(v["total_us"] for v in hot.values()) / passes / 1e3
        extra = {k: v for k, v in ks.items() if any(f in k for f in PER_PASS)}
        extra_ms = sum(v["total_us"] for v in extra.values()) / passes / 1e3
        window = None
    mean_us = sum(v["total_us"] for v in hot.values()) / n_hot
    f_launch = rf["flop_per_sample_per_launch"]
    spl = rf["samples_per_launch"]
    ach = f_launch * spl / (mean_us * 1e-6) / 1e12
    # the bench line's own peak: the fp32 MFMA peak, or for the split-MFMA configs (cfg2: layer 2
    # as six bf16 piece products per fp32 multiply-add) the bf16 peak / 6
    peak = rf.get("peak") or PEAK
    res = {
        "config": name, "round": rtag, "lib_sha256": bench.get("lib_sha256"),
        "bench": {k: bench.get(k) for k in ("value", "ms_per_step", "steps", "warmup", "n_gpus")},
        "bench_roofline": {k: rf.get(k) for k in ("kernel", "mean_launch_ms", "launches", "frac",
                                                    "frac_executed", "flop_per_sample_per_launch",
                                                    "samples_per_launch")},
        "kernels_process": ks, "timed_window": window, "hot_kernels": sorted(hot), "launches_per_step": lps,
        "passes_counted": passes,
        "rocprof_mean_launch_us": mean_us,
        "rocprof_hot_ms_per_step": hot_ms,
        "rocprof_ms_per_step": hot_ms + extra_ms,
        "fits_bench_step": hot_ms + extra_ms <= bench["ms_per_step"],
        "rocprof_achieved_tflops": ach, "rocprof_frac": ach / peak, "peak_tflops": peak,
        # dense-count fracs on both sides (cfg4's headline frac is the executed one)
        "event_frac": rf.get("frac_dense", rf["frac"]),
        "frac_rel_diff": abs(ach / peak - rf.get("frac_dense", rf["frac"])) / rf.get("frac_dense", rf["frac"]),
        "source": {"kernel_stats": os.path.relpath(ks_path, ROOT),
                   "bench": os.path.relpath(os.path.join(cdir, "bench.json"), ROOT)},
    }
    if rf.get("frac_executed"):
        fe = rf["flop_per_sample_executed"]
        res["rocprof_frac_executed"] = fe * spl / (mean_us * 1e-6) / 1e12 / peak
        res["event_frac_executed"] = rf["frac_executed"]
    fetch = _newest(os.path.join(cdir, "fetch", "*", "*counter_collection.csv"))
    write = _newest(os.path.join(cdir, "write", "*", "*counter_collection.csv"))
    if fetch and write:
        fv, wv = _counter(fetch, "FETCH_SIZE"), _counter(write, "WRITE_SIZE")
        fs = [v for k, vs in fv.items() if k in hot for v in vs]
        ws = [v for k, vs in wv.items() if k in hot for v in vs]
        if fs and ws:
            fb = 2 * 1024 * sum(fs) / len(fs)  # KB, doubled (gfx950 FETCH_SIZE correction)
            wb = 1024 * sum(ws) / len(ws)
            res["hbm_bytes_per_launch"] = fb + wb
            res["fetch_bytes_corrected"] = fb
            res["write_bytes"] = wb
            res["pmc_dispatches"] = len(fs)
            res["pmc_note"] = ("FETCH_SIZE (KB) doubled per MI355X_MICROARCH.md (gfx950 reports half of a wide "
                               "streaming read), WRITE_SIZE as reported; mean over the hot kernel's dispatches")
    mf = _newest(os.path.join(cdir, "mfma", "*", "*counter_collection.csv"))
    mt = _newest(os.path.join(cdir, "mfma", "*", "*kernel_trace.csv"))
    if mf:
        res.update(mfma_busy(mf, mt, hot))
        if rf.get("peak_basis"):
            # mixed bf16 (32-cycle) and fp32 (64-cycle) MFMAs: the busy fraction stands, the
            # fp32-only issue count and identity do not apply
            res["mfma_issue_frac"] = None
            res["mfma_identity"] = {"note": "split-MFMA kernel (bf16 32x32x16 + fp32 32x32x2): the busy fraction "
                                            "counts both; frac is against the bf16 peak / 6 (bench peak_basis)"}
        else:
            busy_identity(res, f_launch, spl)
    out = os.path.join(ROOT, "profiles", f"{rtag}_{name}.json")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    shutil.copy(ks_path, os.path.join(ROOT, "profiles", f"{rtag}_{name}_kernel_stats.csv"))
    # the file bench.py quotes for this config (profiles/rocprof_<cfg>[_<batch>].json: a shard run
    # with --batch B quotes rocprof_<cfg>_<B>.json)
    if cfg in HOT:
        with open(os.path.join(ROOT, "profiles", f"rocprof_{name}.json"), "w") as fh:
            json.dump(res, fh, indent=1)
    return res


def main():
    pdir, rtag = sys.argv[1], sys.argv[2]
    for cdir in sorted(glob.glob(os.path.join(pdir, "*"))):
        if not os.path.isfile(os.path.join(cdir, "bench.json")):
            continue
        try:
            r = reconcile(cdir, rtag)
        except Exception as e:  # noqa: BLE001 - report and continue with the other configs
            print(f"{cdir}: {e}")
            continue
        print(f"{r['config']:>18}: step {r['bench']['ms_per_step']:.4f} ms, rocprof kernels/step "
              f"{r['rocprof_ms_per_step']:.4f} ms (fits: {r['fits_bench_step']}), mean {r['rocprof_mean_launch_us']:.1f} us"
              f" x {r['launches_per_step']:.0f}, frac rocprof {r['rocprof_frac']:.3f} / events {r['event_frac']:.3f}"
              + (f", HBM {r['hbm_bytes_per_launch']/1e6:.1f} MB/launch" if "hbm_bytes_per_launch" in r else ""))


if __name__ == "__main__":
    main()
