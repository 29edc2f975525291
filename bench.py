"""Benchmark: log_prob throughput of the gfx950 flow-transform hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5f|cfg5i|...]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

`--gpus N` with no launcher around it (WORLD_SIZE unset) starts the N ranks itself as child
processes (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1) and relays rank
0's line; under a launcher WORLD_SIZE must equal --gpus. The line records the world size and
every rank's device.

One step = one log_prob pass over the batch: every flow layer's fused kernel (conditioner MLP
on fp32 MFMA + transform + log-det accumulate), the fused Gaussian base term with the float64
NLL partial sum, and (N > 1) ONE RCCL all-reduce of the 16-byte partial [sum log p, count] —
the whole data-parallel exchange of the path.

Scaling (default STRONG, north_star's ">= 6x strong scaling at 8 GPUs"): the BASELINE batch
(cfg2 1M, cfg4 4M, cfg5 8,192 / 524,288) is split over the ranks; `--weak` gives every rank the
whole batch instead. The weights are the reference's own (tests/golden/*.npz, produced by
importing the reference) and the input is the G8 seeded batch, so the line also carries the
global NLL against the reference's full-scale NLL ("test-NLL match", BASELINE.json metric).
Eval steps of the cfg* workloads launch eagerly (one chain / layer launch per step; `--graph`
replays a captured HIP graph instead): with the host issuing ahead of the device, a plain launch
leaves less idle between steps than a graph replay (measured, `profiles/r05_graph_vs_eager.jsonl`:
cfg2 125k 164.7 vs 167.0 us, cfg3 125k 131.9 vs 136.0 us, cfg5i 1Ki 32.1 vs 36.3 us, cfg2 1M
equal). The sample4k* steps (several small launches each) keep the graph (`--eager` opts out).

At the default config (cfg2, RealNVP d=2) the line nests the second half of the metric, MAF
d=63 (cfg4, 5x MAF(63,64), 4M samples split over the ranks), with its own roofline and CPU
baseline under "maf_d63".

Rank 0 prints ONE JSON line with the throughput, the roofline of the dominant kernel (HIP
events on the launch stream, over the timed steps) and, at N=1, the oracle CPU baseline timed on
this host (threads = physical cores within this process's CPU allotment) on a bounded sample of
the same workload.
"""
import argparse
import glob
import json
import math
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
sys.path.insert(0, ROOT)

import nfs_amd  # noqa: E402

PEAK_FP32_TFLOPS = 157.3  # MI355X dense FP32 (vector = matrix), MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 2516.6  # MI355X dense BF16 MFMA: 256 CUs x 4 SIMDs x 1024 flop/clk x 2.4 GHz
# The streaming affine kernels (cfg2) run layer 2 of each conditioner net as six bf16 piece
# products per fp32 multiply-add (csrc/nfx_affine_kernel.h, affine_net_split): the ceiling of
# that scheme, in the fp32 flops the layer computes, is the bf16 peak / 6.
PEAK_SPLIT_TFLOPS = PEAK_BF16_TFLOPS / 6
SPLIT_CONFIGS = ("cfg2",)
METRIC = "log_prob samples/sec/GPU + test-NLL match; RealNVP d=2 and MAF d=63"


def perturb(model, sigma, seed):
    """Same recipe as tests/golden/make_golden.py: no layer is the identity, BN stats non-trivial."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for _, p in model.named_parameters():
            p.add_(sigma * torch.randn(p.shape, generator=g))
        for _, mod in model.named_modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.copy_(0.1 * torch.randn(mod.running_mean.shape, generator=g))
                mod.running_var.copy_(0.5 + torch.rand(mod.running_var.shape, generator=g))


# the G16 figure-model training configs: fixture key prefix and Adam learning rate
FIG_TRAIN = {"trainfig_spline": ("spline", 5e-4), "trainfig_maf": ("maf", 1e-3), "trainfig_iaf": ("iaf", 1e-3)}


def build(config):
    """(model, d, flops_per_sample_per_layer, oracle spec, description)."""
    if config == "cfg2":
        torch.manual_seed(0)
        m = nfs_amd.RealNVP(2, 8, 64)
        perturb(m, 0.1, 1)
        H, d = 64, 2
        # 2 nets x 2 flop x (n_c*H + H*H + H*n_t), n_c = n_t = 1
        f = 2 * 2 * (1 * H + H * H + H * 1)
        import oracle
        return m, d, f, oracle.realnvp_spec(8), "cfg2 RealNVP(data_dim=2, n_layers=8, hidden_dim=64) log_prob, eval"
    if config == "cfg3":
        torch.manual_seed(10)
        layers = []
        for i in range(8):
            mask = torch.zeros(2)
            if i % 2 == 0:
                mask[:1] = 1
            else:
                mask[1:] = 1
            layers.append(nfs_amd.SplineCouplingLayer(2, 64, mask, num_bins=8))
        m = nfs_amd.NormalizingFlowModel(layers)
        perturb(m, 0.1, 11)
        H, K = 64, 8
        f = 2 * (1 * H + H * H + H * (3 * K - 1))
        import oracle
        return m, 2, f, [("spline", f"flows.{i}.", {"K": 8}) for i in range(8)], \
            "cfg3 8x SplineCouplingLayer(2, 64, K=8) log_prob, eval"
    if config == "cfg4":
        torch.manual_seed(30)
        m = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(63, 64) for _ in range(5)])
        perturb(m, 0.02, 31)
        d, H = 63, 64
        f = 2 * (d * H + 2 * H * H + 2 * d * H)
        import oracle
        return m, d, f, oracle.maf_spec(5), "cfg4 5x MaskedAutoregressiveFlow(63, 64) log_prob, eval"
    if config in ("sample4k_fused", "sample4k_spline_fused"):
        m, d, f, spec, desc = build(config[:-len("_fused")])
        return m, d, f, spec, desc.replace("sampling: model.forward(z)", "sampling with the N(0, I) draw fused on the "
                                                                         "device: model.sample_fused(n)")
    if config == "sample4k":
        torch.manual_seed(3)
        m = nfs_amd.RealNVP(2, 10, 128)
        perturb(m, 0.1, 4)
        H = 128
        f = 2 * 2 * (1 * H + H * H + H * 1)
        import oracle
        return m, 2, f, oracle.realnvp_spec(10), \
            "sample4k RealNVP(2,10,128) sampling: model.forward(z), n=4000 per call (plots/_common.py:264-274)"
    if config == "sample4k_spline":
        torch.manual_seed(5)
        m = nfs_amd.RealNVPSpline(2, 8, 64)
        perturb(m, 0.1, 6)
        H, K = 64, 10
        # 2 flop x (n_c*H + H*H + H*n_t*(3K-1)), n_c = n_t = 1
        f = 2 * (1 * H + H * H + H * (3 * K - 1))
        import oracle
        return m, 2, f, oracle.spline_model_spec(8), \
            "sample4k_spline RealNVPSpline(2,8,64) (K=10) sampling: model.forward(z), n=4000 per call " \
            "(plots/_common.py:163,264-274)"
    if config in ("sample4k_maf", "sample4k_iaf"):
        torch.manual_seed(7)
        cls = nfs_amd.MaskedAutoregressiveFlow if config == "sample4k_maf" else nfs_amd.InverseAutoregressiveFlow
        m = nfs_amd.NormalizingFlowModel([cls(2, 64) for _ in range(6)])
        perturb(m, 0.02, 8)
        d, H = 2, 64
        f = 2 * (d * H + 2 * H * H + 2 * d * H)
        import oracle
        kind = "maf" if config == "sample4k_maf" else "iaf"
        spec = [(kind, f"flows.{i}.", {}) for i in range(6)]
        what = "MAF forward = sequential over d" if kind == "maf" else "IAF forward = parallel"
        return m, d, f, spec, \
            f"{config} 6x{kind.upper()}(2,64) sampling ({what}): model.forward(z), n=4000 per call " \
            f"(plots/_common.py:165-167,264-274)"
    if config == "trainfig":
        # the reference's benchmark-figure model in its training loop (plots/_common.py:161,
        # 178-183, 194-211): RealNVP(2, 10, 128), full batch of 2,000 two-moons points, train-mode
        # BatchNorm, Adam lr 1e-3, clip_grad_norm_ 5.0; weights + data from the G15 fixture
        m = nfs_amd.RealNVP(2, 10, 128)
        H = 128
        f = 2 * (3 * 2 * H * H + 2 * H + 2 * 2 * H)  # BWD2 per net, as cfg2t
        import oracle
        return m, 2, f, oracle.realnvp_spec(10, training=True), \
            ("trainfig RealNVP(2,10,128) training step, full batch of 2,000 two-moons points "
             "(plots/_common.py:161,194-211: train-mode BatchNorm, Adam lr 1e-3, clip_grad_norm_ 5.0)")
    if config in FIG_TRAIN:
        # the reference's other benchmark-figure models in its training loop (plots/_common.py:
        # 157-169, 178-183, 194-211), weights + data from the G16 fixture
        import oracle
        if config == "trainfig_spline":
            m, H, K = nfs_amd.RealNVPSpline(2, 8, 64), 64, 10
            P = 3 * K - 1
            f = 2 * (3 * H * H + 3 * H + 3 * H * P)  # fused spline backward, as cfg3t
            return m, 2, f, oracle.spline_model_spec(8), \
                ("trainfig_spline RealNVPSpline(2,8,64) K=10 training step, full batch of 2,000 two-moons "
                 "points (plots/_common.py:163,194-211: Adam lr 5e-4, clip_grad_norm_ 5.0)")
        kind = "maf" if config == "trainfig_maf" else "iaf"
        cls = nfs_amd.MaskedAutoregressiveFlow if kind == "maf" else nfs_amd.InverseAutoregressiveFlow
        m = nfs_amd.NormalizingFlowModel([cls(2, 64) for _ in range(6)])
        d, H = 2, 64
        f = 2 * 2 * (d * H + 2 * H * H + 2 * d * H)  # forward recompute + data-gradient chain
        spec = [(kind, f"flows.{i}.", {}) for i in range(6)]
        return m, d, f, spec, \
            (f"{config} 6x{kind.upper()}(2,64) training step, full batch of 2,000 two-moons points "
             f"(plots/_common.py:165-167,194-211: Adam lr 1e-3, clip_grad_norm_ 5.0)")
    if config in ("cfg2t", "train5k"):
        torch.manual_seed(0)
        m = nfs_amd.RealNVP(2, 8, 64)
        perturb(m, 0.03, 1)
        H = 64
        # dominant kernel = BWD2 of the train-mode backward, per net: (diag(r2) W2)^T e2 and
        # dW2 = sum e2 a1^T (2 x 2H^2) + layer 1 (2H) + W3^T delta3 (2H), the layer-2
        # pre-activations read from the copy the statistics pass kept (run_config re-prices it
        # from coupling.KEEP_STATS when a layer recomputed instead: NFX_TRAIN_KEEP=0 or over the
        # keep budget, where the kernel also recomputes layer 2 and the output layer,
        # 3 x 2H^2 + 2H + 2 x 2H)
        f = 2 * (2 * 2 * H * H + 2 * H + 2 * H)
        import oracle
        what = ("cfg2t RealNVP(2,8,64) training step (train-mode BatchNorm: batch statistics + "
                "running-stat update, -log_prob mean, fused backward, Adam)") if config == "cfg2t" else \
            ("train5k RealNVP(2,8,64) full-batch training step on 5,000 samples (README.md:107-117: "
             "two-moons-sized batch, train-mode BatchNorm, Adam)")
        return m, 2, f, oracle.realnvp_spec(8, training=True), what
    if config == "cfg4t":
        m, d, f, spec, _ = build("cfg4")
        # training step: forward recompute + data-gradient chain in the fused backward kernel
        return m, d, 2 * f, spec, "cfg4t 5x MaskedAutoregressiveFlow(63, 64) training step " \
                                  "(-log_prob mean, fused backward, Adam), train mode"
    if config == "cfg3t":
        m, d, _, spec, _ = build("cfg3")
        H, P = 64, 3 * 8 - 1
        # fused spline backward per sample: MLP recompute (H + H^2 + H P), data-gradient chain
        # (P H + H^2 + H) and weight-gradient contractions (P H + H^2 + H), 2 flop each
        f = 2 * (3 * H * H + 3 * H + 3 * H * P)
        return m, d, f, spec, "cfg3t 8x SplineCouplingLayer(2, 64, K=8) training step " \
                              "(-log_prob mean, fused spline backward, Adam)"
    if config in ("cfg5f", "cfg5i"):
        torch.manual_seed(40)
        m = nfs_amd.NormalizingFlowModel([nfs_amd.InverseAutoregressiveFlow(784, 64)])
        perturb(m, 0.01, 41)
        d, H = 784, 64
        # one MADE evaluation per sample in both directions: the sequential inverse kernel
        # computes every hidden unit once, when the input of its degree is known
        f = 2 * (d * H + 2 * H * H + 2 * d * H)
        import oracle
        spec = [("iaf", "flows.0.", {})]
        if config == "cfg5f":
            return m, d, f, spec, "cfg5f IAF(784, 64) forward (sampling, parallel), eval"
        return m, d, f, spec, "cfg5i IAF(784, 64) log_prob (sequential inverse), eval"
    raise ValueError(config)

TRAIN_CONFIGS = ("cfg4t", "cfg2t", "train5k", "cfg3t", "trainfig", "trainfig_spline", "trainfig_maf", "trainfig_iaf")

# Batch of each config: the BASELINE global batch (strong scaling splits it over the ranks,
# --weak gives every rank all of it).
DEFAULT_BATCH = {"cfg2": 1_000_000, "cfg2t": 1_000_000, "train5k": 5_000, "trainfig": 2_000, "trainfig_spline": 2_000,
                 "trainfig_maf": 2_000, "trainfig_iaf": 2_000, "cfg3": 1_000_000, "cfg3t": 1_000_000,
                 "cfg4": 4_000_000, "cfg4t": 500_000, "cfg5f": 524_288, "cfg5i": 8_192,
                 "sample4k": 4_000, "sample4k_spline": 4_000, "sample4k_maf": 4_000, "sample4k_iaf": 4_000,
                 "sample4k_fused": 4_000, "sample4k_spline_fused": 4_000}
# The reference's only published throughput (assets/benchmark.png via
# plots/_common.py:264-274): RealNVP(2,10,128) sampling, model.forward(z) on n = 4,000, CPU.
# The same figure's other sampling numbers: Spline = RealNVPSpline(2,8,64) K=10,
# MAF = 6x MaskedAutoregressiveFlow(2,64), IAF = 6x InverseAutoregressiveFlow(2,64) (plots/_common.py:161-167).
PUBLISHED_SAMPLING = {"sample4k": ("RealNVP(2,10,128)", 186_000.0),
                      "sample4k_spline": ("RealNVPSpline(2,8,64), K=10", 334_000.0),
                      "sample4k_maf": ("6x MAF(2,64)", 602_000.0),
                      "sample4k_iaf": ("6x IAF(2,64)", 1_121_000.0),
                      # the same models with the base draw inside the timed step (the reference's
                      # figure times forward(z) on a fixed z: this line does strictly more work)
                      "sample4k_fused": ("RealNVP(2,10,128), draw included", 186_000.0),
                      "sample4k_spline_fused": ("RealNVPSpline(2,8,64), K=10, draw included", 334_000.0)}
# Reference-pinned workloads: weights from the golden fixture (written by importing the
# reference, tests/golden/make_golden.py), input = the G8 seeded batch, result vs the reference's
# own full-scale NLL / checksums (tests/golden/g8_full_nll.json).
REFERENCE_RUN = {
    "cfg2": {"npz": "g2_realnvp.npz", "prefix": "", "sub": "", "g8": "cfg2_realnvp_d2_B1M"},
    "cfg3": {"npz": "g3_spline.npz", "prefix": "k8.", "sub": "", "g8": "cfg3_spline_k8_d2_B1M"},
    "cfg4": {"npz": "g5_maf63.npz", "prefix": "", "sub": "", "g8": "cfg4_maf_d63_B4M"},
    "cfg5i": {"npz": "g6_iaf784.npz", "prefix": "", "sub": "flows.0.", "g8": "cfg5i_iaf_d784_B8192"},
    "cfg5f": {"npz": "g6_iaf784.npz", "prefix": "", "sub": "flows.0.", "g8": "cfg5f_iaf_d784_B524288"},
}
GOLDEN = os.path.join(ROOT, "tests", "golden")


def load_reference_weights(model, config):
    import numpy as np
    spec = REFERENCE_RUN[config]
    with np.load(os.path.join(GOLDEN, spec["npz"]), allow_pickle=False) as z:
        arrs = {k: z[k] for k in z.files}
    sd = {}
    for k, v in model.state_dict().items():
        gk = spec["prefix"] + (k[len(spec["sub"]):] if spec["sub"] and k.startswith(spec["sub"]) else k)
        sd[k] = torch.from_numpy(np.array(arrs[gk])) if gk in arrs else v
    model.load_state_dict(sd)


def figure_batch(name="g15_fig_train.npz"):
    """G15 / G16: the figure models' initial weights and the 2,000 standardized two-moons points
    (plots/_common.py:103-112), as the reference generated them."""
    import numpy as np
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        arrs = {k: z[k] for k in z.files}
    return arrs


def g8_meta(config):
    with open(os.path.join(GOLDEN, "g8_full_nll.json")) as fh:
        return json.load(fh)[REFERENCE_RUN[config]["g8"]]


def made_executed_flop_per_sample(d, H):
    """fp32 MFMA flops per sample the MADE tile kernel actually issues: per output tile of 32
    rows, the k-loop stops at the last 32x32 block with a nonzero masked weight (structural
    zeros of the sorted MADE degrees, DESIGN.md 'Structural zeros'); 16 v_mfma_f32_32x32x2_f32
    (4,096 flop each) per block per 32 samples."""
    from nfs_amd.flows.autoregressive import made_degrees
    deg = torch.tensor(made_degrees(d, H))
    i = torch.arange(d)
    masks = [(i[None, :] <= deg[:, None]), (deg[None, :] <= deg[:, None]), (deg[None, :] <= deg[:, None]),
             (deg[None, :] < i[:, None]), (deg[None, :] < i[:, None])]  # W1, W2, W3, W4 mu rows, W4 alpha rows
    blocks = 0
    for m in masks:
        R, C = m.shape
        for t in range((R + 31) // 32):
            rows = m[32 * t:32 * t + 32]
            nz = [kb for kb in range((C + 31) // 32) if bool(rows[:, 32 * kb:32 * kb + 32].any())]
            blocks += (max(nz) + 1) if nz else 0
    return blocks * 16 * 4096 / 32


def cpu_info():
    """Host CPU facts for the baseline: model, physical cores, logical CPUs, this process's
    allotment (affinity / OMP_NUM_THREADS), and the thread count used = physical cores capped by
    the allotment (the GPU box grants 16 CPUs per GPU via OMP_NUM_THREADS; more threads would
    oversubscribe a host shared with other jobs)."""
    model = "?"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cores = set()
    for cpu in glob.glob("/sys/devices/system/cpu/cpu[0-9]*/topology"):
        try:
            with open(os.path.join(cpu, "core_id")) as a, open(os.path.join(cpu, "physical_package_id")) as b:
                cores.add((a.read().strip(), b.read().strip()))
        except OSError:
            pass
    physical = len(cores) or (os.cpu_count() or 1)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    allot = min(affinity, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else affinity
    return {"cpu_model": model, "physical_cores": physical, "logical_cpus": os.cpu_count(),
            "affinity_cpus": affinity, "omp_num_threads": omp, "threads": max(1, min(physical, allot))}


def cpu_baseline(model, spec, x_cpu, budget_s=20.0, forward=False, bn_prefix=None):
    """The oracle (op-for-op CPU restatement of the reference) timed on this host."""
    import oracle
    info = cpu_info()
    threads = info["threads"]
    torch.set_num_threads(threads)
    n = x_cpu.shape[0]
    x = x_cpu.float()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    times = []

    def run():
        if forward:
            return oracle.flow_model(sd, spec, x, 1, bn_prefix=bn_prefix)
        z, ld = oracle.flow_model(sd, spec, x, -1, bn_prefix=bn_prefix)
        return z, oracle.gauss_log_prob(z, ld)

    with torch.no_grad():
        _, lp = run()  # warm-up
        t_end = time.perf_counter() + budget_s
        while len(times) < 5 and (time.perf_counter() < t_end or len(times) < 2):
            t0 = time.perf_counter()
            run()
            times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    what = "forward (sampling)" if forward else "log_prob"
    out = {"value": n / med, "unit": "samples/s", "cores": threads, "kind": "port",
           "sample": f"{n} rows of the same seeded batch, {what} via oracle/flows_ref.py "
                     f"(torch CPU, {threads} threads), median of {len(times)} runs after 1 warm-up"}
    out.update({k: info[k] for k in ("cpu_model", "physical_cores", "logical_cpus", "affinity_cpus",
                                     "omp_num_threads")})
    return out, (None if forward else oracle.nll_f64(lp))


def cpu_training_baseline(model, spec, x_gpu, budget_s=12.0, max_rows=32768):
    """One training step of the oracle on this host: autograd through oracle/flows_ref.py."""
    import oracle
    info = cpu_info()
    threads = info["threads"]
    torch.set_num_threads(threads)
    n = min(x_gpu.shape[0], max_rows)
    x = x_gpu[:n].detach().float().cpu()
    sd = {k: v.detach().cpu().clone().requires_grad_(v.is_floating_point() and not k.endswith(
        ("running_mean", "running_var", "mask"))) for k, v in model.state_dict().items()}
    times = []

    def run():
        for v in sd.values():
            v.grad = None
        z, ld = oracle.flow_model(sd, spec, x, -1)
        (-oracle.gauss_log_prob(z, ld).mean()).backward()

    with torch.enable_grad():
        run()
        t_end = time.perf_counter() + budget_s
        while len(times) < 5 and (time.perf_counter() < t_end or len(times) < 2):
            t0 = time.perf_counter()
            run()
            times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    out = {"value": n / med, "unit": "samples/s", "cores": threads, "kind": "port",
           "sample": f"{n} rows, loss + backward via autograd through oracle/flows_ref.py "
                     f"(torch CPU, {threads} threads), median of {len(times)} runs after 1 warm-up"}
    out.update({k: info[k] for k in ("cpu_model", "physical_cores", "logical_cpus", "affinity_cpus",
                                     "omp_num_threads")})
    return out


# CPU-baseline sample per config (rows of the same batch): the full batch where one oracle pass
# takes a few seconds; cfg4 times 1M of the 4M rows (the full batch would be ~4x the 20 s budget);
# the IAF d=784 passes are bounded by the oracle's sequential inverse (0.7k samples/s).
CPU_ROWS = {"cfg2": 1_000_000, "cfg3": 1_000_000, "cfg4": 1_000_000, "cfg5f": 16_384, "cfg5i": 1_024}


def run_config(config, a, world, rank, dev, strong, graph, with_cpu):
    """One benchmark line (dict on rank 0, None elsewhere)."""
    model, d, f_layer, spec, desc = build(config)
    training = config in TRAIN_CONFIGS
    coupling_train = config in ("cfg2t", "train5k", "trainfig")
    from nfs_amd.flows import coupling as _cpk
    _cpk.KEEP_STATS.update(kept=0, recompute=0)
    clip = 5.0 if (config == "trainfig" or config in FIG_TRAIN) else None
    lr = 1e-3 if config == "trainfig" else (FIG_TRAIN[config][1] if config in FIG_TRAIN else 1e-5)
    sampling = config == "cfg5f" or config.startswith("sample4k")
    pinned = config in REFERENCE_RUN
    if pinned:
        load_reference_weights(model, config)
    fig = None
    if config == "trainfig":
        fig = figure_batch()
        model.load_state_dict({k: (torch.from_numpy(fig["fig.init." + k].copy()) if "fig.init." + k in fig else v)
                               for k, v in model.state_dict().items()})
    elif config in FIG_TRAIN:
        g16 = figure_batch("g16_fig_models.npz")
        pre = FIG_TRAIN[config][0] + ".init."
        model.load_state_dict({k: (torch.from_numpy(g16[pre + k].copy()) if pre + k in g16 else v)
                               for k, v in model.state_dict().items()})
        fig = {"fig.x": g16["x"]}
    if coupling_train and world > 1:
        from nfs_amd.distributed import enable_sync_batchnorm
        enable_sync_batchnorm(True)  # batch statistics over all ranks = the full-batch step
    model = model.to(dev).train(training)
    from nfs_amd.distributed import average_gradients, broadcast_parameters, shard_range
    broadcast_parameters(model)  # replicate rank 0's weights (one-time, < 1 MB)
    B_unit = (a.batch if config == a.config else None) or DEFAULT_BATCH[config]
    if strong:
        lo, hi = shard_range(B_unit, rank, world)
        B, B_global = hi - lo, B_unit
    else:
        lo, hi = 0, B_unit
        B, B_global = B_unit, B_unit * world
    x_ref = None
    if fig is not None:
        x = torch.from_numpy(fig["fig.x"][lo:hi].copy()).to(dev)
    elif pinned and B_unit == g8_meta(config)["B"]:
        meta = g8_meta(config)
        x_ref = torch.randn(meta["B"], meta["d"], generator=torch.Generator().manual_seed(meta["seed"]))
        x = x_ref[lo:hi].to(dev)
    else:
        g = torch.Generator(device=dev).manual_seed(1234 + rank)
        x = torch.randn(B, d, device=dev, generator=g)
    flow = model.flow if hasattr(model, "flow") else model

    fused_draw = config.endswith("_fused")
    graphed = None
    if graph and not training:
        graphed = nfs_amd.GraphedFlow(flow, x, mode=("sample" if fused_draw else "forward") if sampling else "log_prob",
                                      strict=False)
    # Adam (the reference's optimizer, plots/_common.py:194-211) in torch's fused form: one
    # multi-tensor kernel per step instead of a few dozen per-parameter elementwise launches
    opt = torch.optim.Adam(model.parameters(), lr=lr, capturable=graph, fused=True) if training else None
    graphed_train = None
    if graph and training:
        if world > 1:
            raise SystemExit("--graph training is single-GPU (the SyncBN / gradient collectives run eagerly)")
        graphed_train = nfs_amd.GraphedTrainStep(flow, x, opt, warmup=a.warmup, clip_grad_norm=clip)

    eager_only = [False]  # the per-kernel event pass runs eager steps (a graph replay records no events)
    # Eval steps all-reduce their float64 [sum log p, count] pair asynchronously: every step's
    # 16 bytes still cross RCCL, but the next step's kernels do not queue behind the collective
    # (the pair is copied out of the graph's reused output buffer first); all pending reductions
    # are waited for before the closing synchronize + barrier, inside the timed region.
    pending = []

    def drain():
        for w in pending:
            w.wait()
        pending.clear()

    def step():
        if graphed_train is not None and not eager_only[0]:
            loss = graphed_train()
            return torch.stack([-loss.double() * B, torch.full((), float(B), device=dev, dtype=torch.float64)])
        if training:
            # data-parallel training step: HIP forward, fused HIP backward, one bucketed RCCL
            # all-reduce of the flat gradient (412 KB at cfg4), Adam
            opt.zero_grad(set_to_none=True)
            logp = flow.log_prob(x)
            loss = -logp.mean()
            loss.backward()
            average_gradients(model, local_count=B)
            if clip is not None:
                torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
            opt.step()
            return torch.stack([-loss.detach().double() * B, torch.tensor(float(B), device=dev, dtype=torch.float64)])
        if graphed is not None:
            out = graphed()
            if sampling:
                return out
            sums = out[1]
        elif sampling and fused_draw:  # z ~ N(0, I) drawn inside the chain kernel, x = forward(z)
            return flow.sample_fused(B, dev)
        elif sampling:  # sampling pass: x = forward(z), no exchange
            return flow.forward(x)
        else:
            logp, sums = flow.log_prob(x, return_sums=True)
        if world > 1:
            sums = sums.clone()
            pending.append(dist.all_reduce(sums, async_op=True))  # RCCL over xGMI: 16 bytes
        return sums

    from nfs_amd.flows import autoregressive as _ar
    from nfs_amd.flows import spline as _sp
    bwd_mod = _sp if config in ("cfg3t", "trainfig_spline") else _ar
    with torch.set_grad_enabled(training):
        for _ in range(a.warmup):
            step()
        drain()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        nfs_amd.reset_stats()
        w0 = time.monotonic_ns()  # the timed window on the clock rocprofv3 stamps kernels with
        t0 = time.perf_counter()
        for _ in range(a.steps):
            out = step()
        drain()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = time.perf_counter() - t0
        w1 = time.monotonic_ns()
        torch_calls = nfs_amd.STATS["torch"]
        hip_calls = nfs_amd.STATS["hip"]
        # Kernel durations: the same K steps again with HIP events around every layer launch
        # on the launch stream. Kept out of the headline loop because each event record adds
        # ~5 us of GPU idle between kernels (measured, profiles/).
        eager_only[0] = True
        aux_events = []
        # A spin kernel ahead of every recorded pass keeps the GPU busy while the host enqueues the
        # pass (eager: ~20 us of Python + ctypes per layer), so an event pair brackets the kernel
        # itself, not the host's launch latency (which dominated short kernels: a 22 us layer read
        # 35 us without it).
        # The spin kernel idles the chip, and its clocks drop with it: one untimed pass right after
        # it brings the clocks back to the timed loop's steady state before the recorded pass (a
        # compute-bound layer read 4% slower straight after the spin than in the timed loop).
        def preroll():
            torch.cuda._sleep(int(1.2e7 if training else 2e6))
        if coupling_train:
            from nfs_amd.flows import coupling as _cp
            rec = []
            for _ in range(a.steps):
                preroll()
                _cp.TRAIN_EVENTS = None
                step()
                _cp.TRAIN_EVENTS = rec
                step()
            torch.cuda.synchronize()
            events = [e for e in rec if e[0].endswith("<BWD2>")]
            _cp.TRAIN_EVENTS = None
        elif training:
            rec = []
            for _ in range(a.steps):
                preroll()
                bwd_mod.BACKWARD_EVENTS = None
                step()
                bwd_mod.BACKWARD_EVENTS = rec
                step()
            torch.cuda.synchronize()
            events = [e for e in rec if e[0] != "made_wgrad_kernel"]
            aux_events = [e for e in rec if e[0] == "made_wgrad_kernel"]
            bwd_mod.BACKWARD_EVENTS = None
        else:
            rec = []
            for _ in range(a.steps):
                preroll()
                for r in (None, rec):
                    flow.layer_events = r
                    if sampling and fused_draw:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        flow.sample_fused(B, dev)
                        e1.record()
                        if r is not None:
                            r.append((nfs_amd._lib.last_kernel(), e0, e1))
                    elif sampling:
                        flow.forward(x)
                    else:
                        flow.log_prob(x, return_sums=True)
            torch.cuda.synchronize()
            events = rec
            flow.layer_events = None
    if torch_calls != 0 or (hip_calls == 0 and graphed is None and graphed_train is None):
        raise RuntimeError(f"hot path did not run on the HIP kernels: {nfs_amd.STATS}")
    t_all = torch.tensor([t], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t_all, op=dist.ReduceOp.MAX)
    t_max = float(t_all.item())

    keep_note = None
    if config in ("cfg2t", "train5k"):
        # price BWD2 by what the forwards actually did: kept pre-activations, or the
        # recompute kernel (NFX_TRAIN_KEEP=0 / a copy over the keep budget)
        H = 64
        kept, rec = _cpk.KEEP_STATS["kept"], _cpk.KEEP_STATS["recompute"]
        f_keep, f_rec = 2 * (2 * 2 * H * H + 2 * H + 2 * H), 2 * (3 * 2 * H * H + 2 * H + 2 * 2 * H)
        if kept + rec:
            f_layer = (kept * f_keep + rec * f_rec) / (kept + rec)
        keep_note = {"layers_kept": kept, "layers_recomputed": rec}
    # dominant kernel: the per-layer fused kernel (every launch of the timed steps), named by the
    # library as dispatched (nfx_last_kernel)
    durs = [e0.elapsed_time(e1) for _, e0, e1 in events]
    kname = events[0][0] if events else "?"
    mean_ms = sum(durs) / max(1, len(durs))
    # one-launch coupling chains (nfx_affine_chain / nfx_spline_chain): one event covers every layer
    layers_per_launch = len(flow.flows) if kname in ("affine_chain_kernel", "affine_schain_kernel",
                                                     "spline_chain_kernel", "spline_schain_kernel") else 1
    f_launch = f_layer * layers_per_launch
    achieved = f_launch * B / (mean_ms * 1e-3) / 1e12

    # result vs the reference's own full-scale run (global over ranks)
    ref_check = None
    nll = None
    if sampling and x_ref is not None:
        with torch.no_grad():
            xo, ldo = flow.forward(x)
            cs = torch.stack([xo.double().sum(), xo.double().abs().sum(), ldo.double().sum()])
        if world > 1:
            dist.all_reduce(cs)
        meta = g8_meta(config)
        scale = 1 if strong else world
        cs = [float(v) / scale for v in cs.cpu()]
        ref_check = {"out_abs_sum_rel_diff": abs(cs[1] - meta["out_abs_sum_f64"]) / meta["out_abs_sum_f64"],
                     "out_sum_diff_rel_to_abs_sum": abs(cs[0] - meta["out_sum_f64"]) / meta["out_abs_sum_f64"],
                     "ld_mean_abs_diff": abs(cs[2] - meta["ld_sum_f64"]) / meta["B"],
                     "source": "tests/golden/g8_full_nll.json " + REFERENCE_RUN[config]["g8"]}
    elif not sampling and not training:
        sums = out  # the last timed step's [sum log p, count], all-reduced over the ranks
        nll = -float(sums[0] / sums[1])
        if x_ref is not None:
            meta = g8_meta(config)
            tol = 1e-5 if config in ("cfg2", "cfg3") else 1e-6 * abs(meta["nll_f64"])
            ref_check = {"nll_gpu": nll, "nll_reference": meta["nll_f64"], "abs_diff": abs(nll - meta["nll_f64"]),
                         "tolerance": tol, "match": abs(nll - meta["nll_f64"]) <= tol,
                         "source": "tests/golden/g8_full_nll.json " + REFERENCE_RUN[config]["g8"]}

    if rank != 0:
        return None
    traffic = None
    rocprof = None
    # rocprofv3 evidence for this config (tools/profile_bench.sh + tools/reconcile_profile.py):
    # the trace of bench.py itself, the kernels inside ITS timed window, the same process's
    # ms_per_step, and the PMC HBM bytes per launch of the hot kernel. Quoted beside the live
    # event-timed numbers, with both step checks (same-run, and against this run's step).
    rp_name = config if B == DEFAULT_BATCH.get(config) else f"{config}_{B}"
    tp = os.path.join(ROOT, "profiles", f"rocprof_{rp_name}.json")
    lib_sha = lib_digest()
    rj = None
    if os.path.exists(tp):
        with open(tp) as fh:
            rj = json.load(fh)
    if rj is not None and rj.get("lib_sha256") != lib_sha:
        # profiled with another build of libnfx.so: its kernels may no longer exist as profiled
        rocprof = {"stale": True, "profiled_lib_sha256": rj.get("lib_sha256"), "source": os.path.relpath(tp, ROOT),
                   "round": rj.get("round"),
                   "note": "profile taken with a different libnfx.so build; figures withheld "
                           "(re-run tools/profile_bench.sh + tools/reconcile_profile.py)"}
    elif rj is not None:
        spl = rj["bench_roofline"]["samples_per_launch"]
        if rj.get("hbm_bytes_per_launch") and spl:
            traffic = rj["hbm_bytes_per_launch"] / spl * B
        rocprof = {"kernels": rj["hot_kernels"], "mean_launch_us": rj["rocprof_mean_launch_us"],
                   "launches_per_step": rj["launches_per_step"], "samples_per_launch": spl,
                   "achieved": rj["rocprof_achieved_tflops"], "frac": rj["rocprof_frac"],
                   "frac_executed": rj.get("rocprof_frac_executed"),
                   "kernel_ms_per_step": rj["rocprof_ms_per_step"],
                   "profiled_run_ms_per_step": rj["bench"]["ms_per_step"],
                   "fits_profiled_step": rj["fits_bench_step"],
                   "profiled_run_event_frac": rj["event_frac"],
                   "source": os.path.relpath(tp, ROOT), "round": rj.get("round")}
        if rj.get("mfma_busy_frac") is not None:
            # the MFMA-busy PMC pass (tools/reconcile_profile.py mfma_busy): share of the SIMD-cycles
            # the matrix pipe ran, the clock, and VALU instructions per MFMA of the hot kernel;
            # frac = busy x clock / 2.4 GHz x (algorithmic / issued MFMA flop)
            rocprof.update({"mfma_busy_frac": rj["mfma_busy_frac"], "mfma_issue_frac": rj.get("mfma_issue_frac"),
                            "clock_ghz": rj.get("clock_ghz"), "valu_insts_per_mfma": rj.get("valu_insts_per_mfma"),
                            "non_mfma_valu_per_mfma": rj.get("non_mfma_valu_per_mfma"),
                            "busy_cycles_per_mfma": rj["pmc_mfma"].get("busy_cycles_per_mfma"),
                            "valu_issue_frac": rj.get("valu_issue_frac"),
                            "pmc_pass_mean_launch_us": rj["pmc_mfma"].get("mean_duration_us"),
                            "identity": rj.get("mfma_identity"),
                            "busy_note": ("busy and clock come from the counter pass, whose dispatches run a little "
                                          "slower than the trace pass and this run (pmc_pass_mean_launch_us vs "
                                          "mean_launch_us); within that pass frac = busy x clock / 2.4 GHz x "
                                          "algorithmic/issued exactly (identity.rebuilt_frac = "
                                          "identity.frac_pmc_pass), so busy >= frac at any clock <= 2.4 GHz")})
    peak = PEAK_SPLIT_TFLOPS if config in SPLIT_CONFIGS else PEAK_FP32_TFLOPS
    result = {
        "metric": METRIC,
        "value": B_global * a.steps / t_max,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * t_max / a.steps,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": ("synthetic: the reference's seeded G8 batch (torch.randn, CPU generator) with the reference's own "
                 "weights from tests/golden (written by importing the reference)") if x_ref is not None else
                ("synthetic: x ~ N(0,1) generated on device (seed 1234+rank); seeded random-init weights "
                 "perturbed N(0, sigma^2) with non-trivial BatchNorm running stats"),
        "config": {"workload": desc, "batch_per_gpu": B, "global_batch": B_global,
                   "parallelism": (f"dp{world} (sample shards, 1 bucketed RCCL all-reduce of the flat gradient per step)"
                                   if training else f"dp{world} (sample shards, 1 RCCL all-reduce of 16 B per step)"),
                   "launch": "hip-graph replay" if graph else "eager"},
        "nll_f64": nll,
        "reference_check": ref_check,
        "timed_window_monotonic_ns": [w0, w1],
        # cfg5i's sequential kernel issues no MFMA (its dot products are VALU FMAs): bound = the
        # fp32 VALU rate, whose peak (packed FMA) equals the fp32 MFMA peak, 157.3 TFLOP/s
        "roofline": {"bound": "valu" if config == "cfg5i" else "mfma", "pipe": "valu" if config == "cfg5i" else "mfma",
                     "kernel": kname, "achieved": achieved,
                     "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                     "traffic": traffic, "flop_per_sample_per_launch": f_launch,
                     "layers_per_launch": layers_per_launch,
                     "samples_per_launch": B, "mean_launch_ms": mean_ms, "launches": len(durs),
                     "traffic_source": os.path.relpath(tp, ROOT) if traffic is not None else None,
                     "rocprof": rocprof},
        "cpu_baseline": None,
    }
    result["lib_sha256"] = lib_sha
    if rocprof is not None and not rocprof.get("stale"):
        # rocprof kernel time per step vs THIS run's step (a different process; the profiled run's
        # own check is fits_profiled_step) and the rocprof frac vs this run's event frac
        rocprof["fits_this_step"] = rocprof["kernel_ms_per_step"] <= result["ms_per_step"]
        # (kernels run a little slower under rocprofv3 than unprofiled: the ratio says how much)
        rocprof["kernel_ms_over_this_step"] = rocprof["kernel_ms_per_step"] / result["ms_per_step"]
        rocprof["frac_rel_diff_vs_events"] = abs(rocprof["frac"] - result["roofline"]["frac"]) / result["roofline"]["frac"]
    if config in SPLIT_CONFIGS:
        result["dtype_note"] = ("fp32 in, out and accumulate; layer 2 of each conditioner net multiplies as bf16 "
                                "piece products (each exact in fp32, six per fp32 multiply-add, dropped terms below "
                                "2^-25): vs the fp32 chain max |dz|/(1+|z|) 1.0e-6, mean dlogp 4.7e-9 at 1M rows "
                                "(tools/split_precision.py, profiles/r06_split/); nll_f64 vs the reference above")
        result["roofline"].update({
            "peak_basis": ("bf16 MFMA peak / 6: layer 2 of every conditioner net runs as six bf16 piece products "
                           "per fp32 multiply-add (v_mfma_f32_32x32x16_bf16, fp32 accumulate; fp32-accurate, not the "
                           "fp32 chain's bits); achieved counts the fp32 flops of the reference's arithmetic"),
            "frac_of_fp32_peak": achieved / PEAK_FP32_TFLOPS, "peak_fp32": PEAK_FP32_TFLOPS,
            "peak_bf16": PEAK_BF16_TFLOPS})
    if config == "cfg4":
        fe = made_executed_flop_per_sample(63, 64)
        ach_e = fe * B / (mean_ms * 1e-3) / 1e12
        rl = result["roofline"]
        result["roofline"]["note"] = (
            "headline achieved/frac = the flops the MFMA pipe executes: the tile kernel skips the 32x32 "
            "blocks that are structurally zero under the MADE mask. achieved_dense / frac_dense count the "
            "masked GEMMs as dense (SURVEY §8(d)'s algorithmic figure)")
        rl.update({"achieved_dense": rl["achieved"], "frac_dense": rl["frac"], "flop_per_sample_dense": f_launch,
                   "flop_per_sample_executed": fe, "achieved_executed": ach_e,
                   "frac_executed": ach_e / PEAK_FP32_TFLOPS, "achieved": ach_e, "frac": ach_e / PEAK_FP32_TFLOPS})
        if rocprof is not None and rocprof.get("frac_executed"):
            rocprof.update({"frac_dense": rocprof["frac"], "frac": rocprof["frac_executed"]})
            rocprof["frac_rel_diff_vs_events"] = abs(rocprof["frac"] - rl["frac"]) / rl["frac"]
    if config in PUBLISHED_SAMPLING:
        mname, pub = PUBLISHED_SAMPLING[config]
        result["metric"] = f"sampling samples/sec ({mname}, n=4000 per forward call)"
        result["vs_baseline"] = result["value"] / pub
        result["published_baseline"] = {"value": pub, "unit": "samples/s", "hardware": "CPU (unspecified)",
                                        "source": "assets/benchmark.png via plots/_common.py:264-274"}
        result["nll_f64"] = None
    if coupling_train:
        result["metric"] = "training samples/sec/GPU (RealNVP d=2 train-mode step)"
        if fig is not None:
            result["metric"] = "training samples/sec/GPU (RealNVP(2,10,128) figure-model train-mode step)"
            result["data"] = ("the reference's own initial weights and 2,000 standardized two-moons points "
                              "(tests/golden/g15_fig_train.npz, written by importing the reference)")
        result["nll_f64"] = None
        if keep_note is not None:
            result["roofline"]["pre_activations"] = keep_note
        result["roofline"]["note"] = ("dominant kernel = BWD2 of the train-mode coupling backward "
                                      "(W2^T e2 and the sample-contraction dW2 on MFMA, one net per "
                                      "workgroup); a layer runs STATS1, STATS2 (keeps the layer-2 "
                                      "pre-activations, 512 B/sample), OUT, BWD1-3")
        if world > 1:
            result["config"]["parallelism"] = (f"dp{world} (sample shards, SyncBN: 4 all-gathers/all-reduces "
                                               f"of <= 3 KB per layer + 1 bucketed gradient all-reduce)")
    elif config in FIG_TRAIN:
        result["metric"] = f"training samples/sec/GPU ({desc.split(' training')[0].split(' ', 1)[1]} figure-model step)"
        result["data"] = ("the reference's own initial weights and 2,000 standardized two-moons points "
                          "(tests/golden/g16_fig_models.npz, written by importing the reference)")
        result["nll_f64"] = None
        result["roofline"]["note"] = ("dominant kernel = the layer's fused backward (spline: MLP recompute, "
                                      "spline adjoint, data-gradient chain and weight contractions; MADE: "
                                      "forward recompute + data-gradient chain); at 2,000 samples the step "
                                      "is launch-bound, frac is small by construction")
    elif config == "cfg3t":
        result["metric"] = "training samples/sec/GPU (8x RQ-spline coupling d=2 density step)"
        result["nll_f64"] = None
        result["roofline"]["note"] = ("dominant kernel = the fused spline backward (MLP recompute, "
                                      "spline adjoint, data-gradient chain and the sample-contraction "
                                      "weight gradients on MFMA, 3x the layer's forward MLP flops)")
    elif training:
        result["metric"] = "training samples/sec/GPU (MAF d=63 density step)"
        result["nll_f64"] = None
        result["roofline"]["note"] = ("dominant kernel = the fused backward (forward recompute + "
                                      "data-gradient chain, 2x the layer's forward flops); the "
                                      "weight gradients run as the MFMA sample-contraction kernel "
                                      "(made_wgrad_kernel, HBM-bound: reads the factor rows once). "
                                      "frac counts the dense flops; the recompute and the transposed "
                                      "chains skip the structurally-zero 32x32 blocks (the transposed "
                                      "staircase has as many blocks as the forward one): frac_executed")
        fe = 2 * made_executed_flop_per_sample(63, 64)
        ach_e = fe * B / (mean_ms * 1e-3) / 1e12
        result["roofline"].update({"flop_per_sample_executed": fe, "achieved_executed": ach_e,
                                   "frac_executed": ach_e / PEAK_FP32_TFLOPS})
        if aux_events:
            wd = [e0.elapsed_time(e1) for _, e0, e1 in aux_events]
            wms = sum(wd) / len(wd)
            fac_bytes = 4 * B * (2 * 63 + 3 * 64 + 3 * 64 + 63)  # δ + input rows the contraction reads
            result["roofline"]["wgrad"] = {"kernel": "made_wgrad_kernel", "bound": "hbm", "mean_launch_ms": wms,
                                           "bytes_per_launch": fac_bytes,
                                           "achieved": fac_bytes / (wms * 1e-3) / 1e9, "peak": 8000.0,
                                           "unit": "GB/s", "frac": fac_bytes / (wms * 1e-3) / 1e9 / 8000.0}
    if world == 1 and with_cpu and training:
        result["cpu_baseline"] = cpu_training_baseline(model, spec, x)
    elif world == 1 and with_cpu:
        rows = CPU_ROWS.get(config, 4000 if config.startswith("sample4k") else 262144)
        xs = (x_ref if x_ref is not None else x.cpu())[:rows]
        cb, cpu_nll = cpu_baseline(model, spec, xs, forward=sampling)
        if not sampling:
            gpu_nll = flow.nll(xs.to(dev))
            cb["nll_abs_diff_vs_gpu"] = abs(cpu_nll - gpu_nll)
        result["cpu_baseline"] = cb
    return result


def lib_digest():
    """sha256 (first 16 hex digits) of the libnfx.so this process loaded: ties a reconciled
    rocprof profile to the build it measured."""
    import hashlib
    from nfs_amd import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher around it: start N child ranks of this script (one
    process per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets
    them, rendezvous on 127.0.0.1), relay rank 0's JSON line, and return non-zero when any rank
    fails (the others are then terminated). This process never touches the GPU: the ranks are
    children started with fork + exec before anything here initialised HIP."""
    import signal
    import subprocess
    import tempfile
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs, outs = [], []
    libc = None
    try:
        import ctypes
        libc = ctypes.CDLL("libc.so.6", use_errno=True)
    except OSError:
        pass

    def die_with_parent():  # runs in the child between fork and exec: no GPU state exists there
        if libc is not None:
            libc.prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG

    def stop_all(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old_term = signal.signal(signal.SIGTERM, lambda *a: (stop_all(), sys.exit(143)))
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port, NFX_BENCH_LAUNCHER="bench.py")
            out = tempfile.TemporaryFile(mode="w+") if r == 0 else None
            outs.append(out)
            procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                                          stdout=out if r == 0 else sys.stderr, preexec_fn=die_with_parent))
        rc = 0
        live = list(range(n))
        while live:
            for r in list(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.remove(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print(f"bench.py launcher: rank {r} exited with {c}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    stop_all()
            time.sleep(0.05)
        outs[0].seek(0)
        text = outs[0].read()
    finally:
        stop_all()
        signal.signal(signal.SIGTERM, old_term)
    lines = [ln for ln in text.splitlines() if ln.strip()]
    for ln in lines[:-1]:
        print(ln, file=sys.stderr)
    if lines:
        try:
            res = json.loads(lines[-1])
            res["launcher"] = f"bench.py --gpus {n}: {n} child ranks (RANK/LOCAL_RANK/WORLD_SIZE, 127.0.0.1:{port})"
            print(json.dumps(res), flush=True)
        except json.JSONDecodeError:
            print(lines[-1], flush=True)
    elif rc == 0:
        print("bench.py launcher: rank 0 printed nothing", file=sys.stderr)
        rc = 1
    return rc


def launch_check(world, rank, local):
    """NFX_BENCH_LAUNCH_CHECK=1: the ranks join a gloo group and report who they are, with no GPU
    call — the CPU test of the `--gpus N` launcher (tests/test_bench_cpu.py). NFX_BENCH_FAIL_RANK=r
    makes rank r exit 3 before joining (the launcher must then fail and stop the others)."""
    if os.environ.get("NFX_BENCH_FAIL_RANK") == str(rank):
        raise SystemExit(3)
    dist.init_process_group("gloo")
    me = {"rank": dist.get_rank(), "local_rank": local, "pid": os.getpid(), "env_rank": rank}
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, me)
    if rank == 0:
        print(json.dumps({"launch_check": True, "world_size": dist.get_world_size(), "ranks": allr}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2",
                    choices=["cfg2", "cfg2t", "train5k", "trainfig", "trainfig_spline", "trainfig_maf", "trainfig_iaf", "cfg3", "cfg3t", "cfg4", "cfg4t", "cfg5f", "cfg5i",
                             "sample4k",
                             "sample4k_spline", "sample4k_maf", "sample4k_iaf", "sample4k_fused",
                             "sample4k_spline_fused"])
    ap.add_argument("--batch", type=int, default=None,
                    help="global batch (default: the BASELINE batch, 1M; 4M cfg4; 512Ki cfg5f; 8Ki cfg5i)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay a captured HIP graph of the step (training: nfs_amd.GraphedTrainStep; "
                         "cfg* eval: nfs_amd.GraphedFlow)")
    ap.add_argument("--eager", action="store_true",
                    help="sample4k* configs: eager launches instead of the captured HIP graph (GraphedFlow)")
    ap.add_argument("--weak", action="store_true", help="weak scaling: every rank processes the whole batch")
    ap.add_argument("--strong", action="store_true", help="(default) strong scaling: split the batch over the ranks")
    ap.add_argument("--no-secondary", action="store_true", help="cfg2: skip the nested MAF d=63 (cfg4) line")
    a = ap.parse_args(argv)
    if a.gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {a.gpus})")

    if "WORLD_SIZE" not in os.environ:
        if a.gpus > 1:
            # no launcher around us: start the N ranks ourselves (one process per GPU)
            raise SystemExit(launch_ranks(a.gpus, sys.argv[1:] if argv is None else list(argv)))
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if world != a.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={world} from the launcher but --gpus {a.gpus}; "
                             f"they must agree (one rank per GPU)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("NFX_BENCH_LAUNCH_CHECK") == "1":
        return launch_check(world, rank, local)
    # NFX_BENCH_REHEARSE=1: every rank on cuda:0 with gloo collectives — exercises the N > 1 code
    # path (sharding, barriers, max-over-ranks timing, reductions) on a one-GPU box; its numbers
    # are not a scaling measurement (the ranks share one GPU)
    rehearse = os.environ.get("NFX_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    elif world > 1 and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py: --gpus {world} but only {torch.cuda.device_count()} GPU(s) visible")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rank_devices = None
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        props = torch.cuda.get_device_properties(dev)
        mine = f"rank {rank}: cuda:{local} {props.name} pci {getattr(props, 'pci_bus_id', '?')}"
        rank_devices = [None] * dist.get_world_size()
        dist.all_gather_object(rank_devices, mine)
    training = a.config in TRAIN_CONFIGS
    graph = a.graph if training else ((not a.eager) if a.config.startswith("sample4k") else (a.graph and not a.eager))
    strong = not a.weak
    result = run_config(a.config, a, world, rank, dev, strong, graph, not a.no_cpu)
    if a.config == "cfg2" and not a.no_secondary:
        sec = run_config("cfg4", a, world, rank, dev, strong, graph, not a.no_cpu)
        if rank == 0:
            result["maf_d63"] = sec
    if rank == 0:
        if rehearse:
            result["rehearsal"] = "NFX_BENCH_REHEARSE=1: all ranks shared cuda:0 over gloo (not a scaling result)"
        result["world_size"] = dist.get_world_size() if world > 1 else 1
        result["rank_devices"] = rank_devices or [f"rank 0: cuda:{local} {torch.cuda.get_device_name(dev)}"]
        result["backend"] = (dist.get_backend() if world > 1 else None)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
