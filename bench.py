"""Benchmark: log_prob throughput of the gfx950 flow-transform hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5f|cfg5i]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One step = one log_prob pass over the per-GPU batch: every flow layer's fused kernel
(conditioner MLP on fp32 MFMA + transform + log-det accumulate), the fused Gaussian base term
with the float64 NLL partial sum, and (N > 1) ONE RCCL all-reduce of the 16-byte partial
[sum log p, count] — the whole data-parallel exchange of the path.
Weak scaling: each rank owns a fixed 1M-sample shard (configs[1] of BASELINE.json at N=1).
cfg5f / cfg5i (BASELINE configs[4], IAF(784, 64)): one step = the sampling pass forward(z)
(parallel MADE kernel) / the density pass log_prob(x) through the sequential IAF inverse.

Rank 0 prints ONE JSON line with the throughput, the roofline of the dominant kernel (HIP
events on the launch stream, over the timed steps) and, at N=1, the oracle CPU baseline timed on
this host on a bounded sample of the same workload.
"""
import argparse
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
    if config in ("cfg2t", "train5k"):
        torch.manual_seed(0)
        m = nfs_amd.RealNVP(2, 8, 64)
        perturb(m, 0.03, 1)
        H = 64
        # dominant kernel = BWD2 of the train-mode backward: per net layer-2 forward recompute,
        # (diag(r2) W2)^T e2 and dW2 = sum e2 a1^T (3 x 2H^2) + layer 1 (2H) + output layer and
        # W3^T delta3 (2 x 2H), n_c = n_t = 1
        f = 2 * (3 * 2 * H * H + 2 * H + 2 * 2 * H)
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

# per-GPU batch of each config (weak scaling unit)
DEFAULT_BATCH = {"cfg2": 1_000_000, "cfg2t": 1_000_000, "train5k": 5_000, "cfg3": 1_000_000, "cfg3t": 1_000_000,
                 "cfg4": 500_000,
                 "cfg4t": 500_000, "cfg5f": 524_288,
                 "cfg5i": 8_192, "sample4k": 4_000, "sample4k_spline": 4_000, "sample4k_maf": 4_000,
                 "sample4k_iaf": 4_000}
# The reference's only published throughput (assets/benchmark.png via
# plots/_common.py:264-274): RealNVP(2,10,128) sampling, model.forward(z) on n = 4,000, CPU.
# The same figure's other sampling numbers: Spline = RealNVPSpline(2,8,64) K=10,
# MAF = 6x MaskedAutoregressiveFlow(2,64), IAF = 6x InverseAutoregressiveFlow(2,64) (plots/_common.py:161-167).
PUBLISHED_SAMPLING = {"sample4k": ("RealNVP(2,10,128)", 186_000.0),
                      "sample4k_spline": ("RealNVPSpline(2,8,64), K=10", 334_000.0),
                      "sample4k_maf": ("6x MAF(2,64)", 602_000.0),
                      "sample4k_iaf": ("6x IAF(2,64)", 1_121_000.0)}


def cpu_baseline(model, spec, x_gpu, budget_s=12.0, forward=False, max_rows=262144):
    """The oracle (op-for-op CPU restatement of the reference) timed on this host."""
    import oracle
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    n = min(x_gpu.shape[0], max_rows)
    x = x_gpu[:n].float().cpu()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    times = []

    def run():
        if forward:
            return oracle.flow_model(sd, spec, x, 1)
        z, ld = oracle.flow_model(sd, spec, x, -1)
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
    return {"value": n / med, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{n} rows of the same seeded batch, {what} via oracle/flows_ref.py "
                      f"(torch CPU, {threads} threads), median of {len(times)} runs after 1 warm-up"}, \
        (None if forward else oracle.nll_f64(lp)), x


def cpu_training_baseline(model, spec, x_gpu, budget_s=12.0, max_rows=32768):
    """One training step of the oracle on this host: autograd through oracle/flows_ref.py."""
    import oracle
    threads = min(16, os.cpu_count() or 1)
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
    return {"value": n / med, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{n} rows, loss + backward via autograd through oracle/flows_ref.py "
                      f"(torch CPU, {threads} threads), median of {len(times)} runs after 1 warm-up"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2",
                    choices=["cfg2", "cfg2t", "train5k", "cfg3", "cfg3t", "cfg4", "cfg4t", "cfg5f", "cfg5i", "sample4k",
                             "sample4k_spline", "sample4k_maf", "sample4k_iaf"])
    ap.add_argument("--batch", type=int, default=None,
                    help="samples per GPU (default 1M; 500k cfg4; 512Ki cfg5f; 8Ki cfg5i)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay the captured HIP graph of the pass (nfs_amd.GraphedFlow) instead of eager launches")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: split ONE global batch (default 1M) over the ranks")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    model, d, f_layer, spec, desc = build(a.config)
    training = a.config in ("cfg4t", "cfg2t", "train5k", "cfg3t")
    coupling_train = a.config in ("cfg2t", "train5k")
    if coupling_train and world > 1:
        from nfs_amd.distributed import enable_sync_batchnorm
        enable_sync_batchnorm(True)  # batch statistics over all ranks = the full-batch step
    model = model.to(dev).train(training)
    from nfs_amd.distributed import average_gradients, broadcast_parameters, shard_range
    broadcast_parameters(model)  # replicate rank 0's weights (one-time, < 1 MB)
    B_unit = a.batch or DEFAULT_BATCH[a.config]
    sampling = a.config == "cfg5f" or a.config.startswith("sample4k")
    if a.strong:
        lo, hi = shard_range(B_unit, rank, world)
        B, B_global = hi - lo, B_unit
    else:
        B, B_global = B_unit, B_unit * world
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.randn(B, d, device=dev, generator=g)
    flow = model.flow if hasattr(model, "flow") else model

    graphed = None
    if a.graph and not training:
        graphed = nfs_amd.GraphedFlow(flow, x, mode="forward" if sampling else "log_prob", strict=False)
    opt = torch.optim.Adam(model.parameters(), lr=1e-5, capturable=a.graph) if training else None
    graphed_train = None
    if a.graph and training:
        if world > 1:
            raise SystemExit("--graph training is single-GPU (the SyncBN / gradient collectives run eagerly)")
        graphed_train = nfs_amd.GraphedTrainStep(flow, x, opt, warmup=a.warmup)

    eager_only = [False]  # the per-kernel event pass runs eager steps (a graph replay records no events)

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
            average_gradients(model)
            opt.step()
            return torch.stack([-loss.detach().double() * B, torch.tensor(float(B), device=dev, dtype=torch.float64)])
        if graphed is not None:
            out = graphed()
            if sampling:
                return out
            sums = out[1]
        elif sampling:  # sampling pass: x = forward(z), no exchange
            return flow.forward(x)
        else:
            logp, sums = flow.log_prob(x, return_sums=True)
        if world > 1:
            dist.all_reduce(sums)  # RCCL over xGMI: 16 bytes
        return sums

    from nfs_amd.flows import autoregressive as _ar
    from nfs_amd.flows import spline as _sp
    bwd_mod = _sp if a.config == "cfg3t" else _ar
    with torch.set_grad_enabled(training):
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        nfs_amd.reset_stats()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            sums = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = time.perf_counter() - t0
        # Kernel durations: the same K steps again with HIP events around every layer launch
        # on the launch stream. Kept out of the headline loop because each event record adds
        # ~5 us of GPU idle between kernels (measured, profiles/).
        eager_only[0] = True
        if coupling_train:
            from nfs_amd.flows import coupling as _cp
            _cp.TRAIN_EVENTS = []
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            events = [e for e in _cp.TRAIN_EVENTS if e[0].endswith("<BWD2>")]
            _cp.TRAIN_EVENTS = None
        elif training:
            bwd_mod.BACKWARD_EVENTS = []
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            events = bwd_mod.BACKWARD_EVENTS
            bwd_mod.BACKWARD_EVENTS = None
        else:
            flow.layer_events = []
            for _ in range(a.steps):
                if sampling:
                    flow.forward(x)
                else:
                    flow.log_prob(x, return_sums=True)
            torch.cuda.synchronize()
            events = flow.layer_events
            flow.layer_events = None
    if nfs_amd.STATS["torch"] != 0 or (nfs_amd.STATS["hip"] == 0 and graphed is None and graphed_train is None):
        raise RuntimeError(f"hot path did not run on the HIP kernels: {nfs_amd.STATS}")
    t_all = torch.tensor([t], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t_all, op=dist.ReduceOp.MAX)
    t_max = float(t_all.item())

    # dominant kernel: the per-layer fused kernel (every launch of the timed steps)
    durs = [e0.elapsed_time(e1) for _, e0, e1 in events]
    kname = events[0][0] if events else "?"
    mean_ms = sum(durs) / max(1, len(durs))
    achieved = f_layer * B / (mean_ms * 1e-3) / 1e12
    nll = None if sampling else -float(sums[0] / sums[1])

    result = None
    if rank == 0:
        traffic = None
        tp = os.path.join(ROOT, "profiles", f"pmc_traffic_{a.config}.json")
        if os.path.exists(tp):
            with open(tp) as fh:
                traffic = json.load(fh).get("hbm_bytes_per_launch")
        result = {
            "metric": METRIC,
            "value": B_global * a.steps / t_max,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * t_max / a.steps,
            "higher_is_better": True,
            "scaling": "strong" if a.strong else "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic: x ~ N(0,1) generated on device (seed 1234+rank); seeded random-init "
                    "weights perturbed N(0, 0.1^2) with non-trivial BatchNorm running stats",
            "config": {"workload": desc, "batch_per_gpu": B, "global_batch": B_global,
                       "parallelism": (f"dp{world} (sample shards, 1 bucketed RCCL all-reduce of the flat gradient per step)"
                            if training else f"dp{world} (sample shards, 1 RCCL all-reduce of 16 B per step)"),
                       "launch": "hip-graph replay" if a.graph else "eager"},
            "nll_f64": nll,
            "roofline": {"bound": "mfma", "pipe": "valu" if a.config == "cfg5i" else "mfma",
                         "kernel": kname, "achieved": achieved,
                         "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": achieved / PEAK_FP32_TFLOPS,
                         "traffic": traffic, "flop_per_sample_per_launch": f_layer,
                         "samples_per_launch": B, "mean_launch_ms": mean_ms, "launches": len(durs)},
            "cpu_baseline": None,
        }
        if a.config in PUBLISHED_SAMPLING:
            mname, pub = PUBLISHED_SAMPLING[a.config]
            result["metric"] = f"sampling samples/sec ({mname}, n=4000 per forward call)"
            result["vs_baseline"] = result["value"] / pub
            result["published_baseline"] = {"value": pub, "unit": "samples/s", "hardware": "CPU (unspecified)",
                                            "source": "assets/benchmark.png via plots/_common.py:264-274"}
            result["nll_f64"] = None
        if coupling_train:
            result["metric"] = "training samples/sec/GPU (RealNVP d=2 train-mode step)"
            result["nll_f64"] = None
            result["roofline"]["note"] = ("dominant kernel = BWD2 of the train-mode coupling backward "
                                          "(layer-2 recompute, W2^T e2 and the sample-contraction dW2 on "
                                          "MFMA); a layer runs STATS1, STATS2, the fused forward, BWD1-3")
            if world > 1:
                result["config"]["parallelism"] = (f"dp{world} (sample shards, SyncBN: 4 all-gathers/all-reduces "
                                                   f"of <= 3 KB per layer + 1 bucketed gradient all-reduce)")
        elif a.config == "cfg3t":
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
                                          "weight gradients run as batched library GEMMs")
        if world == 1 and not a.no_cpu and training:
            result["cpu_baseline"] = cpu_training_baseline(model, spec, x)
        elif world == 1 and not a.no_cpu:
            rows = {"cfg5f": 16384, "cfg5i": 256}.get(a.config, 4000 if a.config.startswith("sample4k") else 262144)
            cb, cpu_nll, xs = cpu_baseline(model, spec, x, forward=sampling, max_rows=rows)
            if not sampling:
                gpu_nll = flow.nll(xs.to(dev))
                cb["nll_abs_diff_vs_gpu"] = abs(cpu_nll - gpu_nll)
            result["cpu_baseline"] = cb
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
