"""HIP-graph capture of the fused layer chain (replaces a tracing compiler for the hot path).

Every libnfx.so entry point is stream-ordered and allocation-free, so a whole eval pass —
`log_prob` (every layer kernel, the fused Gaussian epilogue, the float64 partial sums) or the
sampling pass `forward` — is captured once with `torch.cuda.CUDAGraph` and replayed as one
graph launch: the ~20 us of Python/ctypes issue cost per layer disappears, which is what a
small per-GPU shard (strong scaling, or the reference's 4,000-sample throughput runs) is
bound by. Inputs go through a static buffer; outputs are the graph's static tensors (valid
until the next replay).

mode="sample" is the fused sampling path (`Flow.sample`, flow.py:40-54,
and the reference's sampling throughput loop, plots/_common.py:217-222,264-274): z ~ N(0, I) is
drawn on the device and forward(z) runs in one graph launch per batch of samples, no host round
trip. For chains of eval CouplingLayers (RealNVP) the draw is fused INTO the chain kernel
(nfx_affine_chain_sample: Philox4x32-10 in the kernel's prologue, the generator state advanced on
the device, so every replay draws afresh — the graph holds one kernel); other models draw with
torch's graph-safe Philox generator (normal_) ahead of their forward. The example tensor only
gives the shape [n, d]; `static_in` holds the last z.

The packed weight images are built before capture and baked into the graph. With
`strict=True` (default) every call checks that no parameter or buffer changed since capture
(in-place optimizer steps and load_state_dict bump tensor versions) and raises instead of
replaying stale weights; `strict=False` skips that check.

GraphedTrainStep captures a whole full-batch TRAINING step — loss = -log_prob(x).mean(),
backward (the train-mode coupling kernels and the fused backward passes, BatchNorm running
statistics included), optional gradient clipping, optimizer.step() — as one graph. The
reference trains full-batch on a few thousand points (README.md:107-117: 5,000 two-moons
samples; plots/_common.py:194-211: 2,000), where an eager step is bound by the ~150 kernel
launches it issues, not by the GPU.
"""
import torch

from . import flows as _flows


def _tensor_versions(model):
    return tuple((t.data_ptr(), t._version) for t in list(model.parameters()) + list(model.buffers()))


class GraphedFlow:
    """Capture `model.log_prob(x, return_sums=True)` (mode="log_prob"), `model.forward(x)`
    (mode="forward"), `model.inverse(x)` (mode="inverse") or z ~ N(0, I) + `model.forward(z)`
    (mode="sample") for inputs shaped like `example`."""

    def __init__(self, model, example, mode="log_prob", strict=True, warmup=2):
        if mode not in ("log_prob", "forward", "inverse", "sample"):
            raise ValueError(f"mode must be log_prob/forward/inverse/sample, got {mode}")
        if example.device.type != "cuda":
            raise ValueError("GraphedFlow needs a ROCm device tensor")
        self.model = model.flow if hasattr(model, "flow") and hasattr(model.flow, "log_prob") else model
        self.mode = mode
        self.strict = strict
        self.static_in = example.detach().clone().contiguous()
        # the graph's own log_prob workspace (float64 partials + arrival word): replays of two
        # graphs, or a replay beside eager calls, never share one
        self.workspace = None
        if mode == "log_prob":
            from .models.normalizing_flow_model import new_gauss_workspace
            self.workspace = new_gauss_workspace(example.shape[0], example.device)
        fn = self._call
        stream = torch.cuda.Stream(device=example.device)
        stream.wait_stream(torch.cuda.current_stream(example.device))
        with torch.no_grad(), torch.cuda.stream(stream):
            for _ in range(warmup):  # builds the packed weight images outside the capture
                fn()
        torch.cuda.current_stream(example.device).wait_stream(stream)
        hip0 = _flows.STATS["hip"]
        torch0 = _flows.STATS["torch"]
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.static_out = fn()
        if _flows.STATS["torch"] != torch0:
            raise RuntimeError("GraphedFlow: the captured pass ran eager PyTorch layers, not the HIP kernels")
        self.launches = _flows.STATS["hip"] - hip0
        self.versions = _tensor_versions(self.model) if strict else None

    def _call(self):
        if self.mode == "sample":
            n = self.static_in.shape[0]
            if hasattr(self.model, "sample_fused_ok") and self.model.sample_fused_ok(n, self.static_in.device):
                if not hasattr(self, "_sx"):
                    self._sx = torch.empty_like(self.static_in)
                    self._sld = torch.empty(n, device=self.static_in.device)
                self.fused_draw = True
                x, ld, _ = self.model.sample_fused(n, self.static_in.device, out=(self.static_in, self._sx, self._sld))
                return x, ld
            self.fused_draw = False
            self.static_in.normal_()
            return self.model.forward(self.static_in)
        if self.mode == "log_prob":
            return self.model.log_prob(self.static_in, return_sums=True, workspace=self.workspace)
        if self.mode == "forward":
            return self.model.forward(self.static_in)
        return self.model.inverse(self.static_in)

    def __call__(self, x=None):
        if self.strict and _tensor_versions(self.model) != self.versions:
            raise RuntimeError("GraphedFlow: parameters changed since capture; capture again")
        if x is not None:
            if self.mode == "sample":
                raise ValueError("GraphedFlow(mode='sample') draws its own z; call it without an input")
            if x.shape != self.static_in.shape:
                raise ValueError(f"GraphedFlow captured shape {tuple(self.static_in.shape)}, got {tuple(x.shape)}")
            self.static_in.copy_(x)
        self.graph.replay()
        return self.static_out


class GraphedTrainStep:
    """One captured training step: `loss_fn(model, x)` (default: -model.log_prob(x).mean()),
    backward, `clip_grad_norm_` (if `clip_grad_norm` is set) and `optimizer.step()`.

    The optimizer must be capturable (e.g. torch.optim.Adam(params, capturable=True)). The
    `warmup` eager steps run before capture (on a side stream, as torch.cuda.graphs requires) are
    REAL training steps: they update the parameters and optimizer state. Each call replays one
    step on the static input (optionally refreshed from `x`) and returns the static loss tensor
    (valid until the next replay)."""

    def __init__(self, model, example, optimizer, loss_fn=None, clip_grad_norm=None, warmup=3):
        if example.device.type != "cuda":
            raise ValueError("GraphedTrainStep needs a ROCm device tensor")
        self.model = model
        self.optimizer = optimizer
        # the step's own log_prob workspace (float64 partials + arrival word), as GraphedFlow:
        # two captured steps, or a replay beside eager calls, never share one
        from .models.normalizing_flow_model import new_gauss_workspace
        self.workspace = new_gauss_workspace(example.shape[0], example.device)
        ws = self.workspace
        self.loss_fn = loss_fn or (lambda m, x: -m.log_prob(x, workspace=ws).mean())
        self.clip = clip_grad_norm
        self.static_in = example.detach().clone().contiguous()
        params = [p for g in optimizer.param_groups for p in g["params"]]
        self._params = params
        dev = example.device
        stream = torch.cuda.Stream(device=dev)
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream):
            for _ in range(warmup):
                self._step()
        torch.cuda.current_stream(dev).wait_stream(stream)
        torch0 = _flows.STATS["torch"]
        optimizer.zero_grad(set_to_none=True)
        # The pack kernels must be IN the graph: every replay's optimizer step changes the
        # parameters, and the next replay has to re-pack them. A cache left from an earlier
        # eager call (e.g. warmup=0 after an eval pass) would otherwise be baked in as a
        # constant image and every replay would silently run the forward on stale weights.
        _flows.drop_pack_caches(model)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_loss = self._step(zero=False)
        if _flows.STATS["torch"] != torch0:
            raise RuntimeError("GraphedTrainStep: the captured step ran eager PyTorch layers, not the HIP kernels")
        # Replays update the parameters without bumping their versions, so the image packed
        # during capture would look current to a later eager call: forget it now and after
        # every replay (the graph keeps its own buffers).
        self._hipflows = [m for m in model.modules() if isinstance(m, _flows.HipFlow)]
        self._forget()

    def _forget(self):
        for m in self._hipflows:
            _flows.drop_layer_pack_caches(m)

    def _step(self, zero=True):
        if zero:
            self.optimizer.zero_grad(set_to_none=True)
        loss = self.loss_fn(self.model, self.static_in)
        loss.backward()
        if self.clip is not None:
            torch.nn.utils.clip_grad_norm_(self._params, self.clip)
        self.optimizer.step()
        return loss.detach()

    def __call__(self, x=None):
        if x is not None:
            if x.shape != self.static_in.shape:
                raise ValueError(f"GraphedTrainStep captured shape {tuple(self.static_in.shape)}, got {tuple(x.shape)}")
            self.static_in.copy_(x)
        self.graph.replay()
        self._forget()
        return self.static_loss
