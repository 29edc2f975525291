"""Flow interface + HIP dispatch.

Mirrors the reference boundary `Flow` / `SequentialFlow` (src/flows/flow/flow.py:4-73,
src/flows/flow/sequential_flow.py:5-34): `forward(z) -> (x, log_det[B])`,
`inverse(x) -> (z, log_det[B])`, `sample`, `log_prob`.

Routing (HipFlow._route):
  * fp32 tensors on a ROCm device  -> the layer's fused gfx950 kernel through libnfx.so.
    If autograd needs gradients, the kernel still computes the outputs and HipFlowFunction's
    backward runs the layer's fused backward kernels (`_hip_backward`: MADE flows in every
    direction, spline coupling, eval-mode affine coupling); shapes outside those kernel
    families recompute through the layer's torch composite on the GPU.
  * CPU tensors or fp64 (gradcheck)  -> the layer's torch composite (same math as the reference).
  * train-mode BatchNorm in a conditioner (CouplingLayer) -> the train-mode kernels
    (batch statistics, running-stat update, fused backward; coupling._CouplingTrainFunction).
A shape outside the compiled kernel family raises NotImplementedError on the GPU instead of
silently running eager (set nfs_amd.flows.flow.ALLOW_TORCH_FALLBACK = True to permit it).
"""
import torch
import torch.nn as nn

from .. import _lib

ALLOW_TORCH_FALLBACK = False

# Counters so tests and the bench can prove which path ran.
STATS = {"hip": 0, "torch": 0}


def reset_stats():
    STATS["hip"] = 0
    STATS["torch"] = 0


class Flow(nn.Module):
    """Base class for normalizing flow layers (src/flows/flow/flow.py:4-73)."""

    def __init__(self):
        super().__init__()
        self.data_dim = None

    def forward(self, z):
        raise NotImplementedError

    def inverse(self, x):
        raise NotImplementedError

    def sample(self, num_samples, base_dist, device="cpu"):
        """flow.py:40-54: z ~ base, return forward(z)[0]."""
        z = base_dist.sample((num_samples,)).to(device)
        x, _ = self.forward(z)
        return x

    def log_prob(self, x, base_dist):
        """flow.py:56-73: log p(x) = base.log_prob(inverse(x)) + log|det J_inv|."""
        z, log_det_inv = self.inverse(x)
        log_p_z = base_dist.log_prob(z)
        if len(log_p_z.shape) > 1:
            log_p_z = log_p_z.sum(dim=1)
        return log_p_z + log_det_inv


class HipFlowFunction(torch.autograd.Function):
    """HIP forward; fused HIP backward where the layer has one (`_hip_backward_ok`), else a
    recompute through the layer's torch composite."""

    @staticmethod
    def forward(ctx, layer, direction, x, *params):
        ctx.layer = layer
        ctx.direction = direction
        ctx.save_for_backward(x)
        with torch.no_grad():
            y, ld = layer._hip_call(x, direction)
        return y, ld

    @staticmethod
    def backward(ctx, gy, gld):
        (x,) = ctx.saved_tensors
        layer = ctx.layer
        params = [p for p in layer.parameters()]
        if getattr(layer, "_hip_backward_ok", None) is not None and layer._hip_backward_ok(x, ctx.direction):
            # fused gfx950 backward (MADE flows, spline coupling, eval-mode affine coupling)
            STATS["hip"] += 1
            gx, gparams = layer._hip_backward(x.detach(), gy, gld, ctx.direction)
            gparams = [g if p.requires_grad else None for p, g in zip(params, gparams)]
            return (None, None, gx, *gparams)
        # composite recompute through ATen on the GPU: counted as a torch call, so
        # STATS["torch"] == 0 after a backward proves every layer ran a fused backward kernel
        STATS["torch"] += 1
        with torch.enable_grad():
            xr = x.detach().requires_grad_(True)
            y, ld = layer._torch_call(xr, ctx.direction)
            outs, grads_out = [], []
            if gy is not None:
                outs.append(y)
                grads_out.append(gy)
            if gld is not None:
                outs.append(ld)
                grads_out.append(gld)
            wrt = [xr] + [p for p in params if p.requires_grad]
            grads = torch.autograd.grad(outs, wrt, grads_out, allow_unused=True)
        gx = grads[0]
        it = iter(grads[1:])
        gparams = [next(it) if p.requires_grad else None for p in params]
        return (None, None, gx, *gparams)


class HipFlow(Flow):
    """A Flow whose eval/sampling math runs in one fused gfx950 kernel per call.

    Subclasses implement:
      _torch_call(x, direction) -> (y, ld)            composite torch math (reference ops)
      _hip_supported(x) -> (bool, reason)             shape/dtype inside the kernel family
      _hip_launch(x, out, log_det, direction, accumulate)   enqueue the kernel
      _torch_only() -> bool                           state that forces the composite path
    """

    def forward(self, z):
        return self._dispatch(z, 1)

    def inverse(self, x):
        return self._dispatch(x, -1)

    # -- routing -----------------------------------------------------------------------
    def _route(self, x):
        if x.device.type != "cuda" or x.dtype != torch.float32:
            return "torch"
        if self._torch_only():
            return "torch"
        ok, why = self._hip_supported(x)
        if not ok:
            if ALLOW_TORCH_FALLBACK:
                return "torch"
            raise NotImplementedError(
                f"{type(self).__name__}: no gfx950 kernel for this call ({why}); "
                f"set nfs_amd.flows.flow.ALLOW_TORCH_FALLBACK=True to run eager PyTorch")
        return "hip"

    def _dispatch(self, x, direction):
        if self._route(x) == "torch":
            STATS["torch"] += 1
            return self._torch_call(x, direction)
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            return HipFlowFunction.apply(self, direction, x, *list(self.parameters()))
        return self._hip_call(x, direction)

    def _hip_call(self, x, direction):
        x = x.contiguous()
        out = torch.empty_like(x)
        ld = torch.empty(x.shape[0], device=x.device, dtype=torch.float32)
        self._hip_launch_counted(x, out, ld, direction, accumulate=False)
        return out, ld

    def _hip_launch_counted(self, x, out, log_det, direction, accumulate):
        STATS["hip"] += 1
        self._hip_launch(x, out, log_det, direction, accumulate)

    def _hip_launch_logprob(self, x, out, log_det, logp, sums, workspace, accumulate):
        """Inverse + fused Gaussian log_prob epilogue (last layer of a log_prob chain).
        Returns False when this layer has no fused variant (the caller then runs
        nfx_gauss_logprob after the plain inverse)."""
        return False

    # -- packed-weight cache -------------------------------------------------------------
    # The cache key must notice every change of a parameter/buffer (in-place optimizer steps
    # and load_state_dict bump `_version`, `.to()` moves `data_ptr`, assigning a new Parameter
    # or submodule replaces the object). Walking `parameters()` per call costs ~15 us per layer
    # (named_modules traversal), more than a small-batch kernel, so the module tree is resolved
    # once into direct references to each module's `_parameters`/`_buffers` dicts plus the
    # parent->child links, and re-resolved only when one of those links changed.
    def _nfx_binding(self):
        b = self.__dict__.get("_nfx_bind")
        if b is not None:
            for parent, name, child in b[0]:
                if parent.get(name) is not child:
                    b = None
                    break
        if b is None:
            links, slots = [], []
            for mod in self.modules():
                for name, child in mod._modules.items():
                    links.append((mod._modules, name, child))
                for name in mod._parameters:
                    slots.append((mod._parameters, name))
                for name in mod._buffers:
                    slots.append((mod._buffers, name))
            bns = [m for m in self.modules() if isinstance(m, nn.BatchNorm1d)]
            b = (links, slots, bns)
            object.__setattr__(self, "_nfx_bind", b)
        return b

    def _batchnorms(self):
        return self._nfx_binding()[2]

    def _state_key(self, device):
        key = [device]
        for d, name in self._nfx_binding()[1]:
            t = d[name]
            key.append(None if t is None else (t.data_ptr(), t._version))
        return tuple(key)

    def _packed(self, device, build, slot="_nfx_pack_cache"):
        """Return the cached device weight image, rebuilding it when any parameter/buffer
        changed (in-place optimizer steps and load_state_dict bump tensor versions). `slot`
        names the cache, so a layer can keep several images (forward, backward)."""
        key = self._state_key(device)
        cache = self.__dict__.get(slot)
        if cache is not None and cache[0] == key:
            return cache[1]
        packed = build(device)
        object.__setattr__(self, slot, (key, packed))
        return packed

    def _torch_only(self):
        return False


def drop_pack_caches(module):
    """Forget every cached packed-weight image under `module`, so the next call re-packs from
    the live parameters. Needed after writes the version counters cannot see (a collective or
    `p.data.copy_()` writing through `.data`, a graph replay whose optimizer step updated the
    parameters) and before a graph capture that must record the pack kernels."""
    for m in module.modules():
        if isinstance(m, HipFlow):
            drop_layer_pack_caches(m)


def drop_layer_pack_caches(layer):
    """Forget the cached packed-weight images of one HipFlow layer (every `_packed` slot)."""
    for k in [k for k in layer.__dict__ if k.startswith("_nfx_") and k.endswith("pack_cache")]:
        del layer.__dict__[k]


class SequentialFlow(Flow):
    """A sequence of flows applied in order (src/flows/flow/sequential_flow.py:5-34).

    The reference accumulates into torch.zeros(B) (f32) with one `+=` per layer. When every
    layer routes to its gfx950 kernel (and no gradient is needed) the chain runs the kernels
    back to back with the log-det accumulated IN PLACE into that zero vector (accumulate=1):
    0 + ld_0 + ld_1 + ... in the same float32 order, no intermediate tensors."""

    def __init__(self, flows):
        super().__init__()
        if not isinstance(flows, (list, nn.ModuleList)):
            raise ValueError("flows must be a list or nn.ModuleList")
        self.flows = nn.ModuleList(flows)

    def forward(self, z):
        if self._hip_chain_ok(z):
            return self._hip_chain(z, 1)
        total_log_det = torch.zeros(z.size(0), device=z.device)
        for flow in self.flows:
            z, log_det = flow.forward(z)
            total_log_det += log_det
        return z, total_log_det

    def inverse(self, x):
        if self._hip_chain_ok(x):
            return self._hip_chain(x, -1)
        total_log_det = torch.zeros(x.size(0), device=x.device)
        for flow in reversed(self.flows):
            x, log_det = flow.inverse(x)
            total_log_det += log_det
        return x, total_log_det

    def _hip_chain_ok(self, x):
        if x.device.type != "cuda" or x.dtype != torch.float32 or x.dim() != 2 or len(self.flows) == 0:
            return False
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            return False  # per-layer autograd Functions handle gradients
        return all(isinstance(f, HipFlow) and f._route(x) == "hip" for f in self.flows)

    def _hip_chain(self, x, direction):
        x = x.contiguous()
        ld = torch.zeros(x.shape[0], device=x.device, dtype=torch.float32)
        from . import coupling as _coupling
        from . import spline as _spline
        for mod in (_coupling, _spline):  # one launch (csrc/nfx_affine_*chain*, nfx_spline_schain*)
            if mod.chain_ok(list(self.flows), x):
                out = torch.empty_like(x)
                mod.chain_launch(list(self.flows), x, out, ld, direction, True)
                return out, ld
        bufs = [torch.empty_like(x), torch.empty_like(x)]
        cur, k = x, 0
        for f in (self.flows if direction > 0 else reversed(self.flows)):
            f._hip_launch_counted(cur, bufs[k], ld, direction, accumulate=True)
            cur, k = bufs[k], k ^ 1
        return cur, ld


def stream_ptr(t):
    return _lib.stream_of(t)
