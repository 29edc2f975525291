"""NormalizingFlowModel — drop-in for src/models/normalizing_flow_model.py:4-128.

Same constructor, attributes (`flows`, `batch_norms`, `batch_norm_between_layers`) and
state_dict keys. When every layer routes to its gfx950 kernel, forward/inverse run the layers
back to back on the current stream with the per-sample log-det accumulated IN PLACE by the
kernels (accumulate=1), which is exactly the reference's sequential float32
`log_det_jacobian_sum += log_det` (normalizing_flow_model.py:30-65); there are no
intermediate log-det tensors and no Python-side adds.

`log_prob` / `nll` add the fused Gaussian base term and the float64 NLL partial sums
(csrc/nfx_gauss.hip): the log_prob glue the reference's callers write inline
(README.md:113-114, src/utils.py:39-55, plots/_common.py:201-202).
"""
import collections
import math

import torch
import torch.nn as nn

from .. import _lib
from ..distributed import merge_bn_stats, sync_bn_world
from ..flows import coupling as _coupling
from ..flows import spline as _spline
from ..flows.flow import HipFlow, STATS


class NormalizingFlowModel(nn.Module):
    def __init__(self, flows, batch_norm_between_layers=False):
        super().__init__()
        self.batch_norm_between_layers = batch_norm_between_layers
        if self.batch_norm_between_layers:
            data_dim = flows[0].data_dim if hasattr(flows[0], "data_dim") else None
            if data_dim is None:
                raise ValueError("Cannot use batch_norm_between_layers if flows do not have a 'data_dim' attribute.")
            self.batch_norms = nn.ModuleList([nn.BatchNorm1d(data_dim) for _ in range(len(flows))])
        self.flows = nn.ModuleList(flows)
        # Profiling hook: when set to a list, _hip_chain appends (layer name, start, end) HIP
        # events recorded on the launch stream around every layer kernel (bench.py uses it).
        self.layer_events = None

    # -- reference-order chaining ------------------------------------------------------------
    def forward(self, z):
        if self._hip_chain_ok(z):
            return self._hip_chain(z, 1)
        log_det_jacobian_sum = 0
        for i, flow in enumerate(self.flows):
            z, log_det_jacobian = flow(z)
            log_det_jacobian_sum += log_det_jacobian
            if self.batch_norm_between_layers and i < len(self.flows) - 1:
                bn = self.batch_norms[i]
                if _bn_hip_ok(z):
                    if self.training:
                        _bn_update_running_hip(bn, z)
                    z, log_det_jacobian_sum = _FlowBatchNormFn.apply(
                        z, _as_ld(log_det_jacobian_sum, z), bn.weight, bn.bias, bn, 1)
                    continue
                z = self._apply_batch_norm(bn, z)
                log_det_jacobian_sum += self._batch_norm_log_det_jacobian(bn, z)
        return z, log_det_jacobian_sum

    def inverse(self, x):
        if self._hip_chain_ok(x):
            return self._hip_chain(x, -1)
        log_det_jacobian_sum = 0
        for i, flow in reversed(list(enumerate(self.flows))):
            if self.batch_norm_between_layers and i < len(self.flows) - 1:
                bn = self.batch_norms[i]
                if _bn_hip_ok(x):
                    x, log_det_jacobian_sum = _FlowBatchNormFn.apply(
                        x, _as_ld(log_det_jacobian_sum, x), bn.weight, bn.bias, bn, -1)
                else:
                    x = self._inverse_batch_norm(bn, x)
                    log_det_jacobian_sum -= self._batch_norm_log_det_jacobian(bn, x)
            x, log_det_jacobian = flow.inverse(x)
            log_det_jacobian_sum += log_det_jacobian
        return x, log_det_jacobian_sum

    # -- between-layer BatchNorm (normalizing_flow_model.py:67-128) ----------------------------
    # Composite torch versions (CPU, float64); fp32 ROCm tensors run csrc/nfx_flowbn.hip.
    def _apply_batch_norm(self, bn_layer, x):
        if self.training:
            with torch.no_grad():
                momentum = bn_layer.momentum if bn_layer.momentum is not None else 0.1
                if sync_bn_world() > 1:  # SyncBN: the moments of every rank's shard
                    mean, var = _synced_moments(x)
                else:
                    mean, var = x.mean(dim=0), x.var(dim=0, unbiased=False)
                bn_layer.running_mean.mul_(1 - momentum).add_(momentum * mean)
                bn_layer.running_var.mul_(1 - momentum).add_(momentum * var)
        gamma = bn_layer.weight.view(1, -1)
        beta = bn_layer.bias.view(1, -1)
        mean = bn_layer.running_mean.view(1, -1)
        var = bn_layer.running_var.view(1, -1)
        return (x - mean) / torch.sqrt(var + bn_layer.eps) * gamma + beta

    def _batch_norm_log_det_jacobian(self, bn_layer, x):
        log_det_per_dim = torch.log(torch.abs(bn_layer.weight)) - 0.5 * torch.log(bn_layer.running_var + bn_layer.eps)
        return log_det_per_dim.sum()

    def _inverse_batch_norm(self, bn_layer, y):
        gamma = bn_layer.weight.view(1, -1)
        beta = bn_layer.bias.view(1, -1)
        mean = bn_layer.running_mean.view(1, -1)
        var = bn_layer.running_var.view(1, -1)
        return (y - beta) / gamma * torch.sqrt(var + bn_layer.eps) + mean

    # -- gfx950 chain ----------------------------------------------------------------------
    def _needs_grad(self, x):
        if not torch.is_grad_enabled():
            return False
        return x.requires_grad or any(p.requires_grad for p in self.parameters())

    def _hip_chain_ok(self, x):
        if x.device.type != "cuda" or x.dtype != torch.float32 or x.dim() != 2:
            return False
        if self._needs_grad(x):
            return False  # per-layer autograd Functions handle gradients
        for f in self.flows:
            if not isinstance(f, HipFlow) or f._route(x) != "hip":
                return False
        if self.batch_norm_between_layers and len(self.flows) > 1 and not _bn_hip_ok(x):
            return False
        return True

    def _hip_chain(self, x, direction, logprob=None):
        """Run every layer's kernel back to back. With logprob=(logp, sums, workspace) (an
        inverse chain), the last layer also writes the Gaussian log-density and float64 NLL
        partials in its epilogue when it has a fused variant; `fused` in the return says
        whether it did."""
        x = x.contiguous()
        B = x.shape[0]
        ld = torch.empty(B, device=x.device, dtype=torch.float32)
        n = len(self.flows)
        chain = None
        if not self.batch_norm_between_layers:
            chain = next((m for m in (_coupling, _spline) if m.chain_ok(list(self.flows), x)), None)
        if chain is not None:
            # the whole chain in one launch (csrc/nfx_affine_chain.hip / nfx_affine_schain.hip /
            # nfx_spline_schain_kernel.h), the per-layer kernels' roundings
            out = torch.empty_like(x)
            ev = self.layer_events
            if ev is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            chain.chain_launch(list(self.flows), x, out, ld, direction, False, logprob)
            if ev is not None:
                e1.record()
                ev.append((_lib.last_kernel(), e0, e1))
            return (out, ld, True) if logprob is not None else (out, ld)
        bufs = [torch.empty_like(x), torch.empty_like(x)]
        order = range(n) if direction > 0 else reversed(range(n))
        cur, k, first, fused = x, 0, True, False
        for i in order:
            if direction < 0 and self.batch_norm_between_layers and i < n - 1:
                # (never the first op: the last flow has no BatchNorm, so ld is initialised)
                out = bufs[k] if bufs[k] is not cur else bufs[k ^ 1]
                _bn_launch(self.batch_norms[i], cur, out, ld, -1)
                cur = out
            out = bufs[k]
            if out is cur:
                k ^= 1
                out = bufs[k]
            ev = self.layer_events
            if ev is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            if logprob is not None and i == 0 and self.flows[i]._hip_launch_logprob(
                    cur, out, ld, *logprob, accumulate=not first):
                STATS["hip"] += 1
                fused = True
            else:
                self.flows[i]._hip_launch_counted(cur, out, ld, direction, accumulate=not first)
            if ev is not None:
                e1.record()
                ev.append((_lib.last_kernel(), e0, e1))
            first = False
            cur, k = out, k ^ 1
            if direction > 0 and self.batch_norm_between_layers and i < n - 1:
                bn = self.batch_norms[i]
                if self.training:
                    _bn_update_running_hip(bn, cur)
                out = bufs[k] if bufs[k] is not cur else bufs[k ^ 1]
                _bn_launch(bn, cur, out, ld, 1)
                cur = out
        if logprob is not None:
            return cur, ld, fused
        return cur, ld

    # -- log-density -------------------------------------------------------------------------
    def log_prob(self, x, return_sums=False, workspace=None):
        """log p(x) = log N(z; 0, I) + log|det J_inv| per sample, z = inverse(x).

        With return_sums=True also returns a float64 tensor [sum_i log p(x_i), B] on x's device
        (the partial a data-parallel NLL all-reduces). `workspace`: the fused epilogue's float64
        partials + arrival word (uint8 tensor of at least nfx_gauss_workspace_bytes(B) bytes, any
        content: ABI 3 tags the arrival word per launch); by default one cached per (device,
        current stream), so calls on different streams never share one."""
        if self._hip_chain_ok(x) and len(self.flows) > 0:
            B = x.shape[0]
            logp = torch.empty(B, device=x.device, dtype=torch.float32)
            sums = torch.empty(2, device=x.device, dtype=torch.float64)
            ws = check_gauss_workspace(workspace, B, x.device) if workspace is not None else gauss_workspace(B, x.device)
            z, ld, fused = self._hip_chain(x, -1, logprob=(logp, sums, ws))
            if not fused:
                gauss_logprob(z, ld, logp, sums, ws)
            return (logp, sums) if return_sums else logp
        z, ld = self.inverse(x)
        if z.device.type == "cuda" and z.dtype == torch.float32 and z.dim() == 2 and not self._needs_grad(x):
            logp, sums = gauss_logprob(z, ld, ws=workspace)
        elif z.device.type == "cuda" and z.dtype == torch.float32 and z.dim() == 2:
            # training: the same HIP epilogue under autograd, its adjoint in one HIP kernel
            logp, sums = _GaussLogProbFn.apply(z, ld, workspace)
        else:
            d = z.shape[1]
            logp = -0.5 * (d * math.log(2 * math.pi) + z.pow(2).sum(-1)) + ld
            if not return_sums:  # (no host->device scalar copy: the step stays graph-capturable)
                return logp
            sums = torch.stack([logp.detach().double().sum(),
                                torch.tensor(float(z.shape[0]), dtype=torch.float64, device=z.device)])
        return (logp, sums) if return_sums else logp

    # -- sampling with the base draw on the device ---------------------------------------------
    def sample_fused_ok(self, num_samples, device):
        """True when sample_fused runs as one kernel: eval-mode CouplingLayers (d in {2, 4, 8},
        H <= 128, up to 64k samples) or d = 2 SplineCouplingLayers (any batch), no between-layer
        BatchNorm."""
        return not self.batch_norm_between_layers and self._sample_chain(num_samples, device) is not None

    def _sample_chain(self, num_samples, device):
        fl = list(self.flows)
        for m in (_coupling, _spline):
            if m.sample_chain_ok(fl, num_samples, device):
                return m
        return None

    def sample_fused(self, num_samples, device="cuda", out=None):
        """Flow.sample (src/flows/flow/flow.py:40-54) with the N(0, I) base draw fused into the
        sampling forward: z ~ N(0, I) on the device (Philox4x32-10, this model's own generator
        state, seeded from torch's CPU generator on first use) and x = forward(z), ONE launch
        (nfx_affine_chain_sample / nfx_spline_chain_sample). Returns (x, log_det, z); x equals
        forward(z) bit for bit.
        out=(z, x, ld) writes into caller buffers (GraphedFlow(mode="sample"))."""
        dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        if not self.sample_fused_ok(num_samples, dev):
            raise NotImplementedError("sample_fused: the fused sampling chain does not take this model / size")
        st = getattr(self, "_nfx_rng", None)
        if st is None:
            st = self._nfx_rng = {}
        if dev not in st:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            st[dev] = (seed, torch.zeros(2, dtype=torch.int64, device=dev))
        seed, state = st[dev]
        d = self.flows[0].data_dim
        if out is None:
            z = torch.empty(num_samples, d, device=dev)
            x = torch.empty_like(z)
            ld = torch.empty(num_samples, device=dev)
        else:
            z, x, ld = out
        self._sample_chain(num_samples, dev).chain_sample(list(self.flows), state, seed, z, x, ld)
        return x, ld, z

    def nll(self, x):
        """Mean negative log-likelihood, accumulated in float64 (python float)."""
        _, sums = self.log_prob(x, return_sums=True)
        s = sums.cpu()
        return -(s[0] / s[1]).item()


_GAUSS_WS = collections.OrderedDict()
_GAUSS_WS_MAX = 8  # (device, stream) entries kept; least recently used dropped beyond


def gauss_workspace(B, device, stream=None):
    """The per-workgroup float64 partial sums + arrival word of the fused log_prob epilogues
    (nfx_gauss_workspace_bytes), cached per (device, stream). Any content is valid (ABI 3: the
    kernels tag the arrival word per launch). Launches on one stream are ordered; two streams
    never share a workspace (concurrent launches on one would race on its partials). The cache
    holds the _GAUSS_WS_MAX most recently used streams: a transient stream's entry is dropped
    once eight others were used after it (the caching allocator reuses a dropped buffer only on
    the stream it was allocated on, after that stream's queued work). Captured graphs
    (GraphedFlow, GraphedTrainStep) own theirs."""
    dev = torch.device(device)
    if dev.type == "cuda":
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        st = stream if stream is not None else torch.cuda.current_stream(idx)
        key = (dev.type, idx, int(st.cuda_stream))
    else:
        key = (dev.type, dev.index, 0)
    n = _lib.lib().nfx_gauss_workspace_bytes(B)
    ws = _GAUSS_WS.get(key)
    if ws is None or ws.numel() < n:
        ws = new_gauss_workspace(B, dev)
        _GAUSS_WS[key] = ws
    _GAUSS_WS.move_to_end(key)
    while len(_GAUSS_WS) > _GAUSS_WS_MAX:
        _GAUSS_WS.popitem(last=False)
    return ws


def new_gauss_workspace(B, device):
    """A fresh log_prob workspace for B samples (for callers that own one). Any content is valid
    (ABI 3); nfx_gauss_workspace_init writes the clean arrival word up front (on the current
    stream), so even the first call skips the kernels' one-time claim of a foreign word."""
    ws = torch.empty(_lib.lib().nfx_gauss_workspace_bytes(B), device=device, dtype=torch.uint8)
    if ws.device.type == "cuda":
        _lib.check(_lib.lib().nfx_gauss_workspace_init(_lib.ptr(ws), _lib.stream_of(ws)), "nfx_gauss_workspace_init")
    return ws


def check_gauss_workspace(ws, B, device):
    n = _lib.lib().nfx_gauss_workspace_bytes(B)
    if ws.dtype != torch.uint8 or ws.device != torch.device(device) or ws.numel() < n or not ws.is_contiguous():
        raise ValueError(f"log_prob workspace: need a contiguous uint8 tensor of >= {n} bytes on {device}")
    return ws


def gauss_logprob(z, ld, logp=None, sums=None, ws=None):
    """Fused `MultivariateNormal(0,I).log_prob(z) + ld` and float64 [sum, count] (nfx_gauss_logprob)."""
    z = z.contiguous()
    B, d = z.shape
    if logp is None:
        logp = torch.empty(B, device=z.device, dtype=torch.float32)
    if sums is None:
        sums = torch.empty(2, device=z.device, dtype=torch.float64)
    L = _lib.lib()
    ws = gauss_workspace(B, z.device) if ws is None else check_gauss_workspace(ws, B, z.device)
    _lib.check(L.nfx_gauss_logprob(_lib.ptr(z), _lib.ptr(ld), _lib.ptr(logp), _lib.ptr(sums),
                                   _lib.ptr(ws), B, d, _lib.stream_of(z)), "nfx_gauss_logprob")
    STATS["hip"] += 1
    return logp, sums


class _GaussLogProbFn(torch.autograd.Function):
    """log N(z; 0, I) + ld under autograd: nfx_gauss_logprob forward (the eval epilogue, the
    reference's rounding order), nfx_gauss_logprob_backward (dL/dz = -z g, dL/dld = g)."""

    @staticmethod
    def forward(ctx, z, ld, workspace):
        z = z.contiguous()
        logp, sums = gauss_logprob(z, ld.contiguous(), ws=workspace)
        ctx.save_for_backward(z)
        ctx.mark_non_differentiable(sums)
        return logp, sums

    @staticmethod
    def backward(ctx, g, _gs):
        (z,) = ctx.saved_tensors
        B, d = z.shape
        g = g.contiguous().float()
        gz, gld = torch.empty_like(z), torch.empty_like(g)
        _lib.check(_lib.lib().nfx_gauss_logprob_backward(_lib.ptr(z), _lib.ptr(g), _lib.ptr(gz), _lib.ptr(gld), B, d,
                                                         _lib.stream_of(z)), "nfx_gauss_logprob_backward")
        STATS["hip"] += 1
        return gz, gld, None


# ---------------------------------------------------------------------------------------------
# Between-layer BatchNorm on the GPU (csrc/nfx_flowbn.hip)
# ---------------------------------------------------------------------------------------------
_FLOWBN_MAX_D = 1024


def _bn_hip_ok(x):
    return x.device.type == "cuda" and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] <= _FLOWBN_MAX_D


def _bn_ptrs(bn):
    return (_lib.ptr(bn.weight), _lib.ptr(bn.bias), _lib.ptr(bn.running_mean), _lib.ptr(bn.running_var))


def _bn_launch(bn, x, out, ld, direction):
    """out = BN affine of x (running statistics), ld -+= the scalar log-det, in place."""
    B, d = x.shape
    w, b, rm, rv = _bn_ptrs(bn)
    _lib.check(_lib.lib().nfx_flowbn_apply(_lib.ptr(x), _lib.ptr(out), _lib.ptr(ld), w, b, rm, rv,
                                           float(bn.eps), B, d, direction, _lib.stream_of(x)),
               "nfx_flowbn_apply")
    STATS["hip"] += 1


def _bn_workspace(B, d, device):
    return torch.empty(_lib.lib().nfx_flowbn_workspace_bytes(B, d), device=device, dtype=torch.uint8)


def _bn_update_running_hip(bn, x):
    """Train mode (normalizing_flow_model.py:74-79): fold the batch moments of x into the running
    statistics; with SyncBN enabled the moments are those of every rank's shard."""
    x = x.detach().contiguous()
    B, d = x.shape
    L = _lib.lib()
    stats = torch.empty(d, 3, device=x.device, dtype=torch.float64)
    ws = _bn_workspace(B, d, x.device)
    st = _lib.stream_of(x)
    _lib.check(L.nfx_flowbn_moments(_lib.ptr(x), B, d, _lib.ptr(stats), _lib.ptr(ws), st), "nfx_flowbn_moments")
    merge_bn_stats(stats)
    momentum = bn.momentum if bn.momentum is not None else 0.1
    with torch.no_grad():
        _lib.check(L.nfx_flowbn_update_running(_lib.ptr(stats), _lib.ptr(bn.running_mean),
                                               _lib.ptr(bn.running_var), float(momentum), d, st),
                   "nfx_flowbn_update_running")
        # the kernel writes the buffers behind autograd's back; bump their versions so every
        # version-keyed cache (packed images, graph strict checks) sees the change
        torch.autograd.graph.increment_version(bn.running_mean)
        torch.autograd.graph.increment_version(bn.running_var)
    STATS["hip"] += 2


def _synced_moments(x):
    """(mean, biased var) of x over every rank's shard (float64 Chan merge, cast to x's dtype)."""
    xd = x.detach().double()
    n = torch.full((x.shape[1],), float(x.shape[0]), dtype=torch.float64, device=x.device)
    mean = xd.mean(0)
    m2 = ((xd - mean) ** 2).sum(0)
    stats = torch.stack([n, mean, m2], dim=1)
    merge_bn_stats(stats)
    return stats[:, 1].to(x.dtype), (stats[:, 2] / stats[:, 0]).to(x.dtype)


def _as_ld(ld, x):
    """The running log-det sum as a [B] fp32 tensor (the reference starts it as the int 0)."""
    if isinstance(ld, torch.Tensor):
        return ld
    return torch.full((x.shape[0],), float(ld), device=x.device, dtype=x.dtype)


class _FlowBatchNormFn(torch.autograd.Function):
    """One between-layer BatchNorm call on the GPU with a HIP backward: (x, ld) -> (y, ld +- c)."""

    @staticmethod
    def forward(ctx, x, ld, weight, bias, bn, direction):
        x = x.contiguous()
        y = torch.empty_like(x)
        ld_out = ld.detach().to(torch.float32).contiguous().clone()
        _bn_launch(bn, x, y, ld_out, direction)
        ctx.direction = direction
        ctx.eps = float(bn.eps)
        ctx.save_for_backward(x, weight, bias, bn.running_mean.detach().clone(), bn.running_var.detach().clone())
        return y, ld_out

    @staticmethod
    def backward(ctx, gy, gld):
        x, weight, bias, rm, rv = ctx.saved_tensors
        B, d = x.shape
        gx = torch.empty_like(x)
        dg = torch.empty(d, device=x.device, dtype=torch.float32)
        db = torch.empty(d, device=x.device, dtype=torch.float32)
        gy = gy.contiguous() if gy is not None else None
        gld_c = gld.contiguous() if gld is not None else None
        ws = _bn_workspace(B, d, x.device)
        _lib.check(_lib.lib().nfx_flowbn_backward(
            _lib.ptr(x), _lib.ptr(gy), _lib.ptr(gld_c), _lib.ptr(gx), _lib.ptr(weight.detach()),
            _lib.ptr(bias.detach()), _lib.ptr(rm), _lib.ptr(rv), ctx.eps, _lib.ptr(dg), _lib.ptr(db), B, d,
            ctx.direction, _lib.ptr(ws), _lib.stream_of(x)), "nfx_flowbn_backward")
        STATS["hip"] += 1
        return gx, gld, dg, db, None, None
