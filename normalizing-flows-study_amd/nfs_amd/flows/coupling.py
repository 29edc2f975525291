"""Affine coupling layer (RealNVP) — drop-in for src/flows/coupling/coupling_layer.py.

Same constructor, attributes (`data_dim`, `mask` buffer, `s_net`, `b_net`), initialisation and
state_dict keys as the reference `CouplingLayer` (coupling_layer.py:5-111). On a ROCm device
in eval mode the layer runs as ONE fused gfx950 kernel (csrc/nfx_affine*.hip): both conditioner
MLPs on fp32 MFMA with BatchNorm folded from its running statistics, the affine transform,
the NaN/Inf guards and the log-det.

In eval mode under autograd (e.g. fine-tuning with frozen BatchNorm statistics) the same fused
backward kernels run with the running statistics in place of the batch statistics
(`_hip_backward`, nfx_affine_eval_stats), so gradients never recompute through ATen.

In TRAIN mode (the reference's training loops, README.md:107-117 / plots/_common.py:194-211)
the conditioner BatchNorm normalises with batch statistics; on a ROCm device that runs through
the train-mode kernels (csrc/nfx_affine_train.hip, `_CouplingTrainFunction`): two statistics
passes, the fused layer with the batch statistics folded in, and a three-pass fused backward
(BatchNorm backward with batch statistics, weight gradients as MFMA contractions over the
sample dimension). `nfs_amd.distributed.enable_sync_batchnorm()` takes those statistics over
all data-parallel ranks (SyncBN).
"""
import ctypes
import os

import weakref

import torch
import torch.nn as nn

from .. import _lib
from .. import distributed as _dist
from . import generic as _generic
from .flow import HipFlow, STATS

MAX_D = 64          # eval kernels: affine_coupling_kernel (d <= 8) / affine_wide_kernel (d <= 64)
MAX_D_TRAIN = 8     # train-mode / backward kernels
MAX_H = 128
MAX_H_TRAIN = 128  # HT <= 2: affine_train_kernel; HT 3, 4: affine_trainw_kernel (wide)
ctypes_vp = ctypes.c_void_p

# (kernel-name, start-event, end-event) of every train-mode layer pass while a list is installed
# here (bench.py roofline timing); None = no events.
TRAIN_EVENTS = None

# One-launch layer chains (nfx_affine_chain: the small-batch layout of csrc/nfx_affine_chain.hip
# up to 64k samples, the streaming layout of csrc/nfx_affine_schain.hip above) run every batch the
# library accepts (nfx_affine_chain_supported) up to this many samples; 0 disables them (tests
# compare them with the per-layer kernels).
CHAIN_MAX_B = int(os.environ.get("NFX_CHAIN_MAX_B", str(1 << 62)))
# Stacks with H > 64 have no streaming chain: above this many samples they run the per-layer
# streaming kernels (their MFMA tiling, measured in rounds 2-3) rather than the small-batch chain,
# whose large-batch rate at H > 64 has not been measured against them.
CHAIN_MAX_B_WIDE = int(os.environ.get("NFX_CHAIN_MAX_B_WIDE", str(1 << 16)))
# Tests: route every call through the any-shape path (csrc/nfx_generic.hip) even where a fused
# kernel exists, to pin it against the same fixtures.
FORCE_GENERIC = False
GENERIC_MAX_H = 1024  # conditioner BatchNorm moments (nfx_flowbn_moments): <= 1024 features


def chain_ok(flows, x):
    """A run of eval-mode CouplingLayers with one (d, H), d in {2, 4, 8}, H <= 128, on fp32 ROCm
    rows, that a one-launch chain kernel takes (the streaming chain: H <= 64; the small-batch
    chain: up to ~1M rows at d = 2)."""
    if FORCE_GENERIC or not flows or len(flows) > 64 or x.shape[0] > CHAIN_MAX_B or x.shape[0] == 0:
        return False
    f0 = flows[0]
    if not isinstance(f0, CouplingLayer):
        return False
    d, H = f0.data_dim, f0._hidden()
    if d not in (2, 4, 8) or H > MAX_H or x.shape[1] != d:
        return False
    if H > 64 and x.shape[0] > CHAIN_MAX_B_WIDE:
        return False
    if not _lib.lib().nfx_affine_chain_supported(x.shape[0], d, H):
        return False
    for f in flows:
        if type(f) is not CouplingLayer or f.data_dim != d or f._hidden() != H or f._torch_only():
            return False
    return True


def chain_launch(flows, x, out, ld, direction, accumulate, logprob=None):
    """All `flows` (in module order) in one nfx_affine_chain launch; with logprob=(logp, sums,
    workspace) an inverse chain also writes the Gaussian log-density and NLL partials."""
    packs = (ctypes_vp * len(flows))(*[_lib.ptr(f._packed(x.device, f._build_pack)) for f in flows])
    L = _lib.lib()
    d, H = flows[0].data_dim, flows[0]._hidden()
    p = _lib.ptr
    if logprob is not None:
        logp, sums, ws = logprob
        _lib.check(L.nfx_affine_chain_logprob(packs, len(flows), p(x), p(out), p(ld), p(logp), p(sums), p(ws),
                                              x.shape[0], d, H, int(bool(accumulate)), _lib.stream_of(x)),
                   "nfx_affine_chain_logprob")
    else:
        _lib.check(L.nfx_affine_chain(packs, len(flows), p(x), p(out), p(ld), x.shape[0], d, H, int(direction),
                                      int(bool(accumulate)), _lib.stream_of(x)), "nfx_affine_chain")
    STATS["hip"] += 1


def sample_chain_ok(flows, n, device):
    """chain_ok for the fused sampling pass (nfx_affine_chain_sample): eval-mode CouplingLayers of
    one (d, H), d in {2, 4, 8}, H <= 128, n rows within the small-batch chain, a ROCm device."""
    if FORCE_GENERIC or not flows or len(flows) > 64 or n <= 0 or torch.device(device).type != "cuda":
        return False
    f0 = flows[0]
    if type(f0) is not CouplingLayer:
        return False
    d, H = f0.data_dim, f0._hidden()
    if d not in (2, 4, 8) or H > MAX_H or n > SAMPLE_CHAIN_MAX_B:
        return False
    return all(type(f) is CouplingLayer and f.data_dim == d and f._hidden() == H and not f._torch_only()
               and not f.training for f in flows)


# the fused sampling pass runs the small-batch chain layout (one workgroup per 32-row tile up to
# 4 per CU, then several tiles per workgroup): up to 64k rows, the sizes sampling is called at
SAMPLE_CHAIN_MAX_B = 1 << 16


def chain_sample(flows, rng_state, seed, z, x, ld):
    """z ~ N(0, I) drawn on the device and x, ld = forward(z) through every flow, one launch
    (nfx_affine_chain_sample); rng_state = the device uint64[2] generator state it advances."""
    packs = (ctypes_vp * len(flows))(*[_lib.ptr(f._packed(x.device, f._build_pack)) for f in flows])
    d, H = flows[0].data_dim, flows[0]._hidden()
    p = _lib.ptr
    _lib.check(_lib.lib().nfx_affine_chain_sample(packs, len(flows), int(seed) & ((1 << 64) - 1), p(rng_state), p(z),
                                                  p(x), p(ld), x.shape[0], d, H, _lib.stream_of(x)),
               "nfx_affine_chain_sample")
    STATS["hip"] += 1


def _pad_d(d):
    return 2 if d <= 2 else (4 if d <= 4 else 8)


_KEEP_BUDGET = {}
_KEPT_LIVE = {}  # device index -> bytes of kept pre-activations alive (every layer, every model)
# How the train-mode forwards ran since the last reset: layers that kept their pre-activations
# and layers whose backward recomputes them (bench.py prices the backward's flops from this).
KEEP_STATS = {"kept": 0, "recompute": 0}


def _keep_budget(dev):
    """Bytes ONE train-mode layer may keep for its backward: 1/32 of the device's memory."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _KEEP_BUDGET:
        _KEEP_BUDGET[i] = torch.cuda.get_device_properties(i).total_memory // 32
    return _KEEP_BUDGET[i]


def _keep_reserve(dev, nbytes):
    """Admit one more kept copy: within the per-layer cap and with the copies still alive on the
    device (all layers and models together, until their backward frees them) within 1/8 of its
    memory. Returns the device index to release against, or None (the backward recomputes)."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    live = _KEPT_LIVE.get(i, 0)
    if nbytes > _keep_budget(dev) or live + nbytes > 4 * _keep_budget(dev):
        return None
    _KEPT_LIVE[i] = live + nbytes
    return i


def _keep_release(i, nbytes):
    _KEPT_LIVE[i] = _KEPT_LIVE.get(i, 0) - nbytes


class _CouplingTrainFunction(torch.autograd.Function):
    """Train-mode CouplingLayer on the gfx950 kernels: forward (y, log_det) with batch-statistics
    BatchNorm and running-statistics update; backward = the fused three-pass kernel."""

    @staticmethod
    def forward(ctx, layer, direction, x, *params):
        y, ld, tpack, stats = layer._train_forward(x, direction, keep=True)
        ctx.layer = layer
        ctx.direction = direction
        ctx.tpack = tpack
        ctx.stats = stats
        # the kept layer-2 pre-activations go through save_for_backward (not an attribute of the
        # pack): autograd frees them when this node's backward has run
        h2 = getattr(tpack, "_nfx_h2", None)  # (the any-shape path's tpack is a plain list)
        if h2 is not None:
            tpack._nfx_h2 = None
        ctx.save_for_backward(x, h2)
        return y, ld

    @staticmethod
    def backward(ctx, gy, gld):
        x, h2 = ctx.saved_tensors
        gx, grads = ctx.layer._train_backward(x, gy, gld, ctx.direction, ctx.tpack, ctx.stats, h2=h2)
        STATS["hip"] += 1
        params = list(ctx.layer.parameters())
        gparams = [g if p.requires_grad else None for p, g in zip(params, grads)]
        return (None, None, gx, *gparams)


class CouplingLayer(HipFlow):
    def __init__(self, data_dim, hidden_dim, mask):
        super().__init__()
        self.data_dim = data_dim
        self.register_buffer("mask", mask)
        # coupling_layer.py:18-35
        self.s_net = nn.Sequential(
            nn.Linear(data_dim, hidden_dim), nn.BatchNorm1d(hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, hidden_dim), nn.BatchNorm1d(hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, data_dim))
        self.b_net = nn.Sequential(
            nn.Linear(data_dim, hidden_dim), nn.BatchNorm1d(hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, hidden_dim), nn.BatchNorm1d(hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, data_dim))
        self._initialize_weights()

    def _initialize_weights(self):
        # coupling_layer.py:98-111
        for net in [self.s_net, self.b_net]:
            for layer in net[:-1]:
                if isinstance(layer, nn.Linear):
                    nn.init.xavier_normal_(layer.weight, gain=1.0)
                    if layer.bias is not None:
                        nn.init.zeros_(layer.bias)
        nn.init.zeros_(self.s_net[-1].weight)
        nn.init.zeros_(self.s_net[-1].bias)
        nn.init.zeros_(self.b_net[-1].weight)
        nn.init.zeros_(self.b_net[-1].bias)

    # -- composite (autograd / CPU / fp64) path: the reference math -------------------------
    def _torch_call(self, x, direction):
        mask = self.mask
        xa = x * mask
        s = torch.clamp(self.s_net(xa), min=-10.0, max=10.0)
        b = torch.clamp(self.b_net(xa), min=-10.0, max=10.0)
        if direction > 0:  # coupling_layer.py:40-68
            y = xa + (1 - mask) * (x * torch.exp(s) + b)
            ld = ((1 - mask) * s).sum(dim=1)
        else:  # coupling_layer.py:70-96
            y = xa + (1 - mask) * ((x - b) * torch.exp(-s))
            ld = ((1 - mask) * -s).sum(dim=1)
        y = torch.where(torch.isnan(y) | torch.isinf(y), torch.zeros_like(y), y)
        ld = torch.where(torch.isnan(ld) | torch.isinf(ld), torch.zeros_like(ld), ld)
        return y, ld

    # -- HIP path ---------------------------------------------------------------------------
    def _hidden(self):
        return self.s_net[0].out_features

    def _torch_only(self):
        # The eval kernel folds running statistics; train-mode BatchNorm goes through
        # _dispatch -> _CouplingTrainFunction (or the composite when outside its family).
        return any(bn.training or bn.running_mean is None for bn in self._batchnorms())

    # -- train mode (batch-statistics BatchNorm) ----------------------------------------------
    def _train_ok(self, x):
        bns = self._batchnorms()
        if x.device.type != "cuda" or x.dtype != torch.float32 or x.dim() != 2:
            return False
        if not bns or not all(bn.training for bn in bns):
            return False
        if any(not bn.affine or not bn.track_running_stats or bn.momentum is None or bn.running_mean is None
               for bn in bns):
            return False
        return x.shape[1] == self.data_dim and x.shape[0] >= 2 and (self._fused_train() or self._hidden() <= GENERIC_MAX_H)

    def _fused_train(self):
        """Shapes of the fused train-mode / backward kernels (affine_train*_kernel); others run the
        any-shape path (GEMM conditioner, BatchNorm and affine element kernels)."""
        return not FORCE_GENERIC and self.data_dim <= MAX_D_TRAIN and self._hidden() <= MAX_H_TRAIN

    def _fused_family(self):
        """Shapes of the fused eval kernels (affine_coupling_kernel / affine_wide_kernel)."""
        return not FORCE_GENERIC and self.data_dim <= MAX_D and self._hidden() <= MAX_H

    # -- any-shape path (csrc/nfx_generic.hip) ---------------------------------------------------
    def _generic_nets(self):
        return [(n[0], n[1], n[3], n[4], n[6]) for n in (self.s_net, self.b_net)]

    def _generic_bn_eval(self, device):
        """Per conditioner BatchNorm [4][H] = (mean, invstd, scale, shift) from the running
        statistics (nfx_bn_prepare), cached with the parameters."""
        L = _lib.lib()
        H = self._hidden()
        out = []
        for _, bn1, _, bn2, _ in self._generic_nets():
            for bn in (bn1, bn2):
                t = torch.empty(4, H, device=device, dtype=torch.float32)
                _lib.check(L.nfx_bn_prepare(None, _lib.ptr(bn.weight.detach()), _lib.ptr(bn.bias.detach()),
                                            _lib.ptr(bn.running_mean), _lib.ptr(bn.running_var), float(bn.eps), 0.0,
                                            0, H, _lib.ptr(t[0]), _lib.ptr(t[1]), _lib.ptr(t[2]), _lib.ptr(t[3]),
                                            _lib.stream_of(t)), "nfx_bn_prepare")
                out.append(t)
        return out

    def _mask_dev(self, device):
        return self.mask.detach().to(device=device, dtype=torch.float32).contiguous()

    def _generic_launch(self, x, out, log_det, direction, accumulate):
        mask = self._mask_dev(x.device)
        bnp = self._packed(x.device, self._generic_bn_eval, slot="_nfx_generic_pack_cache")
        raw = []
        for i, (l1, _, l2, _, l3) in enumerate(self._generic_nets()):
            p1, p2 = bnp[2 * i], bnp[2 * i + 1]
            h1 = _generic.linear_forward(x, l1, in_scale=mask, relu=True, post=(p1[2], p1[3]))
            h2 = _generic.linear_forward(h1, l2, relu=True, post=(p2[2], p2[3]))
            raw.append(_generic.linear_forward(h2, l3))
        _lib.check(_lib.lib().nfx_affine_elem_forward(
            _lib.ptr(x), _lib.ptr(raw[0]), _lib.ptr(raw[1]), _lib.ptr(mask), _lib.ptr(out), _lib.ptr(log_det),
            x.shape[0], self.data_dim, int(direction), int(bool(accumulate)), _lib.stream_of(x)),
            "nfx_affine_elem_forward")

    def _generic_acts(self, x, mask, bnp):
        """Conditioner recompute with given BatchNorm (mean, invstd, scale, shift): per net
        (z1, h1, z2, h2, raw output)."""
        L = _lib.lib()
        B, H = x.shape[0], self._hidden()
        acts = []
        for i, (l1, _, l2, _, l3) in enumerate(self._generic_nets()):
            z1 = _generic.linear_forward(x, l1, in_scale=mask)
            h1 = torch.empty_like(z1)
            _lib.check(L.nfx_bn_apply_relu(_lib.ptr(z1), _lib.ptr(bnp[2 * i][2]), _lib.ptr(bnp[2 * i][3]),
                                           _lib.ptr(h1), B, H, _lib.stream_of(x)), "nfx_bn_apply_relu")
            z2 = _generic.linear_forward(h1, l2)
            h2 = torch.empty_like(z2)
            _lib.check(L.nfx_bn_apply_relu(_lib.ptr(z2), _lib.ptr(bnp[2 * i + 1][2]), _lib.ptr(bnp[2 * i + 1][3]),
                                           _lib.ptr(h2), B, H, _lib.stream_of(x)), "nfx_bn_apply_relu")
            acts.append((z1, h1, z2, h2, _generic.linear_forward(h2, l3)))
        return acts

    def _generic_train_forward(self, x, direction):
        """Train mode on the any-shape path: per conditioner BatchNorm the batch moments
        (nfx_flowbn_moments, SyncBN-merged), mean/invstd/scale/shift and the running update
        (nfx_bn_prepare), then the affine element map. Returns (y, ld, bnp, counts)."""
        L = _lib.lib()
        x = x.detach().contiguous()
        B, d = x.shape
        H = self._hidden()
        dev = x.device
        st = _lib.stream_of(x)
        p = _lib.ptr
        mask = self._mask_dev(dev)
        ws = torch.empty(max(1, L.nfx_flowbn_workspace_bytes(B, H)), device=dev, dtype=torch.uint8)
        bnp, counts, raw = [], [], []
        for l1, bn1, l2, bn2, l3 in self._generic_nets():
            h = x
            for lin, bn, first in ((l1, bn1, True), (l2, bn2, False)):
                z = _generic.linear_forward(h, lin, in_scale=mask if first else None)
                stats = torch.empty(H, 3, device=dev, dtype=torch.float64)
                _lib.check(L.nfx_flowbn_moments(p(z), B, H, p(stats), p(ws), st), "nfx_flowbn_moments")
                _dist.merge_bn_stats(stats)
                t = torch.empty(4, H, device=dev, dtype=torch.float32)
                _lib.check(L.nfx_bn_prepare(p(stats), p(bn.weight.detach()), p(bn.bias.detach()), p(bn.running_mean),
                                            p(bn.running_var), float(bn.eps), float(bn.momentum), 1, H, p(t[0]),
                                            p(t[1]), p(t[2]), p(t[3]), st), "nfx_bn_prepare")
                torch.autograd.graph.increment_version(bn.running_mean)
                torch.autograd.graph.increment_version(bn.running_var)
                h = torch.empty_like(z)
                _lib.check(L.nfx_bn_apply_relu(p(z), p(t[2]), p(t[3]), p(h), B, H, st), "nfx_bn_apply_relu")
                bnp.append(t)
                counts.append(stats)  # stats[0, 0] = the global sample count
            raw.append(_generic.linear_forward(h, l3))
        bns = [self.s_net[1], self.s_net[4], self.b_net[1], self.b_net[4]]
        torch._foreach_add_([bn.num_batches_tracked for bn in bns], 1)
        y = torch.empty_like(x)
        ld = torch.empty(B, device=dev, dtype=torch.float32)
        _lib.check(L.nfx_affine_elem_forward(p(x), p(raw[0]), p(raw[1]), p(mask), p(y), p(ld), B, d, int(direction), 0,
                                             st), "nfx_affine_elem_forward")
        return y, ld, bnp, counts

    def _generic_backward(self, x, gy, gld, direction, bnp, counts):
        """dL/dx and the parameter gradients (parameters() order) on the any-shape path: the
        conditioner recomputed with the call's BatchNorm normalisation, the affine element adjoint,
        then per net the Linear / BatchNorm / ReLU backward (train: batch-statistics BatchNorm
        backward with SyncBN-summed float64 sums; counts = None: eval, running statistics)."""
        L = _lib.lib()
        B, d = x.shape
        H = self._hidden()
        st = _lib.stream_of(x)
        p = _lib.ptr
        mask = self._mask_dev(x.device)
        acts = self._generic_acts(x, mask, bnp)
        gs, gb, gx = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
        _lib.check(L.nfx_affine_elem_backward(p(x), p(acts[0][4]), p(acts[1][4]), p(mask), p(gy), p(gld), p(gs), p(gb),
                                              p(gx), B, d, int(direction), st), "nfx_affine_elem_backward")
        ws = torch.empty(max(1, L.nfx_bn_workspace_bytes(B, H)), device=x.device, dtype=torch.uint8)
        train = counts is not None
        grads = []
        for i, ((l1, bn1, l2, bn2, l3), g_out) in enumerate(zip(self._generic_nets(), (gs, gb))):
            z1, h1, z2, h2, _ = acts[i]
            w3 = _generic.linear_backward_weight(g_out, h2, l3)
            g = _generic.linear_backward_data(g_out, l3, act=h2)
            per = []
            for z, hin, lin, bn, k in ((z2, h1, l2, bn2, 2 * i + 1), (z1, x, l1, bn1, 2 * i)):
                t = bnp[k]
                sums = torch.empty(2, H, device=x.device, dtype=torch.float64)
                _lib.check(L.nfx_bn_backward_sums(p(g), p(z), p(t[0]), p(t[1]), p(sums), B, H, p(ws), st),
                           "nfx_bn_backward_sums")
                if train:
                    _dist.allreduce_bn_sums(sums)
                gz = torch.empty_like(g)
                # train: the global sample count = n of the merged moments triple (device float64)
                _lib.check(L.nfx_bn_backward_apply(p(g), p(z), p(t[0]), p(t[1]), p(bn.weight.detach()), p(sums),
                                                   p(counts[k]) if train else None, int(train), p(gz), B, H, st),
                           "nfx_bn_backward_apply")
                first = lin is l1
                wl = _generic.linear_backward_weight(gz, hin, lin, in_scale=mask if first else None)
                if first:
                    _generic.linear_backward_data(gz, lin, out_scale=mask, out=gx)
                else:
                    g = _generic.linear_backward_data(gz, lin, act=hin)
                per.append((wl, sums[1].float(), sums[0].float()))
            (w2, dg2, db2), (w1, dg1, db1) = per
            grads += [w1[0], w1[1], dg1, db1, w2[0], w2[1], dg2, db2, w3[0], w3[1]]
        return gx, grads

    def _dispatch(self, x, direction):
        if self._train_ok(x):
            STATS["hip"] += 1
            if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
                return _CouplingTrainFunction.apply(self, direction, x, *list(self.parameters()))
            y, ld, _, _ = self._train_forward(x, direction)
            return y, ld
        return super()._dispatch(x, direction)

    def _raw_nets(self):
        s_raw, k1 = _lib.mlp_raw([self.s_net[0], self.s_net[3], self.s_net[6]], [self.s_net[1], self.s_net[4]])
        b_raw, k2 = _lib.mlp_raw([self.b_net[0], self.b_net[3], self.b_net[6]], [self.b_net[1], self.b_net[4]])
        return s_raw, b_raw, (k1, k2)

    def _train_forward(self, x, direction, keep=False):
        """Batch statistics (2 passes, SyncBN merge between them), the fused layer with the
        statistics folded in, running-statistics update. Returns (y, ld, tpack, stats). keep=True
        (a forward the backward will follow): the layer-2 statistics pass also keeps the raw
        layer-2 pre-activations in HBM (tpack._nfx_h2, 512 B per sample at H = 64) for the
        backward's first two passes, which then skip recomputing layers 1-2."""
        if not self._fused_train():
            return self._generic_train_forward(x, direction)
        L = _lib.lib()
        x = x.detach().contiguous()
        B, d = x.shape
        H = self._hidden()
        dev = x.device
        st = _lib.stream_of(x)
        s_raw, b_raw, keep_src = self._raw_nets()
        mask = self.mask.detach().to(device=dev, dtype=torch.float32).contiguous()
        nst = L.nfx_affine_train_stats_doubles(H)
        stats = torch.empty(2, nst, device=dev, dtype=torch.float64)
        tpack = torch.empty(L.nfx_affine_train_pack_floats(d, H), device=dev, dtype=torch.float32)
        epack = torch.empty(L.nfx_affine_packed_floats(d, H), device=dev, dtype=torch.float32)
        ws = torch.empty(L.nfx_affine_train_workspace_bytes(B, d, H), device=dev, dtype=torch.uint8)
        keep = keep and os.environ.get("NFX_TRAIN_KEEP", "1") != "0"  # 0: the backward recomputes
        nkeep = L.nfx_affine_train_keep_floats(B, d, H) if keep else 0
        # a layer's kept copy is capped at 1/32 of HBM (9 GB, 17.6M samples at H = 64), the live
        # copies of all layers at 1/8; beyond that the backward recomputes layers 1-2
        rel = _keep_reserve(dev, 4 * nkeep) if nkeep else None
        h2 = None
        if rel is not None:
            h2 = torch.empty(nkeep, device=dev, dtype=torch.float32)
            weakref.finalize(h2, _keep_release, rel, 4 * nkeep)
        KEEP_STATS["kept" if h2 is not None else "recompute"] += 1
        ev = TRAIN_EVENTS
        p = _lib.ptr
        _lib.check(L.nfx_affine_train_pack(s_raw, b_raw, p(mask), None, None, d, H, p(tpack), None, st),
                   "nfx_affine_train_pack")
        for layer in (1, 2):
            if ev is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            _lib.check(L.nfx_affine_train_stats_keep(p(tpack), p(x), B, d, H, layer, p(stats[layer - 1]), p(ws),
                                                     p(h2) if (h2 is not None and layer == 2) else None, st),
                       "nfx_affine_train_stats")
            if ev is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                kn = "affine_trainw_kernel" if H > 64 else "affine_train_kernel"
                ev.append((f"{kn}<STATS{layer}>", e0, e1))
            _dist.merge_bn_stats(stats[layer - 1].view(2, -1, 3))
            _lib.check(L.nfx_affine_train_pack(s_raw, b_raw, p(mask), p(stats[0]),
                                               p(stats[1]) if layer == 2 else None, d, H, p(tpack),
                                               p(epack) if (layer == 2 and h2 is None) else None, st),
                       "nfx_affine_train_pack")  # (kept pre-activations: OUTK needs no eval image)
        y = torch.empty_like(x)
        ld = torch.empty(B, device=dev, dtype=torch.float32)
        if ev is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if h2 is not None:  # from the kept pre-activations (no layer 1-2 recompute)
            _lib.check(L.nfx_affine_train_output(p(tpack), p(x), p(h2), p(y), p(ld), B, d, H, int(direction), st),
                       "nfx_affine_train_output")
        else:
            _lib.check(L.nfx_affine_coupling(p(epack), p(x), p(y), p(ld), B, d, H, int(direction), 0, st),
                       "nfx_affine_coupling")
        if ev is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            ev.append(("affine_train_kernel<OUTK>" if h2 is not None else "affine_coupling_kernel", e0, e1))
        bns = [self.s_net[1], self.s_net[4], self.b_net[1], self.b_net[4]]
        rm = (ctypes_vp * 4)(*[bn.running_mean.data_ptr() for bn in bns])
        rv = (ctypes_vp * 4)(*[bn.running_var.data_ptr() for bn in bns])
        counted = all(bn.num_batches_tracked is not None and bn.num_batches_tracked.dtype == torch.int64
                      and bn.num_batches_tracked.device == dev for bn in bns)
        nb = (ctypes_vp * 4)(*[bn.num_batches_tracked.data_ptr() for bn in bns]) if counted else None
        _lib.check(L.nfx_affine_train_update_running_counted(p(stats[0]), p(stats[1]), rm, rv, nb, H,
                                                             float(bns[0].momentum), st),
                   "nfx_affine_train_update_running")
        for bn in bns:
            torch.autograd.graph.increment_version(bn.running_mean)
            torch.autograd.graph.increment_version(bn.running_var)
            if counted:
                torch.autograd.graph.increment_version(bn.num_batches_tracked)
        if not counted:
            torch._foreach_add_([bn.num_batches_tracked for bn in bns], 1)
        tpack._nfx_keep = (keep_src, mask, epack, ws)  # sources alive while the kernels are queued
        tpack._nfx_h2 = h2
        return y, ld, tpack, stats

    # -- eval mode under autograd (running-statistics BatchNorm) -----------------------------
    def _hip_backward_ok(self, x, direction):
        """Eval-mode call under autograd: the train-mode backward kernels with the BatchNorm
        running statistics in place of batch statistics (nfx_affine_eval_stats)."""
        bns = self._batchnorms()
        if x.dtype != torch.float32 or x.dim() != 2 or len(bns) != 4:
            return False
        if any(bn.training or not bn.affine or bn.running_mean is None for bn in bns):
            return False
        return x.shape[1] == self.data_dim  # fused (d <= 8, H <= 128) or the any-shape path

    def _build_eval_backward_pack(self, device):
        L = _lib.lib()
        d, H = self.data_dim, self._hidden()
        s_raw, b_raw, keep = self._raw_nets()
        mask = self.mask.detach().to(device=device, dtype=torch.float32).contiguous()
        stats = torch.empty(2, L.nfx_affine_train_stats_doubles(H), device=device, dtype=torch.float64)
        st = _lib.stream_of(stats)
        bns = [self.s_net[1], self.s_net[4], self.b_net[1], self.b_net[4]]
        rm = (ctypes_vp * 4)(*[bn.running_mean.data_ptr() for bn in bns])
        rv = (ctypes_vp * 4)(*[bn.running_var.data_ptr() for bn in bns])
        p = _lib.ptr
        _lib.check(L.nfx_affine_eval_stats(rm, rv, H, p(stats[0]), p(stats[1]), st), "nfx_affine_eval_stats")
        tpack = torch.empty(L.nfx_affine_train_pack_floats(d, H), device=device, dtype=torch.float32)
        _lib.check(L.nfx_affine_train_pack(s_raw, b_raw, p(mask), p(stats[0]), p(stats[1]), d, H, p(tpack), None, st),
                   "nfx_affine_train_pack")
        tpack._nfx_keep = (keep, mask)
        return tpack, stats

    def _hip_backward(self, x, gy, gld, direction):
        if not self._fused_train():
            x = x.contiguous()
            gy = torch.zeros_like(x) if gy is None else gy.contiguous().float()
            gld = torch.zeros(x.shape[0], device=x.device) if gld is None else gld.contiguous().float()
            bnp = self._packed(x.device, self._generic_bn_eval, slot="_nfx_generic_pack_cache")
            return self._generic_backward(x, gy, gld, direction, bnp, None)
        tpack, stats = self._packed(x.device, self._build_eval_backward_pack, slot="_nfx_evalbwd_pack_cache")
        return self._train_backward(x, gy, gld, direction, tpack, stats, sync=False)

    def _train_backward(self, x, gy, gld, direction, tpack, stats, sync=True, h2=None):
        """dL/dx and the parameter gradients (parameters() order) of one train-mode call
        (sync=False: eval mode, the BatchNorm sums are plain parameter-gradient partials)."""
        L = _lib.lib()
        x = x.contiguous()
        B, d = x.shape
        H = self._hidden()
        dev = x.device
        st = _lib.stream_of(x)
        gy = torch.zeros_like(x) if gy is None else gy.contiguous().float()
        gld = torch.zeros(B, device=dev) if gld is None else gld.contiguous().float()
        if not self._fused_train():  # tpack, stats = the any-shape path's (bnp, counts)
            return self._generic_backward(x, gy, gld, direction, tpack, stats)
        G = torch.empty(L.nfx_affine_train_grad_doubles(d, H), device=dev, dtype=torch.float64)
        gx = torch.empty_like(x)
        ws = torch.empty(L.nfx_affine_train_workspace_bytes(B, d, H), device=dev, dtype=torch.uint8)
        Hp, D = 32 * ((H + 31) // 32), _pad_d(d)
        s_blocks = {1: G[0:4 * Hp], 2: G[4 * Hp + 2 * (D * Hp + D):][:4 * Hp]}
        if h2 is None:  # kept by a train-mode forward (else: recompute)
            h2 = getattr(tpack, "_nfx_h2", None)
        p = _lib.ptr
        ev = TRAIN_EVENTS
        for stage in (1, 2, 3):
            if ev is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            kept = h2 if stage < 3 else None
            _lib.check(L.nfx_affine_train_backward_keep(p(tpack), p(x), p(gy), p(gld), p(gx), B, d, H,
                                                        int(direction), stage, p(stats[1]), p(G), p(ws),
                                                        p(kept) if kept is not None else None, st),
                       "nfx_affine_train_backward")
            if ev is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                kn = "affine_trainw_kernel" if H > 64 else "affine_train_kernel"
                ev.append((f"{kn}<BWD{stage}>", e0, e1))
            if sync and stage in s_blocks:
                _dist.allreduce_bn_sums(s_blocks[stage])
        grads = torch.empty(L.nfx_affine_train_param_floats(d, H), device=dev, dtype=torch.float32)
        _lib.check(L.nfx_affine_train_assemble(p(G), p(stats[0]), p(stats[1]), d, H, float(self.s_net[1].eps),
                                               p(grads), st), "nfx_affine_train_assemble")
        out, o = [], 0
        for prm in self.parameters():
            n = prm.numel()
            out.append(grads[o:o + n].view_as(prm))
            o += n
        grads._nfx_keep = (ws, G)
        return gx, out

    def _hip_supported(self, x):
        d = self.data_dim
        if x.dim() != 2 or x.shape[1] != d:
            return False, f"input shape {tuple(x.shape)} vs data_dim={d}"
        return True, ""  # beyond the fused family: the any-shape path (_generic_launch)

    def _build_pack(self, device):
        d, H = self.data_dim, self._hidden()
        L = _lib.lib()
        n = L.nfx_affine_packed_floats(d, H)
        packed = torch.empty(n, device=device, dtype=torch.float32)
        s_raw, k1 = _lib.mlp_raw([self.s_net[0], self.s_net[3], self.s_net[6]],
                                 [self.s_net[1], self.s_net[4]])
        b_raw, k2 = _lib.mlp_raw([self.b_net[0], self.b_net[3], self.b_net[6]],
                                 [self.b_net[1], self.b_net[4]])
        mask = self.mask.detach().to(device=device, dtype=torch.float32).contiguous()
        _lib.check(L.nfx_affine_pack(s_raw, b_raw, _lib.ptr(mask), d, H, _lib.ptr(packed),
                                     _lib.stream_of(packed)), "nfx_affine_pack")
        packed._nfx_keep = (k1, k2, mask)  # sources stay alive while the pack kernel is queued
        return packed

    def _hip_launch(self, x, out, log_det, direction, accumulate):
        if not self._fused_family():
            return self._generic_launch(x, out, log_det, direction, accumulate)
        packed = self._packed(x.device, self._build_pack)
        _lib.check(_lib.lib().nfx_affine_coupling(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), x.shape[0],
            self.data_dim, self._hidden(), int(direction), int(bool(accumulate)),
            _lib.stream_of(x)), "nfx_affine_coupling")

    def _hip_launch_logprob(self, x, out, log_det, logp, sums, workspace, accumulate):
        if not self._fused_family():
            return False
        packed = self._packed(x.device, self._build_pack)
        _lib.check(_lib.lib().nfx_affine_coupling_logprob(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), _lib.ptr(logp),
            _lib.ptr(sums), _lib.ptr(workspace), x.shape[0], self.data_dim, self._hidden(),
            int(bool(accumulate)), _lib.stream_of(x)), "nfx_affine_coupling_logprob")
        return True
