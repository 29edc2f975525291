"""MADE-masked autoregressive affine flows — drop-ins for src/flows/autoregressive/.

  MaskedLinear               masked_linear.py:4-18
  MADE                       made.py:6-140 (degrees :24-41, masks :47-79, net :81-134)
  MaskedAutoregressiveFlow   masked_autoregressive_flow.py:5-78
  InverseAutoregressiveFlow  inverse_autoregressive_flow.py:5-103

Constructors, attributes (`conditioner.net[...]`, `dim`, `data_dim`), initialisation order and
state_dict keys (`conditioner.net.{0,2,4,6}.{weight,bias,mask}`) match the reference. On a
ROCm device every direction runs as one gfx950 kernel (csrc/nfx_made*.hip):
  * MAF.inverse / IAF.forward (parallel): the dense masked MADE on fp32 MFMA, W*M pre-applied
    once at pack time (bit-identical to the per-call weight*mask, masks are 0/1).
  * MAF.forward / IAF.inverse (sequential over d in the reference: d full MADE calls): a
    level-scheduled kernel that computes each hidden unit once, as soon as the inputs of its
    degree are known, and each output once — the same values (masked weights multiply exact
    zeros) at the cost of ONE MADE evaluation instead of d.
"""
import ctypes

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from .. import distributed as _dist
from . import generic as _generic
from .flow import HipFlow, STATS

MAX_H = 256       # eval kernels (H > 128: nfx_made_big.hip)
MAX_H_BWD = 128   # fused backward kernels; wider layers: the any-shape path (csrc/nfx_generic.hip)
MAX_D = 4096
# Tests: route every call through the any-shape path (csrc/nfx_generic.hip) even where a fused
# kernel exists, to pin it against the same fixtures.
FORCE_GENERIC = False
# Profiling hook (bench.py): when set to a list, every fused backward launch appends
# (name, start, end) HIP events recorded on the launch stream around the kernel.
BACKWARD_EVENTS = None


def made_degrees(input_dim, hidden_dim):
    """Hidden-unit degrees m[0] of MADE (made.py:24-41), restated exactly.

    d == 2: the [0,0,1,1]* pattern; d == 1: zeros; otherwise floor(numpy.linspace(0, d-1, H)),
    i.e. floor(i * ((d-1)/(H-1))) in float64 with the last entry pinned to d-1 (numpy's
    linspace sets y[-1] = stop). An integer i*(d-1)//(H-1) is NOT equivalent."""
    if input_dim > 1:
        if input_dim == 2:
            return np.array([0, 0, 1, 1] * (hidden_dim // 4 + 1))[:hidden_dim]
        if hidden_dim == 1:
            return np.zeros(1, dtype=int)
        step = float(input_dim - 1) / float(hidden_dim - 1)
        deg = [int(np.floor(float(i) * step)) for i in range(hidden_dim)]
        deg[-1] = input_dim - 1
        return np.array(deg, dtype=int)
    return np.zeros(hidden_dim, dtype=int)


class MaskedLinear(nn.Linear):
    """A linear layer with a fixed binary mask (masked_linear.py:4-18)."""

    def __init__(self, in_features, out_features, mask, bias=True):
        super().__init__(in_features, out_features, bias)
        self.register_buffer("mask", mask)

    def forward(self, input):
        mask = self.mask.to(dtype=self.weight.dtype)
        return F.linear(input, self.weight * mask, self.bias)


class MADE(nn.Module):
    def __init__(self, input_dim, hidden_dim, output_dim_multiplier=2, use_batch_norm=False):
        super().__init__()
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.output_dim_multiplier = output_dim_multiplier
        self.use_batch_norm = use_batch_norm
        self.m = {-1: np.arange(input_dim), 0: made_degrees(input_dim, hidden_dim), 1: np.arange(input_dim)}
        self.masks = self.create_masks()
        self.net = self.create_network()

    def create_masks(self):
        m_in, m_h, m_out = self.m[-1], self.m[0], self.m[1]
        # input -> hidden: deg(j) <= deg(a) (made.py:56)
        m1 = (m_in[np.newaxis, :] <= m_h[:, np.newaxis]).astype(np.float32)
        # hidden -> hidden: deg(b) <= deg(a) (made.py:63)
        mhh = (m_h[np.newaxis, :] <= m_h[:, np.newaxis]).astype(np.float32)
        # hidden -> output k*d + i: deg(a) < i, strict (made.py:72-78)
        row = (m_h[np.newaxis, :] < m_out[:, np.newaxis]).astype(np.float32)
        m2 = np.concatenate([row] * self.output_dim_multiplier, axis=0)
        return [torch.from_numpy(m1), torch.from_numpy(mhh), torch.from_numpy(np.ascontiguousarray(m2))]

    def create_network(self):
        d, H = self.input_dim, self.hidden_dim
        first = MaskedLinear(d, H, mask=self.masks[0])
        second = MaskedLinear(H, H, mask=self.masks[1])
        third = MaskedLinear(H, H, mask=self.masks[1])
        final = MaskedLinear(H, d * self.output_dim_multiplier, mask=self.masks[2])
        layers = []
        for lin in (first, second, third):
            layers.append(lin)
            if self.use_batch_norm:
                layers.append(nn.BatchNorm1d(H))
            layers.append(nn.ReLU())
        layers.append(final)
        # made.py:117-132 (same order as the reference so seeded inits match)
        for lin in (first, second, third):
            nn.init.xavier_normal_(lin.weight, gain=0.5)
            if lin.bias is not None:
                nn.init.zeros_(lin.bias)
        nn.init.normal_(final.weight, mean=0.0, std=0.01)
        if final.bias is not None:
            nn.init.zeros_(final.bias)
        return nn.Sequential(*layers)

    def forward(self, x):
        return self.net(x)

    # pieces the kernels need
    def linears(self):
        return [m for m in self.net if isinstance(m, MaskedLinear)]

    def batchnorms(self):
        return [m for m in self.net if isinstance(m, nn.BatchNorm1d)]


class _MadeAffineFlow(HipFlow):
    """Shared HIP plumbing of MAF / IAF (conditioner = MADE(dim, H, 2))."""

    def __init__(self, dim, hidden_dim=64, use_batch_norm=False):
        super().__init__()
        self.data_dim = dim
        self.dim = dim
        self.conditioner = MADE(dim, hidden_dim, 2, use_batch_norm=use_batch_norm)

    def _torch_only(self):
        return any(bn.training or bn.running_mean is None for bn in self._batchnorms())

    def _hip_supported(self, x):
        d = self.dim
        if x.dim() != 2 or x.shape[1] != d:
            return False, f"input shape {tuple(x.shape)} vs dim={d}"
        return True, ""  # beyond the fused family: the any-shape path (_generic_launch)

    def _fused_family(self):
        """Shapes of the fused eval kernels (nfx_made*.hip); wider ones run the any-shape path."""
        return not FORCE_GENERIC and self.dim <= MAX_D and self.conditioner.hidden_dim <= MAX_H

    # -- any-shape path (csrc/nfx_generic.hip): the MADE one MaskedLinear at a time on MFMA ------
    def _generic_pack(self, device):
        """(masks, eval-BatchNorm post affines) on the device, cached with the parameters."""
        lins = self.conditioner.linears()
        masks = [lin.mask.detach().to(device=device, dtype=torch.float32).contiguous() for lin in lins]
        posts = [None, None, None]
        bns = self.conditioner.batchnorms()
        if bns:
            for i, bn in enumerate(bns):
                sc = (bn.weight.detach() / torch.sqrt(bn.running_var.detach() + bn.eps)).float().contiguous()
                sh = (bn.bias.detach() - bn.running_mean.detach() * sc).float().contiguous()
                posts[i] = (sc, sh)
        return masks, posts

    def _generic_made(self, x):
        masks, posts = self._packed(x.device, self._generic_pack, slot="_nfx_generic_pack_cache")
        return masks, _generic.made_forward(x, self.conditioner.linears(), masks, posts)

    def _generic_bn_eval(self, device):
        """Per MADE BatchNorm [mean, invstd, scale, shift] from the running statistics."""
        return made_bn_eval_params(self.conditioner, device)

    def _generic_made_bn(self, x, bnp=None):
        """MADE with BatchNorm (eval: running statistics unless bnp is given): (masks, acts, params)."""
        masks, _ = self._packed(x.device, self._generic_pack, slot="_nfx_generic_pack_cache")
        if bnp is None:
            bnp = self._packed(x.device, self._generic_bn_eval, slot="_nfx_generic_bn_pack_cache")
        acts, prm = _generic.made_bn_forward(x, self.conditioner.linears(), masks, bnp)
        return masks, bnp, acts, prm

    def _parallel(self, direction):
        return self._variant(direction) in (_lib.NFX_MAF_INVERSE, _lib.NFX_IAF_FORWARD)

    # -- train-mode BatchNorm in the MADE (use_batch_norm=True) ---------------------------------------
    def _bn_train_any(self, x):
        return bn_train_supported(self.conditioner, x, self.dim)

    def _bn_train_ok(self, x, direction):
        """Parallel direction: one MADE call with batch statistics."""
        return self._bn_train_any(x) and self._parallel(direction)

    def _bn_train_seq_ok(self, x, direction):
        """Sequential direction: the reference's d MADE calls, each with its own batch statistics."""
        return self._bn_train_any(x) and not self._parallel(direction)

    def _dispatch(self, x, direction):
        grad = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters()))
        if self._bn_train_ok(x, direction):
            STATS["hip"] += 1
            if grad:
                return _MadeTrainFunction.apply(self, direction, x, *list(self.parameters()))
            y, ld, _, _ = self._generic_train_forward(x, direction)
            return y, ld
        if self._bn_train_seq_ok(x, direction):
            STATS["hip"] += 1
            if grad:
                return _MadeSeqTrainFunction.apply(self, direction, x, *list(self.parameters()))
            return self._generic_seq_train_forward(x, direction)[:2]
        return super()._dispatch(x, direction)

    def _generic_made_bn_train(self, h):
        """One train-mode MADE call on h (made_bn_train_call): (params, bnp, counts)."""
        masks, _ = self._packed(h.device, self._generic_pack, slot="_nfx_generic_pack_cache")
        return made_bn_train_call(self.conditioner, masks, h)

    def _generic_seq_train_forward(self, x, direction):
        """A sequential direction with train-mode BatchNorm, as the reference runs it: d MADE calls
        on the partial vector, each normalising with its own batch statistics and updating the
        running statistics (so d updates per forward), one element step each; then the guards.
        Returns (y, ld, work, wld, bnps, counts)."""
        L = _lib.lib()
        x = x.detach().contiguous()
        B, d = x.shape
        variant = self._variant(direction)
        st = _lib.stream_of(x)
        p = _lib.ptr
        work = torch.zeros_like(x)
        wld = torch.zeros(B, device=x.device, dtype=torch.float32)
        bnps, counts = [], []
        for i in range(d):
            prm, bnp, cnt = self._generic_made_bn_train(work)
            _lib.check(L.nfx_made_elem_step(p(x), p(prm), p(work), p(wld), B, d, i, variant, st), "nfx_made_elem_step")
            bnps.append(bnp)
            counts.append(cnt)
        y = torch.empty_like(x)
        ld = torch.empty(B, device=x.device, dtype=torch.float32)
        _lib.check(L.nfx_made_elem_finish(p(x), p(work), p(wld), p(y), p(ld), B, d, variant, 0, st),
                   "nfx_made_elem_finish")
        return y, ld, work, wld, bnps, counts

    def _generic_seq_train_backward(self, x, gy, gld, direction, work, wld, bnps, counts):
        """Autograd through the d train-mode calls, in reverse: lam = the total dL/dwork (the output
        guard's share of gy, then every later call's input VJP); for call i the conditioner input
        is work with columns >= i zeroed, its MADE is recomputed with its own batch statistics, the
        step adjoint gives (dmu_i, dalpha_i) and dL/dx_i, and the batch-statistics MADE backward
        adds the call's parameter gradients and its input VJP into lam (columns >= i get exact
        zeros through the masks)."""
        L = _lib.lib()
        B, d = x.shape
        variant = self._variant(direction)
        st = _lib.stream_of(x)
        p = _lib.ptr
        lam = torch.empty_like(x)
        _lib.check(L.nfx_made_elem_seq_backward(p(x), None, p(work), None, p(gy), p(gld), p(lam), B, d, variant, 0, st),
                   "nfx_made_elem_seq_backward")
        gx = torch.empty_like(x)
        wi = torch.empty_like(x)
        lins = self.conditioner.linears()
        bns = self.conditioner.batchnorms()
        acc = None
        for i in range(d - 1, -1, -1):
            _lib.check(L.nfx_made_elem_prefix(p(work), p(wi), B, d, i, st), "nfx_made_elem_prefix")
            masks, bnp, acts, prm = self._generic_made_bn(wi, bnps[i])
            dprm = torch.empty_like(prm)
            _lib.check(L.nfx_made_elem_seq_step_backward(p(x), p(prm), p(work), p(wld), p(lam), p(gy), p(gld),
                                                         p(dprm), p(gx), B, d, i, variant, st),
                       "nfx_made_elem_seq_step_backward")
            grads = _generic.made_bn_backward(wi, lins, masks, bns, bnp, acts, dprm, lam if i > 0 else None, True,
                                              counts[i], _dist.allreduce_bn_sums)
            acc = grads if acc is None else [a + g if g is not None else a for a, g in zip(acc, grads)]
        return gx, acc

    def _generic_train_forward(self, x, direction):
        """One train-mode MADE call on x (made_bn_train_call: batch moments, SyncBN merge, running
        update, normalisation), then the parallel element map. Returns (y, ld, bnp, counts)."""
        L = _lib.lib()
        x = x.detach().contiguous()
        B, d = x.shape
        p = _lib.ptr
        prm, bnp, counts = self._generic_made_bn_train(x)
        y = torch.empty_like(x)
        ld = torch.empty(B, device=x.device, dtype=torch.float32)
        _lib.check(L.nfx_made_elem_forward(p(x), p(prm), p(y), p(ld), B, d, self._variant(direction), 0,
                                           _lib.stream_of(x)), "nfx_made_elem_forward")
        return y, ld, bnp, counts

    def _generic_bn_backward(self, x, gz, gld, direction, bnp=None, counts=None):
        """Parallel direction with a BatchNorm MADE (eval: running statistics; train: the call's
        batch statistics bnp / counts from _generic_train_forward)."""
        B, d = x.shape
        train = counts is not None
        masks, bnp, acts, prm = self._generic_made_bn(x, bnp)
        gprm = torch.empty_like(prm)
        gx = torch.empty_like(x)
        _lib.check(_lib.lib().nfx_made_elem_backward(_lib.ptr(x), _lib.ptr(prm), _lib.ptr(gz), _lib.ptr(gld),
                                                     _lib.ptr(gprm), _lib.ptr(gx), B, d, self._variant(direction),
                                                     _lib.stream_of(x)), "nfx_made_elem_backward")
        grads = _generic.made_bn_backward(x, self.conditioner.linears(), masks, self.conditioner.batchnorms(), bnp,
                                          acts, gprm, gx, train, counts, _dist.allreduce_bn_sums)
        return gx, grads

    def _generic_launch(self, x, out, log_det, direction, accumulate):
        variant = self._variant(direction)
        L = _lib.lib()
        B, d = x.shape
        st = _lib.stream_of(x)
        if variant in (_lib.NFX_MAF_INVERSE, _lib.NFX_IAF_FORWARD):
            _, (_, _, _, prm) = self._generic_made(x)
            _lib.check(L.nfx_made_elem_forward(_lib.ptr(x), _lib.ptr(prm), _lib.ptr(out), _lib.ptr(log_det), B, d,
                                               variant, int(bool(accumulate)), st), "nfx_made_elem_forward")
            return
        work, wld = self._generic_seq_work(x, variant)
        _lib.check(L.nfx_made_elem_finish(_lib.ptr(x), _lib.ptr(work), _lib.ptr(wld), _lib.ptr(out), _lib.ptr(log_det),
                                          B, d, variant, int(bool(accumulate)), st), "nfx_made_elem_finish")

    def _generic_seq_work(self, x, variant):
        """A sequential direction as the reference runs it: d MADE calls, one element step each
        (nfx_made_elem_step); returns the raw vector and log-det before the final guards."""
        B, d = x.shape
        L = _lib.lib()
        st = _lib.stream_of(x)
        work = torch.zeros_like(x)
        wld = torch.zeros(B, device=x.device, dtype=torch.float32)
        for i in range(d):
            _, (_, _, _, prm) = self._generic_made(work)
            _lib.check(L.nfx_made_elem_step(_lib.ptr(x), _lib.ptr(prm), _lib.ptr(work), _lib.ptr(wld), B, d, i,
                                            variant, st), "nfx_made_elem_step")
        return work, wld

    def _generic_seq_backward(self, x, gz, gld, variant):
        """A sequential direction beyond the fused backward: autograd through the reference's d
        MADE calls, computed at the finished vector w (params = MADE(w) equal every step's params,
        masks): the total adjoint lam of w solves lam = g_w + VJP_w(dparams(lam)), a strictly
        triangular system, by d - 1 substitution passes (each one MADE input-VJP, 4 GEMMs);
        then the weight gradients for dparams(lam) and dL/dx."""
        B, d = x.shape
        L = _lib.lib()
        st = _lib.stream_of(x)
        p = _lib.ptr
        work, _ = self._generic_seq_work(x, variant)
        lins = self.conditioner.linears()
        bns = self.conditioner.batchnorms()
        if bns:  # eval-mode BatchNorm: a fixed per-feature affine inside the MADE
            masks, bnp, acts, prm = self._generic_made_bn(work)
        else:
            masks, (h1, h2, h3, prm) = self._generic_made(work)
        gw = torch.empty_like(x)
        _lib.check(L.nfx_made_elem_seq_backward(p(x), p(prm), p(work), None, p(gz), p(gld), p(gw), B, d, variant, 0,
                                                st), "nfx_made_elem_seq_backward")
        lam = gw
        dprm = torch.empty_like(prm)
        for _ in range(d - 1):
            _lib.check(L.nfx_made_elem_seq_backward(p(x), p(prm), p(work), p(lam), p(gz), p(gld), p(dprm), B, d,
                                                    variant, 1, st), "nfx_made_elem_seq_backward")
            if bns:
                lam = _generic.made_bn_input_vjp(dprm, lins, masks, bns, bnp, acts, gw.clone())
            else:
                lam = _generic.made_input_vjp(dprm, lins, masks, h1, h2, h3, gw.clone())
        _lib.check(L.nfx_made_elem_seq_backward(p(x), p(prm), p(work), p(lam), p(gz), p(gld), p(dprm), B, d,
                                                variant, 1, st), "nfx_made_elem_seq_backward")
        gx = torch.empty_like(x)
        _lib.check(L.nfx_made_elem_seq_backward(p(x), p(prm), p(work), p(lam), p(gz), p(gld), p(gx), B, d,
                                                variant, 2, st), "nfx_made_elem_seq_backward")
        if bns:
            return gx, _generic.made_bn_backward(work, lins, masks, bns, bnp, acts, dprm, None)
        return gx, _generic.made_backward(work, lins, masks, h1, h2, h3, dprm, None)

    def _generic_backward(self, x, gz, gld, direction):
        """Beyond the fused backward: parallel directions — MADE recompute (GEMMs), the element
        adjoint (nfx_made_elem_backward), then the MADE's backward GEMMs; sequential directions —
        _generic_seq_backward."""
        variant = self._variant(direction)
        if variant in (_lib.NFX_MAF_FORWARD, _lib.NFX_IAF_INVERSE):
            return self._generic_seq_backward(x, gz, gld, variant)
        if self.conditioner.batchnorms():
            return self._generic_bn_backward(x, gz, gld, direction)
        B, d = x.shape
        masks, (h1, h2, h3, prm) = self._generic_made(x)
        gprm = torch.empty_like(prm)
        gx = torch.empty_like(x)
        _lib.check(_lib.lib().nfx_made_elem_backward(_lib.ptr(x), _lib.ptr(prm), _lib.ptr(gz), _lib.ptr(gld),
                                                     _lib.ptr(gprm), _lib.ptr(gx), B, d, variant, _lib.stream_of(x)),
                   "nfx_made_elem_backward")
        grads = _generic.made_backward(x, self.conditioner.linears(), masks, h1, h2, h3, gprm, gx)
        return gx, grads

    def _build_pack(self, device):
        d, H = self.dim, self.conditioner.hidden_dim
        L = _lib.lib()
        packed = torch.empty(L.nfx_made_packed_floats(d, H), device=device, dtype=torch.float32)
        lins = self.conditioner.linears()
        bns = self.conditioner.batchnorms() or ()
        raw, keep = _lib.mlp_raw(lins, bns, masks=[lin.mask for lin in lins])
        # the parallel image (+ degree tables, extents); the sequential directions' image and chunk
        # schedule are added on the first sequential launch of this pack (_seq_packed): a training
        # step re-packs every layer, and the parallel directions never read them
        _lib.check(L.nfx_made_pack_parallel(raw, d, H, _lib.ptr(packed), _lib.stream_of(packed)),
                   "nfx_made_pack_parallel")
        _lib.check(L.nfx_made_pack_backward(raw, d, H, _lib.ptr(packed), _lib.stream_of(packed)),
                   "nfx_made_pack_backward")
        packed._nfx_keep = keep
        packed._nfx_seq = False
        return packed

    def _seq_packed(self, packed, variant):
        """`packed` with the sequential part built (nfx_made_pack_sequential) when `variant` is a
        sequential direction."""
        if variant in (_lib.NFX_MAF_FORWARD, _lib.NFX_IAF_INVERSE) and not getattr(packed, "_nfx_seq", True):
            _lib.check(_lib.lib().nfx_made_pack_sequential(self.dim, self.conditioner.hidden_dim, _lib.ptr(packed),
                                                           _lib.stream_of(packed)), "nfx_made_pack_sequential")
            # under graph capture the build is only recorded: an eager call before the first
            # replay must build it again
            if not torch.cuda.is_current_stream_capturing():
                packed._nfx_seq = True
        return packed

    # -- training: fused backward of every direction (§8(f) item 1) --------------------------
    def _hip_backward_ok(self, x, direction):
        if x.dtype != torch.float32:
            return False
        bns = self.conditioner.batchnorms()
        if bns and (any(bn.training or not bn.affine or bn.running_mean is None for bn in bns)
                    or bns[0].num_features > _generic_bn_max()):
            return False
        return True  # fused backward kernels, or the any-shape path (_generic_backward)

    def _fused_backward_ok(self):
        # parallel directions: made_bwd_kernel (d, H <= 64) / made_bwdw_kernel; sequential
        # directions: made_seq_bwd_kernel
        return (not FORCE_GENERIC and not self.conditioner.batchnorms() and self.dim <= MAX_D
                and self.conditioner.hidden_dim <= MAX_H_BWD)

    def _hip_backward(self, x, gz, gld, direction):
        """dL/dx and the parameter gradients (in self.parameters() order) of one call. Batches
        above nfx_made_backward_max_batch (32-bit factor offsets) run in chunks: dL/dx is per
        sample and every parameter gradient is a sum over samples."""
        x = x.contiguous()
        B, d = x.shape
        H = self.conditioner.hidden_dim
        gz = torch.zeros_like(x) if gz is None else gz.contiguous().float()
        gld = torch.zeros(B, device=x.device) if gld is None else gld.contiguous().float()
        if not self._fused_backward_ok():
            return self._generic_backward(x, gz, gld, direction)
        cap = int(_lib.lib().nfx_made_backward_max_batch(d, H))
        if B > cap:
            gxs, acc = [], None
            for lo in range(0, B, cap):
                gxc, gpc = self._hip_backward_chunk(x[lo:lo + cap], gz[lo:lo + cap], gld[lo:lo + cap], direction)
                gxs.append(gxc)
                acc = gpc if acc is None else [a + g for a, g in zip(acc, gpc)]
            return torch.cat(gxs), acc
        return self._hip_backward_chunk(x, gz, gld, direction)

    def _hip_backward_chunk(self, x, gz, gld, direction):
        B, d = x.shape
        H = self.conditioner.hidden_dim
        packed = self._packed(x.device, self._build_pack)
        L = _lib.lib()
        gx = torch.empty_like(x)
        fac = torch.empty(L.nfx_made_backward_factor_floats(B, d, H), device=x.device, dtype=torch.float32)
        variant = self._variant(direction)
        parallel = variant in (_lib.NFX_MAF_INVERSE, _lib.NFX_IAF_FORWARD)
        ev = BACKWARD_EVENTS
        if ev is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        fn = L.nfx_made_affine_backward if parallel else L.nfx_made_seq_backward
        _lib.check(fn(_lib.ptr(packed), _lib.ptr(x), _lib.ptr(gz), _lib.ptr(gld), _lib.ptr(gx), _lib.ptr(fac),
                      B, d, H, variant, _lib.stream_of(x)),
                   "nfx_made_affine_backward" if parallel else "nfx_made_seq_backward")
        if ev is not None:
            e1.record()
            ev.append(("made_bwd_kernel" if parallel else "made_seq_bwd_kernel", e0, e1))
        return gx, self._weight_grads(fac, B)

    def _weight_grads(self, fac, B):
        """MADE parameter gradients (parameters() order) from the feature-major factors:
        nfx_made_backward_weights (MFMA sample contractions, masks applied)."""
        d, H = self.dim, self.conditioner.hidden_dim
        L = _lib.lib()
        dev = fac.device
        grads = torch.empty(L.nfx_made_param_floats(d, H), device=dev, dtype=torch.float32)
        ws = torch.empty(max(1, L.nfx_made_wgrad_workspace_bytes(B, d, H)), device=dev, dtype=torch.uint8)
        masks = [lin.mask.to(device=dev, dtype=torch.float32).contiguous() for lin in self.conditioner.linears()]
        mp = (ctypes.c_void_p * 4)(*[_lib.ptr(m) for m in masks])
        ev = BACKWARD_EVENTS
        if ev is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        _lib.check(L.nfx_made_backward_weights(_lib.ptr(fac), B, d, H, mp, _lib.ptr(grads), _lib.ptr(ws),
                                               _lib.stream_of(fac)), "nfx_made_backward_weights")
        if ev is not None:
            e1.record()
            ev.append(("made_wgrad_kernel", e0, e1))
        grads._nfx_keep = (masks, ws)
        out, o = [], 0
        for p in self.conditioner.parameters():
            n = p.numel()
            out.append(grads[o:o + n].view_as(p))
            o += n
        return out

    def _hip_launch(self, x, out, log_det, direction, accumulate):
        if not self._fused_family():
            return self._generic_launch(x, out, log_det, direction, accumulate)
        variant = self._variant(direction)
        packed = self._seq_packed(self._packed(x.device, self._build_pack), variant)
        _lib.check(_lib.lib().nfx_made_affine(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), x.shape[0], self.dim,
            self.conditioner.hidden_dim, variant, int(bool(accumulate)),
            _lib.stream_of(x)), "nfx_made_affine")

    def _hip_launch_logprob(self, x, out, log_det, logp, sums, workspace, accumulate):
        if not self._fused_family():
            return False
        variant = self._variant(-1)
        packed = self._seq_packed(self._packed(x.device, self._build_pack), variant)
        rc = _lib.lib().nfx_made_affine_logprob(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), _lib.ptr(logp),
            _lib.ptr(sums), _lib.ptr(workspace), x.shape[0], self.dim,
            self.conditioner.hidden_dim, variant, int(bool(accumulate)), _lib.stream_of(x))
        if rc == _lib.NFX_EUNSUPPORTED:
            return False  # no fused kernel for this (d, H): nothing was launched
        _lib.check(rc, "nfx_made_affine_logprob")
        return True


def made_bn_train_call(conditioner, masks, h):
    """One train-mode call of a BatchNorm MADE (use_batch_norm=True, made.py:93-106) on h: per
    BatchNorm the batch moments (nfx_flowbn_moments, SyncBN-merged), the running update and the
    normalisation (nfx_bn_prepare), ReLU; returns (params, bnp, counts), bnp / counts being what the
    batch-statistics backward (generic.made_bn_backward(train=True)) needs."""
    L = _lib.lib()
    B = h.shape[0]
    dev = h.device
    st = _lib.stream_of(h)
    p = _lib.ptr
    lins = conditioner.linears()
    bns = conditioner.batchnorms()
    bnp, counts = [], []
    for i, bn in enumerate(bns):
        z = _generic.linear_forward(h, lins[i], wmask=masks[i])
        H = z.shape[1]
        ws = torch.empty(max(1, L.nfx_flowbn_workspace_bytes(B, H)), device=dev, dtype=torch.uint8)
        stats = torch.empty(H, 3, device=dev, dtype=torch.float64)
        _lib.check(L.nfx_flowbn_moments(p(z), B, H, p(stats), p(ws), st), "nfx_flowbn_moments")
        _dist.merge_bn_stats(stats)
        t = torch.empty(4, H, device=dev, dtype=torch.float32)
        _lib.check(L.nfx_bn_prepare(p(stats), p(bn.weight.detach()), p(bn.bias.detach()), p(bn.running_mean),
                                    p(bn.running_var), float(bn.eps), float(bn.momentum), 1, H, p(t[0]), p(t[1]),
                                    p(t[2]), p(t[3]), st), "nfx_bn_prepare")
        torch.autograd.graph.increment_version(bn.running_mean)
        torch.autograd.graph.increment_version(bn.running_var)
        h = _generic.bn_apply_relu(z, t)
        bnp.append(t)
        counts.append(stats)  # stats[0, 0] = the global sample count
    torch._foreach_add_([bn.num_batches_tracked for bn in bns], 1)
    return _generic.linear_forward(h, lins[3], wmask=masks[3]), bnp, counts


def made_bn_eval_params(conditioner, device):
    """Per MADE BatchNorm [mean, invstd, scale, shift] from the running statistics (eval mode)."""
    L = _lib.lib()
    out = []
    for bn in conditioner.batchnorms():
        H = bn.num_features
        t = torch.empty(4, H, device=device, dtype=torch.float32)
        _lib.check(L.nfx_bn_prepare(None, _lib.ptr(bn.weight.detach()), _lib.ptr(bn.bias.detach()),
                                    _lib.ptr(bn.running_mean), _lib.ptr(bn.running_var), float(bn.eps), 0.0, 0,
                                    H, _lib.ptr(t[0]), _lib.ptr(t[1]), _lib.ptr(t[2]), _lib.ptr(t[3]),
                                    _lib.stream_of(t)), "nfx_bn_prepare")
        out.append(t)
    return out


def bn_train_supported(conditioner, x, dim):
    """Train-mode BatchNorm MADE on the HIP path: every BatchNorm affine, tracking running
    statistics with a momentum, <= 1024 features; fp32 ROCm rows, B >= 2."""
    bns = conditioner.batchnorms()
    if not bns or not all(bn.training for bn in bns) or x.device.type != "cuda" or x.dtype != torch.float32:
        return False
    if any(not bn.affine or not bn.track_running_stats or bn.momentum is None or bn.running_mean is None
           or bn.num_features > _generic_bn_max() for bn in bns):
        return False
    return x.dim() == 2 and x.shape[1] == dim and x.shape[0] >= 2


def _generic_bn_max():
    return 1024  # nfx_flowbn_moments: <= 1024 features


class _MadeTrainFunction(torch.autograd.Function):
    """MAF.inverse / IAF.forward with train-mode BatchNorm in the MADE: batch statistics and
    running update in the forward, the batch-statistics BatchNorm backward (SyncBN sums) after."""

    @staticmethod
    def forward(ctx, layer, direction, x, *params):
        y, ld, bnp, counts = layer._generic_train_forward(x, direction)
        ctx.layer, ctx.direction, ctx.bnp, ctx.counts = layer, direction, bnp, counts
        ctx.save_for_backward(x)
        return y, ld

    @staticmethod
    def backward(ctx, gy, gld):
        (x,) = ctx.saved_tensors
        x = x.detach().contiguous()
        gy = torch.zeros_like(x) if gy is None else gy.contiguous().float()
        gld = torch.zeros(x.shape[0], device=x.device) if gld is None else gld.contiguous().float()
        gx, grads = ctx.layer._generic_bn_backward(x, gy, gld, ctx.direction, ctx.bnp, ctx.counts)
        STATS["hip"] += 1
        params = list(ctx.layer.parameters())
        return (None, None, gx, *[g if p.requires_grad else None for p, g in zip(params, grads)])


class _MadeSeqTrainFunction(torch.autograd.Function):
    """MAF.forward / IAF.inverse with train-mode BatchNorm in the MADE: the reference's d calls,
    each with its own batch statistics and running update; backward call by call
    (_generic_seq_train_backward)."""

    @staticmethod
    def forward(ctx, layer, direction, x, *params):
        y, ld, work, wld, bnps, counts = layer._generic_seq_train_forward(x, direction)
        ctx.layer, ctx.direction, ctx.bnps, ctx.counts = layer, direction, bnps, counts
        ctx.save_for_backward(x, work, wld)
        return y, ld

    @staticmethod
    def backward(ctx, gy, gld):
        x, work, wld = ctx.saved_tensors
        x = x.detach().contiguous()
        gy = torch.zeros_like(x) if gy is None else gy.contiguous().float()
        gld = torch.zeros(x.shape[0], device=x.device) if gld is None else gld.contiguous().float()
        gx, grads = ctx.layer._generic_seq_train_backward(x, gy, gld, ctx.direction, work, wld, ctx.bnps, ctx.counts)
        STATS["hip"] += 1
        params = list(ctx.layer.parameters())
        return (None, None, gx, *[g if p.requires_grad else None for p, g in zip(params, grads)])


class MaskedAutoregressiveFlow(_MadeAffineFlow):
    def _variant(self, direction):
        return _lib.NFX_MAF_INVERSE if direction < 0 else _lib.NFX_MAF_FORWARD

    def _torch_call(self, x, direction):
        if direction < 0:  # masked_autoregressive_flow.py:18-44 (parallel)
            mu, alpha = self.conditioner(x).chunk(2, dim=1)
            alpha = torch.clamp(alpha, min=-3, max=3)
            z = (x - mu) * torch.exp(torch.clamp(-alpha, min=-5, max=5))
            ld = -torch.sum(alpha, dim=1)
            z = torch.where(torch.isnan(z) | torch.isinf(z), torch.zeros_like(z), z)
        else:  # masked_autoregressive_flow.py:46-78 (sequential)
            B = x.size(0)
            z = torch.zeros(B, self.dim, device=x.device, dtype=x.dtype)
            ld = torch.zeros(B, device=x.device, dtype=x.dtype)
            for i in range(self.dim):
                mu, alpha = self.conditioner(z).chunk(2, dim=1)
                alpha = torch.clamp(alpha, min=-3, max=3)
                scale = torch.exp(torch.clamp(alpha[:, i], min=-5, max=5))
                z_new = z.clone()
                z_new[:, i] = x[:, i] * scale + mu[:, i]
                z = z_new
                ld += alpha[:, i]
            z = torch.where(torch.isnan(z) | torch.isinf(z), torch.zeros_like(z), z)
        ld = torch.where(torch.isnan(ld) | torch.isinf(ld), torch.zeros_like(ld), ld)
        return z, torch.clamp(ld, min=-100, max=100)


class InverseAutoregressiveFlow(_MadeAffineFlow):
    def __init__(self, dim, hidden_dim=64, use_batch_norm=False):
        super().__init__(dim, hidden_dim, use_batch_norm)
        self._initialize_conditioner()

    def _initialize_conditioner(self):
        # inverse_autoregressive_flow.py:21-28
        final = self.conditioner.net[-1]
        if hasattr(final, "weight"):
            torch.nn.init.normal_(final.weight, mean=0.0, std=0.01)
        if hasattr(final, "bias"):
            torch.nn.init.zeros_(final.bias)

    def _variant(self, direction):
        return _lib.NFX_IAF_FORWARD if direction > 0 else _lib.NFX_IAF_INVERSE

    def _torch_call(self, x, direction):
        if direction > 0:  # inverse_autoregressive_flow.py:30-63 (parallel)
            mu, alpha = self.conditioner(x).chunk(2, dim=1)
            alpha = torch.clamp(alpha, min=-2, max=2)
            mu = torch.clamp(mu, min=-10, max=10)
            y = x * torch.exp(torch.clamp(alpha, min=-3, max=3)) + mu
            ld = torch.sum(alpha, dim=1)
        else:  # inverse_autoregressive_flow.py:65-103 (sequential)
            B = x.size(0)
            y = torch.zeros(B, self.dim, device=x.device, dtype=x.dtype)
            ld = torch.zeros(B, device=x.device, dtype=x.dtype)
            for i in range(self.dim):
                mu, alpha = self.conditioner(y).chunk(2, dim=1)
                alpha = torch.clamp(alpha, min=-2, max=2)
                mu = torch.clamp(mu, min=-10, max=10)
                scale = torch.exp(torch.clamp(-alpha[:, i], min=-3, max=3))
                y_new = y.clone()
                y_new[:, i] = (x[:, i] - mu[:, i]) * scale
                y = y_new
                ld -= alpha[:, i]
        y = torch.where(torch.isnan(y) | torch.isinf(y), x, y)
        ld = torch.where(torch.isnan(ld) | torch.isinf(ld), torch.zeros_like(ld), ld)
        return y, torch.clamp(ld, min=-50, max=50)
