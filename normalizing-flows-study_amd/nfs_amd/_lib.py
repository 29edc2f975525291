"""ctypes binding of libnfx.so (the C-ABI declared in include/nfx.h).

The product path fails loudly when the library is missing: every HIP entry point goes through
`lib()`, which raises NfxLibraryError instead of silently falling back to eager PyTorch.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NFX_LIB", os.path.join(_HERE, "libnfx.so"))

NFX_OK = 0
NFX_EINVAL = -1
NFX_EUNSUPPORTED = -2
NFX_ELAUNCH = -3
NFX_FORWARD = 1
NFX_INVERSE = -1
NFX_MAF_INVERSE = 0
NFX_IAF_FORWARD = 1
NFX_MAF_FORWARD = 2
NFX_IAF_INVERSE = 3
NFX_AFFINE_AUTO = 0
NFX_AFFINE_STREAMING = 1
NFX_AFFINE_SMALL = 2
NFX_MADE_SEQ_AUTO = 0
NFX_MADE_SEQ_SEGMENT = 1
NFX_MADE_SEQ_WAVE = 2
NFX_MADE_SEQ_PUSH = 3

# Every symbol include/nfx.h declares (tests check the built library exports all of them).
EXPORTED_SYMBOLS = (
    "nfx_abi_version", "nfx_last_error", "nfx_last_kernel", "nfx_debug_fill_lds",
    "nfx_affine_packed_floats", "nfx_affine_pack", "nfx_affine_coupling", "nfx_affine_coupling_logprob",
    "nfx_affine_kernel_policy", "nfx_affine_chain", "nfx_affine_chain_logprob", "nfx_affine_chain_supported",
    "nfx_affine_chain_sample",
    "nfx_spline_packed_floats", "nfx_spline_pack", "nfx_spline_coupling", "nfx_spline_coupling_logprob",
    "nfx_spline_chain_supported", "nfx_spline_chain", "nfx_spline_chain_logprob", "nfx_spline_chain_sample",
    "nfx_rqs_unit", "nfx_rqs_unit_backward",
    "nfx_arqs_packed_floats", "nfx_arqs_pack", "nfx_arqs",
    "nfx_made_packed_floats", "nfx_made_pack", "nfx_made_pack_parallel", "nfx_made_pack_sequential", "nfx_made_affine", "nfx_made_affine_logprob", "nfx_made_seq_policy",
    "nfx_made_pack_backward", "nfx_made_backward_factor_floats", "nfx_made_backward_max_batch",
    "nfx_made_affine_backward",
    "nfx_made_seq_backward", "nfx_made_factor_pitch", "nfx_made_param_floats", "nfx_made_wgrad_workspace_bytes", "nfx_made_backward_weights",
    "nfx_affine_train_pack_floats", "nfx_affine_train_stats_doubles", "nfx_affine_train_grad_doubles",
    "nfx_affine_train_param_floats", "nfx_affine_train_workspace_bytes", "nfx_affine_train_pack",
    "nfx_affine_train_stats", "nfx_affine_train_update_running", "nfx_affine_train_backward",
    "nfx_affine_train_assemble", "nfx_affine_eval_stats", "nfx_affine_train_keep_floats",
    "nfx_affine_train_stats_keep", "nfx_affine_train_backward_keep", "nfx_affine_train_output", "nfx_affine_train_update_running_counted",
    "nfx_spline_backward_packed_floats", "nfx_spline_backward_param_floats",
    "nfx_spline_backward_workspace_bytes", "nfx_spline_pack_backward", "nfx_spline_coupling_backward",
    "nfx_gauss_workspace_bytes", "nfx_gauss_workspace_init", "nfx_gauss_logprob", "nfx_gauss_logprob_backward",
    "nfx_flowbn_workspace_bytes", "nfx_flowbn_apply", "nfx_flowbn_moments", "nfx_flowbn_update_running",
    "nfx_flowbn_backward",
    "nfx_linear_forward", "nfx_linear_backward_data", "nfx_linear_workspace_bytes", "nfx_linear_backward_weight",
    "nfx_spline_elem_forward", "nfx_spline_elem_backward", "nfx_spline_elem_forward_bounded",
    "nfx_spline_elem_backward_bounded", "nfx_spline_rescale", "nfx_arqs_bounds",
    "nfx_made_elem_forward", "nfx_made_elem_step", "nfx_made_elem_finish", "nfx_made_elem_backward",
    "nfx_made_elem_seq_backward", "nfx_made_elem_seq_step_backward", "nfx_made_elem_prefix",
    "nfx_affine_elem_forward", "nfx_affine_elem_backward", "nfx_bn_prepare", "nfx_bn_apply_relu",
    "nfx_bn_workspace_bytes", "nfx_bn_backward_sums", "nfx_bn_backward_apply", "nfx_arqs_step",
)


class NfxLibraryError(RuntimeError):
    pass


class NfxError(RuntimeError):
    pass


class NfxMlpRaw(ctypes.Structure):
    """Mirror of `NfxMlpRaw` in include/nfx.h (device pointers of one conditioner MLP)."""
    _fields_ = [
        ("w", ctypes.c_void_p * 4),
        ("b", ctypes.c_void_p * 4),
        ("mask", ctypes.c_void_p * 4),
        ("bn_w", ctypes.c_void_p * 3),
        ("bn_b", ctypes.c_void_p * 3),
        ("bn_rm", ctypes.c_void_p * 3),
        ("bn_rv", ctypes.c_void_p * 3),
        ("bn_eps", ctypes.c_float),
        ("n_layers", ctypes.c_int),
    ]


_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t

_SIGNATURES = {
    "nfx_abi_version": (_int, []),
    "nfx_last_error": (ctypes.c_char_p, []),
    "nfx_last_kernel": (ctypes.c_char_p, []),
    "nfx_debug_fill_lds": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_void_p]),
    "nfx_affine_packed_floats": (_sz, [_int, _int]),
    "nfx_affine_pack": (_int, [ctypes.POINTER(NfxMlpRaw), ctypes.POINTER(NfxMlpRaw), _vp, _int, _int, _vp, _vp]),
    "nfx_affine_coupling": (_int, [_vp, _vp, _vp, _vp, _i64, _int, _int, _int, _int, _vp]),
    "nfx_affine_coupling_logprob": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_affine_kernel_policy": (_int, [_int]),
    "nfx_linear_forward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_linear_backward_data": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_linear_workspace_bytes": (_sz, [_i64, _int, _int]),
    "nfx_linear_backward_weight": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _vp, _vp]),
    "nfx_made_elem_forward": (_int, [_vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_made_elem_step": (_int, [_vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_made_elem_finish": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_made_elem_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _vp]),
    "nfx_made_elem_seq_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_made_elem_seq_step_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int,
                                               _vp]),
    "nfx_made_elem_prefix": (_int, [_vp, _vp, _i64, _int, _int, _vp]),
    "nfx_affine_elem_forward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_affine_elem_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _vp]),
    "nfx_bn_prepare": (_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double, _int, _int, _vp, _vp, _vp,
                              _vp, _vp]),
    "nfx_bn_apply_relu": (_int, [_vp, _vp, _vp, _vp, _i64, _int, _vp]),
    "nfx_arqs_step": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _int, _int, _f, _f, _f,
                             _vp]),
    "nfx_bn_workspace_bytes": (_sz, [_i64, _int]),
    "nfx_bn_backward_sums": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _int, _vp, _vp]),
    "nfx_bn_backward_apply": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _int, _vp, _i64, _int, _vp]),
    "nfx_spline_elem_forward": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _f, _f, _f, _f, _int, _int, _vp]),
    "nfx_spline_elem_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _f, _f, _f, _f, _int,
                                        _vp]),
    "nfx_spline_elem_forward_bounded": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _f, _f, _f, _f, _int,
                                               _int, _vp]),
    "nfx_spline_elem_backward_bounded": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _f, _f, _f,
                                                _f, _int, _vp]),
    "nfx_spline_rescale": (_int, [_vp, _vp, _vp, _i64, _int, _f, _vp]),
    "nfx_arqs_bounds": (_int, [_vp, _vp, _vp, _i64, _int, _int, _vp]),
    "nfx_affine_chain_supported": (_int, [_i64, _int, _int]),
    "nfx_affine_chain": (_int, [ctypes.POINTER(_vp), _int, _vp, _vp, _vp, _i64, _int, _int, _int, _int, _vp]),
    "nfx_affine_chain_logprob": (_int, [ctypes.POINTER(_vp), _int, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int,
                                        _int, _vp]),
    "nfx_affine_chain_sample": (_int, [ctypes.POINTER(_vp), _int, ctypes.c_uint64, _vp, _vp, _vp, _vp, _i64, _int, _int,
                                       _vp]),
    "nfx_arqs_packed_floats": (_sz, [_int, _int, _int]),
    "nfx_arqs_pack": (_int, [ctypes.POINTER(NfxMlpRaw), _int, _int, _int, _vp, _vp]),
    "nfx_arqs": (_int, [_vp, _vp, _vp, _vp, _i64, _int, _int, _int, _f, _f, _f, _int, ctypes.c_double,
                        ctypes.c_double, _int, _int, _vp]),
    "nfx_spline_packed_floats": (_sz, [_int, _int, _int]),
    "nfx_spline_pack": (_int, [ctypes.POINTER(NfxMlpRaw), _vp, _int, _int, _int, _vp, _vp]),
    "nfx_spline_coupling": (_int, [_vp, _vp, _vp, _vp, _i64, _int, _int, _int, _f, _f, _f, _f,
                                   _int, _f, _f, _int, _int, _vp]),
    "nfx_spline_coupling_logprob": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _f, _f,
                                           _f, _f, _int, _f, _f, _int, _vp]),
    "nfx_spline_chain_supported": (_int, [_i64, _int, _int, _int]),
    "nfx_spline_chain": (_int, [ctypes.POINTER(_vp), _int, _vp, _vp, _vp, _i64, _int, _int, _int, _f, _f, _f, _f,
                                _int, _int, _vp]),
    "nfx_spline_chain_logprob": (_int, [ctypes.POINTER(_vp), _int, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int,
                                        _int, _f, _f, _f, _f, _int, _vp]),
    "nfx_spline_chain_sample": (_int, [ctypes.POINTER(_vp), _int, ctypes.c_uint64, _vp, _vp, _vp, _vp, _i64, _int, _int,
                                       _int, _f, _f, _f, _f, _vp]),
    "nfx_rqs_unit": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _f, _f, _f, _int, _vp]),
    "nfx_rqs_unit_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _f, _f, _f, _int,
                                     _vp]),
    "nfx_made_packed_floats": (_sz, [_int, _int]),
    "nfx_made_pack": (_int, [ctypes.POINTER(NfxMlpRaw), _int, _int, _vp, _vp]),
    "nfx_made_pack_parallel": (_int, [ctypes.POINTER(NfxMlpRaw), _int, _int, _vp, _vp]),
    "nfx_made_pack_sequential": (_int, [_int, _int, _vp, _vp]),
    "nfx_made_seq_policy": (_int, [_int]),
    "nfx_made_affine": (_int, [_vp, _vp, _vp, _vp, _i64, _int, _int, _int, _int, _vp]),
    "nfx_made_affine_logprob": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _int, _vp]),
    "nfx_made_pack_backward": (_int, [ctypes.POINTER(NfxMlpRaw), _int, _int, _vp, _vp]),
    "nfx_made_backward_factor_floats": (_sz, [_i64, _int, _int]),
    "nfx_made_backward_max_batch": (_i64, [_int, _int]),
    "nfx_made_affine_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_made_seq_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_made_factor_pitch": (_i64, [_i64]),
    "nfx_made_param_floats": (_sz, [_int, _int]),
    "nfx_made_wgrad_workspace_bytes": (_sz, [_i64, _int, _int]),
    "nfx_made_backward_weights": (_int, [_vp, _i64, _int, _int, ctypes.POINTER(_vp), _vp, _vp, _vp]),
    "nfx_affine_train_pack_floats": (_sz, [_int, _int]),
    "nfx_affine_train_stats_doubles": (_sz, [_int]),
    "nfx_affine_train_grad_doubles": (_sz, [_int, _int]),
    "nfx_affine_train_param_floats": (_sz, [_int, _int]),
    "nfx_affine_train_workspace_bytes": (_sz, [_i64, _int, _int]),
    "nfx_affine_train_pack": (_int, [ctypes.POINTER(NfxMlpRaw), ctypes.POINTER(NfxMlpRaw), _vp, _vp, _vp, _int,
                                     _int, _vp, _vp, _vp]),
    "nfx_affine_train_stats": (_int, [_vp, _vp, _i64, _int, _int, _int, _vp, _vp, _vp]),
    "nfx_affine_train_update_running": (_int, [_vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _int,
                                               ctypes.c_double, _vp]),
    "nfx_affine_train_update_running_counted": (_int, [_vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                                       ctypes.POINTER(_vp), _int, ctypes.c_double, _vp]),
    "nfx_affine_train_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _int, _vp, _vp, _vp,
                                         _vp]),
    "nfx_affine_train_assemble": (_int, [_vp, _vp, _vp, _int, _int, _f, _vp, _vp]),
    "nfx_affine_train_keep_floats": (_sz, [_i64, _int, _int]),
    "nfx_affine_train_stats_keep": (_int, [_vp, _vp, _i64, _int, _int, _int, _vp, _vp, _vp, _vp]),
    "nfx_affine_train_backward_keep": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _int, _vp, _vp,
                                              _vp, _vp, _vp]),
    "nfx_affine_train_output": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _vp]),
    "nfx_affine_eval_stats": (_int, [ctypes.POINTER(_vp), ctypes.POINTER(_vp), _int, _vp, _vp, _vp]),
    "nfx_spline_backward_packed_floats": (_sz, [_int, _int, _int]),
    "nfx_spline_backward_param_floats": (_sz, [_int, _int, _int]),
    "nfx_spline_backward_workspace_bytes": (_sz, [_i64, _int, _int, _int]),
    "nfx_spline_pack_backward": (_int, [ctypes.POINTER(NfxMlpRaw), _vp, _int, _int, _int, _vp, _vp]),
    "nfx_spline_coupling_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _int, _int,
                                            _f, _f, _f, _f, _int, _vp]),
    "nfx_gauss_workspace_bytes": (_sz, [_i64]),
    "nfx_gauss_workspace_init": (_int, [_vp, _vp]),
    "nfx_gauss_logprob": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _int, _vp]),
    "nfx_gauss_logprob_backward": (_int, [_vp, _vp, _vp, _vp, _i64, _int, _vp]),
    "nfx_flowbn_workspace_bytes": (_sz, [_i64, _int]),
    "nfx_flowbn_apply": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _i64, _int, _int, _vp]),
    "nfx_flowbn_moments": (_int, [_vp, _i64, _int, _vp, _vp, _vp]),
    "nfx_flowbn_update_running": (_int, [_vp, _vp, _vp, ctypes.c_double, _int, _vp]),
    "nfx_flowbn_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp, _i64, _int, _int,
                                   _vp, _vp]),
}

_lock = threading.Lock()
_lib = None


def load(path=LIB_PATH):
    """Load libnfx.so without touching the GPU (safe on CPU-only hosts)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NfxLibraryError(
                f"libnfx.so not found at {path}: build it with "
                f"`python normalizing-flows-study_amd/build.py` (or __graft_entry__.build()). "
                f"The HIP path has no eager fallback.")
        l = ctypes.CDLL(path)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(l, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = l
        return l


def lib():
    l = _lib
    return l if l is not None else load()


def available():
    try:
        load()
        return True
    except NfxLibraryError:
        return False


def check(rc, what):
    if rc != NFX_OK:
        msg = lib().nfx_last_error().decode(errors="replace")
        raise NfxError(f"{what} failed (rc={rc}): {msg}")


def ptr(t):
    """Device address of a tensor as a plain int (ctypes c_void_p arguments accept ints)."""
    return None if t is None else t.data_ptr()


try:
    _raw_stream = torch._C._cuda_getCurrentRawStream
except AttributeError:  # pragma: no cover - older torch
    _raw_stream = None


def stream_of(t):
    """hipStream_t of torch's current stream on t's device (the stream kernels are enqueued on)."""
    if _raw_stream is not None and t.device.type == "cuda":
        return _raw_stream(t.device.index if t.device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(t.device).cuda_stream


def mlp_raw(linears, batchnorms=(), masks=None):
    """Build an NfxMlpRaw from nn.Linear modules (+ optional BatchNorm1d after hidden layers).

    Returns (struct, keepalive) — keepalive holds the contiguous tensors the pointers refer to.
    """
    raw = NfxMlpRaw()
    keep = []

    def p(t):
        t = t.detach().contiguous().float()
        keep.append(t)
        return t.data_ptr()

    raw.n_layers = len(linears)
    for i, lin in enumerate(linears):
        raw.w[i] = p(lin.weight)
        raw.b[i] = p(lin.bias) if lin.bias is not None else None
        if masks is not None and masks[i] is not None:
            raw.mask[i] = p(masks[i])
    eps = 1e-5
    for i, bn in enumerate(batchnorms):
        if bn is None:
            continue
        raw.bn_w[i] = p(bn.weight) if bn.weight is not None else p(torch.ones_like(bn.running_var))
        raw.bn_b[i] = p(bn.bias) if bn.bias is not None else p(torch.zeros_like(bn.running_var))
        raw.bn_rm[i] = p(bn.running_mean)
        raw.bn_rv[i] = p(bn.running_var)
        eps = bn.eps
    raw.bn_eps = eps
    return raw, keep


def last_kernel():
    """Name of the last kernel this thread launched through libnfx (profiling aid)."""
    return lib().nfx_last_kernel().decode()
