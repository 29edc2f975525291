"""The C-ABI library (libnfx.so) loads without a GPU and exports every symbol include/nfx.h
declares; host-only entry points (sizes, version, argument validation) behave."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

import nfs_amd
from nfs_amd import _lib

HEADER = os.path.join(ROOT, "include", "nfx.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(nfx_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 14
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(_lib.EXPORTED_SYMBOLS) == syms


def test_abi_version_and_sizes():
    L = _lib.lib()
    assert L.nfx_abi_version() == 3
    assert L.nfx_affine_packed_floats(2, 64) > 0
    assert L.nfx_affine_packed_floats(2, 64) % 4 == 0
    assert L.nfx_spline_packed_floats(2, 64, 8) % 4 == 0
    assert L.nfx_made_packed_floats(63, 64) % 4 == 0
    assert L.nfx_affine_packed_floats(0, 64) == 0
    assert L.nfx_gauss_workspace_bytes(1 << 20) >= 8


def test_invalid_arguments_fail_before_any_launch():
    """Argument validation happens on the host: no device pointer is touched."""
    L = _lib.lib()
    rc = L.nfx_affine_coupling(None, None, None, None, 16, 2, 64, 0, 0, None)
    assert rc == -1 and b"direction" in L.nfx_last_error()
    rc = L.nfx_affine_coupling(None, None, None, None, 16, 9, 64, 1, 0, None)
    assert rc in (-1, -2)
    rc = L.nfx_spline_coupling(None, None, None, None, 16, 2, 64, 12, 5.0, 1e-3, 1e-3, 1e-3, 0, 0.0, 0.0, 1, 0, None)
    assert rc == -2 and b"K=12" in L.nfx_last_error()
    rc = L.nfx_made_affine(None, None, None, None, 16, 63, 64, 7, 0, None)
    assert rc == -1
    rc = L.nfx_rqs_unit(None, None, None, None, None, None, 16, 40, 1e-3, 1e-3, 1e-3, 0, None)
    assert rc == -2
    # B == 0 is a valid no-op
    assert L.nfx_affine_coupling(None, None, None, None, 0, 2, 64, 1, 0, None) == 0
    # between-layer BatchNorm
    rc = L.nfx_flowbn_apply(None, None, None, 1, 1, 1, 1, 1e-5, 16, 2, 0, None)
    assert rc == -1 and b"direction" in L.nfx_last_error()
    rc = L.nfx_flowbn_apply(None, None, None, 1, 1, 1, 1, 1e-5, 16, 2000, 1, None)
    assert rc == -2
    assert L.nfx_flowbn_apply(None, None, None, 1, 1, 1, 1, 1e-5, 0, 2, 1, None) == 0
    assert L.nfx_flowbn_workspace_bytes(1 << 20, 63) >= 8 * 63 * 2


def test_product_raises_without_library(monkeypatch, tmp_path):
    """No silent eager fallback: a missing libnfx.so is a loud error."""
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.NfxLibraryError):
        _lib.load(str(tmp_path / "missing.so"))


def test_affine_kernel_policy_roundtrip():
    """Host-only entry point: set/read the affine kernel policy (no GPU call)."""
    f = _lib.load().nfx_affine_kernel_policy
    prev = f(-1)
    assert prev in (_lib.NFX_AFFINE_AUTO, _lib.NFX_AFFINE_STREAMING, _lib.NFX_AFFINE_SMALL)
    assert f(_lib.NFX_AFFINE_SMALL) == prev
    assert f(-1) == _lib.NFX_AFFINE_SMALL
    assert f(7) == _lib.NFX_EINVAL
    assert f(prev) == _lib.NFX_AFFINE_SMALL
    assert f(-1) == prev


def test_any_shape_entry_points_validate_on_the_host():
    """The any-shape path (csrc/nfx_generic.hip): shape / variant / mode checks and the B == 0
    no-ops return before any device call; workspace sizes are host arithmetic."""
    L = _lib.lib()
    EINVAL, EUNSUP = _lib.NFX_EINVAL, _lib.NFX_EUNSUPPORTED
    assert L.nfx_linear_forward(None, None, None, None, None, None, None, None, -1, 4, 4, 0, None) == EINVAL
    assert L.nfx_linear_forward(None, None, None, None, None, None, None, None, 0, 4, 4, 0, None) == 0
    assert L.nfx_linear_forward(None, None, None, None, None, None, None, None, 8, 4, 4, 0, None) == EINVAL
    ps = ctypes.c_void_p(1)
    assert L.nfx_linear_forward(ps, ps, None, None, None, ps, None, ps, 8, 4, 4, 0, None) == EINVAL
    assert b"post_scale" in L.nfx_last_error()
    assert L.nfx_linear_backward_data(None, None, None, None, None, None, 8, 0, 4, 0, None) == EINVAL
    assert L.nfx_linear_backward_weight(None, None, None, None, None, None, 8, 4, 4, None, None) == EINVAL
    assert L.nfx_linear_workspace_bytes(1 << 20, 128, 128) >= 128 * 128 * 4
    assert L.nfx_linear_workspace_bytes(0, 128, 128) == 0
    assert L.nfx_spline_elem_forward(None, None, None, None, None, 8, 2, 12, 5.0, 1e-3, 1e-3, 1e-3, 1, 0,
                                     None) == EUNSUP
    assert L.nfx_spline_elem_backward(None, None, None, None, None, None, None, 8, 2, 8, 5.0, 1e-3, 1e-3, 1e-3, 0,
                                      None) == EINVAL
    # the MADE element map: parallel variants only; a sequential step needs a sequential variant
    assert L.nfx_made_elem_forward(None, None, None, None, 8, 4, _lib.NFX_MAF_FORWARD, 0, None) == EINVAL
    assert L.nfx_made_elem_step(None, None, None, None, 8, 4, 0, _lib.NFX_MAF_INVERSE, None) == EINVAL
    assert L.nfx_made_elem_step(None, None, None, None, 8, 4, 4, _lib.NFX_MAF_FORWARD, None) == EINVAL
    assert L.nfx_made_elem_seq_backward(None, None, None, None, None, None, None, 8, 4, _lib.NFX_IAF_INVERSE, 3,
                                        None) == EINVAL
    assert L.nfx_made_elem_backward(None, None, None, None, None, None, 0, 4, _lib.NFX_IAF_FORWARD, None) == 0
    assert L.nfx_affine_elem_forward(None, None, None, None, None, None, 8, 4, 0, 0, None) == EINVAL
    assert L.nfx_arqs_step(None, None, None, None, None, None, None, None, 8, 4, 1, 0, 1, 0, 1e-3, 1e-3, 1e-3,
                           None) == EUNSUP
    assert L.nfx_arqs_step(None, None, None, None, None, None, None, None, 8, 4, 8, 0, 1, 5, 1e-3, 1e-3, 1e-3,
                           None) == EINVAL
    assert L.nfx_bn_prepare(None, None, None, None, None, 1e-5, 0.1, 0, 0, None, None, None, None, None) == EINVAL
    assert L.nfx_bn_workspace_bytes(1 << 20, 64) >= 2 * 64 * 8
