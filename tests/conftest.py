import json
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "normalizing-flows-study_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libnfx.so")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def state_dict_from(arrs, prefix, module):
    """Build a state dict for `module` from golden arrays stored under `prefix`."""
    sd = {}
    for k, v in module.state_dict().items():
        key = prefix + k
        if key in arrs:
            sd[k] = torch.from_numpy(np.array(arrs[key]))
        else:
            sd[k] = v  # num_batches_tracked
    return sd


def oracle_sd(arrs, prefix=""):
    """Golden arrays -> {key: tensor} for the oracle (keys without `prefix`)."""
    return {k[len(prefix):]: torch.from_numpy(np.array(v)) for k, v in arrs.items() if k.startswith(prefix)}


@pytest.fixture(scope="session")
def cuda_device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def assert_fp32_parity(gpu, cpu32, ref64, slack=1e-5, floor=5e-4, what=""):
    """Error model for ill-conditioned fp32 math (RQ spline chains).

    The reference's own fp32 result (cpu32) is not exact: for some inputs the softmax/exp/log
    chain and the citardauq root lose up to ~1e-3 in log-det against the float64 evaluation of
    the same math (ref64 = the oracle run in double). A kernel rounding differently lands on a
    different but equally-conditioned value, so the check is statistical over the tensor:
      per element  |gpu - ref64| <= 8 |cpu32 - ref64| + slack (1 + |ref64|)
      mean         mean|gpu - ref64| <= 1.5 mean|cpu32 - ref64| + 1e-7
      max          max|gpu - ref64|  <= 4 max|cpu32 - ref64| + slack
      floor        every element within floor (1 + |ref64|) of the float64 value
    i.e. the kernel is as accurate as the reference's fp32, never systematically worse. The
    per-element 8x bound is waived below `floor`: near a knot with steep end derivatives the
    log-det has a condition number ~100 per ulp of the knot position (measured: a 1-ulp
    softmax/exp difference moves ld by 1e-4 while the reference happens to land within 1e-6).
    NaN patterns must agree with the reference."""
    g = np.asarray(gpu, np.float64).ravel()
    c = np.asarray(cpu32, np.float64).ravel()
    r = np.asarray(ref64, np.float64).ravel()
    assert np.array_equal(np.isnan(g), np.isnan(c)), f"{what}: NaN pattern differs from the reference"
    ok = ~np.isnan(c) & ~np.isnan(r)
    g, c, r = g[ok], c[ok], r[ok]
    if g.size == 0:
        return
    eg, ec = np.abs(g - r), np.abs(c - r)
    bound = np.maximum(8 * ec + slack * (1 + np.abs(r)), floor * (1 + np.abs(r)))
    bad = eg > bound
    assert not bad.any(), (f"{what}: {bad.sum()} elements exceed the fp32 error model; worst "
                           f"{eg[bad].max():.3g} (ref err {ec[bad][eg[bad].argmax()]:.3g})")
    assert eg.mean() <= 1.5 * ec.mean() + 1e-7, f"{what}: mean err {eg.mean():.3g} vs reference {ec.mean():.3g}"
    assert eg.max() <= 4 * ec.max() + slack, f"{what}: max err {eg.max():.3g} vs reference {ec.max():.3g}"
