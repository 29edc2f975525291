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
