"""CPU checks of bench.py's bookkeeping: the executed-flop count DESIGN.md quotes for cfg4, the
libnfx.so digest that ties a reconciled rocprof profile to the build it measured, and the
reconcile tool's hot-kernel map covering every config the profiles are taken for."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_made_executed_flops_cfg4():
    import bench
    # d = 63, H = 64: the tile kernel's k-loops stop at the last nonzero 32x32 block
    assert bench.made_executed_flop_per_sample(63, 64) == 30720.0


def test_lib_digest_is_stable():
    import bench
    a, b = bench.lib_digest(), bench.lib_digest()
    assert a == b and re.fullmatch(r"[0-9a-f]{16}", a)


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg4", "cfg5f", "cfg5i", "cfg4t", "cfg2t", "cfg3t"])
def test_reconcile_knows_config(cfg):
    import reconcile_profile
    assert cfg in reconcile_profile.HOT
