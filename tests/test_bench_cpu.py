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


def _bench(env_extra, *args, timeout=180):
    import subprocess
    env = dict(os.environ, **env_extra)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if k not in env_extra:
            env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_flag_launches_ranks(n):
    """`bench.py --gpus N` with no launcher around it starts N ranks itself and they join one
    process group (NFX_BENCH_LAUNCH_CHECK: gloo, no GPU call); rank 0's line is relayed."""
    import json
    r = _bench({"NFX_BENCH_LAUNCH_CHECK": "1"}, "--gpus", str(n))
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["launch_check"] and line["world_size"] == n
    assert sorted(x["rank"] for x in line["ranks"]) == list(range(n))
    assert [x["local_rank"] for x in sorted(line["ranks"], key=lambda x: x["rank"])] == list(range(n))
    assert len({x["pid"] for x in line["ranks"]}) == n
    assert f"{n} child ranks" in line["launcher"]


def test_gpus_flag_rank_failure_fails_the_run():
    r = _bench({"NFX_BENCH_LAUNCH_CHECK": "1", "NFX_BENCH_FAIL_RANK": "1"}, "--gpus", "2")
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr


def test_world_size_must_match_gpus():
    r = _bench({"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"}, "--gpus", "2")
    assert r.returncode != 0 and "must agree" in r.stderr
