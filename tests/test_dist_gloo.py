"""Multi-process data-parallel log_prob on CPU (gloo, world_size 2): the sharded NLL with ONE
all-reduce equals the single-process NLL, shards are balanced and contiguous, and the weight
broadcast replicates rank 0's parameters."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nfs_amd.distributed import shard_range
from _dist_worker import _model, _worker


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("kind", ["realnvp", "spline", "maf"])
def test_sharded_nll_matches_single_process(kind):
    world, n = 2, 1001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    # every rank sees the same global NLL
    assert res[0][1] == res[1][1]
    # the broadcast made rank 1's weights rank 0's
    for k in res[0][2]:
        assert (res[0][2][k] == res[1][2][k]).all(), k
    # equals the single-process NLL of rank 0's model on the full batch
    m = _model(1000, kind)
    d = 2 if kind != "maf" else 5
    x = torch.randn(n, d, generator=torch.Generator().manual_seed(7))
    with torch.no_grad():
        ref = m.nll(x) if hasattr(m, "nll") else None
    assert abs(res[0][1] - ref) < 1e-9


def test_shard_range_balanced_and_contiguous():
    for n in (0, 1, 7, 1000, 1_000_003):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, _) in zip(rs, rs[1:]):
                assert b == c
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1
