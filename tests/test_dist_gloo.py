"""Multi-process data-parallel log_prob on CPU (gloo, world_size 2): the sharded NLL with ONE
all-reduce equals the single-process NLL, shards are balanced and contiguous, and the weight
broadcast replicates rank 0's parameters."""
import os
import socket

import numpy as np
import pytest
import torch

import nfs_amd
import torch.distributed as dist
import torch.multiprocessing as mp

from nfs_amd.distributed import shard_range
from _dist_worker import _model, _syncbn_worker, _train_worker, _train_worker_weighted, _worker


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


@pytest.mark.parametrize("kind", ["maf", "spline"])
def test_data_parallel_gradients_match_full_batch(kind):
    """Equal shards + mean loss per rank + one averaged-gradient all-reduce == the full-batch
    gradient of the single-process model (the training exchange of bench.py cfg4t). Models
    without train-mode BatchNorm only: RealNVP's conditioner BatchNorm normalises with batch
    statistics, which would need a SyncBN all-reduce per layer."""
    world, n = 2, 800
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, world, port, kind, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m = _model(1000, kind).train()
    d = 2 if kind != "maf" else 5
    x = torch.randn(n, d, generator=torch.Generator().manual_seed(9))
    (-m.log_prob(x).mean()).backward()
    for k, p in m.named_parameters():
        for r in range(world):
            assert torch.allclose(torch.from_numpy(res[r][1][k]), p.grad, rtol=1e-4, atol=1e-6), k



def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_syncbn_merge_and_sums_match_full_batch():
    """merge_bn_stats / allreduce_bn_sums (nfs_amd/distributed.py, used between the train-mode
    coupling kernels' passes) called directly on CPU float64 tensors over 2 gloo ranks with
    unequal shards: the merged (n, mean, M2) and the summed BatchNorm-backward blocks equal the
    single-process full-batch values; and the between-layer BatchNorm of a train-mode forward
    (normalizing_flow_model.py:74-79) updates the running statistics from the moments of the
    whole batch, identical on every rank."""
    n = 1001
    res = _spawn(_syncbn_worker, 2, n)
    X = torch.randn(n, 6, generator=torch.Generator().manual_seed(11), dtype=torch.float64) * 3 + 1
    mean = X.mean(0)
    for _, stats, sums, _ in res:
        np.testing.assert_allclose(stats[:, 0], n)
        np.testing.assert_allclose(stats[:, 1], mean.numpy(), rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(stats[:, 2], ((X - mean) ** 2).sum(0).numpy(), rtol=1e-12)
        np.testing.assert_allclose(sums[0], X.sum(0).numpy(), rtol=1e-13)
        np.testing.assert_allclose(sums[1], (X * X).sum(0).numpy(), rtol=1e-13)
    torch.manual_seed(5)
    m = nfs_amd.RealNVPSpline(2, 4, 16, batch_norm_between_layers=True).train()
    z = torch.randn(n, 2, generator=torch.Generator().manual_seed(12))
    with torch.no_grad():
        m.forward(z)
    ref = {k: v.numpy() for k, v in m.state_dict().items() if "batch_norms" in k and "running" in k}
    assert ref
    for k, v in ref.items():
        assert np.array_equal(res[0][3][k], res[1][3][k]), k
        np.testing.assert_allclose(res[0][3][k], v, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("kind", ["maf", "spline"])
def test_unequal_shards_weighted_gradients_match_full_batch(kind):
    """n % world != 0: average_gradients(local_count=...) weights each rank's mean-loss
    gradient by its shard size, giving exactly the full-batch gradient."""
    n = 801
    res = _spawn(_train_worker_weighted, 2, kind, n)
    m = _model(1000, kind).train()
    d = 2 if kind != "maf" else 5
    x = torch.randn(n, d, generator=torch.Generator().manual_seed(9))
    (-m.log_prob(x).mean()).backward()
    for k, p in m.named_parameters():
        for r in range(2):
            assert torch.allclose(torch.from_numpy(res[r][1][k]), p.grad, rtol=1e-4, atol=1e-6), k
