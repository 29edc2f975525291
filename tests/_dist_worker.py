"""Process entry of tests/test_dist_gloo.py (importable by spawned children: sets sys.path)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "normalizing-flows-study_amd"), HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import nfs_amd  # noqa: E402
from nfs_amd.distributed import average_gradients, broadcast_parameters, shard_range, sharded_nll  # noqa: E402


def _model(seed, kind):
    torch.manual_seed(seed)
    if kind == "realnvp":
        m = nfs_amd.RealNVP(2, 4, 16)
    elif kind == "spline":
        m = nfs_amd.RealNVPSpline(2, 2, 16)
    else:
        m = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(5, 16) for _ in range(2)])
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.1 * torch.randn_like(p))
    return m.eval()


def _worker(rank, world, port, kind, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _model(1000 + rank, kind)          # different init per rank ...
        broadcast_parameters(m, src=0)          # ... replicated from rank 0
        d = 2 if kind != "maf" else 5
        x = torch.randn(n, d, generator=torch.Generator().manual_seed(7))
        a, b = shard_range(n, rank, world)
        with torch.no_grad():
            nll = sharded_nll(m, x[a:b])
        sd = {k: v.numpy().copy() for k, v in m.state_dict().items()}
        q.put((rank, nll, sd))
    finally:
        dist.destroy_process_group()


def _train_worker(rank, world, port, kind, n, q):
    """One data-parallel training step: mean loss on this rank's shard, averaged gradients."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _model(1000 + rank, kind).train()
        broadcast_parameters(m, src=0)
        d = 2 if kind != "maf" else 5
        x = torch.randn(n, d, generator=torch.Generator().manual_seed(9))
        a, b = shard_range(n, rank, world)
        loss = -m.log_prob(x[a:b]).mean()
        loss.backward()
        average_gradients(m)
        q.put((rank, {k: p.grad.numpy().copy() for k, p in m.named_parameters()}))
    finally:
        dist.destroy_process_group()



def _syncbn_worker(rank, world, port, n, q):
    """SyncBN pieces on CPU tensors: the (n, mean, M2) merge, the BatchNorm-backward sum
    all-reduce, and the between-layer BatchNorm running-stat update of a train-mode forward."""
    from nfs_amd.distributed import allreduce_bn_sums, enable_sync_batchnorm, merge_bn_stats
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        enable_sync_batchnorm(True)
        X = torch.randn(n, 6, generator=torch.Generator().manual_seed(11), dtype=torch.float64) * 3 + 1
        a, b = shard_range(n, rank, world)
        xs = X[a:b]
        mean = xs.mean(0)
        stats = torch.stack([torch.full((6,), float(b - a), dtype=torch.float64), mean,
                             ((xs - mean) ** 2).sum(0)], dim=1)
        merge_bn_stats(stats)
        sums = torch.stack([xs.sum(0), (xs * xs).sum(0)])
        allreduce_bn_sums(sums)
        # between-layer BatchNorm in train mode (normalizing_flow_model.py:74-79) under SyncBN
        torch.manual_seed(5)
        m = nfs_amd.RealNVPSpline(2, 4, 16, batch_norm_between_layers=True).train()
        z = torch.randn(n, 2, generator=torch.Generator().manual_seed(12))
        with torch.no_grad():
            m.forward(z[a:b])
        rs = {k: v.numpy().copy() for k, v in m.state_dict().items() if "batch_norms" in k and "running" in k}
        q.put((rank, stats.numpy().copy(), sums.numpy().copy(), rs))
    finally:
        enable_sync_batchnorm(False)
        dist.destroy_process_group()


def _train_worker_weighted(rank, world, port, kind, n, q):
    """Unequal shards (n % world != 0): gradients weighted by the local sample count."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _model(1000 + rank, kind).train()
        broadcast_parameters(m, src=0)
        d = 2 if kind != "maf" else 5
        x = torch.randn(n, d, generator=torch.Generator().manual_seed(9))
        a, b = shard_range(n, rank, world)
        loss = -m.log_prob(x[a:b]).mean()
        loss.backward()
        average_gradients(m, local_count=b - a)
        q.put((rank, {k: p.grad.numpy().copy() for k, p in m.named_parameters()}))
    finally:
        dist.destroy_process_group()
