"""Data-parallel log_prob over the GPUs of one node (one process per GPU).

The reference has no distributed code. Its hot path shards by sample with no
per-layer communication: samples are independent in eval mode (the per-sample results of a
half batch are bit-identical to the full batch). The ONLY exchange is the mean NLL: each rank
reduces its shard to a float64 [sum log p, count] pair on device (fused in nfx_gauss_logprob)
and one all-reduce of those 16 bytes runs over RCCL/xGMI (torch.distributed backend "nccl" is
RCCL on ROCm). Weights are replicated once with a broadcast from rank 0.
"""
import torch
import torch.distributed as dist


def shard_range(n, rank, world):
    """Contiguous, balanced [start, stop) of n samples for `rank` of `world`."""
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def broadcast_parameters(module, src=0, group=None):
    """Replicate every parameter and buffer of `module` from rank `src` (one-time, <1 MB)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t, src=src, group=group)
            # the collective writes behind autograd's back: bump the version so any packed
            # weight image keyed on (data_ptr, _version) is rebuilt from the broadcast values
            torch.autograd.graph.increment_version(t)
    from .flows.flow import drop_pack_caches
    drop_pack_caches(module)


def sharded_nll(model, x_local, group=None, return_log_prob=False):
    """Global mean NLL of the samples spread over all ranks; x_local is this rank's shard.

    `model` is a NormalizingFlowModel / RealNVP / RealNVPSpline (anything with
    log_prob(x, return_sums=True)). Returns a python float (identical on every rank)."""
    flow = model.flow if hasattr(model, "flow") and hasattr(model.flow, "log_prob") else model
    logp, sums = flow.log_prob(x_local, return_sums=True)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(sums, group=group)
    s = sums.detach().cpu()
    nll = -(s[0] / s[1]).item() if float(s[1]) > 0 else float("nan")
    return (nll, logp) if return_log_prob else nll


def average_gradients(module, group=None, local_count=None):
    """Data-parallel training exchange: average every parameter gradient over the ranks with
    ONE bucketed all-reduce of the flattened gradients (412 KB for 5 x MAF(63, 64); a single
    message is latency-optimal on xGMI at that size). Parameters without a gradient are skipped.

    Each rank's loss is a mean over its own shard. With `local_count` (this rank's sample
    count, e.g. from shard_range, which hands out shards differing by one when n % world != 0)
    every rank's gradient is weighted by its count and the counts ride in the same all-reduce,
    so the result is exactly the full-batch mean-loss gradient: sum_r n_r g_r / sum_r n_r.
    Without it the ranks are assumed to hold equal shards (plain mean over ranks)."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    params = [p for p in module.parameters() if p.grad is not None]
    if not params:
        return
    grads = [p.grad.reshape(-1) for p in params]
    if local_count is None:
        flat = torch.cat(grads)
        dist.all_reduce(flat, group=group)
        flat /= world
    else:
        n = torch.full((1,), float(local_count), device=grads[0].device, dtype=grads[0].dtype)
        flat = torch.cat([torch.cat(grads) * n, n])
        dist.all_reduce(flat, group=group)
        flat = flat[:-1] / flat[-1]
    o = 0
    for p in params:
        n = p.numel()
        p.grad.copy_(flat[o:o + n].view_as(p))
        o += n


# ---------------------------------------------------------------------------------------------
# SyncBN for data-parallel TRAINING of coupling layers (SURVEY.md §8(e) "when it breaks", §8(f)
# item 2). In train mode CouplingLayer's BatchNorm1d normalises with batch statistics
# (coupling_layer.py:18-35), so a sample-sharded step only equals the full-batch step if the
# statistics and the BatchNorm-backward sums are taken over ALL ranks. The train-mode kernels
# (csrc/nfx_affine_train.hip) hand the host exact float64 pieces between passes:
#   * statistics triples (n, mean, M2) per feature -> all_gather + Chan merge (merge_bn_stats)
#   * backward sums (sum g, sum g x^) per feature   -> all_reduce SUM (allreduce_bn_sums)
# Off by default: a single process reproduces the reference's single-process BatchNorm.
# ---------------------------------------------------------------------------------------------
_SYNC_BN = {"enabled": False, "group": None}


def enable_sync_batchnorm(enabled=True, group=None):
    """Take train-mode coupling BatchNorm statistics over every rank of `group` (SyncBN)."""
    _SYNC_BN["enabled"] = bool(enabled)
    _SYNC_BN["group"] = group


def sync_bn_world():
    """World size SyncBN reduces over (1 when disabled or not distributed)."""
    if not _SYNC_BN["enabled"] or not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(_SYNC_BN["group"])


def merge_bn_stats(stats):
    """In place: per-rank float64 triples [..., 3] = (n, mean, M2) -> the triple of the union
    of all ranks' samples (same on every rank; exact two-level merge in float64)."""
    world = sync_bn_world()
    if world == 1:
        return stats
    group = _SYNC_BN["group"]
    parts = [torch.empty_like(stats) for _ in range(world)]
    dist.all_gather(parts, stats.contiguous(), group=group)
    g = torch.stack(parts)
    n_r, mean_r, m2_r = g[..., 0], g[..., 1], g[..., 2]
    n = n_r.sum(0)
    mean = (n_r * mean_r).sum(0) / n.clamp_min(1.0)
    m2 = m2_r.sum(0) + (n_r * (mean_r - mean) ** 2).sum(0)
    stats[..., 0] = n
    stats[..., 1] = mean
    stats[..., 2] = m2
    return stats


def allreduce_bn_sums(t):
    """In place SUM over the SyncBN group of a float64 block of BatchNorm-backward sums."""
    if sync_bn_world() > 1:
        dist.all_reduce(t, group=_SYNC_BN["group"])
    return t
