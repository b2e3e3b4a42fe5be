"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL
("nccl" on ROCm) across the xGMI mesh (gloo on CPU for tests).

The reference is single-device (train_denoise.py:83-90).  Data parallelism is
exact for every term of the denoise step that is a mean over equal shards (mel
L1, VQ commitment MSE, per-sample SNR mean): plain gradient averaging of the
rank-local losses equals the single-device gradient on the global batch.  Two
reference quantities are *batch-global* and need an explicit exchange:
  * add_noise (dataloader/data_utils.py:15-16): ||speech||, ||noise|| over the
    whole batch -> all-reduce the two sums of squares (add_noise_global);
  * spectral convergence (losses/stft_loss.py:56): ||y-x||_F / ||y||_F over
    the whole batch -> all-reduce the per-rank partial sums (sum (y-x)^2,
    sum y^2, sum |ln y - ln x|, element count) before the ratio
    (global_loss_sums; used by sel/spectral.py's STFT-loss autograd ops).
"""
import os

import torch
import torch.distributed as dist

from . import _lib as L


def is_dist():
    return dist.is_available() and dist.is_initialized()


def rank_world():
    if is_dist():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend=None):
    """Initialise from RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or is_dist():
        return rank_world()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return rank_world()


def shard(t, rank=None, world=None):
    """Rank's equal slice of a global batch along dim 0."""
    if rank is None:
        rank, world = rank_world()
    if t.shape[0] % world:
        raise ValueError(f"global batch {t.shape[0]} not divisible by world size {world}")
    n = t.shape[0] // world
    return t[rank * n:(rank + 1) * n]


# Spectral-convergence / log-magnitude losses over the GLOBAL batch when data
# parallel (the reference's value on the concatenated batch).  Set False to get
# rank-local losses (e.g. when only some ranks evaluate a loss).
GLOBAL_BATCH_LOSSES = True


def global_loss_sums(sums, n):
    """Data-parallel exchange of the STFT-loss partial sums.

    sums: float64 (3,) = [sum (y-x)^2, sum y^2, sum |ln y - ln x|] of this
    rank's shard, n = its element count.  Returns (global sums, global n,
    grad_scale).  The loss computed from the global sums is the same scalar on
    every rank; DDP then AVERAGES the parameter gradients over the W ranks, so
    each rank back-propagates W x d(global loss)/d(local sums) (grad_scale = W):
    the average is then exactly the single-device gradient on the global batch
    (the SC ratio is not a mean over shards).  Data parallel, the
    global count stays on device as the 4th element of the returned sums and
    the returned n is 0 (sel_stft_loss_finish / _coef then read it there): no
    host sync per resolution and step."""
    if not (GLOBAL_BATCH_LOSSES and is_dist()) or dist.get_world_size() == 1:
        return sums, n, 1.0
    t = torch.empty(4, dtype=torch.float64, device=sums.device)
    t[:3] = sums.detach()
    t[3] = float(n)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t, 0, float(dist.get_world_size())


def allreduce_sum_(t):
    if is_dist() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def _local_sumsq(speech, noise):
    """{sum speech^2, sum noise^2} of this rank's shard (sel_sumsq2, fp64 on device)."""
    L.need_device(speech, noise)
    sums = torch.empty(2, dtype=torch.float64, device=speech.device)
    ws = L.workspace(L.lib().sel_add_noise_workspace(speech.numel()), speech.device)
    L.call("sel_sumsq2", L.ptr(speech), L.ptr(noise), speech.numel(), L.ptr(sums), L.ptr(ws), ws.numel(),
           L.stream())
    return sums


def _mix(speech, noise, sums, snr):
    out = torch.empty_like(speech)
    L.call("sel_mix_noise", L.ptr(speech), L.ptr(noise), speech.numel(), L.ptr(sums), float(snr), L.ptr(out),
           L.stream())
    return out


def add_noise_global(speech, noise, snr):
    """add_noise with norms over the GLOBAL batch (all ranks' shards) — equal to
    the reference's add_noise applied to the concatenated global batch."""
    assert speech.shape == noise.shape, "Shapes are not equal!"
    snr = float(snr.item() if torch.is_tensor(snr) else snr)
    a = speech.contiguous().float()
    b = noise.contiguous().float()
    sums = allreduce_sum_(_local_sumsq(a, b))
    return _mix(a, b, sums, snr)


DDP_BUCKET_MB = float(os.environ.get("SEL_DDP_BUCKET_MB", "4"))


def wrap_ddp(module, device=None, bucket_cap_mb=DDP_BUCKET_MB, force=False):
    """DistributedDataParallel over the trainable parameters only (frozen
    decoder/quantizer of trainer/denoise.py are skipped).  Gradient buckets are
    all-reduced by RCCL while the backward is still running.  4 MB buckets:
    the denoise trainer's 15.6 MB of fp32 encoder grads span 4-5 ring
    all-reduces, the first of which start while the encoder's earlier layers
    are still in their backward (one 16 MB bucket would only start after the
    last of them).  The sel reducer (sel.ddp.SelDDP)
    keeps the weight-gradient reductions batched per bucket and writes them
    straight into the buckets (sel.ddp).  SEL_DDP=torch: torch's
    DistributedDataParallel instead (its own bucket copies; the weight-gradient
    reductions then run per layer).  force: wrap under a one-rank group too
    (bench.py's SEL_BENCH_FORCE_DDP rehearsal of the data-parallel schedule on
    one GPU)."""
    if not is_dist() or (dist.get_world_size() == 1 and not force):
        return module
    if os.environ.get("SEL_DDP", "sel") == "torch":
        from torch.nn.parallel import DistributedDataParallel as DDP
        kw = dict(broadcast_buffers=False, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True)
        if device is not None and device.type == "cuda":
            kw["device_ids"] = [device.index]
        return DDP(module, **kw)
    from .ddp import SelDDP
    return SelDDP(module, bucket_cap_mb=bucket_cap_mb)
