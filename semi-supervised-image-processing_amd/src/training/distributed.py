"""Data parallelism for the drop-in pipelines (build extension: the reference
is single-process).

Launch any of the three CLIs under torchrun (one process per GPU, RCCL via
torch.distributed "nccl"); without WORLD_SIZE > 1 everything here is the
identity and the pipelines are exactly the single-process reference path.

What is sharded, and how the result stays equal to the single-process one:
  * evaluation / pseudo-labelling / triage / extraction (forward-only, eval-mode
    BN: every image's output is independent of its batch): the loader's BATCHES
    are split contiguously over the ranks (``shard_loader``), so every rank sees
    the same batch compositions as the single process, and per-batch results
    are gathered in rank order (``gather_list``) -- the reference's per-batch
    loss mean, prediction order and pseudo-label list come out identical
    (reference: semi_supervised.py:44-72, common.py:317-342,439-506,
    feature_extraction.py:251-313);
  * training: the balanced WeightedRandomSampler stream is drawn identically on
    every rank (same global RNG) and rank-strided (``RankStridedSampler``); the
    gradients are all-reduced in buckets during the backward (ssip.dist) and the
    1/world average is folded into the fused AdamW (DDP semantics: per-rank
    BatchNorm statistics, initial weights and buffers broadcast from rank 0);
  * artifacts are written by rank 0 only (``is_main``).
"""
from __future__ import annotations

import math
import os
from typing import Iterator, List, Optional

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, Sampler, Subset

from ssip.dist import GradBucketer, gather_objects, init_from_env, shard_range


def setup(device: torch.device) -> torch.device:
    """Initialise the process group when launched by torchrun (WORLD_SIZE > 1)
    and return this rank's device (cuda:LOCAL_RANK)."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        _, _, local = init_from_env()
        if device.type == "cuda":
            n = torch.cuda.device_count()
            device = torch.device("cuda", local % n if n else 0)
            torch.cuda.set_device(device)
    return device


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def is_main() -> bool:
    return rank() == 0


def shard_loader(loader: DataLoader, even: bool = False) -> DataLoader:
    """This rank's contiguous run of the loader's batches (same batch size,
    collate and workers; sequential loaders only).  even=True (training: every
    batch is a step with gradient all-reduces, so every rank must run the same
    number) pads the batch list to a multiple of world by wrapping around to
    its first batches, as RankStridedSampler / DistributedSampler pad: every
    rank runs ceil(nb / world) batches and no batch of the epoch is dropped."""
    w = world()
    if w == 1:
        return loader
    if loader.batch_size is None:
        raise ValueError("shard_loader needs a batched loader")
    ds = loader.dataset
    n, bs = len(ds), loader.batch_size
    nb = math.ceil(n / bs) if not loader.drop_last else n // bs
    if not even:
        blo, bhi = shard_range(nb, rank(), w)
        idx = list(range(blo * bs, min(bhi * bs, n)))
        return DataLoader(Subset(ds, idx), batch_size=bs, shuffle=False, num_workers=loader.num_workers,
                          pin_memory=loader.pin_memory, collate_fn=loader.collate_fn, drop_last=loader.drop_last)
    total = -(-nb // w) * w if nb > 0 else 0
    blo, bhi = shard_range(total, rank(), w)
    batches = [list(range((b % nb) * bs, min((b % nb + 1) * bs, n))) for b in range(blo, bhi)]
    out = DataLoader(ds, batch_sampler=batches, num_workers=loader.num_workers, pin_memory=loader.pin_memory,
                     collate_fn=loader.collate_fn)
    # which of this rank's batches are wrap-around repeats: they run as steps
    # (the gradient all-reduce needs every rank) but a caller keeps them out of
    # the epoch's loss / accuracy averages, so those cover each batch once, as
    # the single-process epoch does
    out.ssip_padded = [b >= nb for b in range(blo, bhi)]
    return out


def gather_list(local: list) -> list:
    """Per-rank lists concatenated in rank order (identity on one process)."""
    return gather_objects(local) if world() > 1 else list(local)


class RankStridedSampler(Sampler):
    """The base sampler's stream, drawn identically on every rank (it consumes
    the global torch RNG like the reference's WeightedRandomSampler does at each
    epoch's iter), padded to a multiple of world by repeating its head (as
    torch's DistributedSampler pads) and rank-strided: rank r trains on draws
    r, r + world, ...  Every rank gets ceil(n / world) draws, so every rank runs
    the same number of batches (each one a step with gradient all-reduces)."""

    def __init__(self, base: Sampler, rank_: Optional[int] = None, world_: Optional[int] = None):
        self.base = base
        self.r = rank() if rank_ is None else rank_
        self.w = world() if world_ is None else world_

    def __iter__(self) -> Iterator[int]:
        draws = list(self.base)
        n = len(draws)
        if n == 0:
            return iter([])
        total = -(-n // self.w) * self.w
        while len(draws) < total:
            draws += draws[: total - len(draws)]
        return iter(draws[self.r::self.w])

    def __len__(self) -> int:
        n = len(self.base)
        return -(-n // self.w) if n > 0 else 0


def broadcast_model(model) -> None:
    """Rank 0's weights and BN buffers on every rank (DDP initial sync)."""
    if world() == 1:
        return
    arena = model.flatten_parameters()
    dist.broadcast(arena.flat, 0)
    sync_buffers(model)


def sync_buffers(model) -> None:
    """Rank 0's BatchNorm buffers (running_mean / running_var /
    num_batches_tracked) on every rank, in one broadcast per dtype.

    Training updates each rank's running statistics from its own batches
    (DDP: local batch statistics, no SyncBN), so they drift apart; DDP
    re-broadcasts rank 0's buffers (broadcast_buffers=True) and the model the
    pipelines save and report is rank 0's.  Every sharded forward-only pass
    (evaluation, pseudo-labelling, triage) therefore runs after this, so each
    shard is computed with the statistics of that one model (reference: one
    model evaluated in common.py:317-342,439-506; semi_supervised.py:44-72)."""
    if world() == 1:
        return
    bufs = [b for b in model.buffers()]
    for dt in sorted({b.dtype for b in bufs}, key=str):
        group = [b for b in bufs if b.dtype == dt]
        flat = torch.cat([b.reshape(-1) for b in group])
        dist.broadcast(flat, 0)
        o = 0
        with torch.no_grad():
            for b in group:
                n = b.numel()
                b.copy_(flat[o:o + n].view_as(b))
                o += n


def attach_grad_allreduce(model, optimizer) -> None:
    """Bucketed gradient all-reduce launched from inside the backward; the
    optimizer's step() waits for it and averages (grad_scale = 1/world)."""
    if world() == 1:
        return
    broadcast_model(model)
    bucketer = GradBucketer(model.flatten_parameters())
    model.grad_ready_hook = bucketer.mark_ready
    optimizer.dp_bucketer = bucketer



def rank_sum(values: List[float]) -> List[float]:
    """Element-wise sum over ranks (host floats; over RCCL the values travel
    in a device tensor: the "nccl" backend has no CPU tensors)."""
    if world() == 1:
        return list(values)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor(values, dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return t.cpu().tolist()
