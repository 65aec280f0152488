"""Data parallelism over RCCL (torch.distributed backend "nccl" on ROCm).

The reference is single-device (no collectives); this is the
build's DP extension for configs 4/5.  One process per GPU; each rank runs
the full train step on its own shard of the batch; the only exchange is an
all-reduce of the flat fp32 gradient arena (44.7 MB for ResNet-18).

Bucketing: the arena is cut at parameter boundaries into buckets of about
`bucket_bytes`.  The engine's backward calls `mark_ready(params)` as each
block's gradients are enqueued (layer4 first); a bucket whose parameters are
all ready is all-reduced immediately with `async_op=True`, so RCCL runs on
its own stream over xGMI while the remaining backward kernels run.  The
1/world average is folded into the AdamW launch (grad_scale), so no extra
pass over the gradients is needed.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


def init_from_env(backend: Optional[str] = None):
    """Initialise the default process group from torchrun's env (127.0.0.1
    rendezvous).  Returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend is None:
            backend = os.environ.get("SSIP_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        elif torch.cuda.is_available():
            # gloo rehearsal of the DP path (several ranks may share one device)
            torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


class GradBucketer:
    """``premul`` != 1 (RCCL only): each rank's bucket is multiplied by it
    inside the all-reduce (ncclPreMulSum) and the AdamW grad scale divides it
    back out.  With a power of two the result is bit-identical to premul 1;
    tests use it so that a world-size-1 all-reduce is not an identity (a
    bucket reduced before its gradients landed, or an AdamW launch that does
    not wait for the reduction, then changes the weights)."""

    def __init__(self, arena, bucket_bytes: int = 16 << 20, group=None, premul: float = 1.0):
        self.arena = arena
        self.group = group
        self.premul = float(premul)
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # collectives whenever a process group exists, also at world size 1
        # (RCCL then copies in place: the one-GPU RCCL test runs this path)
        self.active = dist.is_initialized()
        # buckets in reverse parameter order (the backward produces the last params first)
        params = list(arena.params)
        spans = [arena.span(p) for p in params]
        buckets: List[List[int]] = []
        cur: List[int] = []
        cur_bytes = 0
        for i in range(len(params) - 1, -1, -1):
            cur.append(i)
            cur_bytes += spans[i][1] * 4
            if cur_bytes >= bucket_bytes:
                buckets.append(cur)
                cur, cur_bytes = [], 0
        if cur:
            buckets.append(cur)
        self.params = params
        self.buckets = buckets
        self.bucket_of = {}
        for b, idxs in enumerate(buckets):
            for i in idxs:
                self.bucket_of[id(params[i])] = b
        self.ranges = []
        for idxs in buckets:
            lo = min(spans[i][0] for i in idxs)
            hi = max(spans[i][0] + spans[i][1] for i in idxs)
            self.ranges.append((lo, hi))
        # Every bucket a multiple of 4 floats: RCCL 2.26.6's ncclPreMulSum
        # (premul != 1) leaves the last count % 4 elements of a call unscaled
        # (tools/rccl_premul_probe.py: the 2-float fc bias at the end of a
        # 2,361,346-float bucket).  A boundary moves UP to a multiple of 4, so
        # the up-to-3 boundary floats (the lowest parameter of the bucket
        # above, produced earlier in the backward) join the bucket below,
        # which launches later: still reduced once, after they are complete.
        # The first bucket ends at the arena's padded end (zeros).
        end = getattr(arena, "padded", arena.numel)
        for b in range(len(self.ranges)):
            lo, hi = self.ranges[b]
            hi = end if b == 0 else self.ranges[b - 1][0]
            lo = lo if lo == 0 else -(-lo // 4) * 4
            self.ranges[b] = (lo, hi)
        # What a bucket waits for and whether it launches at all follow the
        # final ranges, not the parameter lists: a bucket covers every
        # parameter whose span meets its range (the boundary floats of the
        # parameter above included), so it launches once all of those are
        # ready, and whenever any of them trains -- also if its own
        # parameters are all frozen (those moved floats of a
        # trainable parameter were otherwise never reduced).
        self.covers: List[List[int]] = []
        for lo, hi in self.ranges:
            self.covers.append([i for i, (o, n) in enumerate(spans) if n > 0 and o < hi and o + n > lo])
        self.buckets_of = {}
        for b, idxs in enumerate(self.covers):
            for i in idxs:
                self.buckets_of.setdefault(id(params[i]), []).append(b)
        # hipGraph mode (SemiStep(graph=True)): the backward is captured
        # without collectives (ROCm allows no external event nodes in a graph,
        # so a bucket cannot signal mid-replay); after each replay
        # launch_after_graph() all-reduces the buckets in backward order on a
        # comm stream behind the replay
        self.capture_mode = False
        self._comm = None
        self._op = None
        self.reset()

    def _reduce_op(self):
        if self.premul == 1.0:
            return dist.ReduceOp.SUM
        if self._op is None:
            self._op = dist._make_nccl_premul_sum(self.premul)
        return self._op

    def trains(self, b: int) -> bool:
        """Bucket b holds gradient elements of a trainable parameter."""
        return any(self.params[i].requires_grad for i in self.covers[b])

    def reset(self):
        self.pending = [set(i for i in idxs if self.params[i].requires_grad) for idxs in self.covers]
        self.handles = []
        self.launched = [False] * len(self.buckets)

    def _launch(self, b: int):
        if self.launched[b]:
            return
        self.launched[b] = True
        if self.capture_mode:
            return
        lo, hi = self.ranges[b]
        if self.active:
            self.handles.append(dist.all_reduce(self.arena.grad[lo:hi], op=self._reduce_op(), group=self.group,
                                                async_op=True))

    def end_capture(self) -> None:
        """Close the capture-time bookkeeping (nothing was launched)."""
        self.launched = [True] * len(self.buckets)

    def launch_after_graph(self) -> None:
        """All-reduce every bucket with trainable parameters, in backward
        order, on the comm stream once the replayed backward is done."""
        if self._comm is None:
            self._comm = torch.cuda.Stream()
        self._comm.wait_stream(torch.cuda.current_stream())
        self.handles = []
        for b in range(len(self.buckets)):
            if self.active and self.trains(b):
                lo, hi = self.ranges[b]
                with torch.cuda.stream(self._comm):
                    self.handles.append(dist.all_reduce(self.arena.grad[lo:hi], op=self._reduce_op(),
                                                        group=self.group, async_op=True))
        self.launched = [True] * len(self.buckets)

    def mark_ready(self, params) -> None:
        idx = {id(p): i for i, p in enumerate(self.params)}
        for p in params:
            for b in self.buckets_of.get(id(p), ()):
                self.pending[b].discard(idx[id(p)])
                if not self.pending[b] and self.trains(b):
                    self._launch(b)

    def grad_scale(self) -> float:
        """The factor AdamW applies to the reduced gradients: the 1/world
        average, and the premultiplier divided back out."""
        return 1.0 / (self.world * (self.premul if self.active else 1.0))

    def finish(self) -> float:
        """Launch anything left, wait, and return the grad scale (1 / (world * premul))."""
        for b in range(len(self.buckets)):
            if self.trains(b):
                self._launch(b)
        for h in self.handles:
            h.wait()
        self.handles = []
        if self._comm is not None:  # graph mode: the comm stream also carried the event waits
            torch.cuda.current_stream().wait_stream(self._comm)
        return self.grad_scale()


def shard_range(n: int, rank: int, world: int):
    """Contiguous shard [lo, hi) of n items for `rank` (pseudo-labelling,
    evaluation and embedding extraction shard the file list this way)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def strided_indices(indices: List[int], rank: int, world: int) -> List[int]:
    """Rank-stride a global sample stream (the WeightedRandomSampler draw is
    generated identically on every rank from the same seed)."""
    return list(indices[rank::world])


def gather_objects(local: list, group=None) -> list:
    """Concatenate per-rank Python lists in rank order (pseudo-label tuples,
    evaluation records) — the shards come from `shard_range`, so the result
    equals the single-process order."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return list(local)
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, list(local), group=group)
    out = []
    for p in parts:
        out.extend(p)
    return out


def gather_rows(local: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate per-rank [n_r, D] tensors (n_r may differ) in rank order."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return local
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], device=local.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    m = int(max(int(x) for x in ns))
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[: int(k)] for b, k in zip(bufs, ns)], 0)
