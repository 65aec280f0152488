"""CPU, world_size 2 over gloo: the data-parallel pieces that run over RCCL on
the GPU box — bucketed gradient all-reduce on the flat arena (overlapped
launch order), sharding of the sample stream / file list, and the gathers
used for sharded pseudo-labelling / extraction."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path

        root = Path(__file__).resolve().parents[1]
        sys.path.insert(0, str(root / "semi-supervised-image-processing_amd"))
        from ssip.arena import ParamArena
        from ssip.dist import GradBucketer, gather_objects, gather_rows, shard_range, strided_indices

        torch.manual_seed(0)
        params = [torch.nn.Parameter(torch.randn(n)) for n in (1000, 37, 4096, 5, 20000, 64)]
        arena = ParamArena(params)
        b = GradBucketer(arena, bucket_bytes=16 << 10)
        assert len(b.buckets) > 2
        arena.attach_grads()
        for i, p in enumerate(params):
            p.grad.copy_(torch.full_like(p, float(rank + 1) * (i + 1)))
        b.reset()
        # the backward produces the last parameters first
        for p in reversed(params):
            b.mark_ready([p])
        scale = b.finish()
        ok = abs(scale - 1.0 / world) < 1e-12
        for i, p in enumerate(params):
            ok &= torch.allclose(p.grad, torch.full_like(p, 3.0 * (i + 1)))
        # frozen params are skipped, trainable buckets still complete
        params[0].requires_grad_(False)
        b.reset()
        b.mark_ready(params[1:])
        b.finish()
        lo, hi = shard_range(10, rank, world)
        got = gather_objects([("f%d" % i, i % 2) for i in range(lo, hi)])
        ok &= got == [("f%d" % i, i % 2) for i in range(10)]
        rows = gather_rows(torch.arange(lo, hi, dtype=torch.float32)[:, None].repeat(1, 3))
        ok &= torch.equal(rows[:, 0], torch.arange(10, dtype=torch.float32))
        ok &= strided_indices(list(range(9)), rank, world) == list(range(rank, 9, world))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_bucketed_allreduce_and_sharding_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: True, 1: True}
    assert all(p.exitcode == 0 for p in procs)


def test_shard_range_covers_everything():
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "semi-supervised-image-processing_amd"))
    from ssip.dist import shard_range

    for n in (0, 1, 7, 1406):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


def _pipeline_worker(rank, world, port, q):
    """The drop-in pipelines' DP helpers (src/training/distributed.py)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path

        from torch.utils.data import DataLoader, WeightedRandomSampler

        root = Path(__file__).resolve().parents[1]
        sys.path.insert(0, str(root / "semi-supervised-image-processing_amd"))
        from src.training import distributed as D

        ok = D.world() == world and D.rank() == rank and D.is_main() == (rank == 0)
        # batch-granular sharding: every rank sees whole batches of the
        # single-process loader, and the rank-ordered gather restores its order
        data = [(float(i), i % 3) for i in range(11)]
        full = DataLoader(data, batch_size=3, shuffle=False)
        single = [b[0].tolist() for b in full]
        mine = [b[0].tolist() for b in D.shard_loader(full)]
        ok &= D.gather_list(mine) == single
        # per-batch means (the reference's evaluate_on_loader loss) are unchanged
        ok &= D.gather_list([sum(b) / len(b) for b in mine]) == [sum(b) / len(b) for b in single]
        # the balanced sampler's stream is drawn identically on every rank and strided
        torch.manual_seed(5)
        w = [1.0, 3.0, 1.0, 1.0, 2.0, 1.0, 1.0]
        glob = list(WeightedRandomSampler(w, num_samples=7, replacement=True))
        torch.manual_seed(5)
        s = D.RankStridedSampler(WeightedRandomSampler(w, num_samples=7, replacement=True))
        local = list(s)
        # padded to a multiple of world by repeating the head (DistributedSampler)
        padded = glob + glob[: (-len(glob)) % world]
        ok &= local == padded[rank::world] and len(s) == len(local) == 4
        parts = D.gather_list([local])
        inter = [x for t in zip(*parts) for x in t]
        ok &= inter == padded
        ok &= D.rank_sum([1.0, float(rank)]) == [float(world), float(sum(range(world)))]
        # every rank runs the same number of training batches (each one a step
        # with gradient all-reduces) whatever n % world and n % bs are
        for n, bs in ((7, 2), (9, 4), (5, 3), (13, 3)):
            torch.manual_seed(n)
            smp = D.RankStridedSampler(WeightedRandomSampler([1.0] * n, num_samples=n, replacement=True))
            nbat = len(list(DataLoader(list(range(n)), batch_size=bs, sampler=smp)))
            ok &= len(set(D.gather_list([nbat]))) == 1
            even = D.shard_loader(DataLoader(list(range(n)), batch_size=bs, shuffle=False, drop_last=True), even=True)
            got = [b.tolist() for b in even]
            counts = D.gather_list([len(got)])
            nb = n // bs
            ok &= len(set(counts)) == 1 and counts[0] == -(-nb // world)
            # no batch dropped: the rank-ordered batches are the single-process
            # batches, wrapped around to the first ones up to a multiple of world
            single_b = [list(range(b * bs, (b + 1) * bs)) for b in range(nb)]
            allb = [b for part in D.gather_list([got]) for b in part]
            ok &= allb == [single_b[i % nb] for i in range(len(allb))]
            # the wrap-around repeats are flagged: the unflagged batches over all
            # ranks are each single-process batch exactly once (epoch averages)
            flags = [f for part in D.gather_list([even.ssip_padded]) for f in part]
            ok &= len(flags) == len(allb) and sorted(b for b, f in zip(allb, flags) if not f) == single_b
        # rank 0's BN buffers on every rank, bitwise
        bn = torch.nn.Sequential(torch.nn.BatchNorm2d(5), torch.nn.BatchNorm2d(3))
        bn.train()
        torch.manual_seed(100 + rank)
        bn[0](torch.randn(4, 5, 2, 2) * (rank + 1))
        bn[1](torch.randn(4, 3, 2, 2))
        bn[0].num_batches_tracked += rank
        mine0 = [b.clone() for b in bn.buffers()]
        D.sync_buffers(bn)
        got = D.gather_list([[b.tolist() for b in bn.buffers()]])
        ok &= all(g == got[0] for g in got)
        if rank == 0:
            ok &= all(torch.equal(a, b) for a, b in zip(mine0, bn.buffers()))
        else:
            ok &= not all(torch.equal(a, b) for a, b in zip(mine0, bn.buffers()))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_pipeline_sharding_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: True, 1: True}
    assert all(p.exitcode == 0 for p in procs)


def test_bucket_ranges_cover_arena_in_multiples_of_four():
    """GradBucketer's ranges: the padded arena exactly once, every bucket a
    multiple of 4 floats (RCCL's PreMulSum tail), and every parameter element
    in a bucket that launches no earlier than the parameter's own (a boundary
    float may only move to a LATER bucket: lower addresses, reduced after the
    bucket it came from, when it is already complete)."""
    import torch

    from ssip import SSIPResNet, replace_fc
    from ssip.dist import GradBucketer

    m = replace_fc(SSIPResNet("resnet18", 1000), 2)
    ar = m.flatten_parameters()
    for bb in (8 << 20, 16 << 20, 3 << 20):
        bk = GradBucketer(ar, bucket_bytes=bb)
        cover = torch.zeros(ar.padded, dtype=torch.int32)
        owner = torch.full((ar.padded,), -1, dtype=torch.int64)
        for b, (lo, hi) in enumerate(bk.ranges):
            assert (hi - lo) % 4 == 0 and lo < hi
            cover[lo:hi] += 1
            owner[lo:hi] = b
        assert int(cover.min()) == 1 and int(cover.max()) == 1
        for trainable in (None, {"fc.weight", "fc.bias"}):
            names = {id(p): n for n, p in m.named_parameters()}
            for p in ar.params:
                p.requires_grad_(trainable is None or names[id(p)] in trainable)
            _check_bucket_launches(bk, ar)
        for p in ar.params:
            p.requires_grad_(True)


class _OddArena:
    """An arena stand-in whose parameter spans are not multiples of 4 floats,
    so GradBucketer's rounded boundaries move floats between buckets."""

    def __init__(self, sizes):
        import torch

        self.params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
        self._off = {}
        o = 0
        for p, n in zip(self.params, sizes):
            self._off[id(p)] = (o, n)
            o += n
        self.numel = o
        self.padded = -(-o // 64) * 64
        self.grad = torch.zeros(self.padded)

    def span(self, p):
        return self._off[id(p)]


def _check_bucket_launches(bk, ar):
    """Backward order (last parameter first), one mark_ready per trainable
    parameter (the engine hooks only what it computes gradients for): every element of a trainable parameter lies in a bucket that launches,
    and a bucket launches only once every trainable parameter whose span
    meets its range is ready (a bucket of frozen parameters still
    carries the boundary floats of a trainable one above it)."""
    ready = set()
    launches = {}
    real = bk._launch

    def spy(b):
        if not bk.launched[b]:
            launches[b] = set(ready)
        real(b)

    bk._launch = spy
    try:
        bk.reset()
        for i in range(len(bk.params) - 1, -1, -1):
            if bk.params[i].requires_grad:
                ready.add(i)
                bk.mark_ready([bk.params[i]])
        bk.finish()
    finally:
        bk._launch = real
    for i, p in enumerate(bk.params):
        off, n = ar.span(p)
        for b, (lo, hi) in enumerate(bk.ranges):
            if off < hi and off + n > lo and p.requires_grad:
                assert b in launches, ("bucket with trainable floats never launched", b, i)
                assert i in launches[b], ("bucket launched before a parameter it carries was ready", b, i)


def test_bucket_launches_cover_trainable_boundary_floats():
    """Odd spans: every boundary is rounded up, so the lowest floats of a
    bucket's lowest parameter belong to the bucket below.  With that bucket's
    own parameters all frozen it must still launch (and wait for the
    trainable parameter above)."""
    from ssip.dist import GradBucketer

    ar = _OddArena([6, 3, 5, 10, 7, 9, 2, 13])
    for bb in (24, 40, 60):
        bk = GradBucketer(ar, bucket_bytes=bb)
        assert len(bk.ranges) >= 2
        moved = [b for b in range(1, len(bk.ranges))
                 if min(ar.span(bk.params[i])[0] for i in bk.buckets[b - 1]) % 4]
        assert moved, "the case needs a rounded boundary"
        for b in range(len(bk.buckets)):  # bucket b's own parameters frozen, the rest trainable
            for i, p in enumerate(ar.params):
                p.requires_grad_(i not in bk.buckets[b])
            _check_bucket_launches(bk, ar)
        for keep in range(len(ar.params)):  # one trainable parameter at a time
            for i, p in enumerate(ar.params):
                p.requires_grad_(i == keep)
            _check_bucket_launches(bk, ar)
