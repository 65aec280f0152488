"""Does RCCL apply ncclPreMulSum at world size 1 (GPU box) -- also on the
gradient buckets' slices of the arena (unaligned offsets)?"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "semi-supervised-image-processing_amd"))
import torch
import torch.distributed as dist

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
from ssip import SSIPResNet, replace_fc  # noqa: E402
from ssip.dist import GradBucketer  # noqa: E402

m = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev)
ar = m.flatten_parameters()
bk = GradBucketer(ar, bucket_bytes=8 << 20, premul=2.0)
print("buckets", len(bk.buckets), "ranges", bk.ranges, flush=True)
g = ar.grad
g.copy_(torch.randn(g.numel(), device=dev))
ref = g.clone()
for lo, hi in bk.ranges:
    dist.all_reduce(g[lo:hi], op=dist._make_nccl_premul_sum(2.0))
torch.cuda.synchronize()
bad = (g != 2 * ref).nonzero().flatten()
print("per-call op: mismatches", bad.numel(), bad[:10].tolist(), flush=True)
g.copy_(ref)
op = dist._make_nccl_premul_sum(2.0)
hs = [dist.all_reduce(g[lo:hi], op=op, async_op=True) for lo, hi in bk.ranges]
for h in hs:
    h.wait()
torch.cuda.synchronize()
bad = (g != 2 * ref).nonzero().flatten()
print("shared op, async: mismatches", bad.numel(), bad[:10].tolist(), flush=True)
cover = torch.zeros(g.numel(), dtype=torch.int32)
for lo, hi in bk.ranges:
    cover[lo:hi] += 1
print("coverage: min", int(cover.min()), "max", int(cover.max()), "n", g.numel(), flush=True)
dist.destroy_process_group()
