"""GPU, RCCL: the data-parallel gradient path over the "nccl" backend (RCCL
on ROCm) on the box's one GPU.  RCCL refuses two ranks on one device
("Duplicate GPU detected", tools/rccl_probe.py on a gpurun box), so this runs
world size 1: the bucketer still issues every bucket's all-reduce through
RCCL (ssip.dist.GradBucketer is active whenever a process group exists) --
from the backward's grad-ready hooks (eager), from the launch plan's host
callbacks during a C++ replay (plan), and on the comm stream behind a
hipGraph replay (graph) -- and waits for them before AdamW.  A plain SUM
over one rank is an in-place identity, so the buckets are reduced with
ncclPreMulSum(2) and AdamW divides the 2 back out (GradBucketer(premul=2),
grad_scale 0.5): exact in fp32, so after the steps the weights must equal a
run without any process group bit for bit, while a bucket reduced before its
gradients landed (they are then overwritten undoubled and halved) or an
AdamW launch that does not wait for the reduction (it halves the undoubled
gradients) changes them.  The negative control proves the test bites: a
bucketer that all-reduces every bucket at the first grad-ready hook, before
the wgrads that fill them were enqueued, must NOT reproduce the weights.
The multi-GPU node runs the same code with world size > 1 (bench.py under
torch.distributed.run).
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

from test_gpu_dist import STEPS, _data, _free_port

pytestmark = pytest.mark.gpu

MODES = ("eager", "plan", "graph")


def _make(dev, mode, with_bucketer, early=False):
    from ssip import SSIPResNet, replace_fc
    from ssip.dist import GradBucketer
    from ssip.semi_step import SemiStep

    class EarlyBucketer(GradBucketer):
        """Negative control: every bucket is launched at the first hook."""

        def mark_ready(self, params):
            for b in range(len(self.buckets)):
                self._launch(b)

    torch.manual_seed(0)
    m = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev).train()
    cls = EarlyBucketer if early else GradBucketer
    bucketer = cls(m.flatten_parameters(), bucket_bytes=8 << 20, premul=2.0) if with_bucketer else None
    step = SemiStep(m, lr=1e-3, weight_decay=1e-4, tau=0.5, image_size=64, bucketer=bucketer, seed=0,
                    plan=mode == "plan", graph=mode == "graph")
    step.opt.use_device_schedule()
    return step


def _run_steps(step, dev):
    x_l, y_l, x_u, params = _data(0)
    x_l, y_l, x_u = x_l.to(dev), y_l.to(dev), x_u.to(dev)
    for i in range(STEPS):
        step(x_l, y_l, x_u, params[i])
    torch.cuda.synchronize()
    return step.arena.flat.detach().cpu().clone()


def _worker(port, out):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "semi-supervised-image-processing_amd"), str(root), str(root / "tests")]
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        res = {"backend": dist.get_backend()}
        for mode in MODES:
            step = _make(dev, mode, True)
            assert step.bucketer.active and len(step.bucketer.buckets) > 1
            assert step.bucketer.grad_scale() == 0.5
            res[mode] = _run_steps(step, dev)
            del step
        res["early"] = _run_steps(_make(dev, "eager", True, early=True), dev)
        # the rank-0 broadcast the pipelines use for weights, over RCCL
        t = torch.arange(1 << 16, dtype=torch.float32, device=dev)
        dist.broadcast(t, 0)
        res["bcast_ok"] = bool(torch.equal(t.cpu(), torch.arange(1 << 16, dtype=torch.float32)))
        torch.save(res, os.path.join(out, "rccl.pt"))
    finally:
        dist.destroy_process_group()


def test_semi_step_rccl_world1_equals_single(dev, tmp_path):
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_worker, args=(_free_port(), str(tmp_path)))
    p.start()
    p.join(300)
    if p.exitcode is None:
        p.kill()
    assert p.exitcode == 0, p.exitcode
    r = torch.load(tmp_path / "rccl.pt", weights_only=True)
    assert r["backend"] == "nccl"
    assert r["bcast_ok"]
    for mode in MODES:
        want = _run_steps(_make(dev, mode, False), dev)
        assert torch.equal(r[mode], want), mode
        if mode == "eager":
            # the control: all-reduced before the wgrads landed -> different weights
            assert not torch.equal(r["early"], want)
