"""GPU, data parallel with 2 ranks sharing one MI355X (gloo carries the
collectives; RCCL's "nccl" backend takes its place on a multi-GPU node with
the same code): the benchmarked SemiStep with the bucketed gradient
all-reduce launched from inside the real backward (hook order, wgrad side
stream hand-off), eager and launch-plan execution.

Asserted:
  * after one step the all-reduced gradient arena equals the SUM of the two
    single-process gradients of the ranks' shards (the 1/world average is
    folded into AdamW), to fp32 rounding of one add;
  * after 4 steps both ranks hold identical weights (bitwise), and the
    launch-plan replays equal the eager steps (bitwise).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

S, BL, BU, STEPS = 64, 64, 64, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rank):
    from ssip.augment import draw_params_batch

    g = torch.Generator().manual_seed(100 + rank)
    x_l = torch.randint(0, 256, (BL, S, S, 3), generator=g, dtype=torch.uint8)
    x_u = torch.randint(0, 256, (BU, S, S, 3), generator=g, dtype=torch.uint8)
    y_l = torch.randint(0, 2, (BL,), generator=g)
    params = [(draw_params_batch(BL, S, False, g), draw_params_batch(BU, S, False, g), draw_params_batch(BU, S, True, g))
              for _ in range(STEPS)]
    return x_l, y_l, x_u, params


def _make(dev, bucketer_world=False, plan=False):
    from ssip import SSIPResNet, replace_fc
    from ssip.dist import GradBucketer
    from ssip.semi_step import SemiStep

    torch.manual_seed(0)
    m = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev).train()
    bucketer = GradBucketer(m.flatten_parameters(), bucket_bytes=8 << 20) if bucketer_world else None
    step = SemiStep(m, lr=1e-3, weight_decay=1e-4, tau=0.5, image_size=S, bucketer=bucketer, seed=0, plan=plan)
    step.opt.use_device_schedule()
    return step


def _worker(rank, world, port, plan, out):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "semi-supervised-image-processing_amd"), str(root)]
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        step = _make(dev, bucketer_world=True, plan=plan)
        x_l, y_l, x_u, params = _data(rank)
        x_l, y_l, x_u = x_l.to(dev), y_l.to(dev), x_u.to(dev)
        res = {}
        for i in range(STEPS):
            step(x_l, y_l, x_u, params[i])
            if i == 0:
                torch.cuda.synchronize()
                res["grad0"] = step.arena.grad.detach().cpu().clone()
        torch.cuda.synchronize()
        res["flat"] = step.arena.flat.detach().cpu().clone()
        res["plan_ops"] = step._plan.num_ops if plan else 0
        torch.save(res, os.path.join(out, f"rank{rank}_{'plan' if plan else 'eager'}.pt"))
    finally:
        dist.destroy_process_group()


def _run(world, plan, out):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, plan, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(200)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_semi_step_dp2_gloo(dev, tmp_path):
    _run(2, False, str(tmp_path))
    _run(2, True, str(tmp_path))
    r = {(k, m): torch.load(tmp_path / f"rank{k}_{m}.pt", weights_only=True) for k in (0, 1) for m in ("eager", "plan")}
    # identical weights on both ranks, eager and plan alike, and plan == eager
    for m in ("eager", "plan"):
        assert torch.equal(r[(0, m)]["flat"], r[(1, m)]["flat"]), m
    assert torch.equal(r[(0, "eager")]["flat"], r[(0, "plan")]["flat"])
    assert r[(0, "plan")]["plan_ops"] > 100
    # the reduced gradient = sum of the per-rank single-process gradients
    singles = []
    for rank in (0, 1):
        step = _make(dev)
        x_l, y_l, x_u, params = _data(rank)
        step(x_l.to(dev), y_l.to(dev), x_u.to(dev), params[0])
        torch.cuda.synchronize()
        singles.append(step.arena.grad.detach().cpu().clone())
    want = singles[0] + singles[1]
    for m in ("eager", "plan"):
        got = r[(0, m)]["grad0"]
        err = ((got - want).abs().max() / want.abs().max()).item()
        assert err <= 1e-6, (m, err)
        assert torch.equal(got, r[(1, m)]["grad0"])


def _fe_worker(rank, world, port, data, cwd):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "semi-supervised-image-processing_amd"), str(root)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), SSIP_DIST_BACKEND="gloo")
    os.chdir(cwd)
    import torch.distributed as dist

    from src import feature_extraction as FE

    try:
        FE.main(["--data-dir", data, "--batch-size", "5", "--random-init"])
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_feature_extraction_dp2_equals_single(dev, tmp_path, monkeypatch):
    """`python -m src.feature_extraction` under 2 ranks (file list sharded by
    whole batches, embeddings gathered in rank order) writes the same
    embeddings.npy / embeddings.csv as the single-process run, bit for bit."""
    import numpy as np

    from test_gpu_pipeline import _make_dataset

    data = _make_dataset(tmp_path / "mri", n_per_class=7, n_unl=9, size=80)
    (tmp_path / "dp").mkdir()
    (tmp_path / "single").mkdir()
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_fe_worker, args=(r, 2, port, str(data), str(tmp_path / "dp"))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(200)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    monkeypatch.chdir(tmp_path / "single")
    from src import feature_extraction as FE

    FE.main(["--data-dir", str(data), "--batch-size", "5", "--random-init"])
    a = np.load(tmp_path / "dp/outputs/features/embeddings.npy")
    b = np.load(tmp_path / "single/outputs/features/embeddings.npy")
    assert a.shape == b.shape == (23, 512)
    assert np.array_equal(a, b)
    assert (tmp_path / "dp/outputs/features/embeddings.csv").read_text() == \
        (tmp_path / "single/outputs/features/embeddings.csv").read_text()


# --------------------------------------------------------------------------
# the benchmarked per-rank geometry (BASELINE config 4: 224x224, 128 labelled
# + 128 unlabelled per rank), plus the rank-0 BatchNorm buffer sync the
# sharded forward-only passes of the drop-in pipelines rely on
# --------------------------------------------------------------------------
BS, BBL, BBU, BSTEPS = 224, 128, 128, 2
EVAL_N, EVAL_B, EVAL_S = 22, 4, 64   # 6 batches: 3 per rank


def _bench_data(rank):
    from ssip.augment import draw_params_batch

    g = torch.Generator().manual_seed(200 + rank)
    x_l = torch.randint(0, 256, (BBL, BS, BS, 3), generator=g, dtype=torch.uint8)
    x_u = torch.randint(0, 256, (BBU, BS, BS, 3), generator=g, dtype=torch.uint8)
    y_l = torch.randint(0, 2, (BBL,), generator=g)
    params = [(draw_params_batch(BBL, BS, False, g), draw_params_batch(BBU, BS, False, g),
               draw_params_batch(BBU, BS, True, g)) for _ in range(BSTEPS)]
    return x_l, y_l, x_u, params


def _eval_loaders():
    from torch.utils.data import DataLoader

    g = torch.Generator().manual_seed(9)
    x = torch.randn(EVAL_N, 3, EVAL_S, EVAL_S, generator=g)
    y = torch.tensor([i % 2 for i in range(EVAL_N)])
    labelled = DataLoader([(x[i], int(y[i]), f"img{i:02d}") for i in range(EVAL_N)], batch_size=EVAL_B, shuffle=False)
    pool = DataLoader([(x[i], f"img{i:02d}") for i in range(EVAL_N)], batch_size=EVAL_B, shuffle=False)
    return labelled, pool


def _forward_only_passes(model, dev):
    from src.training.common import evaluate_model
    from src.training.semi_supervised import generate_pseudo_labels

    labelled, pool = _eval_loaders()
    _, yt, yp, prob, paths = evaluate_model(model, labelled, dev, pos_index=0)
    picks = generate_pseudo_labels(model, pool, dev, threshold=0.5)
    return {"y_pred": yp.tolist(), "y_prob": prob.tolist(), "paths": list(paths),
            "picks": [(p, int(l), float(c)) for p, l, c in picks]}


def _bench_worker(rank, world, port, out):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "semi-supervised-image-processing_amd"), str(root)]
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.training import distributed as D
        from ssip import SSIPResNet, replace_fc
        from ssip.dist import GradBucketer
        from ssip.semi_step import SemiStep

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.manual_seed(0)
        m = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev).train()
        D.broadcast_model(m)
        bucketer = GradBucketer(m.flatten_parameters())
        step = SemiStep(m, lr=1e-3, weight_decay=1e-4, tau=0.5, image_size=BS, bucketer=bucketer, seed=0, plan=True,
                        eager_warmup=1)
        x_l, y_l, x_u, params = _bench_data(rank)
        x_l, y_l, x_u = x_l.to(dev), y_l.to(dev), x_u.to(dev)
        res = {}
        for i in range(BSTEPS):
            step(x_l, y_l, x_u, params[i])
            if i == 0:
                torch.cuda.synchronize()
                res["grad0"] = step.arena.grad.detach().cpu().clone()
        torch.cuda.synchronize()
        res["flat"] = step.arena.flat.detach().cpu().clone()
        # per-rank running statistics (each from its own batches) before the sync
        res["buf_before"] = [b.detach().cpu().clone() for b in m.buffers()]
        D.sync_buffers(m)
        res["buf_after"] = [b.detach().cpu().clone() for b in m.buffers()]
        res["state"] = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        res.update(_forward_only_passes(m, dev))
        torch.save(res, os.path.join(out, f"bench_rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_semi_step_dp2_bench_geometry(dev, tmp_path):
    """2 ranks at the benchmarked per-rank workload (224²,
    128 + 128, launch plan, bucketed all-reduce from inside the backward):
      * the all-reduced gradient of step 1 = sum of the two single-process
        gradients (fp32 rounding of one add), identical on both ranks;
      * weights bitwise identical on both ranks after the steps;
      * BN running statistics differ per rank after training (local batch
        statistics) and are bitwise rank 0's on both ranks after sync_buffers;
      * the 2-rank sharded evaluate_model / generate_pseudo_labels equal the
        single-process passes of rank 0's model, bit for bit."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(400)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    r = [torch.load(tmp_path / f"bench_rank{k}.pt", weights_only=True) for k in (0, 1)]
    assert torch.equal(r[0]["flat"], r[1]["flat"])
    assert torch.equal(r[0]["grad0"], r[1]["grad0"])
    assert not all(torch.equal(a, b) for a, b in zip(r[0]["buf_before"], r[1]["buf_before"]))
    assert all(torch.equal(a, b) for a, b in zip(r[0]["buf_after"], r[1]["buf_after"]))
    assert all(torch.equal(a, b) for a, b in zip(r[0]["buf_before"], r[0]["buf_after"]))
    # the reduced gradient = the sum of the per-rank single-process gradients
    from ssip import SSIPResNet, replace_fc
    from ssip.semi_step import SemiStep

    singles = []
    for rank in (0, 1):
        torch.manual_seed(0)
        m = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev).train()
        step = SemiStep(m, lr=1e-3, weight_decay=1e-4, tau=0.5, image_size=BS, seed=0)
        x_l, y_l, x_u, params = _bench_data(rank)
        step(x_l.to(dev), y_l.to(dev), x_u.to(dev), params[0])
        torch.cuda.synchronize()
        singles.append(step.arena.grad.detach().cpu().clone())
        del step, m
    want = singles[0] + singles[1]
    err = ((r[0]["grad0"] - want).abs().max() / want.abs().max()).item()
    assert err <= 1e-6, err
    # single process, rank 0's model (weights + synced buffers)
    torch.manual_seed(0)
    m = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev)
    m.load_state_dict(r[0]["state"])
    single = _forward_only_passes(m, dev)
    for k in ("y_pred", "y_prob", "paths", "picks"):
        assert r[0][k] == single[k], k
        assert r[1][k] == single[k], k


_BWD = ("dgrad", "wgrad")


def _overlap_worker(rank, world, port, out):
    """Eager steps, then a plan recording and replays, logging host-side order:
    every C-ABI launch (eager) / every plan segment's launches (replay) and
    every bucket all-reduce launch."""
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "semi-supervised-image-processing_amd"), str(root)]
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ssip import _lib, ops
        from ssip import plan as P

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        step = _make(dev, bucketer_world=True, plan=True)
        bk = step.bucketer
        log = []            # eager: ("call", name) / ("ar", bucket)
        seg_names = [[]]    # plan recording: launch names per segment
        cur = {"seg": None}  # plan replay: the segment whose callback is running

        real_call = _lib.call

        def call(name, *a):
            log.append(("call", name))
            return real_call(name, *a)

        _lib.call = ops.call = call
        real_on_call, real_cb = P.PlanRecorder.on_call, P.PlanRecorder.callback

        def on_call(self, name, args):
            seg_names[-1].append(name)
            return real_on_call(self, name, args)

        def callback(self, fn, args):
            seg_names.append([])
            return real_cb(self, fn, args)

        P.PlanRecorder.on_call, P.PlanRecorder.callback = on_call, callback

        def replay(self):
            lib = _lib.lib()
            for seg in range(self.segments):
                _lib.check(lib.ssip_plan_run(self.handle, seg), "ssip_plan_run")
                if seg < len(self.callbacks):
                    cur["seg"] = seg
                    fn, args = self.callbacks[seg]
                    fn(*args)
                    cur["seg"] = None

        P.Plan.replay = replay
        real_launch = bk._launch

        def launch(b):
            if not bk.launched[b]:
                log.append(("ar", b, cur["seg"]))
            return real_launch(b)

        bk._launch = launch
        real_reset = bk.reset

        def reset():
            log.append(("reset",))
            return real_reset()

        bk.reset = reset
        x_l, y_l, x_u, params = _data(rank)
        x_l, y_l, x_u = x_l.to(dev), y_l.to(dev), x_u.to(dev)
        for i in range(STEPS):
            step(x_l, y_l, x_u, params[i])
        torch.cuda.synchronize()
        assert step._plan is not None
        torch.save({"log": log, "seg_names": seg_names, "nbuckets": len(bk.buckets),
                    "trains": [bk.trains(b) for b in range(len(bk.buckets))]},
                   os.path.join(out, f"overlap{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_allreduce_overlaps_backward(dev, tmp_path):
    """north_star's "RCCL gradient all-reduce ... overlapped with backward" as a
    tested property (the loop being sharded: reference
    src/training/common.py:376-387).  2 ranks over gloo, SemiStep with 8 MiB
    buckets, eager steps and launch-plan replays: every bucket's all-reduce
    but the last is enqueued while backward work (a dgrad or wgrad launch) is
    still to be enqueued after it in the same step -- in eager steps counted in
    C-ABI launches, in plan replays in plan segments (the bucket launches from
    the callback after segment k; a later segment must still hold a dgrad /
    wgrad)."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(200)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank in (0, 1):
        r = torch.load(tmp_path / f"overlap{rank}.pt", weights_only=False)
        log, seg_names, nb = r["log"], r["seg_names"], r["nbuckets"]
        assert nb >= 3 and all(r["trains"])
        # one step per bucketer reset (eager steps, the recording step and
        # every replay reset it first)
        steps, cur_step = [], None
        for e in log:
            if e[0] == "reset":
                cur_step = []
                steps.append(cur_step)
            elif cur_step is not None:
                cur_step.append(e)
        eager_steps = checked_replays = 0
        for part in steps:
            ars = [(k, e) for k, e in enumerate(part) if e[0] == "ar"]
            if not ars:
                continue
            assert len(ars) == nb, (rank, "every bucket launches once per step", len(ars))
            if all(e[2] is None for _, e in ars):  # eager (or the recording step): C-ABI launches logged
                eager_steps += 1
                for k, e in ars[:-1]:
                    later = [x[1] for x in part[k + 1:] if x[0] == "call"]
                    assert any(t in n for n in later for t in _BWD), \
                        (rank, "bucket all-reduce enqueued after the backward's last launch", e[1])
            else:  # a replay: bucket launches from the callbacks between plan segments
                checked_replays += 1
                for _, e in ars[:-1]:
                    assert e[2] is not None
                    later = [n for sg in seg_names[e[2] + 1:] for n in sg]
                    assert any(t in n for n in later for t in _BWD), \
                        (rank, "bucket all-reduce launched after the backward's final segment", e[1], e[2])
        assert eager_steps >= 2 and checked_replays >= 1, (rank, eager_steps, checked_replays)
