"""North-star benchmark: semi-supervised train-step images/sec, ResNet-18,
224x224, 256 images per GPU per step (128 labelled + 128 unlabelled, weak +
strong views, FixMatch-style consistency loss), bf16 activations with fp32
accumulation / master weights, synthetic uint8 inputs resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One step = GPU augment of 3 views (384 images) + weak forward (128, no grad,
on a second stream) + train forward/backward (256; weight gradients on a
side stream) + bucketed RCCL all-reduce launched from inside the backward
(N > 1) + fused AdamW.  Launches are eager by default (`--graph` replays one
captured hipGraph instead: HIP serialises a graph's parallel branches, so it
is slower here).  `value` = images (labelled + unlabelled) all ranks consumed / the
max-over-ranks wall time of the K timed steps.  The `roofline` object is the
conv implicit-GEMM kernel family (fwd + dgrad + wgrad launches of one step),
timed with HIP events on the launch stream; `cpu_baseline` is the oracle's
CPU restatement of the same step (oracle/step_oracle.py) on rank 0.
"""
from __future__ import annotations

import argparse
import glob
import json
import re
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "semi-supervised-image-processing_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

GFLOP_PER_IMG_TRAIN = 10.64535   # R18 224² fwd+dgrad+wgrad (no stem dgrad)
GFLOP_PER_IMG_FWD = 3.627125
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}  # MI355X dense MFMA (MI355X_MICROARCH.md)
HBM_PEAK_BPS = 8.0e12  # MI355X HBM3E spec peak (MI355X_MICROARCH.md; 6.29 TB/s measured copy)


def _round_of(path: str) -> int:
    m = re.match(r"r(\d+)_", os.path.basename(path))
    return int(m.group(1)) if m else -1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU per step (labelled + unlabelled)")
    ap.add_argument("--labeled", type=int, default=None, help="labelled images per GPU per step (default: batch / 2)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--serial-weak", action="store_true", help="run the weak forward on the main stream (A/B)")
    ap.add_argument("--arch", default="resnet18", choices=["resnet18", "resnet50"],
                    help="resnet50 + --image-size 512 --batch 128 = BASELINE config 5 (per GPU)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--exec", dest="mode", default="plan", choices=["eager", "plan", "graph"],
                    help="eager: Python enqueues every launch; plan: one step recorded, then replayed from C++ "
                         "(ssip/plan.py, same streams and overlap); graph: one captured hipGraph per step (HIP runs "
                         "a graph's parallel branches one after another)")
    ap.add_argument("--graph", action="store_true", help="= --exec graph (older command lines)")
    ap.add_argument("--eager", action="store_true", help="= --exec eager (older command lines)")
    ap.add_argument("--workload", default="semi", choices=["semi", "extract"],
                    help="semi: the north-star train step (default); extract: src.feature_extraction's frozen "
                         "ResNet-18 embedding pass (the reference's only published throughput, 358.6 images/s)")
    ap.add_argument("--extract-images", type=int, default=1506, help="images of the end-to-end extraction run")
    ap.add_argument("--cpu-warmup", type=int, default=10,
                    help="CPU-baseline warm-up steps (BASELINE.md section 3: >= 10)")
    ap.add_argument("--cpu-steps", type=int, default=50, help="CPU-baseline timed steps, median reported "
                    "(BASELINE.md section 3: >= 50)")
    ap.add_argument("--cpu-budget-s", type=float, default=340.0,
                    help="stop the CPU-baseline timed steps after this much wall time (the count timed is reported)")
    ap.add_argument("--cpu-batch", type=int, default=None,
                    help="images per CPU-baseline step (default: the GPU batch; 16 for resnet50 at 512, where one "
                         "full 128-image CPU step takes minutes)")
    ap.add_argument("--profile-leg", default=None, choices=["full", "production"],
                    help="profiling run (no JSON line): warm-up, then --steps repetitions of that roofline leg "
                         "alone, without event timers, for rocprofv3 --kernel-trace / --pmc "
                         "(tools/roofline_from_trace.py takes the last complete step)")
    ap.add_argument("--sclk-out", default=None,
                    help="--profile-leg: write the legs' mean SCLK (amdsmi, the bench line's sampler) to this JSON "
                         "file, so a trace's MFMA busy is normalised by its own box's clock")
    ap.add_argument("--max-inflight", type=int, default=None,
                    help="host waits for step k - N before enqueueing step k (0: never; default: SemiStep's own "
                         "bound on launch-plan replays, $SSIP_MAX_INFLIGHT or 2)")
    return ap.parse_args()


def host_cores() -> dict:
    """The host cores this process can actually run on: the affinity mask,
    capped by a cgroup CPU quota when one is set (a GPU box's CPU share can be
    a quota over a machine-wide affinity mask).  An inherited OMP_NUM_THREADS
    does not cap it."""
    avail = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    cores = avail if quota is None else max(1, min(avail, int(quota + 0.5)))
    return {"cores": cores, "affinity": avail, "cgroup_quota": quota, "total": os.cpu_count()}


class SclkSampler:
    """Mean graphics clock (SCLK, MHz) of the bench's GPU over a timed region,
    sampled every 5 ms from the SMU (amdsmi, by the device's PCI address).  A
    box indicator only: the in-kernel clock under MFMA load can read up to
    ~10 % below it (MI355X_MICROARCH.md, DVFS give-back)."""

    def __init__(self, dev_index: int):
        import threading

        self.samples, self._stop, self.source, self.err = [], threading.Event(), None, None
        try:
            import amdsmi

            p = torch.cuda.get_device_properties(dev_index)
            bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
            amdsmi.amdsmi_init()
            self._h = amdsmi.amdsmi_get_processor_handle_from_bdf(bdf)
            self._read = lambda: float(amdsmi.amdsmi_get_clock_info(self._h, amdsmi.AmdSmiClkType.SYS)["clk"])
            self._read()
            self.source = f"amdsmi SYS clock of {bdf}"
        except Exception as e:  # no SMU access on this box: report null
            self._read, self.err = None, f"{type(e).__name__}: {e}"[:120]
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            try:
                self.samples.append(self._read())
            except Exception:
                pass
            self._stop.wait(0.005)

    def __enter__(self):
        if self._read is not None:
            self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._read is not None:
            self._t.join()

    def summary(self):
        if not self.samples:
            return {"mean_mhz": None, "source": self.source, "error": self.err}
        v = self.samples
        return {"mean_mhz": round(sum(v) / len(v), 1), "min_mhz": min(v), "max_mhz": max(v), "samples": len(v),
                "source": self.source}


def extract_bench(args):
    """Feature extraction (src.feature_extraction, BASELINE config 1's pass):
    frozen eval-mode ResNet-18 -> 512-D avgpool embeddings, Resize(256) ->
    CenterCrop(224) on the device, batch 32.  Two measurements:
      value      = end to end from JPEG files on local disk (synthetic 512x512
                   RGB JPEGs, the dataset's shape): decode on the host threads,
                   uint8 H2D, GPU transform, forward, D2H of the embeddings --
                   the same span as the reference's published 4.20 s for 1,506
                   images (outputs/logs/feature_extraction.log:3-5)
      device_resident = the same forward with the uint8 batch already in HBM."""
    import tempfile

    import numpy as np
    from PIL import Image

    from ssip.augment import GpuTransform
    from src import feature_extraction as FE

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bs, dt = 32, args.dtype
    model = FE.load_model(dev, dt, None, allow_random_init=True)
    tf = FE.build_transform(model.compute_dtype)
    g = torch.Generator().manual_seed(7)
    u8 = torch.randint(0, 256, (bs, 512, 512, 3), generator=g, dtype=torch.uint8).to(dev)
    with torch.no_grad():
        for _ in range(max(3, args.warmup)):
            model(tf(u8))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            feats = model(tf(u8))
        torch.cuda.synchronize()
        dt_dev = (time.perf_counter() - t0) / args.steps
    n = args.extract_images
    with tempfile.TemporaryDirectory() as td:
        root = os.path.join(td, "mri", "sans_label")
        os.makedirs(root)
        rng = np.random.default_rng(0)
        base = rng.integers(0, 256, (8, 512, 512, 3), dtype=np.uint8)
        for i in range(n):
            Image.fromarray(np.roll(base[i % 8], i, axis=1)).save(os.path.join(root, f"{i:05d}.jpg"), quality=90)
        recs = FE.discover_image_records(Path(td) / "mri")
        threads = min(16, len(os.sched_getaffinity(0)))
        FE.extract_embeddings(recs[:64], dev, batch_size=bs, dtype=dt, decode_threads=threads,
                              allow_random_init=True)  # warm-up
        t0 = time.perf_counter()
        res = FE.extract_embeddings(recs, dev, batch_size=bs, dtype=dt, decode_threads=threads,
                                    allow_random_init=True)
        e2e = time.perf_counter() - t0
    assert res.embeddings.shape == (n, 512)
    out = {
        "metric": "images/sec feature extraction (frozen ResNet-18, 512-D embeddings), 224x224 bs=32, 1 MI355X",
        "value": round(n / e2e, 2), "unit": "images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "higher_is_better": True, "scaling": "none", "vs_baseline": round(n / e2e / 358.6, 3), "dtype": dt,
        "data": f"{n} synthetic 512x512 RGB JPEGs (quality 90) on local disk, decoded on {threads} host threads; "
                f"seeded random-init ResNet-18",
        "config": {"workload": "feature_extraction_resnet18_224", "batch": bs, "images": n,
                   "decode_threads": threads},
        "device_resident": {"value": round(bs / dt_dev, 1), "unit": "images/s", "ms_per_batch": round(dt_dev * 1e3, 3),
                            "tflops": round(bs * GFLOP_PER_IMG_FWD / dt_dev / 1e3, 1),
                            "note": "uint8 [32,512,512,3] already in HBM: GPU transform + forward only "
                                    "(3.627 GFLOP/img, SURVEY 8d)"},
        "baseline_note": "358.6 images/s = the reference's own end-to-end run (1,506 images in 4.20 s on an "
                         "unnamed CUDA GPU, outputs/logs/feature_extraction.log:3-5)",
    }
    del feats
    print(json.dumps(out))


def roofline_leg(step, x_l, y_l, x_u, kind, ops, resnet_mod, timer=True, lead=2):
    """One step with every launch on one stream and (timer) HIP events around
    every conv launch.  kind "full": the wgrads at their full-chip grids;
    "production": with the side stream's grid budgets.  Two unsynchronised
    steps are queued first so the host enqueues the eager instrumented step
    while the device is still busy: each event bracket then holds its
    kernel's execution, not device idle time waiting for the host's next
    launch (the brackets agree with rocprofv3's kernel durations,
    profiles/r5_roofline_leg_*.txt)."""
    for _ in range(lead):
        step(x_l, y_l, x_u)
    t = ops.ConvTimer() if timer else None
    ops.set_conv_timer(t)
    saved = (step.graph, step.plan, step.overlap, resnet_mod.WGRAD_SIDE_STREAM, resnet_mod.WGRAD_BUDGET_SERIAL)
    # every launch on one stream: an event bracket must not include queueing
    # behind a kernel of another stream (weak forward, side-stream wgrads)
    step.graph, step.plan, step.overlap = False, False, False
    resnet_mod.WGRAD_SIDE_STREAM = False
    resnet_mod.WGRAD_BUDGET_SERIAL = kind == "production"
    try:
        step(x_l, y_l, x_u)
    finally:
        (step.graph, step.plan, step.overlap, resnet_mod.WGRAD_SIDE_STREAM,
         resnet_mod.WGRAD_BUDGET_SERIAL) = saved
        ops.set_conv_timer(None)
    torch.cuda.synchronize()
    return {"summary": t.summary(), "timer": t} if t is not None else None


def main():
    args = parse()
    if args.workload == "extract":
        return extract_bench(args)
    from ssip import SSIPResNet, ops, replace_fc
    from ssip import resnet as resnet_mod
    from ssip.dist import GradBucketer, init_from_env
    from ssip.semi_step import SemiStep

    rank, world, local = init_from_env()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    prio = int(os.environ.get("SSIP_MAIN_PRIO", "-1"))
    if prio:
        # the step's critical path (train forward, BN / dgrad chain) on a
        # higher-priority queue than the weak-forward and wgrad side streams:
        # their workgroups no longer delay its short BN / finalize launches
        # (A/B, 6 + 6 alternated runs on one box: 7.119 -> 7.024 ms/step;
        # SSIP_MAIN_PRIO=0 keeps the default stream)
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=prio))
    Bl = args.labeled if args.labeled is not None else args.batch // 2
    Bu = args.batch - Bl
    torch.manual_seed(42)
    model = replace_fc(SSIPResNet(args.arch, 1000, dtype=args.dtype), 2).to(dev).train()
    if world > 1:
        # identical initial weights on every rank (rank 0 broadcasts)
        arena = model.flatten_parameters()
        dist.broadcast(arena.flat, 0)
        for b in model.buffers():
            dist.broadcast(b, 0)
    bucketer = GradBucketer(model.flatten_parameters()) if world > 1 else None
    S = args.image_size
    mode = "graph" if args.graph else "eager" if args.eager else args.mode
    step = SemiStep(model, lr=1e-4, weight_decay=1e-4, tau=0.7, image_size=S, bucketer=bucketer, seed=rank,
                    graph=mode == "graph", plan=mode == "plan")
    step.overlap = not args.serial_weak

    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    x_l = torch.randint(0, 256, (Bl, S, S, 3), generator=g, dtype=torch.uint8).to(dev)
    x_u = torch.randint(0, 256, (Bu, S, S, 3), generator=g, dtype=torch.uint8).to(dev)
    y_l = torch.randint(0, 2, (Bl,), generator=g).to(dev)

    for _ in range(args.warmup):
        step(x_l, y_l, x_u)
    if args.profile_leg:
        with SclkSampler(local) as sclk:
            for _ in range(args.steps):
                # every step of the trace after the warm-up is a leg step (no lead-in
                # replays): the profile tools take the last complete one
                roofline_leg(step, x_l, y_l, x_u, args.profile_leg, ops, resnet_mod, timer=False, lead=0)
        sc = sclk.summary()
        print(f"profile-leg {args.profile_leg}: {args.steps} legs done; sclk {json.dumps(sc)}", file=sys.stderr)
        if args.sclk_out:
            with open(args.sclk_out, "w") as f:
                json.dump({"leg": args.profile_leg, "steps": args.steps, "sclk": sc}, f)
        return
    slots = step.input_slots()
    if slots is not None and os.environ.get("SSIP_NO_INPUT_SLOTS") != "1":
        # the synthetic batch written once into the buffers the recorded plan
        # reads (where an input pipeline would land each batch): no copy-in
        for dst, src in zip(slots, (x_l, y_l, x_u)):
            dst.copy_(src)
        x_l, y_l, x_u = slots
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if args.max_inflight is not None:
        step.max_inflight = args.max_inflight
    with SclkSampler(local) as sclk:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step(x_l, y_l, x_u)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss = out.loss.cpu().tolist()

    # step boundaries (after the timed region, same replay path): events on the
    # launch stream at each step's start and end; the stream's idle time
    # between one step's last launch and the next step's first is the time the
    # device waited for the host, and the host's own enqueue time per step
    bounds, enq = [], []
    for _ in range(8):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        h0 = time.perf_counter()
        step(x_l, y_l, x_u)
        enq.append(time.perf_counter() - h0)
        e1.record()
        bounds.append((e0, e1))
    torch.cuda.synchronize()
    gaps = sorted(bounds[i][1].elapsed_time(bounds[i + 1][0]) * 1e3 for i in range(len(bounds) - 1))
    enq.sort()
    boundary = {"gap_us_median": round(gaps[len(gaps) // 2], 1), "gap_us_max": round(gaps[-1], 1),
                "host_enqueue_ms_median": round(enq[len(enq) // 2] * 1e3, 3),
                "note": "launch-stream idle between consecutive steps (event after step k's last launch to "
                        "event before step k+1's first), 8 untraced steps after the timed region; "
                        "host_enqueue_ms is the host time of one step call, which includes the wait for the "
                        "replay two steps back (the in-flight bound), so it equals the device step time once the "
                        "host is ahead"}

    # roofline legs (one instrumented step each, bench_roofline_leg): "full" --
    # the conv family's own rate, every launch at its full-chip grid -- is the
    # line's `frac`; "production" keeps the side-stream wgrads' grid budgets
    # (one workgroup per CU; half the CUs for the layer-1 wgrad) that the
    # overlapped step actually runs, serialised, as `frac_production`
    legs = {}
    for kind in ("production", "full"):
        legs[kind] = roofline_leg(step, x_l, y_l, x_u, kind, ops, resnet_mod)
    summ = legs["full"]["summary"]
    timer = legs["full"]["timer"]
    conv_flops = sum(v[0] for v in summ.values())
    conv_ms = sum(v[1] for v in summ.values())
    conv_launches = sum(v[2] for v in summ.values())
    conv_bytes = sum(v[3] for v in summ.values())
    achieved = conv_flops / (conv_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    # per-launch speed of light: max(FLOPs / MFMA peak, algorithmic bytes / HBM peak)
    # -- layer 1's 64-channel convs sit below the ridge point (~310 FLOP/B), HBM-bound
    sol_s, meas_s = timer.sol(peak * 1e12, HBM_PEAK_BPS)
    psumm = legs["production"]["summary"]
    prod_ms = sum(v[1] for v in psumm.values())
    prod_achieved = sum(v[0] for v in psumm.values()) / (prod_ms * 1e-3) / 1e12
    by_pass = {k: {"tflop": round(v[0] / 1e12, 4), "ms": round(v[1], 3), "launches": v[2],
                   "tflops": round(v[0] / (v[1] * 1e-3) / 1e12, 1)} for k, v in sorted(summ.items())}

    # HBM traffic of the same family from the committed rocprofv3 PMC passes of
    # THIS workload (tools/pmc_traffic.py: FETCH_SIZE*2 + WRITE_SIZE, separate
    # passes, per step): counters cannot be read from inside the run itself, so
    # a file is used only when its `_workload` key equals this run's; else null
    workload_key = f"semi_consistency_{args.arch}_{S} bs{args.batch} labeled{Bl} {args.dtype}"
    traffic, traffic_src = None, None
    for pmc in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                             "r*_pmc_traffic.json")), key=_round_of):
        with open(pmc) as f:
            d = json.load(f)
        if d.get("_workload") == workload_key:
            traffic, traffic_src = d.get("conv", {}).get("total_bytes"), os.path.basename(pmc)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.step_oracle import time_cpu_step

        # one thread per host core this process may use
        hc = host_cores()
        cb = args.cpu_batch or (16 if (args.arch, S) == ("resnet50", 512) else args.batch)
        cbl = max(1, cb * Bl // args.batch)
        c = time_cpu_step(Bl=cbl, Bu=cb - cbl, steps=args.cpu_steps, warmup=args.cpu_warmup, threads=hc["cores"],
                          arch=args.arch, size=S, budget_s=args.cpu_budget_s)
        full = c["warmup"] >= 10 and c["steps_timed"] >= 50
        cpu = {"value": round(c["value"], 3), "unit": "images/s", "cores": c["threads"], "kind": "port",
               "threads": c["threads"], "host_cores": hc["cores"], "host_cpus_affinity": hc["affinity"],
               "host_cgroup_quota": hc["cgroup_quota"], "host_cpus_total": hc["total"],
               "model": args.arch, "image_size": S, "batch": cb,
               "sample": c["sample"] + ("" if full else
                                        f"; BASELINE.md section 3 asks >= 10 warm-up + >= 50 timed steps: "
                                        f"{c['steps_timed']} fitted the --cpu-budget-s {args.cpu_budget_s:g} s "
                                        "bound on the bench's run time")
                         + ("" if cb == args.batch else f"; {cb} images per CPU step (the GPU step's "
                                                        f"{args.batch} take minutes per CPU step), rate per image"),
               "step_times_s": [round(t, 3) for t in c["step_times_s"]]}

    if rank == 0:
        imgs = args.batch * world * args.steps
        value = imgs / elapsed
        res = {
            "metric": "images/sec semi-supervised train step, 224x224 bs=256, 1/2/4/8 MI355X"
                      if (args.arch, S, args.batch) == ("resnet18", 224, 256) else
                      f"images/sec semi-supervised train step, {args.arch} {S}x{S} bs={args.batch}",
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": f"synthetic uint8 {S}x{S}x3 images resident in HBM, random-init {args.arch} (seed 42)",
            "config": {"workload": f"semi_consistency_{args.arch}_{S}",
                       "model": args.arch, "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "labeled_per_gpu": Bl, "unlabeled_per_gpu": Bu, "image_size": S,
                       "parallelism": f"dp{world}", "tau": 0.7,
                       "gflop_per_step_per_gpu": round(Bl * GFLOP_PER_IMG_TRAIN + Bu * (GFLOP_PER_IMG_FWD
                                                                                        + GFLOP_PER_IMG_TRAIN), 1)
                       if (args.arch, S) == ("resnet18", 224) else round(conv_flops / 1e9, 1)},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4), "traffic": traffic,
                         "traffic_note": ("bytes per step for the same conv family, PMC FETCH_SIZE*2 + WRITE_SIZE "
                                          f"(profiles/{traffic_src}; Infinity-Cache hits are counted)")
                         if traffic_src else f"no committed PMC passes for workload '{workload_key}'",
                         "kernel": "conv family: conv_glds / conv_halo / conv_stem_halo / conv_halo_wgrad / "
                                   "conv_stem_bwd_wgrad (fwd+dgrad+wgrad, incl. wgrad slab reduce), "
                                   f"{conv_launches} launches/step, {conv_flops / 1e12:.3f} TFLOP/step "
                                   f"in {conv_ms:.3f} ms (single stream, every launch at its full-chip grid; "
                                   "rocprofv3 of this leg: `python bench.py --profile-leg full`, "
                                   "tools/roofline_from_trace.py)",
                         "by_pass": by_pass,
                         "frac_production": round(prod_achieved / peak, 4),
                         "production": {"achieved": round(prod_achieved, 1), "ms": round(prod_ms, 3),
                                        "note": "the same launches with the side-stream wgrads' grid budgets "
                                                "the overlapped step runs (one workgroup per CU; half the CUs for "
                                                "the layer-1 wgrad), still serialised on one stream: "
                                                "`python bench.py --profile-leg production`"},
                         "sol": {"frac": round(sol_s / meas_s, 4), "sol_ms": round(sol_s * 1e3, 3),
                                 "algorithmic_bytes": conv_bytes, "hbm_peak_gbps": HBM_PEAK_BPS / 1e9,
                                 "note": "sum over the same launches of max(FLOPs / MFMA peak, algorithmic bytes / "
                                         "HBM peak) divided by their measured time: the fraction of each launch's "
                                         "own roofline (HBM-bound below ~312 FLOP/B)"}},
            "cpu_baseline": cpu,
            "sclk": sclk.summary(),
            "step_boundary": boundary,
            "last_loss": [round(v, 5) for v in loss],
        }
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
