"""Probe: can RCCL ("nccl" backend) run several ranks on the one GPU of a
gpurun box?  Spawns `--world` ranks on cuda:0, each all-reduces a tensor of
its rank id, prints one line per rank.  Used to decide whether the 2-rank
RCCL test (tests/test_gpu_rccl.py) can run on a 1-GPU box.

    timeout -k 10 90 python tools/rccl_probe.py --world 2
"""
import argparse
import os
import socket
import sys

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        t = torch.full((1 << 20,), float(rank + 1), device="cuda")
        dist.all_reduce(t)
        torch.cuda.synchronize()
        want = world * (world + 1) / 2
        print(f"rank {rank}: all_reduce -> {t[0].item()} (want {want}) ok={bool((t == want).all())}", flush=True)
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    a = ap.parse_args()
    print("torch", torch.__version__, "nccl version", torch.cuda.nccl.version(), flush=True)
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, a.world, port)) for r in range(a.world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(60)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    codes = [p.exitcode for p in procs]
    print("exit codes", codes, flush=True)
    sys.exit(0 if all(c == 0 for c in codes) else 1)


if __name__ == "__main__":
    main()
