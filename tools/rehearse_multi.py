"""Rehearsal of bench.py's multi-GPU legs on ONE GPU: 2 ranks (torch.distributed.run, gloo, both on cuda:0)
run the key-hash sharded C4 leg (router-owned keys) and the time-range sharded C5 / C5t legs at reduced batch
sizes.  The driver runs the
real thing (nccl, one GPU per rank) at round end; this checks the rank logic, exchange and timing code paths.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \
        tools/rehearse_multi.py
"""
import importlib
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    pkg = importlib.import_module("scotty-window-processor_amd")
    dev = torch.device("cuda", 0)
    c4 = bench.extra_c4(pkg, dev, 1 << 20, 1 << 16, 3, rank=rank, world=world, dist=dist)
    c5 = bench.extra_c5(pkg, dev, 1 << 22, 3, n_windows=100, lo=10_000, hi=200_000, rank=rank, world=world, dist=dist)
    c5t = bench.extra_c5t(pkg, dev, 1 << 20, 3, rank=rank, world=world, dist=dist)
    if rank == 0:
        print(json.dumps({"c4": c4, "c5": c5, "c5t": c5t}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
