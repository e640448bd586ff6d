"""2-rank rehearsal of the multi-GPU bench legs (gloo, both ranks on cuda:0 of a one-GPU box; the driver's N-GPU
run uses RCCL).  Launch: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1
--master-port P tools/rehearse_multi.py [batch].

Checks, for the legs bench.py runs at G > 1:
  * C5 / C5t go through ShardedSlicingWindowOperator.processChunk WITHOUT precomputed bounds, i.e. the real
    {n, first ts, last ts} all-gather of every chunk is inside the timed region, and every rank emits the same
    windows (row lists compared across ranks by an all-gather of their digests);
  * C4's routing (device split by owner rank + all-to-all of the records) is timed and reported as its own field.
Prints one JSON line per rank-0 with the timed fields."""
import hashlib
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def digest(rows):
    h = hashlib.sha256()
    for w in rows:
        h.update(repr(w.key()).encode())
    return int.from_bytes(h.digest()[:8], "little", signed=True)


def sharded_rows(pkg, torch, dist, dev, windows, aggs, batch, steps, rank, world, ts_of):
    op = pkg.ShardedSlicingWindowOperator(device=0)
    for a in aggs:
        op.addWindowFunction(a)
    op.setMaxLateness(1)
    for w in windows:
        op.addWindowAssigner(w)
    g = torch.Generator(device=dev)
    g.manual_seed(100 + rank)
    digs, nrows = [], 0
    for s in range(steps):
        ts = ts_of(s).to(dev)
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize(dev)
        op.processChunk(ts.data_ptr(), v.data_ptr(), batch, 0)
        rows = op.processWatermark(int(ts_of(s).max()) if world == 1 else ts_last(ts_of, s, world, dist))
        nrows += len(rows)
        digs.append(digest(rows))
    return digs, nrows


def ts_last(ts_of, s, world, dist):
    import torch
    t = torch.tensor([int(ts_of(s).max())], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def main():
    import torch
    import torch.distributed as dist
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    pkg = importlib.import_module("scotty-window-processor_amd")
    bench = importlib.import_module("bench")
    out = {"world": world, "batch_per_rank": batch}
    # C5 (count windows) and C5t (count + time windows): every rank the same windows
    Count, Time = pkg.WindowMeasure.Count, pkg.WindowMeasure.Time
    sizes = pkg.workloads.random_count_sizes(50, 10_000, 200_000, seed=10)
    cases = {
        "c5": ([pkg.TumblingWindow(Count, z) for z in sizes],
               lambda s: (torch.arange(batch, dtype=torch.int64) + rank * batch + s * world * batch) // 1000),
        "c5t": ([pkg.TumblingWindow(Count, 1000), pkg.SlidingWindow(Time, 60_000, 1000)],
                lambda s: torch.arange(batch, dtype=torch.int64) + rank * batch + s * world * batch),
    }
    for name, (wins, ts_of) in cases.items():
        digs, nrows = sharded_rows(pkg, torch, dist, dev, wins, [pkg.AGG_SUM_I32, pkg.AGG_COUNT], batch, 4, rank,
                                   world, ts_of)
        mine = torch.tensor(digs + [nrows], dtype=torch.int64)
        allv = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        same = all(torch.equal(allv[0], x) for x in allv)
        out[name + "_ranks_equal"] = bool(same)
        out[name + "_rows_rank0"] = int(allv[0][-1])
        if not same:
            raise SystemExit("rank windows differ on %s" % name)
    # the timed bench legs themselves (bounds exchange inside the timed region; routing as its own field)
    out["c5"] = bench.extra_c5(pkg, dev, batch, 3, warm=1, n_windows=50, lo=10_000, hi=200_000, rank=rank,
                               world=world, dist=dist)
    out["c5t"] = bench.extra_c5t(pkg, dev, batch, 3, warm=1, rank=rank, world=world, dist=dist)
    out["c4"] = bench.extra_c4(pkg, dev, batch, 1 << 16, 3, rank=rank, world=world, dist=dist)
    out["c4_routing"] = bench.c4_routing(pkg, dev, batch, 1 << 16, 2, rank, world, dist)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
