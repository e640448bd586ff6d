"""One rank of a sharded non-keyed run (launched by tests/test_gpu_shard.py through torch.distributed.run).
Every rank feeds its arrival chunk of each global micro-batch and writes the windows of every watermark to
<out>.rank<r> (every rank holds the same slice store, so every rank's rows are checked).  RCCL ("nccl"): no
synchronisation by the test between chunks (and, unless SCOTTY_SHARD_SYNC=1, none by the operator: the exchange is
ordered by events); the exchange buffer is poisoned on torch's stream before each chunk, so
a commit that read it before the collective landed would fold garbage and fail the oracle comparison."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from helpers import product  # noqa: E402
from shard_cases import case  # noqa: E402


def main():
    out, cid = sys.argv[1], int(sys.argv[2])
    backend = sys.argv[3] if len(sys.argv) > 3 else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    pkg = product()
    cfg, ts, vals, sched = case(cid)
    op = pkg.ShardedSlicingWindowOperator(device=0)
    for a in cfg["aggs"]:
        op.addWindowFunction(a)
    if cfg.get("lateness") is not None:
        op.setMaxLateness(cfg["lateness"])
    for w in cfg["windows"]:
        op.addWindowAssigner(w)
    dev = torch.device("cuda", 0)
    res = []
    for st in sched:
        if st[0] == "push":
            lo, hi = st[1], st[2]
            cuts = np.linspace(lo, hi, world + 1).astype(np.int64)
            a, b = int(cuts[rank]), int(cuts[rank + 1])
            t = torch.tensor(ts[a:b], dtype=torch.int64, device=dev)
            v = torch.tensor(vals[a:b], dtype=torch.int32, device=dev)
            if backend == "nccl":
                _, gb = op._bufs()
                gb.fill_(-0x5A5A5A5A5A5A5A5A)  # poison: overwritten by the all-gather before the commit may read it
                torch.cuda.synchronize(dev)  # (the fill runs on torch's stream, the exchange on the op's own)
            # (t and v are dropped at the next push: their memory goes back to torch's allocator while the op's
            # stream may still read them -- the operator orders torch's stream after the chunk, so the reuse waits)
            op.processChunk(t.data_ptr(), v.data_ptr(), b - a, int(ts[0]))
            if backend != "nccl":
                torch.cuda.synchronize(dev)
        else:
            try:
                ws = op.processWatermark(st[1])
            except pkg.ScottyError as e:  # IndexOutOfBoundsException in the reference: the test expects it too
                if e.code != -5:
                    raise
                res.append([["index_error"]])
                continue
            res.append([list(w.key()[:4]) + [list(w.key()[4])] for w in ws] + [["dropped", op.droppedCount()]])
    json.dump(res, open("%s.rank%d" % (out, rank), "w"))
    with open("%s.rank%d.mode" % (out, rank), "w") as f:
        f.write("async" if op.async_exchange else "sync")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
