"""The sharded edge-decision protocol of scotty_shard_push / scotty_shard_commit (slicing_kernels.hip,
shard_export_kernel / shard_commit_kernel), restated in numpy and run on 2 gloo ranks on the CPU: each
rank derives its records from its arrival chunk only, the records are all-gathered, and the committed slice
edges must equal the slice starts the oracle (the reference's StreamSlicer, S/StreamSlicer.java:55-116)
produces for the whole stream.  No GPU: this pins the exchange algebra the GPU kernels implement."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import product
from specs import Tumbling, Sliding, Time, SUM

K = 4096  # candidate slots per rank


def next_grid(windows, x):  # min over windows of assignNextWindowStart (Tumbling / Sliding, x >= 0)
    return min(x + (w.a if w.kind == 0 else w.b) - x % (w.a if w.kind == 0 else w.b) for w in windows)


def local_records(ts, g, lateness):
    """This rank's records for candidate grid points g (ascending): chunk max, reached[k], f_loc[k]."""
    cmax = int(ts.max()) if len(ts) else -(1 << 63)
    pm = np.maximum.accumulate(ts) if len(ts) else ts
    reached = np.zeros(K, np.int64)
    floc = np.zeros(K, np.int64)
    for k, gk in enumerate(g):
        if gk > cmax:
            break
        e_idx = int(np.argmax(ts >= gk))                 # first local tuple reaching g_k
        m_loc = int(pm[e_idx - 1]) if e_idx > 0 else -(1 << 63)
        reached[k] = 1
        floc[k] = 1 if (k > 0 and g[k - 1] <= m_loc) or (int(ts[e_idx]) - gk < lateness) else 0
    return cmax, reached, floc


def commit(recs, g, prev_max):
    """Every rank: owner of g_k = first rank reaching it; emit iff k == 0 or its f_loc or g_{k-1} <= pre_owner."""
    pre, p = [], prev_max
    for cmax, _, _ in recs:
        pre.append(p)
        p = max(p, cmax)
    edges = []
    for k, gk in enumerate(g):
        if gk > p:
            break
        for r, (_, reached, floc) in enumerate(recs):
            if reached[k]:
                if k == 0 or floc[k] or g[k - 1] <= pre[r]:
                    edges.append(gk)
                break
    return edges, p


def _worker(rank, world, port, out):
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    from oracle.oracle import OracleOperator
    wl = product().workloads
    failures = []
    for seed in range(12):
        rng = np.random.default_rng(seed)
        if seed < 6:   # dense streams
            wins = [Tumbling(Time, int(rng.integers(50, 400)) | 1), Sliding(Time, 1200, int(rng.integers(30, 200)) | 1)]
            lateness = int(rng.choice([1, 20, 300]))
            ts, _ = wl.stream(60_000, [5, 20][seed % 2], t0=1000, ooo_frac=[0.0, 0.2][seed % 2],
                              max_delay=int(rng.integers(1, 400)), seed=seed,
                              gaps=[(i, int(rng.integers(10, 2000))) for i in range(3000, 60_000, 9000)])
        else:          # sparse streams: tuples jump over grid points by more than maxLateness at chunk cuts
            wins = [Tumbling(Time, int(rng.integers(2, 9)) | 1), Sliding(Time, 40, int(rng.integers(3, 12)) | 1)]
            lateness = int(rng.choice([1, 2, 3]))
            ts, _ = wl.stream(4000, [0.1, 0.25][seed % 2], t0=1000, ooo_frac=[0.0, 0.1][seed % 2], max_delay=3,
                              seed=seed)
            ts = ts + np.cumsum(rng.integers(0, 4, size=len(ts)))
        ora = OracleOperator()
        ora.addWindowFunction(SUM)
        ora.setMaxLateness(lateness)
        for w in wins:
            ora.addWindowAssigner(w)
        ora.processElements(ts[:1], np.zeros(1, np.int64))          # first tuple: the first-edge walk
        starts = [ora.slice(i).t_start for i in range(ora.store_size())]
        prev_max = int(ts[0])
        pending = next_grid(wins, prev_max)
        nb = 8 if seed < 6 else 200
        bounds = np.linspace(1, len(ts), nb + 1).astype(np.int64)     # global micro-batches
        for b in range(nb):
            lo, hi = int(bounds[b]), int(bounds[b + 1])
            cuts = np.linspace(lo, hi, world + 1).astype(np.int64)
            g = [pending]
            while len(g) < K and g[-1] <= max(prev_max, int(ts[lo:hi].max())):
                g.append(next_grid(wins, g[-1]))
            mine = ts[int(cuts[rank]):int(cuts[rank + 1])]
            cmax, reached, floc = local_records(mine, g, lateness)
            rec = torch.tensor(np.concatenate([[cmax], reached, floc]), dtype=torch.int64)
            allr = [torch.empty_like(rec) for _ in range(world)]
            dist.all_gather(allr, rec)
            recs = [(int(t[0]), t[1:1 + K].numpy(), t[1 + K:].numpy()) for t in allr]
            edges, prev_max = commit(recs, g, prev_max)
            starts += [int(e) for e in edges if e >= 0]
            n_cand = sum(1 for x in g if x <= prev_max)
            pending = g[n_cand] if n_cand < len(g) else next_grid(wins, g[-1])
            ora.processElements(ts[lo:hi], np.zeros(hi - lo, np.int64))
            want = [ora.slice(i).t_start for i in range(ora.store_size())]
            if starts != want:
                failures.append((seed, b, len(starts), len(want)))
                break
    with open(out + ".%d" % rank, "w") as f:
        f.write(repr(failures))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_edge_protocol_two_gloo_ranks_matches_oracle():
    out = os.path.join(tempfile.mkdtemp(), "r")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        assert open(out + ".%d" % r).read() == "[]"
