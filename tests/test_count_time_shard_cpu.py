"""The per-chunk time-edge decision of the sharded count path (CEngine::time_edges with a ShardTime, count_tcand_kernel's
rule), restated in numpy and run on 2 gloo ranks on the CPU: every rank replays the stream's first-tuple edge walk,
decides only the grid points in (max ts before its chunk, chunk max] from its own tuples plus the two gathered
timestamp bounds, and the rank-ordered union of the decided edges must equal the slice starts the oracle (the
reference's StreamSlicer on the whole in-order stream, S/StreamSlicer.java:46-116) produces.  No GPU."""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from specs import Tumbling, Sliding, Time, SUM

JMIN = -(1 << 63)


def next_grid(windows, x):  # min over windows of assignNextWindowStart (Tumbling / Sliding, x >= 0)
    return min(x + (w.a if w.kind == 0 else w.b) - x % (w.a if w.kind == 0 else w.b) for w in windows)


def first_walk(windows, te, lateness):
    """calculateNextFixedEdge from min_next_edge_ts = Long.MIN_VALUE (x >= 0 streams: no wrap-around)."""
    edges, n = [], next_grid(windows, te - lateness)
    while te > n:
        if n >= 0:
            edges.append(n)
        n = next_grid(windows, max(te - lateness, n))
    if n == te:
        edges.append(n)
        n = next_grid(windows, max(te - lateness, n))
    return edges, n


def chunk_edges(ts, start, prev, pending, batch_last, windows, lateness):
    """Edges this chunk appends from position `start`: candidates are the grid points from the pending edge up to the
    batch max, those in (prev, chunk max] are decided here (the first one always, later ones iff the running max
    before their first tuple reached the previous point or that tuple lies within maxLateness)."""
    cand, g, n_all = [], pending, 0
    while g <= batch_last:
        n_all += 1
        if g > prev and start < len(ts) and g <= ts[-1]:
            cand.append(g)
        g = next_grid(windows, g)
    new_pending = g if n_all else pending
    out = []
    for k, gk in enumerate(cand):
        p = start + int(np.searchsorted(ts[start:], gk, side="left"))
        e = int(ts[p])
        m = int(ts[p - 1]) if p > start else prev
        if (k == 0 or cand[k - 1] <= m or e - gk < lateness) and (gk >= 0 or e == gk):
            out.append(gk)
    return out, new_pending


def _worker(rank, world, port, out):
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    from oracle.oracle import OracleOperator
    failures = []
    for seed in range(10):
        rng = np.random.default_rng(700 + seed)
        wins = [Tumbling(Time, int(rng.integers(3, 40)) | 1), Sliding(Time, 200, int(rng.integers(3, 30)) | 1)]
        lateness = int(rng.choice([0, 1, 5, 60]))
        n = 6000
        ts = 500 + np.sort(rng.integers(0, [3000, 60_000][seed % 2], size=n)).astype(np.int64)  # ties when dense
        ora = OracleOperator()
        ora.addWindowFunction(SUM)
        ora.setMaxLateness(lateness)
        for w in wins:
            ora.addWindowAssigner(w)
        starts, started, prev_max, pending = [], False, JMIN, None
        bounds = np.concatenate([[0, 1, 2, 5], np.linspace(9, n, 30).astype(np.int64)])
        for b in range(len(bounds) - 1):
            lo, hi = int(bounds[b]), int(bounds[b + 1])
            cuts = np.linspace(lo, hi, world + 1).astype(np.int64)
            a, z = int(cuts[rank]), int(cuts[rank + 1])
            mine = ts[a:z]
            # the pre-push all-gather: {n, first, last} per rank
            rec = torch.tensor([len(mine), int(mine[0]) if len(mine) else JMIN, int(mine[-1]) if len(mine) else JMIN],
                               dtype=torch.int64)
            allr = [torch.empty_like(rec) for _ in range(world)]
            dist.all_gather(allr, rec)
            g = [t.tolist() for t in allr]
            n_before = sum(x[0] for x in g[:rank])
            before = max([x[2] for x in g[:rank] if x[0] > 0], default=JMIN)
            batch_last = max([x[2] for x in g if x[0] > 0], default=JMIN)
            mine_edges, start, prev = [], 0, max(prev_max, before)
            if not started:
                walk, pending = first_walk(wins, int(ts[0]), lateness)
                if n_before == 0 and len(mine):
                    mine_edges, start = list(walk), 1
                prev = max(prev, int(ts[0]))
            e, pending = chunk_edges(mine, start, prev, pending, batch_last, wins, lateness)
            mine_edges += e
            prev_max = max(prev_max, batch_last)
            started = True
            # rank-ordered union (the commit's record order)
            m = torch.tensor([len(mine_edges)] + mine_edges + [0] * (4096 - len(mine_edges)), dtype=torch.int64)
            alle = [torch.empty_like(m) for _ in range(world)]
            dist.all_gather(alle, m)
            for t in alle:
                starts += t[1:1 + int(t[0])].tolist()
            if not starts:  # time windows only here: a tuple meeting an empty store opens a slice at 0
                starts = [0]  # (S/SliceManager.java:49-51; on the count path the first count edge precedes it)
            ora.processElements(ts[lo:hi], np.zeros(hi - lo, np.int64))
            want = [ora.slice(i).t_start for i in range(ora.store_size())]
            if starts != want:
                failures.append((seed, b, starts[-5:], want[-5:]))
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


def test_count_path_time_edges_two_gloo_ranks_match_oracle():
    out = os.path.join(tempfile.mkdtemp(), "r")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        assert open(out + ".%d" % r).read() == "[]"
