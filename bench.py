"""Headline benchmark: tuples/s of the MI355X slicing operator on BASELINE.json's config (configs[1]).

Workload (N=1): 1000 concurrent tumbling windows with sizes from BenchmarkRunner.randomTumbling(1000,1,20)
(java.util.Random(10)), SUM_I32 + COUNT, in-order synthetic stream, maxLateness 1 (Flink connector default).
One step = one watermark interval: a micro-batch of --batch tuples per GPU covering 1 s of event time,
resident in HBM before the timed region, pushed through the C-ABI (ingest + edge commit kernels) followed by
processWatermark (window assembly + GC + results to host).  N>1: one process per GPU; the ONE non-keyed C2
stream is sharded by arrival (= time) range -- rank r holds chunk r of every global micro-batch of N*batch
tuples -- and one RCCL all-gather over xGMI per micro-batch exchanges the ranks' first-crossing records and
slice partials; every rank then holds the same slice store and emits the same windows.
Weak scaling: tuples per GPU fixed; value = all ranks' tuples / max-over-ranks time.

Prints ONE JSON line (rank 0).  cpu_baseline = the CPU restatement of SlicingWindowOperator (oracle/),
single thread, on a bounded sample of the same workload.
"""
import argparse
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
METRIC = "tuples/sec (1/2/4/8 GPU) at 1000 concurrent windows; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_TUPLE = 12   # int64 ts + int32 value, read once
C4_BATCH = 1 << 26     # GPU runs use N ~ 2^26 tuples per watermark batch (C4: per rank)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(sizes, rate_per_ms, budget_s=12.0):
    """Oracle (C++ restatement of the reference operator, 1 thread) on a bounded prefix of the same stream."""
    from oracle.oracle import OracleOperator
    op = OracleOperator()
    op.addWindowFunction(0)  # SUM_I32
    op.addWindowFunction(1)  # COUNT
    op.setMaxLateness(1)
    for s in sizes:
        op.addWindowAssigner(0, 0, s, 0)
    chunk = 1 << 21
    rng = np.random.default_rng(11)
    done, t_proc, ms_per_chunk = 0, 0.0, chunk / rate_per_ms
    t_start = time.time()
    k = 0
    while time.time() - t_start < budget_s:
        idx = np.arange(done, done + chunk, dtype=np.int64)
        ts = (idx // rate_per_ms).astype(np.int64)
        vals = rng.integers(-2**31, 2**31, size=chunk, dtype=np.int64).astype(np.int32).astype(np.int64)
        t0 = time.perf_counter()
        op.processElements(ts, vals)
        op.processWatermark(int(ts[-1]))
        t_proc += time.perf_counter() - t0
        done += chunk
        k += 1
    return {"value": done / t_proc, "unit": "tuples/s", "cores": 1, "kind": "port",
            "sample": "%d tuples (%.0f ms of event time at %d tuples/ms, %d watermarks) of the same C2 stream, "
                      "oracle/ C++ restatement of SlicingWindowOperator, 1 thread" % (done, done / rate_per_ms,
                                                                                    rate_per_ms, k)}


def extra_c3(pkg, dev, batch, steps, warm=61):
    """BASELINE configs[2] (C3): SlidingWindow(60 s, 60 ms) + SessionWindow(1 s gap), MIN_I32 + MAX_I32, 20 %
    out-of-order tuples late by U[1,500] ms, watermark lag 500 ms, maxLateness 1000; exact engine
    (exact_batch.hip).  Every 10 s of event time the stream pauses for 1.5 s, so sessions close
    (BenchmarkRunner.generateSessionGaps-like).  61 s of warm-up: every timed step emits its sliding windows.
    Inputs resident in HBM; results stay in HBM (processWatermarkDevice)."""
    import torch
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    op = pkg.SlicingWindowOperator(device=dev.index)
    op.addWindowFunction(pkg.AGG_MIN_I32)
    op.addWindowFunction(pkg.AGG_MAX_I32)
    op.setMaxLateness(1000)
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60_000, 60))
    op.addWindowAssigner(pkg.SessionWindow(pkg.WindowMeasure.Time, 1000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    times, rows, events = [], 0, 0
    for s in range(warm + steps):
        t_begin = s * 1000 + 1000 + (s // 10) * 1500
        ts = base + t_begin
        late = torch.rand(batch, device=dev, generator=g) < 0.2
        d = torch.randint(1, 501, (batch,), device=dev, generator=g)
        ts = torch.where(late, torch.clamp(ts - d, min=t_begin - 500), ts).contiguous()
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        n, _ = op.processWatermarkDevice(t_begin + (batch - 1) // rate - 500)
        torch.cuda.synchronize(dev)
        if s >= warm:
            times.append(time.perf_counter() - t0)
            rows += n
    return {"workload": "C3: SlidingWindow(60s,60ms) + SessionWindow(gap 1s), MIN_I32+MAX_I32, 20% out-of-order "
                        "(delay U[1,500] ms), lag 500 ms, 1.5 s pause every 10 s, non-keyed, exact engine",
            "tuples_per_step": batch, "steps": steps, "ms_per_step": 1e3 * sum(times) / len(times),
            "value": batch * len(times) / sum(times), "unit": "tuples/s", "windows_emitted": rows}


def c2s_windows(pkg):
    """1000 concurrent sliding windows: sizes BenchmarkRunner.randomTumbling(1000,1,20) (java.util.Random(10)),
    slide = size/20 (50..1000 ms; a power-of-two slide is bumped by 1 ms, as the reference would hang on it)."""
    out = []
    for size in pkg.workloads.random_tumbling_sizes(1000, 1, 20, seed=10):
        slide = max(1, size // 20)
        if slide & (slide - 1) == 0:
            slide += 1
        out.append((size, slide))
    return out


def extra_c2s(pkg, dev, batch, steps, warm=21, tune=None, ooo=0.2):
    """north_star target workload: 1000 concurrent sliding windows (c2s_windows), SUM_I32 + COUNT, 20 %
    out-of-order tuples late by U[1,500] ms, watermark lag 500 ms, maxLateness 1000; grid path.  Warm-up until the
    largest window (20 s) has been emitted, so every timed step assembles a full set of windows."""
    import torch
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    op = pkg.SlicingWindowOperator(device=dev.index)
    for k, v in (tune or {}).items():
        op.tune(k, v)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1000)
    for size, slide in c2s_windows(pkg):
        op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, size, slide))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    times, rows = [], 0
    op.enableTiming(True)
    for s in range(warm + steps):
        ts = base + s * 1000 + 1000
        late = torch.rand(batch, device=dev, generator=g) < ooo
        d = torch.randint(1, 501, (batch,), device=dev, generator=g)
        ts = torch.where(late, torch.clamp(ts - d, min=1), ts).contiguous()
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        if s == warm:
            op.enableTiming(False)
            op.enableTiming(True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        n, _ = op.processWatermarkRaw(s * 1000 + 1000 + (batch - 1) // rate - 500)
        torch.cuda.synchronize(dev)
        if s >= warm:
            times.append(time.perf_counter() - t0)
            rows += n
    ingest_ms, launches, _ = op.ingestTiming()
    avg_ms = ingest_ms / max(1, launches)
    achieved = batch * BYTES_PER_TUPLE / (avg_ms * 1e-3) / 1e9
    f = op._l.scotty_debug_grid_stat
    f.restype, f.argtypes = ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int]
    log("c2s: tuples added with global atomics since creation:", f(op._h, 0))
    return {"workload": "C2s: 1000 concurrent sliding windows, sizes randomTumbling(1000,1,20) Random(10), slide "
                        "size/20, SUM_I32+COUNT, 20% out-of-order (delay U[1,500] ms), lag 500 ms, maxLateness 1000",
            "tuples_per_step": batch, "steps": steps, "ms_per_step": 1e3 * sum(times) / len(times),
            "value": batch * len(times) / sum(times), "unit": "tuples/s", "windows_emitted": rows,
            "ingest": {"avg_launch_ms": avg_ms, "achieved_GBs": achieved, "frac": achieved / HBM_PEAK_GBS}}


def extra_c5(pkg, dev, batch, steps, warm=3, n_windows=1000, lo=1_000_000, hi=20_000_000, rank=0, world=1,
              dist=None):
    """BASELINE configs[4] (C5): count-based windows, BenchmarkRunner.randomCount(n, lo, hi) (TumblingWindow(Count,
    size), java.util.Random(10)), SUM_I32 + COUNT, in-order non-keyed stream, maxLateness 1; count path (every slice
    a LazySlice, S/slice/SliceFactory.java:17-22).  world > 1: time/arrival-range sharding -- rank r holds arrival
    chunk r of every global micro-batch of world * batch tuples, one all-gather of count-cell records per batch
    (RCCL over xGMI), every rank holds the same slices; weak scaling, max over ranks."""
    import torch
    G = world
    rate = max(1, (batch * G) // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(9 + rank)
    if G > 1:
        op = pkg.ShardedSlicingWindowOperator(device=dev.index)
    else:
        op = pkg.SlicingWindowOperator(device=dev.index)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1)
    for size in pkg.workloads.random_count_sizes(n_windows, lo, hi, seed=10):
        op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Count, size))
    base = (torch.arange(batch, device=dev, dtype=torch.int64) + rank * batch) // rate
    times, rows = [], 0
    for s in range(warm + steps):
        ts = base + s * 1000
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize(dev)
        if dist is not None and s == warm:
            dist.barrier()
        t0 = time.perf_counter()
        if G > 1:
            op.processChunk(ts.data_ptr(), v.data_ptr(), batch, 0, n_before=rank * batch, n_total=G * batch)
            n, _ = op.processWatermarkDevice(s * 1000 + (G * batch - 1) // rate)
        else:
            op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
            n, _ = op.processWatermarkDevice(s * 1000 + (batch - 1) // rate)
        torch.cuda.synchronize(dev)
        if s >= warm:
            times.append(time.perf_counter() - t0)
            rows += n
    elapsed = sum(times)
    if dist is not None:
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    return {"workload": "C5: %d tumbling count windows, sizes randomCount(%d,%d,%d) Random(10), SUM_I32+COUNT, "
                        "in-order, maxLateness=1%s" % (n_windows, n_windows, lo, hi,
                                                       ", time-range sharded over %d GPUs (RCCL all-gather of count "
                                                       "cells)" % G if G > 1 else ""),
            "tuples_per_step": batch * G, "tuples_per_step_per_gpu": batch, "steps": steps,
            "ms_per_step": 1e3 * elapsed / len(times), "value": batch * G * len(times) / elapsed, "unit": "tuples/s",
            "scaling": "weak", "windows_emitted": rows}


def extra_c4(pkg, dev, batch, keys, steps, lane=True, rank=0, world=1, dist=None):
    """BASELINE configs[3] (C4): SlidingWindow(60 s, 1 s) SUM_I32 per key, uniform keys, maxLateness 1 (Flink
    connector default); 61 s of warm-up so every step emits each key's window.  world > 1: key-hash sharding
    with no collective -- rank r owns the keys k with k mod world == r (what an upstream keyBy delivers), `keys`
    is the global key count, `batch` the tuples per rank per step (weak scaling); the timed region is bracketed
    by barriers and the max over ranks is taken."""
    import torch
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(42 + rank)
    op = pkg.KeyedSlicingWindowOperator(device=dev.index)
    if not lane:
        op.tune("keyed_lane", 0)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.setMaxLateness(1)
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60_000, 1_000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    warm = 61
    shard_keys = max(1, keys // world)
    times, rows, elapsed = [], 0, 0.0
    for s in range(warm + steps):
        k = torch.randint(0, shard_keys, (batch,), device=dev, dtype=torch.int32, generator=g) * world + rank
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        ts = base + s * 1000
        torch.cuda.synchronize(dev)
        if dist is not None and s == warm:
            dist.barrier()
        t0 = time.perf_counter()
        op.processElementsDevice(k.data_ptr(), ts.data_ptr(), v.data_ptr(), batch)
        n, _ = op.processWatermarkDevice(s * 1000 + (batch - 1) // rate)
        torch.cuda.synchronize(dev)
        if s >= warm:
            times.append(time.perf_counter() - t0)
            rows += n
    elapsed = sum(times)
    if dist is not None:
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    return {"workload": "C4: keyed SlidingWindow(60s,1s) SUM_I32, %d uniform keys%s, maxLateness=1, results left "
                        "in HBM" % (keys, " key-hash sharded over %d GPUs (no collective)" % world if world > 1 else ""),
            "tuples_per_step": batch * world, "tuples_per_step_per_gpu": batch, "steps": steps,
            "keys_per_gpu": op.keyCount(), "ms_per_step": 1e3 * elapsed / len(times),
            "value": batch * world * len(times) / elapsed, "unit": "tuples/s", "scaling": "weak",
            "windows_emitted_rank0": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 27, help="tuples per step (1 s of event time)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C3 / C4 secondary measurements")
    ap.add_argument("--shard", action="store_true", help="use the sharded (RCCL exchange) path even at N=1")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    pkg = importlib.import_module("scotty-window-processor_amd")

    sizes = pkg.workloads.random_tumbling_sizes(1000, 1, 20, seed=10)
    B = args.batch
    sharded = world > 1 or args.shard
    if sharded and not dist:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%s" % os.environ.get("MASTER_PORT", "29511"),
                                rank=0, world_size=1)
    G = world
    rate = max(1, (B * G) // 1000)  # tuples per ms of event time of the global stream
    nsteps = args.steps + args.warmup

    # ---- inputs resident in HBM before the timed region: this rank's arrival chunk of every global batch
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    batches = []
    base = (torch.arange(B, device=dev, dtype=torch.int64) + rank * B) // rate
    for s in range(nsteps):
        ts = base + s * 1000
        vals = torch.randint(-2**31, 2**31, (B,), device=dev, dtype=torch.int32, generator=gen)
        batches.append((ts, vals, int(s * 1000 + (B * G - 1) // rate)))
    torch.cuda.synchronize(dev)

    op = pkg.ShardedSlicingWindowOperator(device=local) if sharded else pkg.SlicingWindowOperator(device=local)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1)
    for s in sizes:
        op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Time, s))
    n_windows = 0

    def step(i):
        ts, vals, wm = batches[i]
        if sharded:
            op.processChunk(ts.data_ptr(), vals.data_ptr(), B, 0)
        else:
            op.processElementsDevice(ts.data_ptr(), vals.data_ptr(), B)
        nw, _ = op.processWatermarkRaw(wm)
        return nw

    for i in range(args.warmup):
        step(i)
    op.enableTiming(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.warmup, nsteps):
        n_windows += step(i)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    ingest_ms, launches, tuples = op.ingestTiming()
    assert op.processedCount() >= B * nsteps - 1, op.processedCount()

    if rank == 0:
        total = B * args.steps * world
        avg_ms = ingest_ms / max(1, launches)
        achieved = (B * BYTES_PER_TUPLE) / (avg_ms * 1e-3) / 1e9
        traffic = None
        tfile = os.path.join(ROOT, "profiles", "ingest_traffic.json")
        if os.path.exists(tfile):
            try:
                tj = json.load(open(tfile))
                if tj.get("batch") == B:
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        res = {
            "metric": METRIC,
            "value": total / elapsed,
            "unit": "tuples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32 values / int64 timestamps",
            "data": "synthetic (in-HBM, seeded): global stream ts = step*1000 + i//%d ms, int32 uniform values" % rate,
            "config": {"workload": "C2: 1000 concurrent tumbling windows, sizes randomTumbling(1000,1,20) "
                                   "java.util.Random(10), SUM_I32+COUNT, in-order, maxLateness=1",
                       "tuples_per_step": B * world, "tuples_per_step_per_gpu": B, "event_ms_per_step": 1000,
                       "windows_emitted": n_windows,
                       "parallelism": ("time-range shard x%d, RCCL all-gather of slice partials per micro-batch"
                                       % world) if sharded else "single GPU"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "ingest_kernel<VT_I32,NEED_SUM>", "algorithmic_bytes_per_launch":
                             B * BYTES_PER_TUPLE, "avg_launch_ms": avg_ms, "launches": launches},
        }
    if not args.no_extra:
        del batches
        del op
        torch.cuda.empty_cache()
        if world == 1:
            extra = {"c2s": extra_c2s(pkg, dev, 1 << 27, 5), "c3": extra_c3(pkg, dev, 1 << 26, 5),
                     "c4": extra_c4(pkg, dev, C4_BATCH, 1 << 20, 5), "c5": extra_c5(pkg, dev, 1 << 27, 5)}
        else:  # every rank takes part: key-hash sharded C4, no collective on the data path
            extra = {"c4": extra_c4(pkg, dev, C4_BATCH, 1 << 20, 5, rank=rank, world=world, dist=dist),
                     "c5": extra_c5(pkg, dev, 1 << 27, 5, rank=rank, world=world, dist=dist)}
        if rank == 0:
            res["extra"] = extra
    if rank == 0:
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(sizes, rate)
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
