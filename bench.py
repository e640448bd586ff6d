"""Headline benchmark: tuples/s of the MI355X slicing operator on BASELINE.json's config (configs[1]).

Workload (N=1): 1000 concurrent tumbling windows with sizes from BenchmarkRunner.randomTumbling(1000,1,20)
(java.util.Random(10)), SUM_I32 + COUNT, in-order synthetic stream, maxLateness 1 (Flink connector default).
One step = one watermark interval: a micro-batch of --batch tuples per GPU covering 1 s of event time,
resident in HBM before the timed region, pushed through the C-ABI (ingest + edge commit kernels) followed by
processWatermark (triggers, window assembly, GC, one packed transfer of the results to the host).  N>1: one
process per GPU; the ONE non-keyed C2 stream is sharded by arrival (= time) range -- rank r holds chunk r of every
global micro-batch of N*batch tuples -- and one RCCL all-gather over xGMI per micro-batch exchanges the ranks'
first-crossing records and slice partials; every rank then holds the same slice store and emits
the same windows.  Weak scaling: tuples per GPU fixed; value = all ranks' tuples / max-over-ranks time.

`python bench.py --gpus N` without a launcher starts N ranks itself (torch.distributed.run, before any GPU call)
and every rank asserts WORLD_SIZE == N, so an N-GPU run can never silently measure one GPU.

Prints ONE JSON line (rank 0).  roofline: the ingest kernel (frac) and ALL device work of a step (frac_step), from
HIP events on the operator's stream.  extra: the other BASELINE configs (C2s = the north_star target: 1000 sliding
windows, 20 % out-of-order; C3, C4, C5), each with its own CPU baseline (oracle/, the C++ restatement of the
reference operator; keyed: T threads) on a bounded sample of the same stream.
"""
import argparse
import ctypes
import importlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
METRIC = "tuples/sec (1/2/4/8 GPU) at 1000 concurrent windows; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_TUPLE = 12   # int64 ts + int32 value, read once
PCIE_GBS = 64.0        # host link, PCIe Gen5 x16 (32 GT/s x 16 lanes): the bound of host-buffer ingest
KEYED_BYTES_PER_TUPLE = 16  # + uint32 key
C4_BATCH = 1 << 26     # GPU runs use N ~ 2^26 tuples per watermark batch (C4: per rank)
CPU_BUDGET_S = float(os.environ.get("SCOTTY_CPU_BUDGET_S", "12"))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


TUNE = {}  # --tune: scotty_tune knobs for the C2 / C1 / C2s / C3 operators (A/B runs)


def apply_tune(op):
    for k, v in TUNE.items():
        op.tune(k, v)


def device_roofline(op, steps, batch, bytes_per_tuple, kernel):
    """Roofline of the dominant kernel (ingest) and of the whole step (every timed launch/transfer class)."""
    t = op.deviceTiming()
    ing_ms, ing_n = t["ingest"]
    step_ms = sum(v[0] for v in t.values()) / max(1, steps)
    avg = ing_ms / max(1, ing_n)
    algo = batch * bytes_per_tuple
    ach = algo / (avg * 1e-3) / 1e9 if avg > 0 else 0.0
    ach_step = algo / (step_ms * 1e-3) / 1e9 if step_ms > 0 else 0.0
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "kernel": kernel, "algorithmic_bytes_per_launch": algo, "avg_launch_ms": avg, "launches": ing_n,
            "achieved_step": ach_step, "frac_step": ach_step / HBM_PEAK_GBS, "device_ms_per_step": step_ms,
            "device_ms_per_step_by_class": {k: v[0] / max(1, steps) for k, v in t.items()}}


KN_INGEST, KN_KG_HIST, KN_KG_SCATTER, KN_KG_BUCKET, KN_COUNT_INGEST, KN_LANE_SESSION, KN_REPLAY = range(7)  # device_common.h


def kernel_name(pkg, which):
    """rocprofv3 name of this thread's last launch of a measured kernel class (scotty_debug_kernel_name)."""
    f = pkg.lib().scotty_debug_kernel_name
    f.restype, f.argtypes = ctypes.c_char_p, [ctypes.c_int]
    return f(which).decode()


def norm_kernel(name):
    """A kernel name as rocprofv3 prints it, without namespaces, arguments or spaces (for matching)."""
    name = name.split("(")[0].replace("void ", "")
    for ns in ("scotty::", "kg::", "ck::", "wk::", "xq::", "ls::", "lc::", "ln::", "k::", "x::"):
        name = name.replace(ns, "")
    return name.replace(" ", "")


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def pmc_traffic(leg, kernels, batch, algo_bytes):
    """HBM traffic of a leg's measured kernel(s) per launch from profiles/traffic.json (tools/traffic.py: separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, per-pattern corrections calibrated by tools/pmc_calib.hip), used
    only when the file measured exactly these kernels (rocprof names) at this batch size; else None with the reason."""
    try:
        tj = json.load(open(TRAFFIC_FILE))["legs"][leg]
    except (OSError, KeyError, ValueError):
        return {"traffic": None, "traffic_note": "no %s entry in profiles/traffic.json" % leg}
    want = sorted(norm_kernel(k) for k in kernels)
    have = sorted(norm_kernel(k) for k in tj.get("kernels", {}))
    if tj.get("batch") != batch or want != have:
        return {"traffic": None, "traffic_note": "profiles/traffic.json measured %s at batch %s, this run launched %s at "
                                                 "batch %d" % (have, tj.get("batch"), want, batch)}
    hbm = sum(v["hbm_bytes_per_launch"] for v in tj["kernels"].values())
    return {"traffic": hbm, "traffic_kernels": sorted(tj["kernels"]), "traffic_over_algorithmic": hbm / algo_bytes,
            "traffic_source": tj.get("source")}


# ----------------------------------------------------------------------------------------------- CPU baselines
def _cpu_nonkeyed(setup, gen_step, wm_of, steps_range, budget_s, chunk, warm=None, sample=""):
    """Oracle (C++ restatement of SlicingWindowOperator, 1 thread) on the same stream: an untimed sparse warm-up
    (warm: list of (ts, vals, wm)), then the full-rate steps of the GPU leg in chunks of `chunk` tuples, a watermark
    at the end of every step (the GPU cadence), until the budget is spent; a watermark closes the sample."""
    from oracle.oracle import OracleOperator
    op = OracleOperator()
    setup(op)
    for ts, vals, wm in (warm or []):
        op.processElements(ts, vals)
        if wm is not None:
            op.processWatermark(wm)
    done, t_proc, n_wm, last_ts = 0, 0.0, 0, None
    for s in steps_range:
        ts, vals = gen_step(s)
        for c0 in range(0, len(ts), chunk):
            t0 = time.perf_counter()
            op.processElements(ts[c0:c0 + chunk], vals[c0:c0 + chunk])
            t_proc += time.perf_counter() - t0
            done += min(chunk, len(ts) - c0)
            last_ts = int(ts[min(len(ts), c0 + chunk) - 1])
            if t_proc > budget_s:
                break
        t0 = time.perf_counter()
        op.processWatermark(wm_of(s, last_ts) if t_proc <= budget_s else wm_of(s, last_ts, partial=True))
        t_proc += time.perf_counter() - t0
        n_wm += 1
        if t_proc > budget_s:
            break
    return {"value": done / t_proc, "unit": "tuples/s", "cores": 1, "kind": "port",
            "sample": "%d tuples, %d watermarks of the same stream; %s; oracle/ C++ restatement of "
                      "SlicingWindowOperator, 1 thread" % (done, n_wm, sample)}


def host_cores():
    """(effective cores, affinity threads, cgroup CPU quota or None).  Effective = min(the threads this process may
    run on (sched_getaffinity), the cgroup's CPU quota): more threads than the quota only time-slice the same CPUs."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    eff = n if quota is None else max(1, min(n, int(quota)))
    return eff, n, quota


C1_PUBLISHED = 1.56e6  # README.md:50-54, benchmark/configurations/sliding_benchmark_Scotty.json:22 (Flink + Scotty)


def cpu_c1(rate):
    """C1 (BASELINE configs[0]) on the oracle, 1 thread: the reference benchmark's sliding 60 s / 1 s SUM over
    Random(43).nextInt() values, in-order, maxLateness 1; sparse 60 s warm-up (1 tuple/ms) then full-rate steps."""
    pkg = importlib.import_module("scotty-window-processor_amd")
    jr = pkg.workloads.JavaRandomInts(43)

    def setup(op):
        op.addWindowFunction(0)
        op.setMaxLateness(1)
        op.addWindowAssigner(1, 0, 60_000, 1_000)
    warm_ts = np.arange(0, 60_000, dtype=np.int64)
    warm = [(warm_ts, jr.next_ints(len(warm_ts)).astype(np.int64), 59_999)]

    def gen(s):
        ts = 60_000 + s * 1000 + np.arange(rate * 1000, dtype=np.int64) // rate
        return ts, jr.next_ints(len(ts)).astype(np.int64)
    r = _cpu_nonkeyed(setup, gen, lambda s, lt, partial=False: lt, range(1000), CPU_BUDGET_S, 1 << 22, warm,
                      "C1 at %d tuples/ms after a 60 s sparse warm-up (1 tuple/ms), Random(43).nextInt() values" % rate)
    r["published_reference_flink_scotty"] = {"value": C1_PUBLISHED, "unit": "events/s",
                                             "source": "README.md:50-54 (Flink + Scotty, sliding 60 s / 1 s)"}
    return r


def cpu_c2(sizes, rate):
    def setup(op):
        op.addWindowFunction(0)
        op.addWindowFunction(1)
        op.setMaxLateness(1)
        for s in sizes:
            op.addWindowAssigner(0, 0, s, 0)
    rng = np.random.default_rng(11)
    warm_ts = np.arange(0, 21000, dtype=np.int64)
    warm = [(warm_ts, np.zeros(len(warm_ts), np.int64), 20999)]

    def gen(s):
        ts = 21000 + s * 1000 + np.arange(rate * 1000, dtype=np.int64) // rate
        return ts, rng.integers(-2**31, 2**31, size=len(ts), dtype=np.int64)
    return _cpu_nonkeyed(setup, gen, lambda s, lt, partial=False: lt, range(1000), CPU_BUDGET_S, 1 << 22, warm,
                         "C2 at %d tuples/ms after a 21 s sparse warm-up (1 tuple/ms)" % rate)


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


def cpu_c2s(pkg, rate):
    wins = c2s_windows(pkg)

    def setup(op):
        op.addWindowFunction(0)
        op.addWindowFunction(1)
        op.setMaxLateness(1000)
        for size, slide in wins:
            op.addWindowAssigner(1, 0, size, slide)
    rng = np.random.default_rng(12)
    warm_ts = np.arange(1, 21000, dtype=np.int64)
    warm = [(warm_ts, np.zeros(len(warm_ts), np.int64), 20499)]

    def gen(s):
        ts = 21000 + s * 1000 + np.arange(rate * 1000, dtype=np.int64) // rate
        late = rng.random(len(ts)) < 0.2
        d = rng.integers(1, 501, size=len(ts))
        ts = np.where(late, np.maximum(ts - d, 1), ts)
        return ts, rng.integers(-2**31, 2**31, size=len(ts), dtype=np.int64)
    return _cpu_nonkeyed(setup, gen, lambda s, lt, partial=False: 21000 + s * 1000 + 999 - 500, range(1000),
                         CPU_BUDGET_S, 1 << 20, warm,
                         "C2s at %d tuples/ms, 20%% late by U[1,500] ms, after a 21 s sparse warm-up" % rate)


def cpu_c3(rate):
    def setup(op):
        op.addWindowFunction(2)
        op.addWindowFunction(3)
        op.setMaxLateness(1000)
        op.addWindowAssigner(1, 0, 60_000, 60)
        op.addWindowAssigner(2, 0, 1000, 0)
    rng = np.random.default_rng(13)
    warm = []
    for s in range(61):  # sparse warm-up with the same session pauses
        t_begin = s * 1000 + 1000 + (s // 10) * 2000
        ts = t_begin + np.arange(0, 1000, dtype=np.int64)
        warm.append((ts, np.zeros(len(ts), np.int64), t_begin + 999 - 500 if s % 10 == 9 or s == 60 else None))

    def gen(s):
        t_begin = s * 1000 + 1000 + (s // 10) * 2000
        ts = t_begin + np.arange(rate * 1000, dtype=np.int64) // rate
        late = rng.random(len(ts)) < 0.2
        d = rng.integers(1, 501, size=len(ts))
        ts = np.where(late, np.maximum(ts - d, t_begin - 500), ts)
        return ts, rng.integers(-2**31, 2**31, size=len(ts), dtype=np.int64)

    def wm(s, lt, partial=False):
        return s * 1000 + 1000 + (s // 10) * 2000 + 999 - 500 if not partial else lt - 500
    return _cpu_nonkeyed(setup, gen, wm, range(61, 2000), CPU_BUDGET_S, 1 << 20, warm,
                         "C3 at %d tuples/ms, 20%% late, after a 61 s sparse warm-up with the session pauses" % rate)


def cpu_c5(pkg, rate):
    sizes = pkg.workloads.random_count_sizes(1000, 1_000_000, 20_000_000, seed=10)

    def setup(op):
        op.addWindowFunction(0)
        op.addWindowFunction(1)
        op.setMaxLateness(1)
        for size in sizes:
            op.addWindowAssigner(0, 1, size, 0)
    rng = np.random.default_rng(14)

    def gen(s):
        ts = s * 1000 + np.arange(rate * 1000, dtype=np.int64) // rate
        return ts, rng.integers(-2**31, 2**31, size=len(ts), dtype=np.int64)
    return _cpu_nonkeyed(setup, gen, lambda s, lt, partial=False: lt, range(1000), CPU_BUDGET_S, 1 << 22, None,
                         "C5 from the stream start at %d tuples/ms (count windows fire every 1M-20M tuples)" % rate)


def cpu_c5t(step):
    def setup(op):
        op.addWindowFunction(0)
        op.addWindowFunction(1)
        op.setMaxLateness(1)
        op.addWindowAssigner(0, 1, 1000, 0)
        op.addWindowAssigner(1, 0, 60_000, 1000)
    rng = np.random.default_rng(16)

    def gen(s):
        ts = np.arange(s * step, (s + 1) * step, dtype=np.int64)
        return ts, rng.integers(-2**31, 2**31, size=len(ts), dtype=np.int64)
    return _cpu_nonkeyed(setup, gen, lambda s, lt, partial=False: lt, range(100000), CPU_BUDGET_S, 1 << 20, None,
                         "SURVEY C5 from the stream start, unique ts, a watermark per %d tuples (the GPU leg's 2^26 "
                         "would put LazyAggregateStore.aggregate's slices x windows scan at ~10^10 per watermark)"
                         % step)


def cpu_c4(keys, batch, threads):
    """KeyedScottyWindowOperator on T threads (key % T partitions): sparse warm-up (2^20 tuples per second for
    60 s, so every key's operator holds its sliding-window slices), then full-rate steps of the GPU leg."""
    from oracle.oracle import KeyedOracleThreads
    op = KeyedOracleThreads(threads)
    op.addWindowFunction(0)
    op.setMaxLateness(1)
    op.addWindowAssigner(1, 0, 60_000, 1_000)
    rng = np.random.default_rng(15)
    warm_n = 1 << 20
    for s in range(60):
        k = rng.integers(0, keys, size=warm_n).astype(np.uint32)
        ts = s * 1000 + np.arange(warm_n, dtype=np.int64) // (warm_n // 1000)
        op.process(op.partition(k, ts, np.zeros(warm_n, np.int64)), s * 1000 + 999)
    rate = batch // 1000
    done, t_proc, rows, steps = 0, 0.0, 0, 0
    for s in range(60, 1000):
        k = rng.integers(0, keys, size=batch).astype(np.uint32)
        ts = s * 1000 + np.arange(batch, dtype=np.int64) // rate
        v = rng.integers(-2**31, 2**31, size=batch, dtype=np.int64)
        p = op.partition(k, ts, v)
        t0 = time.perf_counter()
        rows += op.process(p, s * 1000 + (batch - 1) // rate)
        t_proc += time.perf_counter() - t0
        done += batch
        steps += 1
        if t_proc > CPU_BUDGET_S:
            break
    eff, affinity, quota = host_cores()
    return {"value": done / t_proc, "unit": "tuples/s", "cores": threads, "kind": "port",
            "affinity_threads": affinity, "cgroup_cpu_quota": quota,
            "sample": "%d steps of %d tuples (%d uniform keys, 1 s of event time each, one watermark per step) after a "
                      "60 s sparse warm-up; oracle/ KeyedScottyWindowOperator restatement on %d threads = the effective "
                      "host cores of this process, min(sched_getaffinity %d, cgroup quota %s); key %% %d partitions"
                      % (steps, batch, keys, threads, affinity, quota, threads)}


def cpu_c4s(keys, batch, threads):
    """C4s on the CPU: KeyedScottyWindowOperator with SessionWindow(1 s) + SlidingWindow(60 s, 1 s) per key on T
    threads (key % T partitions), the GPU leg's stream (20 % of tuples late by U[1,500] ms, 2 s pause every 10 s,
    watermark lag 500 ms), one watermark per step; two untimed steps, then timed steps until the budget."""
    from oracle.oracle import KeyedOracleThreads, JavaError
    op = KeyedOracleThreads(threads)
    op.addWindowFunction(0)
    op.setMaxLateness(1000)
    op.addWindowAssigner(1, 0, 60_000, 1_000)
    op.addWindowAssigner(2, 0, 1000, 0)
    rng = np.random.default_rng(77)
    rate = max(1, batch // 1000)
    base = np.arange(batch, dtype=np.int64) // rate
    done, t_proc, steps = 0, 0.0, 0
    for s in range(1000):
        t_begin = s * 1000 + 1000 + (s // 10) * 2000
        k = rng.integers(0, keys, size=batch).astype(np.uint32)
        late = rng.random(batch) < 0.2
        ts = np.where(late, base + t_begin - rng.integers(1, 501, size=batch), base + t_begin)
        v = rng.integers(-2**31, 2**31, size=batch, dtype=np.int64)
        p = op.partition(k, ts, v)
        t0 = time.perf_counter()
        try:  # the first steps' too-late tuples throw per tuple in the reference (recorded, the batch continues)
            op.process(p, t_begin + (batch - 1) // rate - 500)
        except JavaError:
            pass
        dt = time.perf_counter() - t0
        if s >= 2:
            t_proc += dt
            done += batch
            steps += 1
            if t_proc > CPU_BUDGET_S:
                break
    eff, affinity, quota = host_cores()
    return {"value": done / t_proc, "unit": "tuples/s", "cores": threads, "kind": "port",
            "affinity_threads": affinity, "cgroup_cpu_quota": quota,
            "sample": "%d steps of %d tuples (%d uniform keys, the C4s stream: steps 2.. of one run from event time "
                      "0, a 2 s pause every 10 steps) after 2 untimed steps; oracle/ KeyedScottyWindowOperator "
                      "restatement on %d threads = the effective host cores of this process, min(sched_getaffinity "
                      "%d, cgroup quota %s); key %% %d partitions" % (steps, batch, keys, threads, affinity, quota,
                                                                      threads)}


# ----------------------------------------------------------------------------------------------- GPU legs
def extra_c1(pkg, dev, batch, steps, warm=2):
    """BASELINE configs[0] (C1), the reference benchmark's own workload at GPU batch size: SlidingWindow(Time,
    60000, 1000), SUM_I32 of java.util.Random(43).nextInt() values (restated exactly, generated on the host before
    the timed region), in-order ts = i // rate, maxLateness 1 (Flink connector default), one key; grid path.  A sparse
    60 s warm-up (1 tuple/ms, the same Random(43) sequence) so every step emits its window; then `steps` wall-clock
    steps and as many HIP-event steps (roofline).  Published: Flink + Scotty ~1.56 M events/s (README.md:50-54)."""
    import torch
    rate = max(1, batch // 1000)
    jr = pkg.workloads.JavaRandomInts(43)
    op = pkg.SlicingWindowOperator(device=dev.index)
    apply_tune(op)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.setMaxLateness(1)
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60_000, 1_000))
    wts = torch.arange(0, 60_000, dtype=torch.int64, device=dev)
    wv = torch.from_numpy(jr.next_ints(60_000)).to(dev)
    torch.cuda.synchronize(dev)
    op.processElementsDevice(wts.data_ptr(), wv.data_ptr(), 60_000)
    op.processWatermarkRaw(59_999)
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    inputs = []
    for s in range(warm + 2 * steps):
        inputs.append((base + 60_000 + s * 1000, torch.from_numpy(jr.next_ints(batch)).to(dev)))
    torch.cuda.synchronize(dev)

    def step(s):
        ts, v = inputs[s]
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        return op.processWatermarkRaw(60_000 + s * 1000 + (batch - 1) // rate)[0]
    # full-rate warm-up steps (untimed): the first full-size push sizes the operator's per-batch buffers (cells, tile
    # maxima, the ingest arena) -- C2 has the same warm-up; round 5's C1 timed its first full-size step and showed a
    # ~60 us/step wall-device gap from it
    for s in range(warm):
        step(s)
    torch.cuda.synchronize(dev)
    rows, each = 0, []
    t0 = time.perf_counter()
    for s in range(warm, warm + steps):
        rows += step(s)
        each.append(time.perf_counter())
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    op.enableTiming(True)
    for s in range(warm + steps, warm + 2 * steps):
        step(s)
    torch.cuda.synchronize(dev)
    roof = device_roofline(op, steps, batch, BYTES_PER_TUPLE, kernel_name(pkg, KN_INGEST))
    roof.update(pmc_traffic("c1", [roof["kernel"]], batch, batch * BYTES_PER_TUPLE))
    ms = 1e3 * elapsed / steps
    return {"workload": "C1: SlidingWindow(Time,60000,1000), SUM_I32 of Random(43).nextInt(), in-order, "
                        "maxLateness=1, one key (the reference benchmark's sliding workload)",
            "tuples_per_step": batch, "steps": steps, "warmup_full_rate_steps": warm, "ms_per_step": ms,
            "ms_per_step_each": [round(1e3 * (b - a), 4) for a, b in zip([t0] + each[:-1], each)],
            "wall_minus_device_us_per_step": 1e3 * (ms - roof["device_ms_per_step"]),
            "frac_step_wall": batch * BYTES_PER_TUPLE / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "value": batch * steps / elapsed, "unit": "tuples/s", "windows_emitted": rows,
            "published_reference_flink_scotty": {"value": C1_PUBLISHED, "unit": "events/s",
                                                 "source": "README.md:50-54"},
            "roofline": roof}


def extra_c3(pkg, dev, batch, steps=10, warm=61, tune=None):
    """BASELINE configs[2] (C3): SlidingWindow(60 s, 60 ms) + SessionWindow(1 s gap), MIN_I32 + MAX_I32, 20 %
    out-of-order tuples late by U[1,500] ms, watermark lag 500 ms, maxLateness 1000; exact engine.  Every 10 s of
    event time the stream pauses for 2 s (SURVEY: 1-2 s silences), so sessions close: tuples up to 500 ms late leave
    a 1.5 s silence, more than the 1 s gap (a 1.5 s pause leaves exactly the gap, and the sessions merge again).  61 s of
    warm-up: every timed step emits its sliding windows.  The timed steps cover whole 10-step session periods, so
    the pause step (new session, out-of-order session edits: the event-exact path, exact_batch.hip) is counted
    beside the quiet steps (one pass, exact_quiet.hip) in its true proportion.  Inputs resident in HBM; results
    stay in HBM (processWatermarkDevice).  A second run of as many steps with HIP events gives the device roofline.
    `tune`: scotty_tune knobs (the "c3nb" leg: {"quiet_band": 0}, the start band off, for an A/B in one run)."""
    import torch
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    op = pkg.SlicingWindowOperator(device=dev.index)
    for k, v in (tune or {}).items():
        op.tune(k, v)
    apply_tune(op)
    op.addWindowFunction(pkg.AGG_MIN_I32)
    op.addWindowFunction(pkg.AGG_MAX_I32)
    op.setMaxLateness(1000)
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60_000, 60))
    op.addWindowAssigner(pkg.SessionWindow(pkg.WindowMeasure.Time, 1000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    times, rows, verdicts, rounds = [], 0, [], []
    for s in range(warm + 2 * steps):
        if s % 10 == 0:
            log("c3: step %d" % s)
        if s == warm + steps:
            op.enableTiming(True)  # instrumented steps: after the wall-clock ones
        t_begin = s * 1000 + 1000 + (s // 10) * 2000
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
        if warm <= s < warm + steps:
            times.append(time.perf_counter() - t0)
            rows += n
            verdicts.append(op._debug_stat(8))
            rounds.append((op._debug_stat(0), op._debug_stat(1)))  # events, event-exact rounds of the batch
    roof = device_roofline(op, steps, batch, BYTES_PER_TUPLE, kernel_name(pkg, KN_INGEST))
    roof["kernel_role"] = "the grid ingest on the exact engine's quiet path"
    roof.update(pmc_traffic("c3", [roof["kernel"]], batch, batch * BYTES_PER_TUPLE))
    return {"workload": "C3: SlidingWindow(60s,60ms) + SessionWindow(gap 1s), MIN_I32+MAX_I32, 20% out-of-order "
                        "(delay U[1,500] ms), lag 500 ms, 2 s pause every 10 s, non-keyed, exact engine",
            "tuples_per_step": batch, "steps": steps, "ms_per_step": 1e3 * sum(times) / len(times),
            "ms_per_step_each": [round(1e3 * t, 4) for t in times],
            "quiet_steps": sum(1 for x in verdicts if x == 1), "event_exact_steps": sum(1 for x in verdicts if x != 1),
            "event_prefix_then_quiet_steps": op._debug_stat(12),
            "start_band_moves": op._debug_stat(100), "start_band_moves_no_edge": op._debug_stat(102),
            "jump_pieces": op._debug_stat(101), "tune": tune or {},
            "events_rounds_each": rounds,
            "value": batch * len(times) / sum(times), "unit": "tuples/s", "windows_emitted": rows,
            "roofline": roof,
            "roofline_wall": {"achieved": batch * BYTES_PER_TUPLE * len(times) / sum(times) / 1e9,
                              "frac": batch * BYTES_PER_TUPLE * len(times) / sum(times) / 1e9 / HBM_PEAK_GBS}}


def extra_c2s(pkg, dev, batch, steps, warm=21, tune=None, ooo=0.2):
    """north_star target workload: 1000 concurrent sliding windows (c2s_windows), SUM_I32 + COUNT, 20 %
    out-of-order tuples late by U[1,500] ms, watermark lag 500 ms, maxLateness 1000; grid path.  Warm-up until the
    largest window (20 s) has been emitted, so every timed step assembles a full set of windows.  Inputs are
    generated for every step before the timed region starts (resident in HBM)."""
    import torch
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    op = pkg.SlicingWindowOperator(device=dev.index)
    for k, v in (tune or {}).items():
        op.tune(k, v)
    apply_tune(op)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1000)
    for size, slide in c2s_windows(pkg):
        op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, size, slide))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate

    def gen(s):
        ts = base + s * 1000 + 1000
        late = torch.rand(batch, device=dev, generator=g) < ooo
        d = torch.randint(1, 501, (batch,), device=dev, generator=g)
        ts = torch.where(late, torch.clamp(ts - d, min=1), ts).contiguous()
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        return ts, v
    f = op._l.scotty_debug_grid_stat
    f.restype, f.argtypes = ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int]
    glb = []
    for s in range(warm):
        ts, v = gen(s)
        torch.cuda.synchronize(dev)  # the C-ABI reads the buffers on its own stream
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        op.processWatermarkRaw(s * 1000 + 1000 + (batch - 1) // rate - 500)
        glb.append(f(op._h, 0))
    log("c2s: global-atomic tuples after each warm-up step:", glb)
    # wall-clock steps (no instrumentation), then as many steps with HIP events around every launch group (roofline)
    timed = [gen(s) for s in range(warm, warm + 2 * steps)]
    torch.cuda.synchronize(dev)
    rows = 0
    t0 = time.perf_counter()
    for i, s in enumerate(range(warm, warm + steps)):
        ts, v = timed[i]
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        n, _ = op.processWatermarkRaw(s * 1000 + 1000 + (batch - 1) // rate - 500)
        rows += n
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    op.enableTiming(True)
    for i, s in enumerate(range(warm + steps, warm + 2 * steps)):
        ts, v = timed[steps + i]
        op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        op.processWatermarkRaw(s * 1000 + 1000 + (batch - 1) // rate - 500)
    torch.cuda.synchronize(dev)
    log("c2s: tuples added with global atomics since creation:", f(op._h, 0))
    log("c2s: last ingest launch: %d workgroups, streaming variant %d, slow-path tuples of the last push %d"
        % (f(op._h, 9), f(op._h, 10), f(op._h, 11)))
    log("c2s: cell index base %d shift %d buckets %d full %d span_end %d; slices %d, grid ahead %d, prev_max %d"
        % tuple(f(op._h, k) for k in range(1, 9)))
    roof = device_roofline(op, steps, batch, BYTES_PER_TUPLE, kernel_name(pkg, KN_INGEST))
    roof.update(pmc_traffic("c2s", [roof["kernel"]], batch, batch * BYTES_PER_TUPLE))
    return {"workload": "C2s: 1000 concurrent sliding windows, sizes randomTumbling(1000,1,20) Random(10), slide "
                        "size/20, SUM_I32+COUNT, 20% out-of-order (delay U[1,500] ms), lag 500 ms, maxLateness 1000",
            "tuples_per_step": batch, "steps": steps, "ms_per_step": 1e3 * elapsed / steps,
            "value": batch * steps / elapsed, "unit": "tuples/s", "windows_emitted": rows,
            "roofline": roof}


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
        op.tune("count_path", 1)  # the C5 stream is in timestamp order: no LazySlice record sets needed
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1)
    for size in pkg.workloads.random_count_sizes(n_windows, lo, hi, seed=10):
        op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Count, size))
    base = (torch.arange(batch, device=dev, dtype=torch.int64) + rank * batch) // rate
    times, rows = [], 0
    roof_steps = steps if G == 1 else 0  # G == 1: as many instrumented steps after the timed ones (device roofline)
    for s in range(warm + steps + roof_steps):
        if s == warm + steps:
            op.enableTiming(True)
        ts = base + s * 1000
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize(dev)
        if dist is not None and s == warm:
            dist.barrier()
        t0 = time.perf_counter()
        if G > 1:  # the real bounds exchange: an all-gather of {n, first ts, last ts} per chunk, timed
            op.processChunk(ts.data_ptr(), v.data_ptr(), batch, 0)
            n, _ = op.processWatermarkDevice(s * 1000 + (G * batch - 1) // rate)
        else:
            op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
            n, _ = op.processWatermarkDevice(s * 1000 + (batch - 1) // rate)
        torch.cuda.synchronize(dev)
        if warm <= s < warm + steps:
            times.append(time.perf_counter() - t0)
            rows += n
    elapsed = sum(times)
    roof = None
    if roof_steps:
        roof = device_roofline(op, roof_steps, batch, BYTES_PER_TUPLE, kernel_name(pkg, KN_COUNT_INGEST))
        roof["classes_note"] = ("push_other and watermark are marker-event intervals on the op's stream (any bubble a "
                                "host read inside them leaves counts as device time: an upper bound)")
        roof.update(pmc_traffic("c5", [roof["kernel"]], batch, batch * BYTES_PER_TUPLE))
    if dist is not None:
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    return {"roofline": roof, "workload": "C5: %d tumbling count windows, sizes randomCount(%d,%d,%d) Random(10), SUM_I32+COUNT, "
                        "in-order, maxLateness=1%s" % (n_windows, n_windows, lo, hi,
                                                       ", time-range sharded over %d GPUs (RCCL all-gather of count "
                                                       "cells)" % G if G > 1 else ""),
            "tuples_per_step": batch * G, "tuples_per_step_per_gpu": batch, "steps": steps,
            "ms_per_step": 1e3 * elapsed / len(times), "value": batch * G * len(times) / elapsed, "unit": "tuples/s",
            "scaling": "weak", "windows_emitted": rows,
            "roofline_wall": {"achieved": batch * BYTES_PER_TUPLE * len(times) / (elapsed / G * G) / 1e9,
                              "frac": batch * BYTES_PER_TUPLE * len(times) / elapsed / 1e9 / HBM_PEAK_GBS}}


def extra_c5t(pkg, dev, batch, steps, warm=3, rank=0, world=1, dist=None):
    """TumblingWindow(Count, 1000) + SlidingWindow(Time, 60000, 1000), SUM_I32 + COUNT, non-keyed,
    in-order with unique timestamps (ts = global arrival index), maxLateness 1, one watermark per micro-batch of
    world * batch tuples; count path with time edges (CEngine::time_edges).  world > 1: arrival-range sharding,
    rank r holds chunk r of every micro-batch, one all-gather of count-cell records per batch; weak scaling."""
    import torch
    G = world
    g = torch.Generator(device=dev)
    g.manual_seed(19 + rank)
    if G > 1:
        op = pkg.ShardedSlicingWindowOperator(device=dev.index)
    else:
        op = pkg.SlicingWindowOperator(device=dev.index)
        op.tune("count_path", 1)  # in-order stream: count + time windows on the count path
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.addWindowFunction(pkg.AGG_COUNT)
    op.setMaxLateness(1)
    op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Count, 1000))
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60000, 1000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) + rank * batch
    times, rows = [], 0
    roof_steps = steps if G == 1 else 0  # G == 1: as many instrumented steps after the timed ones (device roofline)
    for s in range(warm + steps + roof_steps):
        if s == warm + steps:
            op.enableTiming(True)
        ts = base + s * G * batch
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize(dev)
        if dist is not None and s == warm:
            dist.barrier()
        t0 = time.perf_counter()
        wm = (s + 1) * G * batch - 1
        if G > 1:  # the real bounds exchange ({n, first ts, last ts} all-gather per chunk), timed
            op.processChunk(ts.data_ptr(), v.data_ptr(), batch, 0)
        else:
            op.processElementsDevice(ts.data_ptr(), v.data_ptr(), batch)
        n, _ = op.processWatermarkDevice(wm)
        torch.cuda.synchronize(dev)
        if warm <= s < warm + steps:
            times.append(time.perf_counter() - t0)
            rows += n
    elapsed = sum(times)
    roof = None
    if roof_steps:
        roof = device_roofline(op, roof_steps, batch, BYTES_PER_TUPLE, kernel_name(pkg, KN_COUNT_INGEST))
        roof["classes_note"] = ("push_other and watermark are marker-event intervals on the op's stream (the time-edge "
                                "pass reads the batch's first / last ts on the host inside the push: upper bound)")
        roof.update(pmc_traffic("c5t", [roof["kernel"]], batch, batch * BYTES_PER_TUPLE))
    if dist is not None:
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    return {"roofline": roof, "workload": "C5 (SURVEY): TumblingWindow(Count,1000) + SlidingWindow(Time,60000,1000), SUM_I32+COUNT, "
                        "in-order unique ts (ts = arrival index), maxLateness=1, a watermark per %d-tuple micro-batch%s"
                        % (batch * G, ", arrival-range sharded over %d GPUs (RCCL all-gather of count cells)" % G
                           if G > 1 else ""),
            "tuples_per_step": batch * G, "tuples_per_step_per_gpu": batch, "steps": steps,
            "ms_per_step": 1e3 * elapsed / len(times), "value": batch * G * len(times) / elapsed, "unit": "tuples/s",
            "scaling": "weak", "windows_emitted": rows,
            "roofline_wall": {"achieved": batch * BYTES_PER_TUPLE * len(times) / elapsed / 1e9,
                              "frac": batch * BYTES_PER_TUPLE * len(times) / elapsed / 1e9 / HBM_PEAK_GBS}}


def c4_routing(pkg, dev, batch, keys, steps, rank, world, dist, seed=4242):
    """The keyBy in front of the keyed operator at G > 1, timed on its own (BENCH field `routing`): each rank holds an
    arrival slice of the global keyed stream (uniform keys), splits it on the device by the owner rank of every key
    (the product router's key-group assignment, KeyedShardRouter / scotty_key_shard, as a device lookup table) with a
    stable sort, and exchanges the parts with one all-to-all of 16-byte records (RCCL over xGMI for "nccl"; host
    staged for "gloo") after an all-to-all of the part sizes.  Reported per step: split ms, exchange ms, and the
    routed tuples/s; the operator legs consume rank-owned batches (what an upstream keyBy delivers)."""
    import torch
    allk = np.arange(keys, dtype=np.uint32)
    parts = pkg.KeyedShardRouter(world).route(allk, allk.astype(np.int64), allk.astype(np.int32))
    owner = np.zeros(keys, dtype=np.int64)
    for r, (k, _, _) in enumerate(parts):
        owner[k] = r
    owner_d = torch.from_numpy(owner).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(seed + rank)
    staged = dist.get_backend() != "nccl"
    rate = max(1, batch // 1000)
    t_split = t_x = 0.0
    got = 0
    for s in range(steps + 1):
        k = torch.randint(0, keys, (batch,), device=dev, dtype=torch.int64, generator=g)
        ts = torch.arange(batch, device=dev, dtype=torch.int64) // rate + s * 1000
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int64, generator=g)
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        own = owner_d[k]
        order = torch.sort(own, stable=True).indices
        rec = torch.stack([ts[order], (k[order] << 32) | (v[order] & 0xFFFFFFFF)], dim=1).contiguous()
        cnt = torch.bincount(own, minlength=world)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        cin = cnt.cpu() if staged else cnt
        cout = torch.empty_like(cin)
        dist.all_to_all_single(cout, cin)
        ins, outs = cin.tolist(), cout.tolist()
        src = rec.cpu() if staged else rec
        dst = torch.empty((sum(outs), 2), dtype=torch.int64, device=src.device)
        dist.all_to_all_single(dst, src, output_split_sizes=outs, input_split_sizes=ins)
        if not staged:
            torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        if s > 0:
            t_split += t1 - t0
            t_x += t2 - t1
            got += int(dst.shape[0])
    t = torch.tensor([t_split, t_x], dtype=torch.float64, device=dev if not staged else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_split, t_x = (float(x) for x in t.tolist())
    return {"what": "device split by owner rank (stable sort) + all-to-all of 16-B records, per rank per step",
            "tuples_per_step_per_gpu": batch, "steps": steps, "split_ms_per_step": 1e3 * t_split / steps,
            "exchange_ms_per_step": 1e3 * t_x / steps,
            "routed_tuples_per_s": batch * world * steps / (t_split + t_x),
            "received_tuples_rank0_per_step": got / steps, "backend": dist.get_backend()}


def extra_c4(pkg, dev, batch, keys, steps, lane=True, rank=0, world=1, dist=None, tune=None, aggs=None, host_steps=0):
    """BASELINE configs[3] (C4): SlidingWindow(60 s, 1 s) SUM_I32 per key, uniform keys, maxLateness 1 (Flink
    connector default); 61 s of warm-up so every step emits each key's window.  world > 1: key-hash sharding
    with no collective -- rank r owns the keys KeyedShardRouter(world) assigns it (what an upstream keyBy delivers), `keys`
    is the global key count, `batch` the tuples per rank per step (weak scaling); the timed region is bracketed
    by barriers and the max over ranks is taken."""
    import torch
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(42 + rank)
    op = pkg.KeyedSlicingWindowOperator(device=dev.index)
    if not lane:
        op.tune("keyed_lane", 0)
    for k, v in (tune or {}).items():
        op.tune(k, v)
    for agg in aggs or (pkg.AGG_SUM_I32,):  # aggs: A/B of the watermark's assembly (tools/c4_run.py minmax)
        op.addWindowFunction(agg)
    op.setMaxLateness(1)
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60_000, 1_000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    warm = 61
    # the keys this rank owns under the product's key-hash router (scotty_key_shard: the SPE's key groups)
    allk = np.arange(keys, dtype=np.uint32)
    own = pkg.KeyedShardRouter(world).route(allk, allk.astype(np.int64), allk.astype(np.int32))[rank][0]
    own = torch.from_numpy(own.astype(np.int32)).to(dev)
    times, rows, elapsed = [], 0, 0.0
    for s in range(warm + 2 * steps):
        if s % 10 == 0:
            log("c4: step %d" % s)
        if s == warm + steps:
            op.enableTiming(True)  # instrumented steps (HIP events per launch class) after the wall-clock ones
        k = own[torch.randint(0, len(own), (batch,), device=dev, dtype=torch.int64, generator=g)]
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        ts = base + s * 1000
        torch.cuda.synchronize(dev)
        if dist is not None and s == warm:
            dist.barrier()
        t0 = time.perf_counter()
        op.processElementsDevice(k.data_ptr(), ts.data_ptr(), v.data_ptr(), batch)
        n, _ = op.processWatermarkDevice(s * 1000 + (batch - 1) // rate)
        torch.cuda.synchronize(dev)
        if warm <= s < warm + steps:
            times.append(time.perf_counter() - t0)
            rows += n
        if dist is not None and s == warm + steps - 1:
            dist.barrier()
    kn = [kernel_name(pkg, k) for k in (KN_KG_HIST, KN_KG_SCATTER, KN_KG_BUCKET)]
    roof = device_roofline(op, steps, batch, KEYED_BYTES_PER_TUPLE,
                           "keyed data pass (class ingest): %s + scans + %s + %s" % tuple(kn))
    roof["kernels"] = kn
    if world == 1 and aggs is None:  # HBM bytes of the data pass per step (tools/traffic.py; scans are not matched)
        roof.update(pmc_traffic("c4", kn, batch, batch * KEYED_BYTES_PER_TUPLE))
    host = None
    if host_steps:  # the same steps with every window's row copied to host memory (scotty_process_watermark)
        op.enableTiming(False)
        ht = []
        for s in range(warm + 2 * steps, warm + 2 * steps + host_steps):
            k = own[torch.randint(0, len(own), (batch,), device=dev, dtype=torch.int64, generator=g)]
            v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
            ts = base + s * 1000
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            op.processElementsDevice(k.data_ptr(), ts.data_ptr(), v.data_ptr(), batch)
            n, _ = op.processWatermarkRaw(s * 1000 + (batch - 1) // rate)
            ht.append(time.perf_counter() - t0)
        host = {"what": "results to host memory (scotty_process_watermark: one packed D2H of the SoA rows), "
                        "as KeyedScottyWindowOperator hands every window to out.collect", "steps": host_steps,
                "windows_per_step": n, "ms_per_step": 1e3 * sum(ht) / len(ht),
                "value": batch * world * len(ht) / sum(ht), "unit": "tuples/s"}
    elapsed = sum(times)
    if dist is not None:
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    per_gpu = batch * len(times) / elapsed
    return {"workload": "C4: keyed SlidingWindow(60s,1s) SUM_I32, %d uniform keys%s, maxLateness=1, results left "
                        "in HBM" % (keys, " key-hash sharded over %d GPUs (no collective)" % world if world > 1 else ""),
            "tuples_per_step": batch * world, "tuples_per_step_per_gpu": batch, "steps": steps,
            "keys_per_gpu": op.keyCount(), "ms_per_step": 1e3 * elapsed / len(times),
            "value": batch * world * len(times) / elapsed, "unit": "tuples/s", "scaling": "weak",
            "windows_emitted_rank0": rows, "roofline": roof, "results_to_host": host,
            "roofline_wall": {"achieved": per_gpu * KEYED_BYTES_PER_TUPLE / 1e9,
                              "frac": per_gpu * KEYED_BYTES_PER_TUPLE / 1e9 / HBM_PEAK_GBS}}


def extra_c4s(pkg, dev, batch, keys, steps=10, warm=12, tune=None):
    """Keyed sessions at scale: KeyedScottyWindowOperator with SessionWindow(gap 1 s) +
    SlidingWindow(60 s, 1 s) per key, SUM_I32, `keys` uniform keys, 20 % out-of-order tuples late by U[1,500] ms,
    watermark lag 500 ms, maxLateness 1000, a 2 s pause every 10 s of event time (every key's session closes, C3's
    shape per key).  Session windows take the lane-per-key session replay (keyed_lane_session.hip: one lane restates one
    key's StreamSlicer / SliceManager / SessionContext, steady-state tuples in registers).  The timed steps cover one
    whole 10-step period (the pause step included); a second period with HIP events gives the device split.
    `tune`: scotty_tune knobs (the "c4s3" leg: {"keyed_lane_session": 2}, the kernel's 3-waves build, A/B;
    profiles/r05/ab_c4s_occupancy.json: 2 waves 8.04 ms/step, 3 waves 8.93)."""
    import torch
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(77)
    op = pkg.KeyedSlicingWindowOperator(device=dev.index)
    for k_, v_ in (tune or {}).items():
        op.tune(k_, v_)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.setMaxLateness(1000)
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 60_000, 1_000))
    op.addWindowAssigner(pkg.SessionWindow(pkg.WindowMeasure.Time, 1000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    times, rows = [], 0
    for s in range(warm + 2 * steps):
        if s % 5 == 0:
            log("keyed leg: step %d" % s)
        if s == warm + steps:
            op.enableTiming(True)
        t_begin = s * 1000 + 1000 + (s // 10) * 2000
        k = torch.randint(0, keys, (batch,), device=dev, dtype=torch.int64, generator=g).to(torch.int32)
        late = torch.rand(batch, device=dev, generator=g) < 0.2
        d = torch.randint(1, 501, (batch,), device=dev, generator=g)
        ts = torch.where(late, base + t_begin - d, base + t_begin).contiguous()
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        op.processElementsDevice(k.data_ptr(), ts.data_ptr(), v.data_ptr(), batch)
        n, _ = op.processWatermarkDevice(t_begin + (batch - 1) // rate - 500)
        torch.cuda.synchronize(dev)
        if warm <= s < warm + steps:
            times.append(time.perf_counter() - t0)
            rows += n
    kn = kernel_name(pkg, KN_LANE_SESSION)
    roof = device_roofline(op, steps, batch, KEYED_BYTES_PER_TUPLE, kn)
    roof["kernel_note"] = ("lane per key, the replay of the batch sorted by key; the sort, segment and key-table passes "
                           "are push_other")
    roof.update(pmc_traffic("c4s", [kn], batch, batch * KEYED_BYTES_PER_TUPLE))
    return {"workload": "C4s: keyed SessionWindow(gap 1s) + SlidingWindow(60s,1s) SUM_I32, %d uniform keys, 20%% "
                        "out-of-order (delay U[1,500] ms), lag 500 ms, 2 s pause every 10 s, maxLateness 1000, "
                        "lane-per-key session replay, results left in HBM" % keys, "tune": tune or {},
            "lane_counters": ([op._debug_stat(103 + i) for i in range(4)] + [op._debug_stat(110 + i) for i in range(10)]
                              if (tune or {}).get("lane_session_counters") else None),
            "tuples_per_step": batch, "steps": steps, "keys": op.keyCount(),
            "ms_per_step": 1e3 * sum(times) / len(times), "ms_per_step_each": [round(1e3 * t, 3) for t in times],
            "value": batch * len(times) / sum(times), "unit": "tuples/s", "windows_emitted": rows, "roofline": roof}


def _numa_of_addr(addr):
    """NUMA node of the page at a host address (get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR), x86-64 syscall 239)."""
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        node = ctypes.c_int(-1)
        rc = libc.syscall(239, ctypes.byref(node), None, ctypes.c_ulong(0), ctypes.c_void_p(addr), ctypes.c_ulong(3))
        return node.value if rc == 0 else None
    except Exception:
        return None


def _node_cpus(node):
    try:
        out = set()
        for part in open("/sys/devices/system/node/node%d/cpulist" % node).read().strip().split(","):
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
        return out
    except (OSError, ValueError):
        return set()


def gpu_numa_node(dev_index):
    """NUMA node of the GPU's PCI function (sysfs), or None."""
    try:
        import torch
        p = torch.cuda.get_device_properties(dev_index)
        path = "/sys/bus/pci/devices/%04x:%02x:%02x.0/numa_node" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        return int(open(path).read().strip())
    except Exception:
        return None


C4C_COUNT = 500  # tuples per count window of the C4c leg (extra_c4c)


def extra_c4c(pkg, dev, batch, keys, steps=10, warm=11, tune=None):
    """Keyed out-of-order count windows at scale: KeyedScottyWindowOperator with
    TumblingWindow(Count, 1000) + SlidingWindow(Time, 10 s, 1 s) per key, SUM_I32, `keys` uniform keys, 20 % of tuples
    late by U[1,500] ms, watermark lag 500 ms, maxLateness 1000.  Count windows make every slice a LazySlice with its
    TreeSet record set, and an out-of-order tuple runs SliceManager's count-shift loop (S/SliceManager.java:64-87) --
    the per-key replay path (one wavefront per key, exact_kernels.hip replay_kernel).  11 s of warm-up fill the sliding
    windows' retention; results stay in HBM; a second run of as many steps with HIP events gives the device split.
    The shape is one the reference runs without throwing: the first step is in order (a late tuple below a key's first
    slice throws IndexOutOfBounds in SliceManager.processElement), and a count window spans 500 tuples = ~7.8 s of a
    key's 64 tuples per step, inside the 11 s the time window keeps (WindowManager.clearAfterWatermark removes slices
    older than watermark - maxLateness - clearDelay, S/WindowManager.java:80-92; Count(1000) would span ~15.6 s and its
    start slice is gone by the time it fires: LazyAggregateStore.aggregate's getSlice(-1), on the oracle and here)."""
    import torch
    rate = max(1, batch // 1000)
    g = torch.Generator(device=dev)
    g.manual_seed(78)
    op = pkg.KeyedSlicingWindowOperator(device=dev.index)
    for k_, v_ in (tune or {}).items():
        op.tune(k_, v_)
    op.addWindowFunction(pkg.AGG_SUM_I32)
    op.setMaxLateness(1000)
    op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Count, C4C_COUNT))
    op.addWindowAssigner(pkg.SlidingWindow(pkg.WindowMeasure.Time, 10_000, 1_000))
    base = torch.arange(batch, device=dev, dtype=torch.int64) // rate
    times, rows, count_rows = [], 0, 0
    for s in range(warm + 2 * steps):
        if s % 5 == 0:
            log("keyed leg: step %d" % s)
        if s == warm + steps:
            op.enableTiming(True)
        t_begin = s * 1000 + 1000
        k = torch.randint(0, keys, (batch,), device=dev, dtype=torch.int64, generator=g).to(torch.int32)
        late = (torch.rand(batch, device=dev, generator=g) < 0.2) & (s > 0)
        d = torch.randint(1, 501, (batch,), device=dev, generator=g)
        ts = torch.where(late, base + t_begin - d, base + t_begin).contiguous()
        v = torch.randint(-2**31, 2**31, (batch,), device=dev, dtype=torch.int32, generator=g)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        op.processElementsDevice(k.data_ptr(), ts.data_ptr(), v.data_ptr(), batch)
        n, _ = op.processWatermarkDevice(t_begin + (batch - 1) // rate - 500)
        torch.cuda.synchronize(dev)
        if warm <= s < warm + steps:
            times.append(time.perf_counter() - t0)
            rows += n
    kn = kernel_name(pkg, KN_REPLAY)
    roof = device_roofline(op, steps, batch, KEYED_BYTES_PER_TUPLE, kn)
    roof["kernel_note"] = ("wavefront-per-key replay of LazySlice record sets (class ingest); the sort by key, segment "
                           "and key-table passes are push_other")
    roof.update(pmc_traffic("c4c", [kn], batch, batch * KEYED_BYTES_PER_TUPLE))
    roof["bound_note"] = ("latency-bound: one wavefront restates one key's operator tuple by tuple (record-set inserts, "
                          "count shifts); the HBM fraction is reported for comparison only")
    return {"workload": "C4c: keyed TumblingWindow(Count,%d) + SlidingWindow(10s,1s) SUM_I32, %d uniform keys, 20%% "
                        "out-of-order after the first step (delay U[1,500] ms), lag 500 ms, maxLateness 1000, per-key "
                        "replay with LazySlice record sets, results left in HBM" % (C4C_COUNT, keys), "tune": tune or {},
            "tuples_per_step": batch, "steps": steps, "keys": op.keyCount(),
            "ms_per_step": 1e3 * sum(times) / len(times), "ms_per_step_each": [round(1e3 * t, 3) for t in times],
            "value": batch * len(times) / sum(times), "unit": "tuples/s", "windows_emitted": rows, "roofline": roof}


def cpu_c4c(keys, batch, threads):
    """C4c on the CPU: KeyedScottyWindowOperator with TumblingWindow(Count, 1000) + SlidingWindow(10 s, 1 s) per key on T
    threads (key % T partitions), the GPU leg's stream shape, one watermark per step; two untimed steps, then timed
    steps until the budget."""
    from oracle.oracle import KeyedOracleThreads
    op = KeyedOracleThreads(threads)
    op.addWindowFunction(0)
    op.setMaxLateness(1000)
    op.addWindowAssigner(0, 1, C4C_COUNT, 0)
    op.addWindowAssigner(1, 0, 10_000, 1_000)
    rng = np.random.default_rng(78)
    rate = max(1, batch // 1000)
    base = np.arange(batch, dtype=np.int64) // rate
    done, t_proc, steps = 0, 0.0, 0
    for s in range(1000):
        t_begin = s * 1000 + 1000
        k = rng.integers(0, keys, size=batch).astype(np.uint32)
        late = (rng.random(batch) < 0.2) & (s > 0)
        ts = np.where(late, base + t_begin - rng.integers(1, 501, size=batch), base + t_begin)
        v = rng.integers(-2**31, 2**31, size=batch, dtype=np.int64)
        p = op.partition(k, ts, v)
        t0 = time.perf_counter()
        op.process(p, t_begin + (batch - 1) // rate - 500)  # the shape never throws (extra_c4c)
        dt = time.perf_counter() - t0
        if s >= 2:
            t_proc += dt
            done += batch
            steps += 1
            if t_proc > CPU_BUDGET_S:
                break
    eff, affinity, quota = host_cores()
    return {"value": done / t_proc, "unit": "tuples/s", "cores": threads, "kind": "port",
            "affinity_threads": affinity, "cgroup_cpu_quota": quota,
            "sample": "%d steps of %d tuples (%d uniform keys, the C4c stream from event time 1 s) after 2 untimed "
                      "steps; oracle/ KeyedScottyWindowOperator restatement on %d threads = the effective host cores "
                      "of this process, min(sched_getaffinity %d, cgroup quota %s); key %% %d partitions"
                      % (steps, batch, keys, threads, affinity, quota, threads)}


def extra_pcie(pkg, sizes, batch, steps):
    """Placement first (the pinned leg split 14.4 vs 17.8 ms across boxes): the GPU's NUMA node,
    this process's CPUs on it, and -- when the process may run there -- the leg runs with its CPU affinity bound to that
    node, so the pinned staging slots are allocated (first touched) there; the node of the slots' pages is recorded."""
    node = gpu_numa_node(0)
    before = os.sched_getaffinity(0)
    local = (_node_cpus(node) & before) if node is not None and node >= 0 else set()
    placement = {"gpu_numa_node": node, "affinity_cpus": len(before), "affinity_cpus_on_gpu_node": len(local),
                 "bound_to_gpu_node": bool(local)}
    if local:
        os.sched_setaffinity(0, local)
    try:
        out = _extra_pcie(pkg, sizes, batch, steps, placement)
    finally:
        os.sched_setaffinity(0, before)
    out["placement"] = placement
    return out


def _extra_pcie(pkg, sizes, batch, steps, placement):
    """PCIe-inclusive C2: the same operator fed from HOST memory through scotty_process_elements --
    (a) the op's pinned staging slots (scotty_host_buffers: DMA in place, double-buffered), (b) pageable numpy
    arrays (chunked through pinned staging).  Timed: push + watermark calls per step, each step ending with its
    results on the host; the producer's writes of the next batch (ts column) are outside the timed calls."""
    import numpy as np
    rate = max(1, batch // 1000)
    out = {"tuples_per_step": batch, "steps": steps, "bytes_per_tuple": BYTES_PER_TUPLE,
           "pcie_bound_tuples_per_s": PCIE_GBS * 1e9 / BYTES_PER_TUPLE}
    rng = np.random.default_rng(77)
    base = np.arange(batch, dtype=np.int64) // rate
    vals0 = rng.integers(-2**31, 2**31, size=batch, dtype=np.int64).astype(np.int32)
    for mode in ("pinned", "pageable"):
        op = pkg.SlicingWindowOperator()
        op.addWindowFunction(pkg.AGG_SUM_I32)
        op.addWindowFunction(pkg.AGG_COUNT)
        op.setMaxLateness(1)
        for sz in sizes:
            op.addWindowAssigner(pkg.TumblingWindow(pkg.WindowMeasure.Time, sz))
        timed = 0.0
        for s in range(steps + 2):
            if mode == "pinned":
                ts, vals = op.hostBuffers(batch)
                np.add(base, s * 1000, out=ts)
                vals[:] = vals0
                if s < 2:  # the two staging slots' page placement
                    placement["pinned_slot%d_numa_node" % s] = _numa_of_addr(ts.ctypes.data)
            else:
                ts, vals = base + s * 1000, vals0
            t0 = time.perf_counter()
            op.processElements(ts, vals)
            op.processWatermarkRaw(s * 1000 + (batch - 1) // rate)
            if s >= 2:
                timed += time.perf_counter() - t0
        out[mode] = {"value": batch * steps / timed, "unit": "tuples/s", "ms_per_step": 1e3 * timed / steps,
                     "frac_of_pcie_bound": batch * steps / timed / out["pcie_bound_tuples_per_s"]}
        op.close()
    return out


def spawn_ranks(args):
    """`--gpus N` without a launcher: run N ranks through torch.distributed.run as a child (no GPU touched here)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log("bench: launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 27, help="tuples per step (1 s of event time)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C2s / C3 / C4 / C5 secondary measurements")
    ap.add_argument("--only", default="", help="comma list of extra legs to run (c1,c2s,c3,c4,c4s,c4c,c5,c5t,pcie; c3nb: C3 with the start band "
                    "off, A/B; c4s3: C4s on the lane-session kernel's 3-waves build, A/B; c4s10: C4s with 10-bit sort digits, A/B; c4cw: C4c on the "
                    "wavefront replay, A/B); default all but c3nb, c4s3, c4s10, c4cw")
    ap.add_argument("--tune", default="", help="k=v[,k=v]: scotty_tune knobs for the C2, C1, C2s and C3 operators (A/B)")
    ap.add_argument("--shard", action="store_true", help="use the sharded (RCCL exchange) path even at N=1")
    ap.add_argument("--roof-steps", type=int, default=10, help="instrumented steps (HIP events) after the timed ones")
    ap.add_argument("--skip-headline", action="store_true",
                    help="profiling runs only (tools/gpu_traffic.sh): run just the --only legs, no C2 headline line")
    args = ap.parse_args()
    for kv in (x for x in args.tune.split(",") if x):
        k, v = kv.split("=")
        TUNE[k] = int(v)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    # stdout carries exactly one line, rank 0's JSON: anything else a library prints to file descriptor 1 (RCCL's
    # version banner at communicator creation, on every rank) goes to stderr
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d: refusing to report a run on a different GPU count"
                         % (args.gpus, world))
    import torch
    ndev = torch.cuda.device_count()
    if local >= ndev:
        raise SystemExit("bench: rank %d needs GPU %d but only %d GPU(s) are visible" % (rank, local, ndev))
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
    nroof = max(1, args.roof_steps)
    nsteps = args.steps + args.warmup + nroof

    legs = set(x for x in args.only.split(",") if x) or {"c1", "c2s", "c3", "c4", "c4s", "c4c", "c5", "c5t", "pcie"}
    pcie = None
    if world == 1 and not args.no_extra and "pcie" in legs:
        # before everything else: once the headline's or C4's device buffers have come and gone, the leg's first pinned
        # staging allocation makes its host-fed steps 17.7-19.4 ms instead of 14.4 (plain pinned copies stay at
        # 57 GB/s; DESIGN.md §4, profiles/r06/ab/pcie_order/)
        pcie = extra_pcie(pkg, sizes, 1 << 26, 5)
        log("bench: PCIe-inclusive C2 done")
    res = {"metric": METRIC, "skipped_headline": True} if rank == 0 else None
    batches = op = None
    if not args.skip_headline:
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
        apply_tune(op)
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
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(args.warmup, args.warmup + args.steps):
            n_windows += step(i)
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        # roofline: the same step with HIP events around every launch group (after the wall-clock region, so the
        # instrumentation does not count in `value`)
        op.enableTiming(True)
        for i in range(args.warmup + args.steps, nsteps):
            step(i)
        torch.cuda.synchronize(dev)
        if dist:
            t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            dist.barrier()
        assert op.processedCount() >= B * nsteps - 1, op.processedCount()
        log("bench: C2 done, %.3f ms/step" % (elapsed * 1e3 / args.steps))

        res = None
        if rank == 0:
            total = B * args.steps * world
            roof = device_roofline(op, nroof, B, BYTES_PER_TUPLE, kernel_name(pkg, KN_INGEST))
            roof.update(pmc_traffic("c2", [roof["kernel"]], B, B * BYTES_PER_TUPLE))
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
                           "parallelism": ("time-range shard x%d, RCCL all-gather of slice partials per micro-batch, "
                                           "%s" % (world, "on the op's stream (no host sync)"
                                                   if op.async_exchange else "host-synchronised"))
                           if sharded else "single GPU",
                           **({"tune": dict(TUNE)} if TUNE else {})},
                "roofline": roof,
            }
    extra = {}
    if not args.no_extra:
        batches = op = None
        torch.cuda.empty_cache()
        if world == 1:
            if pcie is not None:
                extra["pcie_inclusive"] = pcie
            if "c1" in legs:
                extra["c1"] = extra_c1(pkg, dev, 1 << 26, 10)
                log("bench: C1 done")
            if "c2s" in legs:
                extra["c2s"] = extra_c2s(pkg, dev, 1 << 27, 5)
                log("bench: C2s done")
            if "c3" in legs:
                extra["c3"] = extra_c3(pkg, dev, 1 << 26, 10)
                log("bench: C3 done")
            if "c3nb" in args.only.split(","):  # A/B only (not in the default legs): C3 with the start band off
                extra["c3nb"] = extra_c3(pkg, dev, 1 << 26, 10, tune={"quiet_band": 0})
                log("bench: C3 (band off) done")
            if "c4" in legs:
                extra["c4"] = extra_c4(pkg, dev, C4_BATCH, 1 << 20, 5, host_steps=5)
                log("bench: C4 done")
            if "c4s" in legs:
                extra["c4s"] = extra_c4s(pkg, dev, C4_BATCH, 1 << 20)
            if "c4c" in legs:
                extra["c4c"] = extra_c4c(pkg, dev, C4_BATCH, 1 << 20)
                log("bench: C4c (keyed out-of-order count windows) done")
            if "c4cw" in args.only.split(","):  # A/B only: C4c through the wavefront replay (keyed_lane_count 0)
                extra["c4cw"] = extra_c4c(pkg, dev, C4_BATCH, 1 << 20, tune={"keyed_lane_count": 0})
                log("bench: C4c (wavefront replay) done")
            if "c4s10" in args.only.split(","):  # A/B only: the replay sort's 10-bit digits (keyed_sort_digit10 1)
                extra["c4s10"] = extra_c4s(pkg, dev, C4_BATCH, 1 << 20, tune={"keyed_sort_digit10": 1})
                log("bench: C4s (10-bit sort digits) done")
            if "c4s8" in args.only.split(","):  # A/B only: 8-bit digits in every sort pass (keyed_sort_digit10 2)
                extra["c4s8"] = extra_c4s(pkg, dev, C4_BATCH, 1 << 20, tune={"keyed_sort_digit10": 2})
                log("bench: C4s (8-bit last sort pass) done")
            if "c4s3" in args.only.split(","):  # A/B only: the lane-session kernel's 3-waves-per-SIMD build
                extra["c4s3"] = extra_c4s(pkg, dev, C4_BATCH, 1 << 20, tune={"keyed_lane_session": 2})
                log("bench: C4s (keyed sessions) done")
            if "c5" in legs:
                extra["c5"] = extra_c5(pkg, dev, 1 << 27, 5)
                log("bench: C5 done")
            if "c5t" in legs:
                extra["c5t"] = extra_c5t(pkg, dev, 1 << 26, 5)
                log("bench: C5t done")
        else:  # every rank takes part: key-hash sharded C4, no collective on the data path
            extra = {"c4": extra_c4(pkg, dev, C4_BATCH, 1 << 20, 5, rank=rank, world=world, dist=dist),
                     "c5": extra_c5(pkg, dev, 1 << 27, 5, rank=rank, world=world, dist=dist),
                     "c5t": extra_c5t(pkg, dev, 1 << 26, 5, rank=rank, world=world, dist=dist)}
            extra["c4"]["routing"] = c4_routing(pkg, dev, C4_BATCH, 1 << 20, 3, rank, world, dist)
    if rank == 0:
        if extra:
            res["extra"] = extra
        if not args.no_cpu_baseline and world == 1:
            # CPU baselines on this box's host cores, rank 0, N=1 only (bounded samples of the same streams)
            res["cpu_baseline"] = cpu_c2(sizes, rate)
            log("bench: CPU C2 done")
            threads, affinity, quota = host_cores()  # T = the host cores this process may use
            log("bench: host cores: %d effective (%d affinity threads, cgroup quota %s)" % (threads, affinity, quota))
            cb = {"c1": lambda: cpu_c1((1 << 26) // 1000),
                  "c2s": lambda: cpu_c2s(pkg, (1 << 27) // 1000), "c3": lambda: cpu_c3((1 << 26) // 1000),
                  "c4": lambda: cpu_c4(1 << 20, C4_BATCH, threads), "c4s": lambda: cpu_c4s(1 << 20, C4_BATCH, threads),
                  "c4c": lambda: cpu_c4c(1 << 20, C4_BATCH, threads),
                  "c5": lambda: cpu_c5(pkg, (1 << 27) // 1000),
                  "c5t": lambda: cpu_c5t(1 << 20)}
            for name, fn in cb.items():
                if name in extra:
                    extra[name]["cpu_baseline"] = fn()
                    log("bench: CPU %s done" % name)
        print(json.dumps(res), file=json_out, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
