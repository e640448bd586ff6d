/*
 * scotty_mi355x.h -- C-ABI of the MI355X-native general-stream-slicing operator.
 *
 * Drop-in boundary for the reference's operator interface
 *   core/src/main/java/de/tub/dima/scotty/core/WindowOperator.java:9-40
 *   slicing/src/main/java/de/tub/dima/scotty/slicing/SlicingWindowOperator.java:21-69
 * A JVM shim (Panama FFM / JNI) binds exactly these symbols:
 * processElement() calls are buffered off-heap and handed over once per
 * micro-batch; processWatermark() returns the emitted windows.
 *
 * Conventions: plain pointers and sizes, no exceptions across the boundary,
 * int status (0 = OK, <0 = error, >0 = warning) plus scotty_last_error().
 * One op is single-threaded (like the reference: one operator per task thread).
 */
#ifndef SCOTTY_MI355X_H
#define SCOTTY_MI355X_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes */
#define SCOTTY_OK 0
#define SCOTTY_WARN_LATE_DROPPED 1     /* tuples older than the oldest slice were dropped (the reference
                                          throws IndexOutOfBoundsException, S/SliceManager.java:75-76) */
#define SCOTTY_ERR_ARG (-1)            /* bad argument / unknown kind */
#define SCOTTY_ERR_UNSUPPORTED (-2)    /* configuration not implemented on the MI355X path */
#define SCOTTY_ERR_HIP (-3)            /* HIP runtime error / no device */
#define SCOTTY_ERR_STATE (-4)          /* call sequence error */
#define SCOTTY_ERR_INDEX (-5)          /* IndexOutOfBoundsException of the reference */
#define SCOTTY_ERR_NOMEM (-6)

/* ---- window kinds (core/windowType) */
#define SCOTTY_WIN_TUMBLING 0   /* TumblingWindow(measure, size)            C/windowType/TumblingWindow.java */
#define SCOTTY_WIN_SLIDING 1    /* SlidingWindow(measure, size, slide)      C/windowType/SlidingWindow.java */
#define SCOTTY_WIN_SESSION 2    /* SessionWindow(measure, gap)              C/windowType/SessionWindow.java */
#define SCOTTY_WIN_FIXED_BAND 3 /* FixedBandWindow(measure, start, size)    C/windowType/FixedBandWindow.java */
#define SCOTTY_MEASURE_TIME 0   /* C/windowType/WindowMeasure.java */
#define SCOTTY_MEASURE_COUNT 1

/* ---- value column type of an op (the reference's InputType) */
#define SCOTTY_VALUE_I32 0
#define SCOTTY_VALUE_I64 1
#define SCOTTY_VALUE_F64 2

/* ---- aggregate kinds: the GPU recognises these AggregateFunction classes
 * (C/windowFunction/ReduceAggregateFunction.java, InvertibleReduceAggregateFunction.java) */
#define SCOTTY_AGG_SUM_I32 0 /* Integer sum, int32 wrap (B/flinkBenchmark/aggregations/SumAggregation.java:16-18) */
#define SCOTTY_AGG_COUNT 1   /* lift=1, combine=+ (D/storm-demo/.../windowFunctions/Count.java) */
#define SCOTTY_AGG_MIN_I32 2 /* Math.min (D/flink-demo/.../MinWindowFunction.java:12) */
#define SCOTTY_AGG_MAX_I32 3 /* Math.max (D/flink-demo/.../MaxWindowFunction.java:12) */
#define SCOTTY_AGG_SUM_I64 4
#define SCOTTY_AGG_MIN_I64 5
#define SCOTTY_AGG_MAX_I64 6
#define SCOTTY_AGG_SUM_F64 7 /* within 1e-6 relative of the reference's arrival-order fold */
#define SCOTTY_AGG_MIN_F64 8
#define SCOTTY_AGG_MAX_F64 9
/* The arrival index (0-based, counting every tuple pushed to the operator, WindowManager.currentCount order) of the
 * window's FIRST partial: the first tuple added to the first non-empty slice the window contains.  It is what a
 * combine that keeps partialAggregate1's fields returns (B/flinkBenchmark/aggregations/SumAggregation.java:16-18,
 * D/flink-demo/.../SumWindowFunction.java:16-17) under AggregateValueState's lift-first / clone-first-then-fold order
 * (S/state/AggregateValueState.java:23-31, 55-69): the host shim rebuilds those fields from the payload of that tuple
 * (scotty_first_indices tells it which payloads to keep).  Grid path only (non-keyed, context-free time windows);
 * other configurations return SCOTTY_ERR_UNSUPPORTED at the first push.  Value column: int64. */
#define SCOTTY_AGG_FIRST 10
/* OR-able flag: the function is an InvertibleAggregateFunction (C/windowFunction/InvertibleAggregateFunction.java):
 * a record leaving a LazySlice is removed by liftAndInvert instead of recomputing the slice from its record set
 * (S/state/AggregateValueState.java:33-41).  Sums and counts only. */
#define SCOTTY_AGG_INVERTIBLE 0x10000
#define SCOTTY_MAX_AGGS 8

/* ---- create flags */
#define SCOTTY_FLAG_KEYED 0x1u /* keyed operator: one logical SlicingWindowOperator per uint32 key, all with the
                                  same windows / functions / lateness, as the Flink connector builds them
                                  (flink-connector/.../KeyedScottyWindowOperator.java:41-66) */

typedef struct scotty_op scotty_op;

/* Result of one processWatermark: SoA columns owned by the library, valid until the next call on
 * the op.  Row i is the i-th AggregateWindow of the reference's List (S/WindowManager.java:41-80),
 * in the reference's emission order.  values[a][i] is the lowered value of aggregation a
 * (registration order), stored as int64 (integer kinds, already wrapped to the kind's width) or as
 * the bits of a double (F64 kinds).  has_value[i]==0 <=> AggregateWindow.hasValue()==false, in which
 * case getAggValues() is the empty list. */
typedef struct {
  size_t n_windows;
  int32_t n_aggs;
  const int64_t* start;
  const int64_t* end;
  const int32_t* measure;
  const uint8_t* has_value;
  const int64_t* values[SCOTTY_MAX_AGGS];
  const uint32_t* key; /* keyed ops: key of row i (rows of one key are contiguous, in the reference's order);
                          NULL for non-keyed ops */
} scotty_windows;

/* new SlicingWindowOperator(stateFactory)  (S/SlicingWindowOperator.java:30-37) */
int scotty_create(scotty_op** op, int device, int value_type, uint32_t flags);
void scotty_destroy(scotty_op* op);
const char* scotty_last_error(scotty_op* op);

/* WindowOperator.addWindowAssigner(Window)  (C/WindowOperator.java:24; S/WindowManager.java:121-147)
 * a,b = size,0 | size,slide | gap,0 | start,size */
int scotty_add_window(scotty_op* op, int kind, int measure, int64_t a, int64_t b);
/* WindowOperator.addAggregation / SlicingWindowOperator.addWindowFunction (C/WindowOperator.java:30,
 * S/SlicingWindowOperator.java:57-63).  agg_kind: SCOTTY_AGG_* [| SCOTTY_AGG_INVERTIBLE].  Returns the aggregation
 * index (>=0) or an error. */
int scotty_add_aggregation(scotty_op* op, int agg_kind);
/* WindowOperator.setMaxLateness (C/WindowOperator.java:37; default 1000, S/WindowManager.java:24) */
int scotty_set_max_lateness(scotty_op* op, int64_t max_lateness);

/* A micro-batch of WindowOperator.processElement(element, ts) calls (C/WindowOperator.java:14) in
 * arrival order.  Host memory, caller-owned, consumed before return (pageable input is copied through the op's
 * pinned staging while earlier chunks are DMA'd; memory from scotty_host_buffers is DMA'd in place).  val points to
 * n values of the op's value type.  The transfer overlaps the op's queued device work; no device synchronisation. */
int scotty_process_elements(scotty_op* op, const int64_t* ts, const void* val, size_t n);
/* Pinned host staging owned by the op, for up to n tuples: the caller fills ts / val (/ key, keyed ops) -- the
 * off-heap buffer of the Java shim's processElement -- and passes the same pointers to scotty_process_elements /
 * scotty_process_keyed_elements, which DMA them without a CPU copy (PCIe-bound ingest).  Two slots alternate
 * between calls: a slot handed out again is reusable once its previous DMA has finished (the call waits for
 * that), so the caller fills one slot while the other is in flight. */
int scotty_host_buffers(scotty_op* op, size_t n, int64_t** ts, void** val, uint32_t** key);
/* Same, with device pointers already resident in HBM (device `device` of the op).  The buffers must
 * stay valid and unmodified until the next scotty_process_watermark() returns. */
int scotty_process_elements_device(scotty_op* op, const int64_t* d_ts, const void* d_val, size_t n);

/* Keyed micro-batch: processElement(element, ts) of the key's operator, for every tuple in arrival order
 * (KeyedScottyWindowOperator.processElement, flink-connector/.../KeyedScottyWindowOperator.java:56-66).
 * A key seen for the first time gets a fresh operator (:57-60).  Host memory, consumed before return. */
int scotty_process_keyed_elements(scotty_op* op, const uint32_t* key, const int64_t* ts, const void* val, size_t n);
/* Same, device pointers resident in HBM (valid until the call returns; 16-byte aligned). */
int scotty_process_keyed_elements_device(scotty_op* op, const uint32_t* d_key, const int64_t* d_ts,
                                         const void* d_val, size_t n);

/* WindowOperator.processWatermark(wm) (C/WindowOperator.java:19).  Blocks until results are ready.
 * Keyed ops: processWatermark(wm) of every key's operator (KeyedScottyWindowOperator.java:72-86); all
 * windows are returned (the connector's hasValue() filter, :80, is the caller's). */
int scotty_process_watermark(scotty_op* op, int64_t watermark_ts, scotty_windows* out);
/* Same, but the result columns stay in HBM (device pointers, valid until the next call on the op).
 * Exact-engine and count-path ops (keyed, or with session / count windows); grid-path ops (context-free time
 * windows only) return SCOTTY_ERR_UNSUPPORTED. */
int scotty_process_watermark_device(scotty_op* op, int64_t watermark_ts, scotty_windows* out);
/* ---- time/arrival-range sharding of ONE non-keyed stream over G ranks (one GPU each).
 * Every rank creates the same operator (same windows, functions, lateness) and, per micro-batch, holds a
 * contiguous arrival chunk of the global batch (chunk r precedes chunk r+1 in arrival order).  Per batch:
 *   1. scotty_shard_push(op, chunk, ts0, xbuf): ingest the chunk, write this rank's exchange record into the
 *      caller's device buffer xbuf of scotty_shard_xbytes(op) bytes (same size on every rank);
 *      ts0 = timestamp of the global first tuple (only read on the op's first batch: the first-edge walk);
 *   2. the caller all-gathers the G records in rank order into one device buffer (RCCL / NCCL all_gather);
 *   3. scotty_shard_commit(op, gathered, G): every rank decides the same slice edges (StreamSlicer rule from
 *      the global first crossings, S/StreamSlicer.java:55-116) and folds every rank's partials.
 * Without shard_async the push returns after the op's stream finished (the chunk's buffers are free again);
 * with scotty_tune("shard_async", 1) it returns at once and, as for scotty_process_elements_device, the chunk's
 * buffers must stay valid and unmodified until the op's stream has run the push (order the caller's stream after
 * it with scotty_stream_order, or wait for the next watermark).
 * Watermarks then run unchanged (and identically) on every rank.  Context-free time windows only (the grid
 * path), or count windows with optional context-free time windows (the count path, with
 * scotty_shard_push_counted / scotty_shard_push_timed); other configurations return SCOTTY_ERR_UNSUPPORTED. */
size_t scotty_shard_xbytes(scotty_op* op);
int scotty_shard_push(scotty_op* op, const int64_t* d_ts, const void* d_val, size_t n, int64_t ts0, void* d_xbuf);
int scotty_shard_commit(scotty_op* op, const void* d_gathered, int world);
/* Step 1 for operators with count windows (also accepted by time-window operators, which ignore the counts):
 * n_before = tuples of lower ranks in this micro-batch, n_total = the micro-batch's tuples over all ranks (the
 * chunk's first tuple has count currentCount + n_before, S/WindowManager.java:196-198).  Count windows shard
 * only in-order streams; the record holds per-rank count cells (count_common.h). */
int scotty_shard_push_counted(scotty_op* op, const int64_t* d_ts, const void* d_val, size_t n, int64_t ts0,
                              int64_t n_before, int64_t n_total, void* d_xbuf);
/* Step 1 for count-path operators that also hold context-free TIME windows (in-order stream):
 * additionally ts_before = the largest timestamp of the micro-batch's tuples on lower ranks (INT64_MIN if none)
 * and ts_last = the micro-batch's largest timestamp (INT64_MIN if it is empty).  The time edges a chunk appends
 * are decided from them locally (count_engine.cpp, CEngine::time_edges); callers gather {n, first ts, last ts}
 * per rank before the push (one small all-gather, like the counts). */
int scotty_shard_bounds(scotty_op* op, const int64_t* d_ts, size_t n, int64_t* first_last);  /* chunk's first/last ts */
int scotty_shard_push_timed(scotty_op* op, const int64_t* d_ts, const void* d_val, size_t n, int64_t ts0,
                            int64_t n_before, int64_t n_total, int64_t ts_before, int64_t ts_last, void* d_xbuf);

/* ---- key-hash routing of ONE keyed stream over G ranks (no collective on the hot path).
 * The SPE's keyBy: key k goes to rank keyGroup(k) * G / max_parallelism with keyGroup(k) = murmurHash(k) %
 * max_parallelism (Flink's KeyGroupRangeAssignment, which routes tuples to the reference's per-task operators,
 * F/KeyedScottyWindowOperator.java:56-66).  max_parallelism <= 0 means 128 (the SPE's default for G <= 85). */
int32_t scotty_key_shard(uint32_t key, int world, int max_parallelism);
/* Stable split of a host micro-batch by that shard: out_* hold the G sub-batches back to back, shard s at
 * [offsets[s], offsets[s+1]) (offsets has G+1 entries), each in arrival order.  val_bytes = 4 or 8.  threads <= 0:
 * all hardware threads.  Rank s then pushes its sub-batch with scotty_process_keyed_elements. */
int scotty_route_keyed(const uint32_t* key, const int64_t* ts, const void* val, size_t val_bytes, size_t n,
                       int world, int max_parallelism, int threads, uint32_t* out_key, int64_t* out_ts, void* out_val,
                       uint64_t* offsets);

/* Stream ordering for callers that run the exchange on their own stream (e.g. RCCL through torch.distributed):
 * op_waits == 0: `stream` waits for the work queued on the op's stream so far (the exchange record of a shard push
 * is complete before the all-gather reads it); op_waits != 0: the op's stream waits for the work queued on `stream`
 * (the gathered records have landed before scotty_shard_commit reads them).  With scotty_tune("shard_async", 1) the
 * shard pushes then return without a host synchronisation.  `stream` is a hipStream_t (NULL: the default stream) of
 * the HIP runtime this library is bound to.  PyTorch wheels ship their own libamdhip64.so.7: imported first, it also
 * serves this library (same soname, one runtime), and the Python ShardedSlicingWindowOperator orders torch's stream
 * with this call; with two runtimes mapped (this library loaded before torch) it host-synchronises both sides. */
int scotty_stream_order(scotty_op* op, void* stream, int op_waits);

/* The op's own stream (a hipStream_t of the runtime this library is bound to), for a caller that queues its
 * exchange on it directly (the Python ShardedSlicingWindowOperator runs the RCCL all-gather there, wrapped as a
 * torch.cuda.ExternalStream: push, all-gather and commit then follow each other on one stream, no event, no host
 * synchronisation). */
void* scotty_op_stream(scotty_op* op);

/* Number of keys (operators) of a keyed op. */
int64_t scotty_key_count(scotty_op* op);

/* Counters: tuples dropped as too late since creation; tuples processed. */
uint64_t scotty_dropped_count(scotty_op* op);
uint64_t scotty_processed_count(scotty_op* op);
/* Number of retained slices (LazyAggregateStore.size(), S/aggregationstore/LazyAggregateStore.java:54). */
int64_t scotty_slice_count(scotty_op* op);
/* SCOTTY_AGG_FIRST operators: the arrival indices a later window can still return -- the FIRST partial of every
 * retained non-empty slice, ascending -- into out[0 .. cap).  Returns how many there are (may exceed cap), or a
 * negative status.  The shim keeps the payloads of exactly these tuples after each watermark. */
int64_t scotty_first_indices(scotty_op* op, int64_t* out, size_t cap);

/* Optional HIP-event timing of the dominant (ingest) kernel on the op's stream.  When enabled, each
 * push records events around the ingest kernel; scotty_ingest_timing() returns the summed device
 * milliseconds and launch count since the last reset. */
int scotty_enable_timing(scotty_op* op, int on);
int scotty_ingest_timing(scotty_op* op, double* total_ms, uint64_t* launches, uint64_t* tuples);
/* Device time per class since scotty_enable_timing, from HIP events around each launch group on the op's stream
 * (grid path: every launch and transfer of a micro-batch and a watermark is in exactly one class, so the sum over
 * the classes is the device time of the step; count path: the ingest launch, and the rest of each push / watermark as
 * marker-event intervals on the op's stream).  Resolved at each watermark. */
#define SCOTTY_TIME_INGEST 0      /* the ingest kernel (the HBM-bound pass over the tuples) */
#define SCOTTY_TIME_PUSH_OTHER 1  /* the other kernels of a micro-batch (cell index, edge commit) */
#define SCOTTY_TIME_WATERMARK 2   /* triggers, window assembly, GC */
#define SCOTTY_TIME_RESULT_COPY 3 /* the packed result transfer to the host */
int scotty_device_timing(scotty_op* op, int cls, double* total_ms, uint64_t* intervals);

/* Tuning knobs (not semantics): "slice_capacity" / "session_capacity" per operator of the exact engine
 * (set before the first push), "ingest_mode" (grid-path ingest kernel variant, A/B only), "exact_serial"
 * (non-keyed: single-wavefront replay, A/B only), "keyed_lane" 0 (keyed: wavefront-per-key replay instead of
 * the lane-per-key path for context-free time windows, A/B only), "keyed_grid" 0 (keyed: every batch sorted by
 * key and replayed, instead of the sort-free path for in-order batches of context-free time windows, A/B only),
 * "count_path" 1 (a promise that the stream is in
 * timestamp order: non-keyed operators with count windows only keep no LazySlice record sets and run on the
 * segmented-reduction count path; an out-of-order tuple that would move records then fails loudly -- without the
 * promise they run on the exact engine, which keeps the record sets), "ingest_blocks", "shard_cells" / "shard_cands" (cells /
 * edge candidates per rank record of the time-window exchange), "shard_count_cells" (count cells per rank record
 * of the count-window exchange), "count_prefix_one" 0 (the count path's watermark prefix sums by three kernels
 * instead of one workgroup; tests), "shard_async" 1 (shard pushes return without a host synchronisation: the caller
 * orders its collective's stream with scotty_stream_order -- same HIP runtime only, see there), "exact_prefix" n
 * (exact engine, non-keyed: the first event-exact piece of a batch the one-pass quiet path refused, in tuples;
 * 0 = max(batch / 32, 2^20); later pieces grow 4x; the split is invisible in the results), "quiet_band" 1 (exact
 * engine, non-keyed, one session window: one-pass batches may move the last session's start down -- the stream
 * resuming after a silence then costs one pass instead of event-exact rounds; the results are the same; on by
 * default, 0 for A/B), "keyed_lane_session" (keyed session windows: 0 the wavefront-per-key replay, 1 the lane-per-key
 * kernel's 2-waves-per-SIMD build, the default, 2 its 3-waves build; A/B only, before the first push),
 * "keyed_lane_count" 0 (keyed operators with LazySlice record sets and no session window -- count windows -- through
 * the wavefront-per-key replay instead of the lane-per-key kernel; A/B only), "keyed_sort_digit10" 1 (keyed replay:
 * sort 17-20-bit keys in two 10-bit digit passes instead of three 8-bit ones; A/B only, slower),
 * "keyed_pack_records" 0 (keyed lane-session replay: 16-byte sort records even when a batch's key and event-time bits
 * fit the packed 8-byte ones; A/B only), "lane_session_counters" 1 (debugging aid: count the lane-session kernel's
 * paths). */
int scotty_tune(scotty_op* op, const char* key, int64_t value);

/* Wait for all work enqueued on the op's stream. */
int scotty_sync(scotty_op* op);

#ifdef __cplusplus
}
#endif
#endif
