// count_common.h -- data layout of the count-window path, shared by host and gfx950 kernels.
//
// Serves non-keyed operators whose windows are all context-free COUNT windows (tumbling, sliding, fixed band;
// BASELINE configs[4], BenchmarkRunner "randomCount").  With count windows every slice is a LazySlice
// (S/slice/SliceFactory.java:17-22) and StreamSlicer.determineSlices places an edge exactly when the running
// count reaches the pending count edge (S/StreamSlicer.java:36-44, calculateNextFixedEdgeCount :88-101): the
// edges are the union grid of the windows' assignNextWindowStart in COUNT space and do not depend on the data.
// A tuple's slice is therefore a function of its arrival index alone, and one micro-batch is a segmented
// reduction over arrival order:
//   * the slice started by an edge at count g has tStart = maxEventTime at that moment = max ts of all tuples
//     before it (S/StreamSlicer.java:39-41, :83), cStart = g (S/SliceManager.java:27-38);
//   * a tuple with ts >= tStart of its slice is added to it (the in-order branch, or the out-of-order branch
//     landing in the last slice: no count shift, S/SliceManager.java:56-85);
//   * a tuple with ts < tStart of the oldest retained slice throws IndexOutOfBoundsException in the reference
//     (S/aggregationstore/LazyAggregateStore.java:29-37): dropped and counted, its count still consumed;
//   * a tuple with oldest tStart <= ts < tStart of its own slice would be inserted into an earlier LazySlice and
//     shift the last record of every later slice (:77-85): not on this path (SCOTTY_ERR_UNSUPPORTED, loud).
// cLast of a slice = cStart + tuples added (AbstractSlice.addElement, S/slice/AbstractSlice.java:27-31).
#pragma once
#include <stdint.h>

#include "device_common.h"

namespace scotty {

constexpr int CSTEP = 256;  // tuples per wave step (4 per lane), 8 bitmap words

struct CSlices {  // SoA, absolute indices [head, tail)
  int64_t *ts, *tl, *cs;
  unsigned long long* cnt;
  unsigned long long* p[NPART];
};

struct CCells {  // per-batch partials; cell 0 = the slice open before the batch, cell j = the j-th edge's slice
  unsigned long long* cnt;
  long long* tl;  // max ts of added tuples
  long long* tf;  // min ts of added tuples (out-of-order check)
  unsigned long long* p[NPART];
  int64_t* e_pos;  // [E] batch index of edge j
  int64_t* e_ts;   // [E] tStart of edge j's slice
};

struct CMeta {
  int64_t head, tail;      // retained slices
  int64_t prev_max;        // StreamSlicer.maxEventTime (INT64_MIN before the first tuple)
  uint64_t late_total;     // dropped tuples since creation
  int64_t err;             // != 0: a tuple needs a LazySlice record move (unsupported)
  int64_t n_edges;         // edges of the last push
  int64_t first_start;     // tStart of the oldest retained slice when the push began
  // watermark scalars
  int64_t wm_status;       // 0 ok, 1 empty store, 2 watermark before the oldest slice (getSlice(-1))
  int64_t cend;            // cLast of the count-trigger slice (S/WindowManager.java:109-115)
  int64_t oldest;          // tStart of the oldest retained slice
  int64_t r_lo, r_hi;      // aggregate scan range, absolute [r_lo, r_hi)
  int64_t range_err;       // startIndex == -1 with a non-empty loop (getSlice(-1))
  uint64_t late_push;      // dropped tuples of the current push (folded into late_total by the commit)
  int64_t pad[2];
};

// Time/arrival-range sharding of one count-window stream over G ranks (BASELINE configs[4]):
// rank r ingests its arrival chunk at global count C + n_before_r into local cells and exports one record;
// every rank commits the G records in rank order.  Record (int64 words):
//   [0..15]  header: chunk max ts, dropped tuples, edges E_r, chunk size, count of the chunk's first tuple,
//            overflow (E_r + 1 > cap)
//   cells    cap x {cnt, tLast, tFirst, sum, min, max}   cell 0 = tuples before the chunk's first edge
//   edges    cap x {global count of the edge, max ts before it within the chunk (INT64_MIN if none)}
constexpr int CSHARD_HDR = 16;
__host__ __device__ inline int64_t cshard_words(int64_t cap) { return CSHARD_HDR + 8 * cap; }

struct CWin {  // one context-free window, registration order
  int32_t kind;
  int32_t measure;  // SCOTTY_MEASURE_COUNT, or SCOTTY_MEASURE_TIME (time windows on an in-order stream)
  int64_t a, b;
};

struct CPushArgs {
  const int64_t* ts;
  const void* val;
  int64_t n;
  uint32_t* bits;        // edge bitmap over batch positions
  int64_t nwords;
  int64_t C;             // count of the batch's first tuple (WindowManager.currentCount)
  int64_t mark_from;     // smallest count that can be an edge (the pending edge)
  int64_t extra_point;   // count of the very first edge (first tuple of the stream), or -1
  const CWin* wins;
  int32_t n_wins;
  int32_t need, vt;
  int64_t* stepc;        // [nsteps] edges per step
  int64_t* stepbase;     // [nsteps] exclusive scan of stepc
  int64_t* stepte;       // [nsteps + 1] first time edge at or after each step (te_lb), n_te at the end
  uint32_t* steptp;      // [nsteps] the step's time edges as packed in-step offsets (count_stepc_kernel)
  long long* stepmax;    // [nwaves] max ts per ingest wave (every tuple, dropped ones too)
  long long* steppre;    // [nwaves] inclusive prefix max of stepmax
  int64_t nsteps;
  int64_t per_wave;      // steps per wave
  int64_t nwaves;        // ceil(nsteps / per_wave)
  CCells cells;
  int64_t cell_cap;
  CSlices sl;
  CMeta* meta;
  int32_t shard;         // ingest for a shard record: local prefix max only, no own-ts substitution
  int64_t ts0;           // shard: timestamp of the stream's first tuple (first slice start)
  // time edges of the batch (time windows, in-order stream): batch position of the tuple that appends each edge
  // and the edge, sorted by position then edge; at one position they follow the count edge
  // (StreamSlicer.determineSlices checks the count edge first, S/StreamSlicer.java:36-44 then :46-83)
  const int64_t* te_pos;
  const int64_t* te_g;
  int64_t n_te;
  int32_t check_sorted;  // time windows: flag (CMeta.err bit 8) a batch that is not in timestamp order
};

// Time-edge candidates of one in-order batch: the union time grid from the pending edge N up to the batch max
// (host-enumerated); per candidate the first tuple reaching it decides the edge (commit_kernel's rule: g == N, or
// g == nextGrid(m(g)), or e(g) - g < maxLateness, S/StreamSlicer.java:55-84, :103-116).
struct CTimeArgs {
  const int64_t* ts;
  int64_t n;
  int64_t start;         // first batch position the candidates apply to (1 when position 0 is the stream's first)
  int64_t prev_max;      // maxEventTime before position `start`
  int64_t lateness;
  const int64_t* cand;   // [n_cand] ascending (step == 0)
  int64_t step, cand0;   // step > 0: cand[k] = cand0 + k * step (one common period, no array)
  int64_t n_cand;
  int64_t prev0;         // the grid point before cand[0] (JMIN: cand[0] is the pending edge itself)
  int64_t* te_pos;       // out: [n_te] compacted edges
  int64_t* te_g;
  unsigned long long* n_te;
  int64_t* flag;         // scratch [n_cand] 0/1
  int64_t* off;          // scratch [n_cand] exclusive scan of flag
  int64_t* pos;          // scratch [n_cand]
};

struct CShardArgs {
  const int64_t* gathered;  // world records
  int32_t world;
  int64_t cap;
  int64_t ts0;
  int32_t vt;
  long long* plan;          // [2 * world] slice offset, prefix max before the rank
  CSlices sl;
  CMeta* meta;
};

// Window rows of one window's trigger as an arithmetic run: start = first + k * step, end = start + size
// (k < count); generated on the device in registration order (count_rows_kernel)
struct CRowSeg {
  int64_t first, step, count, size;
  int64_t meas;
};

struct CWmArgs {
  CSlices sl;
  CMeta* meta;
  int64_t wm;
  int64_t min_count, max_count;  // LazyAggregateStore.aggregate arguments (count part)
  int64_t gc_before;             // clearAfterWatermark: wm - maxLateness - maxFixedWindowSize
  const int64_t* w_start;        // [nw] windows (count windows in count space)
  const int64_t* w_end;
  const int32_t* w_meas;         // [nw] SCOTTY_MEASURE_* of each window
  int64_t min_ts, max_ts;        // LazyAggregateStore.aggregate arguments (time part)
  int64_t ts_sorted_from;        // slices from here on have nondecreasing tStart / tLast (CEngine::ts_sorted_from)
  int64_t nw;
  int32_t need, vt, n_aggs, prefix;  // prefix: all aggregations invertible integer kinds -> prefix sums
  int32_t agg_kind[8];
  unsigned long long* pre_cnt;   // [r_hi - r_lo + 1] exclusive prefix sums (prefix mode)
  unsigned long long* pre_sum;
  uint8_t* has_value;
  int64_t* values[8];
};

}  // namespace scotty
