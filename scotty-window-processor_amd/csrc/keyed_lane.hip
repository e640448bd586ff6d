// keyed_lane.hip -- one LANE per key: the keyed exact engine's fast path for operators whose windows are all
// context-free time windows (Tumbling / Sliding / FixedBand) on Eager slices -- the Flink connector's common
// case and BASELINE configs[3] (C4).  For this subset the reference's per-tuple work is a short scalar state
// machine (StreamSlicer.determineSlices, S/StreamSlicer.java:36-116, and SliceManager.processElement,
// S/SliceManager.java:47-87, without context-aware windows): a wavefront per key (exact_kernels.hip) spends
// 64 lanes on it, here one lane walks a key's ~16 tuples of a micro-batch with the current slice's partials
// held in registers.  The state layout (XState, slice SoA) is the exact engine's, so configurations can move
// between the two paths mid-stream.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "exact_common.h"
#include "exact_op.h"

namespace scotty {
namespace ln {

constexpr int64_t JMAX = INT64_MAX, JMIN = INT64_MIN;
constexpr int64_t ID_MIN = INT64_MAX;
constexpr int64_t ID_MAX = INT64_MIN;

__device__ __forceinline__ int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
__device__ __forceinline__ int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
__device__ __forceinline__ int64_t jmod(int64_t a, int64_t b) { return b == -1 ? 0 : a % b; }
__device__ __forceinline__ int64_t f64_key(double d) {
  const int64_t b = __double_as_longlong(d);
  return b ^ ((b >> 63) & 0x7FFFFFFFFFFFFFFFLL);
}

// assignNextWindowStart (TumblingWindow.java:29-31, SlidingWindow.java:41-43, FixedBandWindow.java:37-48)
__device__ __forceinline__ int64_t assign_next(const XCfg* c, int w, int64_t t) {
  const int k = c->cf_kind[w];
  const int64_t a = c->cf_a[w], b = c->cf_b[w];
  if (k == 0) return jsub(jadd(t, a), jmod(t, a));
  if (k == 1) return jsub(jadd(t, b), jmod(t, b));
  if (t == JMAX || t < a) return a;
  if (t >= a && t < jadd(a, b)) return jadd(a, b);
  return JMAX;
}

// One key's slice list.  The slice columns are the kernel argument's (uniform, SGPRs); a lane holds only its
// key's base offset, the StreamSlicer / store scalars it changes, and the current slice's aggregation fields
// (VGPR budget: the kernel is latency bound, occupancy is what hides the per-key record and slice loads).
// MM: the operator has a MIN or MAX aggregation (partials p[1] / p[2] live).
template <int VT, bool MM, class V>
struct Lane {
  const XCfg* c;
  V sl;
  int64_t b;  // op * sc
  // XState fields the per-tuple path changes
  int64_t maxEventTime, nextEdgeTs, currentCount;
  int32_t head, tail, started;
  uint32_t dropped;
  int32_t minmod;  // lowest slice position whose cnt / sum changed (slice prefixes above it go stale)
  // register copy of the current (last) slice
  int32_t ci;
  int64_t c_tl, c_tf, c_cl;
  uint64_t c_cnt, c_p0;
  int64_t c_p1, c_p2;
  bool hang;

  __device__ void load_cur() {
    ci = tail - 1;
    if (ci < head) {
      ci = -1;
      c_tl = JMIN;  // empty store: the first tuple appends
      return;
    }
    const int64_t j = b + ci;
    c_tl = sl.tl[j]; c_tf = sl.tf[j]; c_cl = sl.cl[j];
    c_cnt = sl.cnt[j]; c_p0 = sl.p[0][j];
    if (MM) {
      c_p1 = (int64_t)sl.p[1][j];
      c_p2 = (int64_t)sl.p[2][j];
    }
  }
  __device__ void flush_cur() {
    if (ci < 0) return;
    const int64_t j = b + ci;
    sl.tl[j] = c_tl; sl.tf[j] = c_tf; sl.cl[j] = c_cl;
    sl.cnt[j] = c_cnt; sl.p[0][j] = c_p0;
    if (MM) {
      sl.p[1][j] = (unsigned long long)c_p1;
      sl.p[2][j] = (unsigned long long)c_p2;
    }
  }
  // calculateNextFixedEdge (S/StreamSlicer.java:103-116), time windows
  __device__ int64_t next_fixed_edge(int64_t te_) const {
    const int64_t cur = nextEdgeTs == JMIN ? JMAX : nextEdgeTs;
    const int64_t t_c = max(jsub(te_, c->max_lateness), cur);
    int64_t e = JMAX;
    for (int w = 0; w < c->n_cf; w++) e = min(e, assign_next(c, w, t_c));  // all time-measured here
    return e;
  }
  // SliceManager.appendSlice (S/SliceManager.java:27-38); a new slice starts Flexible(1), empty
  __device__ void append(int64_t start, int32_t type) {
    if (ci >= 0) {
      flush_cur();
      sl.te[b + ci] = start;
      sl.ty[b + ci] = type;
    }
    const int64_t j = b + tail;
    sl.ts[j] = start; sl.te[j] = JMAX; sl.cs[j] = currentCount; sl.ty[j] = 1;
    ci = tail;
    tail++;
    c_tl = start; c_tf = JMAX; c_cl = currentCount;
    c_cnt = 0; c_p0 = 0; c_p1 = ID_MIN; c_p2 = ID_MAX;
  }
  __device__ static void lift(int64_t vb, int64_t& mn, int64_t& mx) {
    if (VT == VT_F64) {
      const double d = __longlong_as_double(vb);
      mn = d != d ? INT64_MIN : f64_key(d);
      mx = d != d ? INT64_MAX : f64_key(d);
    } else {
      mn = vb;
      mx = vb;
    }
  }
  __device__ static uint64_t add_sum(uint64_t acc, int64_t vb) {
    if (VT == VT_F64)
      return (uint64_t)__double_as_longlong(__longlong_as_double((long long)acc) + __longlong_as_double(vb));
    return acc + (uint64_t)vb;
  }
  // AbstractSlice.addElement + AggregateState.addElement on the current slice (registers)
  __device__ void add_cur(int64_t t, int64_t vb) {
    c_tl = max(c_tl, t);
    c_tf = min(c_tf, t);
    c_cl = jadd(c_cl, 1);
    c_cnt++;
    if (c->need & NEED_SUM) c_p0 = add_sum(c_p0, vb);
    if (MM) {
      int64_t mn, mx;
      lift(vb, mn, mx);
      c_p1 = min(c_p1, mn);
      c_p2 = max(c_p2, mx);
    }
  }
  // ... on an older slice (out-of-order tuple), in HBM
  __device__ void add_mem(int i, int64_t t, int64_t vb) {
    const int64_t j = b + i;
    minmod = min(minmod, i);
    sl.tl[j] = max(sl.tl[j], t);
    sl.tf[j] = min(sl.tf[j], t);
    sl.cl[j] = jadd(sl.cl[j], 1);
    sl.cnt[j] = sl.cnt[j] + 1;
    if (c->need & NEED_SUM) sl.p[0][j] = add_sum(sl.p[0][j], vb);
    if (MM) {
      int64_t mn, mx;
      lift(vb, mn, mx);
      sl.p[1][j] = (unsigned long long)min((int64_t)sl.p[1][j], mn);
      sl.p[2][j] = (unsigned long long)max((int64_t)sl.p[2][j], mx);
    }
  }
  // LazyAggregateStore.findSliceIndexByTimestamp (:29-37) on a sorted list: last slice with tStart <= t
  __device__ int find_ts(int64_t t) const {
    int lo = head, hi = tail;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sl.ts[b + mid] <= t) lo = mid + 1; else hi = mid;
    }
    return lo - 1 >= head ? lo - 1 : -1;
  }
  // SlicingWindowOperator.processElement (S/SlicingWindowOperator.java:41-44) for this subset
  __device__ void process(int64_t t, int64_t vb) {
    if (t >= maxEventTime) {  // StreamSlicer.determineSlices, in-order branch (:51-86)
      if (nextEdgeTs == JMIN) nextEdgeTs = next_fixed_edge(t);
      while (t > nextEdgeTs) {
        if (nextEdgeTs >= 0) append(nextEdgeTs, XTYPE_FIXED);
        nextEdgeTs = next_fixed_edge(t);
        if (nextEdgeTs == JMIN) {  // the reference loops forever here (power-of-two size / slide)
          hang = true;
          return;
        }
      }
      if (nextEdgeTs == t) {
        append(t, XTYPE_FIXED);
        nextEdgeTs = next_fixed_edge(t);
      }
    }
    currentCount = jadd(currentCount, 1);  // WindowManager.incrementCount
    maxEventTime = max(t, maxEventTime);
    if (tail <= head) append(0, 1);  // SliceManager.processElement: empty store (:49-51)
    started = 1;
    if (t >= c_tl) {
      add_cur(t, vb);
    } else {
      const int idx = find_ts(t);
      if (idx < 0) dropped++;  // IndexOutOfBoundsException in the reference: the tuple is lost
      else if (idx == ci) add_cur(t, vb);
      else add_mem(idx, t, vb);
    }
  }
};

template <int VT, bool MM, class V>
__global__ __launch_bounds__(256) void lane_replay_kernel(XBatchArgs a) {
  const XCfg* cfg = a.cfg;
  const int64_t op = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (op >= a.n_ops) return;
  const int64_t b0 = a.seg_begin[op], b1 = a.seg_end[op];
  if (b1 <= b0) return;
  XState* sp = a.st + op;
  if (sp->err) return;
  if (a.retry && !sp->pending) return;
  const unsigned char* rec = (const unsigned char*)a.ts;
  auto load = [&](int64_t i, int64_t& t, int64_t& vb) {
    const unsigned char* r = rec + i * a.rec_stride;
    t = *(const int64_t*)r;
    if constexpr (VT == VT_I32) vb = (int64_t)*(const int32_t*)(r + 8);
    else vb = *(const int64_t*)(r + 8);
  };
  Lane<VT, MM, V> L{};
  L.c = cfg;
  L.sl = xview<V>(a.sl);
  L.b = op * (int64_t)cfg->sc;
  L.maxEventTime = sp->maxEventTime;
  L.nextEdgeTs = sp->nextEdgeTs;
  L.currentCount = sp->currentCount;
  L.head = sp->head;
  L.tail = sp->tail;
  L.started = sp->started;
  L.dropped = 0;
  L.hang = false;
  int32_t pvalid = sp->pvalid;
  // capacity pre-check (same bound as the wavefront replay): defer the key, the host grows and retries
  // the lane's run is read 4 records per round so 4 scattered loads are in flight at once (the kernel waits on
  // memory, not ALU: SQ_WAIT_ANY is ~80% of its wave cycles)
  int64_t tmin = JMAX, tmax = JMIN;
  int64_t i = b0;
  for (; i + 4 <= b1; i += 4) {
    int64_t t0, t1, t2, t3, v_;
    load(i, t0, v_);
    load(i + 1, t1, v_);
    load(i + 2, t2, v_);
    load(i + 3, t3, v_);
    tmin = min(tmin, min(min(t0, t1), min(t2, t3)));
    tmax = max(tmax, max(max(t0, t1), max(t2, t3)));
  }
  for (; i < b1; i++) {
    int64_t t, vb;
    load(i, t, vb);
    tmin = min(tmin, t);
    tmax = max(tmax, t);
  }
  int64_t from = L.started ? max(L.maxEventTime, jsub(tmin, cfg->max_lateness)) : jsub(tmin, cfg->max_lateness);
  if (from > tmax) from = tmax;
  const double span = (double)tmax - (double)from;
  double bound = 4.0;
  for (int w = 0; w < cfg->n_cf; w++) {
    const int k = cfg->cf_kind[w];
    bound += k == 2 ? 2.0 : span / (double)(k == 0 ? cfg->cf_a[w] : cfg->cf_b[w]) + 2.0;
  }
  const double need_s = (double)(L.tail - L.head) + bound;
  if (need_s > (double)cfg->sc) {
    atomicMax(&a.need[0], (unsigned long long)min(need_s, 1e15) + 2ull);
    sp->pending = 1;
    return;
  }
  sp->pending = 0;
  if ((double)L.tail + bound > (double)cfg->sc && L.head > 0) {  // compact [head, tail) to the front
    const int n = L.tail - L.head;
    const int64_t h = L.b + L.head, d = L.b;
    const V q = xview<V>(a.sl);
    for (int i = 0; i < n; i++) {
      q.ts[d + i] = q.ts[h + i]; q.te[d + i] = q.te[h + i]; q.tl[d + i] = q.tl[h + i]; q.tf[d + i] = q.tf[h + i];
      q.cs[d + i] = q.cs[h + i]; q.cl[d + i] = q.cl[h + i]; q.ty[d + i] = q.ty[h + i];
      q.cnt[d + i] = q.cnt[h + i];
      for (int p = 0; p < NPART; p++) q.p[p][d + i] = q.p[p][h + i];
    }
    L.head = 0;
    L.tail = n;
    pvalid = 0;
  }
  L.minmod = max(L.tail - 1, 0);  // the current slice takes the in-order tuples, appended slices follow it
  L.load_cur();
  // replay with the next record's load issued before the current record is processed
  int64_t t_nx, v_nx;
  load(b0, t_nx, v_nx);
  for (int64_t j = b0; j < b1 && !L.hang; j++) {
    const int64_t t = t_nx, vb = v_nx;
    if (j + 1 < b1) load(j + 1, t_nx, v_nx);
    L.process(t, vb);
  }
  L.flush_cur();
  sp->maxEventTime = L.maxEventTime;
  sp->nextEdgeTs = L.nextEdgeTs;
  sp->currentCount = L.currentCount;
  sp->head = L.head;
  sp->tail = L.tail;
  sp->started = L.started;
  if (L.dropped) sp->dropped += L.dropped;
  if (L.hang) sp->err = XERR_HANG;
  sp->pvalid = min(pvalid, L.minmod);
}

// ---------------------------------------------------------------- watermark, one lane per key
// Triggered context-free time windows of one key (S/WindowManager.java:104-118, C/windowType/*.triggerWindows)
template <bool EMIT>
__device__ int64_t lane_triggers(const XCfg* c, int64_t last, int64_t wm, int64_t* w_start, int64_t* w_end,
                                 int32_t* w_meas, int32_t* w_op, int64_t off, int32_t op, int64_t& minTs,
                                 int64_t& maxTs) {
  int64_t k = 0;
  auto emit = [&](int64_t st, int64_t en) {
    if (EMIT) {
      w_start[off + k] = st;
      w_end[off + k] = en;
      w_meas[off + k] = 0;
      w_op[off + k] = op;
    }
    minTs = min(minTs, st);
    maxTs = max(maxTs, en);
    k++;
  };
  for (int w = 0; w < c->n_cf; w++) {
    const int kind = c->cf_kind[w];
    const int64_t a = c->cf_a[w], b = c->cf_b[w];
    if (kind == 0) {
      const int64_t ls = jsub(last, jmod(jadd(last, a), a));
      for (int64_t ws = ls; jadd(ws, a) <= wm; ws = jadd(ws, a)) emit(ws, jadd(ws, a));
    } else if (kind == 1) {
      const int64_t ls = jsub(wm, jmod(jadd(wm, b), b));
      for (int64_t ws = ls; jadd(ws, a) > last; ws = jsub(ws, b))
        if (ws >= 0 && jadd(ws, a) <= jadd(wm, 1)) emit(ws, jadd(ws, a));
    } else {
      const int64_t e = jadd(a, b);
      if (last <= e && e <= wm) emit(a, e);
    }
  }
  return k;
}

// SessionContext.triggerWindows of each session context (C/windowType/SessionWindow.java:107-116, after the
// context-free windows, S/WindowManager.java:104-118): the sessions with end + gap < wm, oldest first, as windows
// [start, end + gap); EMIT also drops them from the context (the remaining ones move to the front).  Returns -1 for
// an empty context (getWindow(0) throws IndexOutOfBoundsException).
template <bool EMIT>
__device__ int64_t lane_session_triggers(const XCfg* c, const XSess& x, int64_t op, XState& s, int64_t wm,
                                         int64_t* w_start, int64_t* w_end, int32_t* w_meas, int32_t* w_op, int64_t off,
                                         int64_t& minTs, int64_t& maxTs) {
  int64_t k = 0;
  for (int ctx = 0; ctx < c->n_ctx; ctx++) {
    const int64_t gap = c->gap[ctx];
    const int ns = s.ns(ctx);
    if (ns == 0) return -1;
    const int64_t sb = (op * c->ctx_alloc + ctx) * (int64_t)c->sesscap;
    int64_t* const st = x.start + sb;
    int64_t* const en = x.end + sb;
    int i = 0;
    for (; i < ns; i++) {
      const int64_t e = jadd(en[i], gap);
      if (!(e < wm)) break;
      const int64_t b = st[i];
      if (EMIT) {
        w_start[off + k] = b;
        w_end[off + k] = e;
        w_meas[off + k] = 0;  // time-measured contexts only on this path
        w_op[off + k] = (int32_t)op;
      }
      minTs = min(minTs, b);
      maxTs = max(maxTs, e);
      k++;
    }
    if (EMIT && i > 0) {
      for (int j = i; j < ns; j++) {
        st[j - i] = st[j];
        en[j - i] = en[j];
      }
      s.set_ns(ctx, ns - i);
    }
  }
  return k;
}

// The dropped-tuple total and the error bits of a workgroup's keys: one atomic each per workgroup (the compiler
// combines a wavefront's same-address atomics into one, but one per wavefront still serialised 16 K atomics on one
// word per watermark at 1 M keys -- ~90 atomics per us)
template <int T>
__device__ __forceinline__ void block_flush(unsigned long long dropped, int32_t err_bits, unsigned long long* d_total,
                                            int32_t* d_err) {
  __shared__ unsigned long long s_d[T / 64];
  __shared__ int32_t s_e[T / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    dropped += (unsigned long long)__shfl_xor((long long)dropped, o);
    err_bits |= __shfl_xor(err_bits, o);
  }
  if (lane == 0) {
    s_d[wid] = dropped;
    s_e[wid] = err_bits;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long d = 0;
    int32_t e = 0;
    for (int w = 0; w < T / 64; w++) {
      d += s_d[w];
      e |= s_e[w];
    }
    if (d) atomicAdd(d_total, d);
    if (e) atomicOr(d_err, e);
  }
}

constexpr int COUNT_T = 1024;
template <class V>
__global__ __launch_bounds__(COUNT_T) void lane_wm_count_kernel(XWmArgs a) {
  const int64_t op = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = op < a.n_ops;
  XState s{};
  if (live) s = a.st[op];
  block_flush<COUNT_T>(live ? s.dropped : 0, live && s.err ? 1 << s.err : 0, a.dropped_total, a.op_err);
  if (!live) return;
  int64_t k = 0;
  if (!s.err && s.tail > s.head) {
    int64_t last = s.lastWatermark == -1 ? max((int64_t)0, jsub(a.wm, a.cfg->max_lateness)) : s.lastWatermark;
    const int64_t oldest = xview<V>(a.sl).ts[op * (int64_t)a.cfg->sc + s.head];
    if (last < oldest) last = oldest;
    int64_t mn = JMAX, mx = 0;
    k = lane_triggers<false>(a.cfg, last, a.wm, nullptr, nullptr, nullptr, nullptr, 0, 0, mn, mx);
    if (a.cfg->n_ctx > 0) {
      XState s2 = s;
      const int64_t ks = lane_session_triggers<false>(a.cfg, a.ss, op, s2, a.wm, nullptr, nullptr, nullptr, nullptr, 0,
                                                      mn, mx);
      if (ks < 0) atomicOr(a.err_flag, 1);
      else k += ks;
    }
  }
  a.wcount[op] = k;
}

// first position in [lo, hi) where the monotone predicate p turns true (hi if never), probing from lo upward
// (galloping: a target near lo costs a few loads, not a full bisection's chain of dependent ones)
template <typename P>
__device__ __forceinline__ int first_true_up(int lo, int hi, P p) {
  if (lo >= hi || p(lo)) return lo;
  int a = lo, step = 1;  // !p(a)
  while (a + step < hi && !p(a + step)) {
    a += step;
    step <<= 1;
  }
  int c = min(a + step, hi);  // p(c) or c == hi
  while (c - a > 1) {
    const int m = (a + c) >> 1;
    if (p(m)) c = m; else a = m;
  }
  return c;
}
// the same position, probing from hi - 1 downward
template <typename P>
__device__ __forceinline__ int first_true_down(int lo, int hi, P p) {
  if (lo >= hi || !p(hi - 1)) return hi;
  int c = hi - 1, step = 1;  // p(c)
  while (c - step >= lo && p(c - step)) {
    c -= step;
    step <<= 1;
  }
  int a = max(c - step, lo - 1);  // !p(a) or a == lo - 1
  while (c - a > 1) {
    const int m = (a + c) >> 1;
    if (p(m)) c = m; else a = m;
  }
  return c;
}

// WindowManager.processWatermark for one key (S/WindowManager.java:38-61): triggered windows, the
// LazyAggregateStore.aggregate scan range (:83-90, its getSlice(-1) exception included), clearAfterWatermark
// (:82-95).  AGG: also the windows' values -- COUNT and integer SUM from the slice prefixes (extended from
// XState.pvalid to tail first), so a window costs two gallops and two reads instead of a scan of its slices
// (S/slice/SliceManager... AggregateWindowState over the contained slices, S/state/AggregateWindowState.java);
// without AGG the host runs wm_agg_kernel over [wlo, whi) (MIN / MAX / f64 sums).
//
// Rows: with a.row_count the kernel also counts (no separate count pass): each wavefront reserves its keys' rows
// with one atomic, the host having sized the row columns from a bound (lane_row_bound); else at a.woff[op].
constexpr int EMIT_T = 1024;
template <bool AGG, class V>
__global__ __launch_bounds__(EMIT_T) void lane_wm_emit_kernel(XWmArgs a) {
  const int64_t op = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const XCfg* c = a.cfg;
  const V q = xview<V>(a.sl);
  const int64_t base = op * (int64_t)c->sc;
  const auto ts = q.ts + base;
  XState s{};
  bool live = op < a.n_ops;
  int64_t k = 0;
  if (live) s = a.st[op];
  if (a.row_count)  // what the count pass accumulates (uniform: every thread of the workgroup takes this)
    block_flush<EMIT_T>(live ? s.dropped : 0, live && s.err ? 1 << s.err : 0, a.dropped_total, a.op_err);
  if (live) {
    if (s.err) {
      live = false;
    } else {
      if (s.lastWatermark == -1) s.lastWatermark = max((int64_t)0, jsub(a.wm, c->max_lateness));  // :43-44
      if (s.tail <= s.head) {
        s.lastWatermark = a.wm;
        a.st[op] = s;
        live = false;
      } else {
        if (s.lastWatermark < ts[s.head]) s.lastWatermark = ts[s.head];
        if (a.row_count) {
          int64_t mn = JMAX, mx = 0;
          k = lane_triggers<false>(c, s.lastWatermark, a.wm, nullptr, nullptr, nullptr, nullptr, 0, 0, mn, mx);
          if (c->n_ctx > 0) {  // (the host takes this one-kernel mode for context-free windows only)
            XState s2 = s;
            const int64_t ks = lane_session_triggers<false>(c, a.ss, op, s2, a.wm, nullptr, nullptr, nullptr, nullptr,
                                                            0, mn, mx);
            if (ks < 0) {
              atomicOr(a.err_flag, 1);
              live = false;
            } else {
              k += ks;
            }
          }
        }
      }
    }
  }
  int64_t off = 0;
  if (a.row_count) {  // workgroup-aggregated row reservation: one atomic per workgroup (one counter word takes
                      // only ~90 atomics per us, a per-wavefront reservation would serialise on it)
    __shared__ long long s_w[EMIT_T / 64 + 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t inc = k;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t u = (int64_t)__shfl_up((long long)inc, o);
      if (lane >= o) inc += u;
    }
    if (lane == 63) s_w[wid] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
      long long run = 0;
      for (int w = 0; w < EMIT_T / 64; w++) {
        const long long v = s_w[w];
        s_w[w] = run;
        run += v;
      }
      s_w[EMIT_T / 64] = run > 0 ? (long long)atomicAdd(a.row_count, (unsigned long long)run) : 0;
    }
    __syncthreads();
    off = (int64_t)s_w[EMIT_T / 64] + (int64_t)s_w[wid] + inc - k;
    if (live && off + k > a.n_rows) {  // the host bound was wrong: nothing is written, the call fails
      atomicOr(a.err_flag, 4);
      return;
    }
  } else if (live) {
    off = a.woff[op];
  }
  if (!live) return;
  const auto tl = q.tl + base;
  const auto cs = q.cs + base;
  int64_t minTs = JMAX, maxTs = 0;
  k = lane_triggers<true>(c, s.lastWatermark, a.wm, a.w_start, a.w_end, a.w_meas, a.w_op, off, (int32_t)op, minTs,
                          maxTs);
  if (c->n_ctx > 0)  // (the count pass has thrown for an empty context; no single-kernel row bound covers sessions)
    k += lane_session_triggers<true>(c, a.ss, op, s, a.wm, a.w_start, a.w_end, a.w_meas, a.w_op, off + k, minTs, maxTs);
  const int h = s.head, t = s.tail;
  // find_ts / find_count: last slice with key <= x (LazyAggregateStore.findSliceIndexBy*, :29-50), -1 if none
  auto last_ts_le_up = [&](int64_t x) { return first_true_up(h, t, [&](int i) { return ts[i] > x; }) - 1; };
  auto last_ts_le_dn = [&](int64_t x) { return first_true_down(h, t, [&](int i) { return ts[i] > x; }) - 1; };
  auto last_cs_le_up = [&](int64_t x) { return first_true_up(h, t, [&](int i) { return cs[i] > x; }) - 1; };
  auto last_cs_le_dn = [&](int64_t x) { return first_true_down(h, t, [&](int i) { return cs[i] > x; }) - 1; };
  auto fix = [&](int i) { return i < h ? -1 : i; };
  if (AGG) {
    // the scan range only bounds the contained slices, which the prefix lookup finds directly; its getSlice(-1)
    // exception needs cStart[head] > currentCount, impossible here (cStart is the count at append time)
    s.wlo = h;
    s.whi = t;
  } else if (k > 0) {  // LazyAggregateStore.aggregate scan range (:83-90); no count windows: minCount = currentCount
    const int S = t - h;
    auto rel = [&](int i) { return i < 0 ? -1 : i - h; };
    int si = max(rel(fix(last_ts_le_up(minTs))), 0);
    si = min(si, rel(fix(last_cs_le_dn(s.currentCount))));
    int ei = min(S - 1, rel(fix(last_ts_le_dn(maxTs))));
    ei = max(ei, rel(fix(last_cs_le_up(0))));
    if (si < 0 && si <= ei) {
      atomicOr(a.err_flag, 2);
      si = 0;
    }
    s.wlo = h + si;
    s.whi = h + ei + 1;
  } else {
    s.wlo = s.whi = h;
  }
  if (AGG && k > 0) {
    const bool sums = (c->need & NEED_SUM) != 0;
    // MIN / MAX (integer values, key-interleaved store only): block summaries instead of a scan of each window's
    // slices (LazyAggregateStore.aggregate's per-slice AggregateWindowState.addState, :83-111, regrouped: min / max
    // are associative, and the slices of a window's run are combined in blocks)
    constexpr bool KW = std::is_same<V, XKView>::value;
    const bool mmin = KW && (c->need & NEED_MIN) != 0, mmax = KW && (c->need & NEED_MAX) != 0;
    const auto pc = q.pc + base;
    const auto ps = q.ps + base;
    const auto cnt = q.cnt + base;
    const auto p0 = q.p[0] + base;
    const auto p1 = q.p[1] + base;
    const auto p2 = q.p[2] + base;
    int pv = a.prefix_reset ? 0 : s.pvalid;
    if (pv < t) {  // extend the prefixes over the slices changed since the last watermark
      unsigned long long rc = pv > 0 ? pc[pv - 1] : 0, rs = pv > 0 && sums ? ps[pv - 1] : 0;
      for (int i = pv; i < t; i++) {
        rc += cnt[i];
        pc[i] = rc;
        if (sums) {
          rs += p0[i];
          ps[i] = rs;
        }
      }
      if constexpr (KW) {
        if (mmin || mmax) {
          const auto qn = q.qn + base, sn = q.sn + base, qx = q.qx + base, sx = q.sx + base;
          // in-block prefixes of the changed positions (a block's first position starts its own)
          int64_t rn = (pv % XK_MB) ? qn[pv - 1] : ID_MIN, rx = (pv % XK_MB) ? qx[pv - 1] : ID_MAX;
          for (int i = pv; i < t; i++) {
            if (i % XK_MB == 0) {
              rn = ID_MIN;
              rx = ID_MAX;
            }
            if (mmin) qn[i] = rn = min(rn, (int64_t)p1[i]);
            if (mmax) qx[i] = rx = max(rx, (int64_t)p2[i]);
          }
          // in-block suffixes of every complete block that holds a changed position
          for (int b0 = pv - pv % XK_MB; b0 + XK_MB <= t; b0 += XK_MB) {
            int64_t un = ID_MIN, ux = ID_MAX;
            for (int i = b0 + XK_MB - 1; i >= b0; i--) {
              if (mmin) sn[i] = un = min(un, (int64_t)p1[i]);
              if (mmax) sx[i] = ux = max(ux, (int64_t)p2[i]);
            }
          }
        }
      }
      pv = t;
    }
    s.pvalid = pv;
    const bool sorted = !(s.unsorted & 3);
    const int lo0 = (int)s.wlo, hi0 = (int)s.whi;
    const uint32_t key = a.slot_key ? a.slot_key[op] : (uint32_t)op;
    for (int64_t r = off; r < off + k; r++) {
      const int64_t ws = a.w_start[r], we = a.w_end[r];
      uint64_t cn = 0, sw = 0;
      int64_t mn = ID_MIN, mx = ID_MAX;
      if (sorted) {  // the contained slices (ws <= tStart, tLast < we) are the run [lo, hi): tLast increases
        const int lo = first_true_up(lo0, hi0, [&](int i) { return ts[i] >= ws; });
        const int hi = first_true_down(lo, hi0, [&](int i) { return tl[i] >= we; });
        if (hi > lo) {
          cn = pc[hi - 1] - (lo > 0 ? pc[lo - 1] : 0ull);
          if (sums) sw = ps[hi - 1] - (lo > 0 ? ps[lo - 1] : 0ull);
          if constexpr (KW) {
            if (mmin || mmax) {
              const auto qn = q.qn + base, sn = q.sn + base, qx = q.qx + base, sx = q.sx + base;
              const int bl = lo / XK_MB, bh = (hi - 1) / XK_MB;
              if (bl == bh) {  // within one block: its slices (at most XK_MB)
                for (int i = lo; i < hi; i++) {
                  if (mmin) mn = min(mn, (int64_t)p1[i]);
                  if (mmax) mx = max(mx, (int64_t)p2[i]);
                }
              } else {  // suffix of lo's (complete) block, whole blocks, prefix of hi - 1's block
                if (mmin) mn = min(sn[lo], qn[hi - 1]);
                if (mmax) mx = max(sx[lo], qx[hi - 1]);
                for (int b = bl + 1; b < bh; b++) {
                  const int e = b * XK_MB + XK_MB - 1;
                  if (mmin) mn = min(mn, (int64_t)qn[e]);
                  if (mmax) mx = max(mx, (int64_t)qx[e]);
                }
              }
            }
          }
        }
      } else {
        for (int i = lo0; i < hi0; i++) {
          if (!(ws <= ts[i] && we > tl[i])) continue;
          cn += cnt[i];
          if (sums) sw += p0[i];
          if (mmin) mn = min(mn, (int64_t)p1[i]);
          if (mmax) mx = max(mx, (int64_t)p2[i]);
        }
      }
      const bool present = cn != 0;
      a.has_value[r] = present ? 1 : 0;
      if (a.w_key) a.w_key[r] = key;
      for (int q = 0; q < c->n_aggs; q++)
        a.values[q][r] = present ? x::lower_value(c->agg_kind[q], cn, sw, mn, mx) : 0;
    }
  }
  s.lastWatermark = a.wm;
  s.lastCount = s.currentCount;
  // clearAfterWatermark (:82-95): below the oldest session start of any context as well
  const int64_t cw = jsub(a.wm, c->max_lateness);
  int64_t first = cw;
  for (int ctx = 0; ctx < c->n_ctx; ctx++) {
    const int64_t* st = a.ss.start + (op * c->ctx_alloc + ctx) * (int64_t)c->sesscap;
    for (int i = 0; i < s.ns(ctx); i++) first = min(first, st[i]);
  }
  const int64_t gt = min(jsub(cw, c->max_fixed), first);
  const int idx = fix(last_ts_le_up(gt));
  if (idx > s.head) s.head = idx;
  a.st[op] = s;
}

}  // namespace ln

hipError_t launch_lane_replay(const XBatchArgs& a, const XCfg& host_cfg, hipStream_t st) {
  if (a.n_ops <= 0) return hipSuccess;
  const dim3 grid((unsigned)((a.n_ops + 255) / 256)), block(256);
  const bool mm = (host_cfg.need & (NEED_MIN | NEED_MAX)) != 0;
  const int vt = host_cfg.vt;
  if (a.sl.kw) {  // key-interleaved store: integer values (COUNT, SUM, MIN, MAX; no f64)
    if (vt == VT_I32) {
      if (mm) hipLaunchKernelGGL((ln::lane_replay_kernel<VT_I32, true, XKView>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((ln::lane_replay_kernel<VT_I32, false, XKView>), grid, block, 0, st, a);
    } else {
      if (mm) hipLaunchKernelGGL((ln::lane_replay_kernel<VT_I64, true, XKView>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((ln::lane_replay_kernel<VT_I64, false, XKView>), grid, block, 0, st, a);
    }
    return hipGetLastError();
  }
#define SCOTTY_LANE(V, M) hipLaunchKernelGGL((ln::lane_replay_kernel<V, M, XSlices>), grid, block, 0, st, a)
  if (vt == VT_I32) { if (mm) SCOTTY_LANE(VT_I32, true); else SCOTTY_LANE(VT_I32, false); }
  else if (vt == VT_I64) { if (mm) SCOTTY_LANE(VT_I64, true); else SCOTTY_LANE(VT_I64, false); }
  else { if (mm) SCOTTY_LANE(VT_F64, true); else SCOTTY_LANE(VT_F64, false); }
#undef SCOTTY_LANE
  return hipGetLastError();
}
hipError_t launch_lane_wm_count(const XWmArgs& a, hipStream_t st) {
  if (a.n_ops <= 0) return hipSuccess;
  const dim3 grid((unsigned)((a.n_ops + ln::COUNT_T - 1) / ln::COUNT_T)), block(ln::COUNT_T);
  if (a.sl.kw) hipLaunchKernelGGL(ln::lane_wm_count_kernel<XKView>, grid, block, 0, st, a);
  else hipLaunchKernelGGL(ln::lane_wm_count_kernel<XSlices>, grid, block, 0, st, a);
  return hipGetLastError();
}
hipError_t launch_lane_wm_emit(const XWmArgs& a, bool agg, hipStream_t st) {
  if (a.n_ops <= 0) return hipSuccess;
  const dim3 grid((unsigned)((a.n_ops + ln::EMIT_T - 1) / ln::EMIT_T)), block(ln::EMIT_T);
  if (a.sl.kw) hipLaunchKernelGGL((ln::lane_wm_emit_kernel<true, XKView>), grid, block, 0, st, a);
  else if (agg) hipLaunchKernelGGL((ln::lane_wm_emit_kernel<true, XSlices>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((ln::lane_wm_emit_kernel<false, XSlices>), grid, block, 0, st, a);
  return hipGetLastError();
}

}  // namespace scotty
