// keyed_lane_count.hip -- lane-per-key replay of keyed operators that keep LazySlice record sets and have no session
// windows: count windows beside context-free time windows on out-of-order streams.
//
// The reference runs one SlicingWindowOperator per key (flink-connector/.../KeyedScottyWindowOperator.java:56-86).
// With a count window every slice is a LazySlice holding its tuples in a TreeSet ordered by ts
// (S/slice/SliceFactory.java:17-22, S/slice/LazySlice.java:14-54), and an out-of-order tuple runs SliceManager's
// count-shift loop: every later slice hands its last record to the next one so each slice keeps its count
// (S/SliceManager.java:64-87).  The wavefront replay (exact_kernels.hip replay_kernel) restates that with one
// wavefront per key: every out-of-order tuple is an "event" of ~10-20 dependent memory round trips that one wavefront
// waits for alone (C4c, 2^20 keys: 78 ms per 2^26-tuple batch).  Here one LANE restates one key's operator tuple by
// tuple, exactly as exact_op.h's Op does for the same store (XSlices columns, the op's record arena, XState), so 64
// keys wait on their chains side by side and the watermark kernels read the result unchanged.  The record moves
// become per-lane loops, eight records in flight per round.
//
// Scope (exact_engine.h lane_count_mode): keyed, records mode, no session contexts -- so no slice is ever split or
// merged (those come from session edits only, S/SliceManager.java:89-166) and findSliceIndexByTimestamp works on a
// list in tStart order unless an append broke it (the `unsorted` bit, handled by the backward scan as in the
// reference).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "exact_common.h"
#include "exact_op.h"

namespace scotty {
namespace lc {
using namespace x;

// U: records per round of a record move (U loads in flight per lane)
template <int VT, int U>
struct LOp {
  const XCfg* c;
  int64_t *ts, *te, *tl, *tf, *cs, *cl;
  int32_t* ty;
  unsigned long long *cnt, *p0, *p1, *p2;
  int64_t *rlo, *rhi, *rts, *rv;
  int32_t* nn;
  XState s;
  int32_t exc;

  __device__ void bind(const XCfg* cf, const XSlices& sl, int64_t op) {
    c = cf;
    const int64_t b = op * (int64_t)cf->sc;
    ts = sl.ts + b; te = sl.te + b; tl = sl.tl + b; tf = sl.tf + b; cs = sl.cs + b; cl = sl.cl + b;
    ty = sl.ty + b; cnt = sl.cnt + b; p0 = sl.p[0] + b; p1 = sl.p[1] + b; p2 = sl.p[2] + b;
    rlo = sl.rlo + b; rhi = sl.rhi + b; nn = sl.nn + b;
    rts = sl.rts + op * cf->rcap; rv = sl.rv + op * cf->rcap;
    exc = 0;
  }

  // ---------------------------------------------------------------- slice list (exact_op.h Op, one lane)
  __device__ void copy_slice(int dst, int src) {
    ts[dst] = ts[src]; te[dst] = te[src]; tl[dst] = tl[src]; tf[dst] = tf[src];
    cs[dst] = cs[src]; cl[dst] = cl[src]; ty[dst] = ty[src];
    cnt[dst] = cnt[src]; p0[dst] = p0[src]; p1[dst] = p1[src]; p2[dst] = p2[src];
    rlo[dst] = rlo[src]; rhi[dst] = rhi[src]; nn[dst] = nn[src];
  }
  __device__ bool ensure_room() {  // compacts [head, tail) to the front when the store is full (dst < src: forward)
    if (s.tail < c->sc) return true;
    if (s.head == 0) {
      exc = XERR_SLICE_CAP;
      return false;
    }
    for (int i = 0; i < s.tail - s.head; i++) copy_slice(i, s.head + i);
    s.tail -= s.head;
    s.head = 0;
    return true;
  }
  __device__ void init_slice(int i, int64_t start, int64_t end, int64_t c_s, int64_t c_l, int32_t type, int64_t rpos) {
    ts[i] = start; te[i] = end; tl[i] = start; tf[i] = JMAX; cs[i] = c_s; cl[i] = c_l; ty[i] = type;
    cnt[i] = 0; p0[i] = 0; p1[i] = (unsigned long long)ID_MIN; p2[i] = (unsigned long long)ID_MAX;
    rlo[i] = rpos; rhi[i] = rpos; nn[i] = 0;
  }
  __device__ bool valid(int i) {
    if (i < s.head || i >= s.tail) {
      exc = XERR_INDEX;
      return false;
    }
    return true;
  }
  // LazyAggregateStore.findSliceIndexByTimestamp (:29-37): the last slice with tStart <= t, -1 if none -- a bisection
  // on a list in tStart order, else the reference's backward scan
  __device__ int find_ts(int64_t t) const {
    if (s.tail <= s.head) return -1;
    if (!(s.unsorted & 1)) {
      int lo = s.head, hi = s.tail;  // first index with ts > t
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (ts[m] <= t) lo = m + 1; else hi = m;
      }
      return lo - 1 >= s.head ? lo - 1 : -1;
    }
    for (int i = s.tail - 1; i >= s.head; i--)
      if (ts[i] <= t) return i;
    return -1;
  }

  // ---------------------------------------------------------------- partials
  __device__ void fold_partial(int i, int64_t vbits) {
    const Lift l = lift(VT, vbits);
    if (c->need & NEED_SUM) {
      if (VT == VT_F64)
        p0[i] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)p0[i]) +
                                                         __longlong_as_double((long long)l.sum));
      else
        p0[i] = p0[i] + l.sum;
    }
    if (c->need & NEED_MIN) p1[i] = (unsigned long long)min((int64_t)p1[i], l.mn);
    if (c->need & NEED_MAX) p2[i] = (unsigned long long)max((int64_t)p2[i], l.mx);
  }
  // AbstractSlice.addElement + AggregateState.addElement; LazySlice.addElement adds the record (:23-27)
  __device__ void add_element(int i, int64_t t, int64_t vbits) {
    tl[i] = max(tl[i], t);
    tf[i] = min(tf[i], t);
    cl[i] = jadd(cl[i], 1);
    cnt[i] = cnt[i] + 1;
    fold_partial(i, vbits);
    nn[i] = 1;
    if (ty_lazy(ty[i])) rec_insert(i, t, vbits);
  }

  // ---------------------------------------------------------------- LazySlice record sets
  // n records from src to dst in the op's arena, overlap-safe: U loaded before the U stores, rounds in the
  // direction of the move (a round's stores only overwrite records already loaded)
  __device__ void rec_move(int64_t dst, int64_t src, int64_t n) {
    if (n <= 0 || dst == src) return;
    if (dst < src) {
      int64_t i = 0;
      for (; i + U <= n; i += U) {
        int64_t a[U], v[U];
#pragma unroll
        for (int u = 0; u < U; u++) { a[u] = rts[src + i + u]; v[u] = rv[src + i + u]; }
#pragma unroll
        for (int u = 0; u < U; u++) { rts[dst + i + u] = a[u]; rv[dst + i + u] = v[u]; }
      }
      for (; i < n; i++) { const int64_t a = rts[src + i], v = rv[src + i]; rts[dst + i] = a; rv[dst + i] = v; }
    } else {
      int64_t i = n;
      for (; i - U >= 0; i -= U) {
        int64_t a[U], v[U];
#pragma unroll
        for (int u = 0; u < U; u++) { a[u] = rts[src + i - U + u]; v[u] = rv[src + i - U + u]; }
#pragma unroll
        for (int u = 0; u < U; u++) { rts[dst + i - U + u] = a[u]; rv[dst + i - U + u] = v[u]; }
      }
      for (; i > 0; i--) { const int64_t a = rts[src + i - 1], v = rv[src + i - 1]; rts[dst + i - 1] = a; rv[dst + i - 1] = v; }
    }
  }
  __device__ void rec_adjust(int from, int64_t d) {  // record ranges of slices [from, tail) move by d
#pragma unroll 4
    for (int i = from; i < s.tail; i++) {
      rlo[i] += d;
      rhi[i] += d;
    }
  }
  __device__ int64_t rec_lb(int64_t lo, int64_t hi, int64_t t) const {  // first p in [lo, hi) with rts[p] >= t
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (rts[m] < t) lo = m + 1; else hi = m;
    }
    return lo;
  }
  // TreeSet.add: insert (t, v) into slice i's sorted set unless a record with ts t exists (S/slice/StreamRecord.java:25-27)
  __device__ void rec_insert(int i, int64_t t, int64_t vbits) {
    // an in-order tuple (most of them) lands after the slice's last record: one probe instead of a bisection
    const int64_t lo = rlo[i], hi = rhi[i];
    const int64_t p = (hi == lo || rts[hi - 1] < t) ? hi : rec_lb(lo, hi - 1, t);
    if (p < rhi[i] && rts[p] == t) return;
    if (s.rend >= c->rcap) {
      exc = XERR_REC_CAP;
      return;
    }
    rec_move(p + 1, p, s.rend - p);
    rts[p] = t;
    rv[p] = vbits;
    rhi[i] += 1;
    rec_adjust(i + 1, 1);
    s.rend++;
  }
  __device__ void rec_delete(int i, int64_t p) {  // the arena record at p, owned by slice i
    rec_move(p, p + 1, s.rend - p - 1);
    rhi[i] -= 1;
    rec_adjust(i + 1, -1);
    s.rend--;
  }
  // AggregateValueState.recompute over the slice's record set (S/state/AggregateValueState.java:43-49)
  __device__ void rec_recompute(int i) {
    uint64_t n = 0, sw = 0;
    double sf = 0.0;
    int64_t mn = ID_MIN, mx = ID_MAX;
    for (int64_t p = rlo[i]; p < rhi[i]; p++) {
      const Lift l = lift(VT, rv[p]);
      n++;
      if (VT == VT_F64) sf += __longlong_as_double((long long)l.sum);
      else sw += l.sum;
      mn = min(mn, l.mn);
      mx = max(mx, l.mx);
    }
    cnt[i] = n;
    p0[i] = VT == VT_F64 ? (uint64_t)__double_as_longlong(sf) : sw;
    p1[i] = (unsigned long long)mn;
    p2[i] = (unsigned long long)mx;
    nn[i] = n != 0;
  }
  // AggregateState.removeElement (S/state/AggregateValueState.java:33-41): liftAndInvert of every (invertible)
  // function, else recompute from the records; have == false: the record is Java null
  __device__ void part_remove(int i, bool have, int64_t vbits) {
    if (c->invertible) {
      if (!have) {
        exc = XERR_NPE;
        return;
      }
      const Lift l = lift(VT, vbits);
      cnt[i] = cnt[i] - 1;
      if (VT == VT_F64)
        p0[i] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)p0[i]) -
                                                         __longlong_as_double((long long)l.sum));
      else
        p0[i] = p0[i] - l.sum;
    } else {
      rec_recompute(i);
    }
  }
  // AbstractSlice.addElement + AggregateState.addElement of a moved record (LazySlice.prependElement :29-33)
  __device__ void part_add(int i, int64_t t, int64_t vbits) {
    tl[i] = max(tl[i], t);
    tf[i] = min(tf[i], t);
    cl[i] = jadd(cl[i], 1);
    cnt[i] = cnt[i] + 1;
    nn[i] = 1;
    const Lift l = lift(VT, vbits);
    if (VT == VT_F64)
      p0[i] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)p0[i]) +
                                                       __longlong_as_double((long long)l.sum));
    else
      p0[i] = p0[i] + l.sum;
    p1[i] = (unsigned long long)min((int64_t)p1[i], l.mn);
    p2[i] = (unsigned long long)max((int64_t)p2[i], l.mx);
  }
  // slice(i).dropLastElement() -> slice(i+1).prependElement(record) (LazySlice.java:29-44): the record changes owner
  // by moving the boundary of the adjacent sets, then takes its sorted place in slice i+1 (a duplicate ts is dropped)
  __device__ void move_last_to_next(int i) {
    const int j = i + 1;
    const bool have = rhi[i] > rlo[i];
    int64_t t = 0, v = 0;
    if (have) {
      t = rts[rhi[i] - 1];
      v = rv[rhi[i] - 1];
      rhi[i] -= 1;
      rlo[j] -= 1;
    }
    cl[i] = jsub(cl[i], 1);
    if (rhi[i] > rlo[i]) tl[i] = rts[rhi[i] - 1];
    part_remove(i, have, v);
    if (exc) {  // the record left slice i but never reached slice i+1
      if (have) rec_delete(j, rlo[j]);
      return;
    }
    if (!have) {  // prependElement(null)
      exc = XERR_NPE;
      return;
    }
    part_add(j, t, v);
    const int64_t p = rec_lb(rlo[j] + 1, rhi[j], t);
    if (p < rhi[j] && rts[p] == t) {
      rec_delete(j, rlo[j]);
    } else if (p > rlo[j] + 1) {
      rec_move(rlo[j], rlo[j] + 1, p - 1 - rlo[j]);
      rts[p - 1] = t;
      rv[p - 1] = v;
    }
  }
  // arena compaction: live records [rlo[head], rend) move to the arena start
  __device__ void rec_compact() {
    if (s.tail <= s.head) {
      s.rend = 0;
      return;
    }
    const int64_t base = rlo[s.head];
    if (base <= 0) return;
    rec_move(0, base, s.rend - base);
    for (int i = s.head; i < s.tail; i++) {
      rlo[i] -= base;
      rhi[i] -= base;
    }
    s.rend -= base;
  }

  // SliceManager.appendSlice (S/SliceManager.java:27-38)
  __device__ void append_slice(int64_t start, int32_t type) {
    if (s.tail > s.head) {
      const int k = s.tail - 1;
      te[k] = start;
      ty[k] = type | (ty[k] & XTYPE_LAZY);
    }
    if (!ensure_room()) return;
    const int i = s.tail;
    init_slice(i, start, JMAX, s.currentCount, s.currentCount, 1 | (c->lazy ? XTYPE_LAZY : 0), s.rend);
    s.tail++;
    if (i > s.head && ts[i - 1] > start) s.unsorted |= 1;
  }

  // ---------------------------------------------------------------- StreamSlicer (S/StreamSlicer.java:36-116)
  // assignNextWindowStart: TumblingWindow.java:29-31, SlidingWindow.java:41-43, FixedBandWindow.java:37-48
  __device__ int64_t assign_next(int w, int64_t t) const {
    const int k = c->cf_kind[w];
    const int64_t a = c->cf_a[w], b = c->cf_b[w];
    if (k == 0) return jsub(jadd(t, a), jmod(t, a));
    if (k == 1) return jsub(jadd(t, b), jmod(t, b));
    if (t == JMAX || t < a) return a;
    if (t >= a && t < jadd(a, b)) return jadd(a, b);
    return JMAX;
  }
  __device__ int64_t next_edge(int64_t t_c, int measure) const {  // min over the windows of one measure
    int64_t e = JMAX;
    for (int w = 0; w < c->n_cf; w++)
      if (c->cf_measure[w] == measure) e = min(e, assign_next(w, t_c));
    return e;
  }
  __device__ int64_t next_fixed_edge(int64_t te_) const {  // calculateNextFixedEdge (:103-116)
    const int64_t cur = s.nextEdgeTs == JMIN ? JMAX : s.nextEdgeTs;
    return next_edge(max(jsub(te_, c->max_lateness), cur), 0);
  }
  __device__ int64_t next_count_edge() const {  // calculateNextFixedEdgeCount (:88-101)
    const int64_t cur = s.nextEdgeCount == JMIN ? 0 : s.nextEdgeCount;
    return next_edge(max(s.currentCount, cur), 1);
  }
  __device__ void determine_slices(int64_t te_) {  // :36-86 (no session context: no flexible edge)
    if (c->has_count) {
      if (s.nextEdgeCount == JMIN || s.currentCount == s.nextEdgeCount) {
        if (s.maxEventTime == JMIN) s.maxEventTime = te_;
        append_slice(s.maxEventTime, XTYPE_FIXED);
        if (exc) return;
        s.nextEdgeCount = next_count_edge();
      }
    }
    if (c->has_time && te_ >= s.maxEventTime) {
      if (c->has_fixed && s.nextEdgeTs == JMIN) s.nextEdgeTs = next_fixed_edge(te_);
      while (c->has_fixed && te_ > s.nextEdgeTs) {
        if (s.nextEdgeTs >= 0) append_slice(s.nextEdgeTs, XTYPE_FIXED);
        if (exc) return;
        s.nextEdgeTs = next_fixed_edge(te_);
        if (s.nextEdgeTs == JMIN) {
          exc = XERR_HANG;
          return;
        }
      }
      if (s.nextEdgeTs == te_) {
        append_slice(te_, XTYPE_FIXED);
        if (exc) return;
        s.nextEdgeTs = next_fixed_edge(te_);
      }
    }
    s.currentCount = jadd(s.currentCount, 1);  // WindowManager.incrementCount (:196-198)
    s.maxEventTime = max(te_, s.maxEventTime);
  }
  // SliceManager.processElement (S/SliceManager.java:47-87), no session context
  __device__ void manager_process(int64_t t, int64_t vbits) {
    if (s.tail <= s.head) append_slice(0, 1);
    if (exc) return;
    s.started = 1;
    const int cur = s.tail - 1;
    if (t >= tl[cur]) {
      add_element(cur, t, vbits);
      return;
    }
    const int idx = find_ts(t);
    if (!valid(idx)) return;
    add_element(idx, t, vbits);
    if (exc) return;
    if (c->has_count && idx <= s.tail - 2) {  // shift count in slices: each later slice's last record (:77-85)
      for (int i = idx; i <= s.tail - 2 && !exc; i++) {
        if (!ty_lazy(ty[i]) || !ty_lazy(ty[i + 1])) {  // (LazySlice) cast of an EagerSlice
          exc = XERR_UNSUPPORTED;
          return;
        }
        move_last_to_next(i);
      }
    }
  }
};

template <int VT>
__device__ __forceinline__ void load_rec(const XBatchArgs& a, int64_t i, int64_t& t, int64_t& vb) {
  const unsigned char* r = (const unsigned char*)a.ts + i * a.rec_stride;
  t = *(const int64_t*)r;
  if constexpr (VT == VT_I32) vb = (int64_t)*(const int32_t*)(r + 8);
  else vb = *(const int64_t*)(r + 8);
}

// one lane per key: the key's tuples [seg_begin, seg_end) of the batch sorted by key (arrival order kept), AoS records
template <int VT, int U>
__global__ __launch_bounds__(256) void lane_count_kernel(XBatchArgs a) {
  const int64_t op = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (op >= a.n_ops) return;
  const int64_t b0 = a.seg_begin[op], b1 = a.seg_end[op];
  if (b1 <= b0) return;
  const XCfg* cfg = a.cfg;
  LOp<VT, U> o;
  o.bind(cfg, a.sl, op);
  o.s = a.st[op];
  if (o.s.err) return;
  if (a.retry && !o.s.pending) return;
  o.s.pending = 0;
  // capacity pre-check (replay_kernel's bound): a key that might overflow its slice store or record arena is deferred
  // untouched; the host grows the capacities and relaunches the deferred keys (retry)
  const int64_t seglen = b1 - b0;
  if (a.need) {
    int64_t tmin = JMAX, tmax = JMIN;
    for (int64_t i = b0; i < b1; i++) {
      int64_t t_, v_;
      load_rec<VT>(a, i, t_, v_);
      tmin = min(tmin, t_);
      tmax = max(tmax, t_);
    }
    int64_t from = o.s.started ? max(o.s.maxEventTime, jsub(tmin, cfg->max_lateness)) : jsub(tmin, cfg->max_lateness);
    if (from > tmax) from = tmax;
    const double span = (double)tmax - (double)from;
    double bound = 0.0;
    for (int w = 0; w < cfg->n_cf; w++) {
      const int k = cfg->cf_kind[w];
      const double step = k == 0 ? (double)cfg->cf_a[w] : (double)cfg->cf_b[w];
      if (k == 2) bound += 2.0;
      else if (cfg->cf_measure[w] == 1) bound += (double)seglen / step + 2.0;
      else bound += span / step + 2.0;
    }
    const double need_s = (double)(o.s.tail - o.s.head) + bound + 2.0;
    const int64_t live = o.s.tail > o.s.head ? o.s.rend - o.rlo[o.s.head] : 0;
    const int64_t need_r = live + seglen + 64;
    if (need_s > (double)cfg->sc || need_r > cfg->rcap) {
      atomicMax(&a.need[0], (unsigned long long)min(need_s, 1e15) + 2ull);
      atomicMax(&a.need[2], (unsigned long long)need_r);
      o.s.pending = 1;
      a.st[op] = o.s;
      return;
    }
  }
  if (o.s.rend + seglen + 64 > cfg->rcap) o.rec_compact();
  // The current (last) slice in registers.  Most tuples are in order and open no slice: determineSlices only counts
  // them (no count edge due, no time edge crossed, S/StreamSlicer.java:36-86) and processElement's in-order branch adds
  // them to the last slice (S/SliceManager.java:56-63), whose record set they extend at its end (ts above its last
  // record: TreeSet.add appends; an equal ts adds no record).  Those tuples touch only these registers and the two
  // record words they append -- about 26 scattered lines per tuple otherwise (the slice's fields read and written, its
  // record range), which bounded the kernel at 140 GB of line traffic per C4c batch (profiles/r06/prof).  Every other
  // tuple flushes the registers and runs the restatement above, which then sees the store exactly as it would have.
  int ci = -1;
  bool dirty = false, c_lazy = false;
  int64_t c_tl = 0, c_tf = 0, c_cl = 0, c_rhi = 0, c_last = JMIN;
  uint64_t c_cnt = 0, c_p0 = 0;
  int64_t c_p1 = 0, c_p2 = 0;
  auto load_cur = [&]() {
    ci = o.s.tail > o.s.head ? o.s.tail - 1 : -1;
    dirty = false;
    if (ci < 0) return;
    c_tl = o.tl[ci]; c_tf = o.tf[ci]; c_cl = o.cl[ci]; c_cnt = o.cnt[ci];
    c_p0 = o.p0[ci]; c_p1 = (int64_t)o.p1[ci]; c_p2 = (int64_t)o.p2[ci];
    c_lazy = ty_lazy(o.ty[ci]);
    c_rhi = o.rhi[ci];
    c_last = c_rhi > o.rlo[ci] ? o.rts[c_rhi - 1] : JMIN;
  };
  auto flush_cur = [&]() {
    if (ci < 0 || !dirty) return;
    o.tl[ci] = c_tl; o.tf[ci] = c_tf; o.cl[ci] = c_cl; o.cnt[ci] = c_cnt;
    o.p0[ci] = c_p0; o.p1[ci] = (unsigned long long)c_p1; o.p2[ci] = (unsigned long long)c_p2;
    o.nn[ci] = 1;
    o.rhi[ci] = c_rhi;
    dirty = false;
  };
  load_cur();
  for (int64_t i = b0; i < b1 && !o.s.err; i++) {
    int64_t t, vb;
    load_rec<VT>(a, i, t, vb);
    // the fast tuple: no count edge (nextEdgeCount pending and not reached), no time edge (t below the pending fixed
    // edge, or out of order), in order in the last slice, and its record (if any) appended at the arena's end
    bool fast = ci >= 0 && t >= c_tl && (!c_lazy || (c_last <= t && c_rhi == o.s.rend && o.s.rend < cfg->rcap));
    if (fast && cfg->has_count) fast = o.s.nextEdgeCount != JMIN && o.s.currentCount != o.s.nextEdgeCount;
    if (fast && cfg->has_time && t >= o.s.maxEventTime)
      fast = cfg->has_fixed ? (o.s.nextEdgeTs != JMIN && t < o.s.nextEdgeTs) : t != o.s.nextEdgeTs;
    if (fast) {
      o.s.currentCount = jadd(o.s.currentCount, 1);
      o.s.maxEventTime = max(t, o.s.maxEventTime);
      o.s.started = 1;
      c_tl = max(c_tl, t);
      c_tf = min(c_tf, t);
      c_cl = jadd(c_cl, 1);
      c_cnt++;
      const Lift l = lift(VT, vb);
      if (cfg->need & NEED_SUM) {
        if (VT == VT_F64)
          c_p0 = (uint64_t)__double_as_longlong(__longlong_as_double((long long)c_p0) +
                                                __longlong_as_double((long long)l.sum));
        else
          c_p0 += l.sum;
      }
      if (cfg->need & NEED_MIN) c_p1 = min(c_p1, l.mn);
      if (cfg->need & NEED_MAX) c_p2 = max(c_p2, l.mx);
      dirty = true;
      if (c_lazy && c_last != t) {  // LazySlice.addElement: records.add, at the end of the set and of the arena
        o.rts[o.s.rend] = t;
        o.rv[o.s.rend] = vb;
        o.s.rend++;
        c_rhi++;
        c_last = t;
      }
      continue;
    }
    flush_cur();
    o.exc = 0;
    o.determine_slices(t);
    if (!o.exc) o.manager_process(t, vb);
    if (xerr_tuple_failed(o.exc)) {
      o.s.dropped++;
      o.exc = 0;
    } else if (o.exc) {
      o.s.err = o.exc;
    }
    load_cur();
  }
  flush_cur();
  a.st[op] = o.s;
}

}  // namespace lc

// 8 records per round of a record move: 162 VGPRs, 3 waves per SIMD (16 per round, 194 VGPRs and 2 waves: C4c lane
// kernel 46.3 vs 42.3 ms per 2^26-tuple batch, profiles/r06/ab/ab_c4c_lane.json)
hipError_t launch_lane_count(const XBatchArgs& a, int vt, hipStream_t st) {
  if (a.n_ops <= 0) return hipSuccess;
  if (a.rec_stride != (vt == VT_I32 ? 16 : 24)) return hipErrorInvalidValue;  // AoS records {ts, value, ...}
  const dim3 grid((unsigned)((a.n_ops + 255) / 256)), block(256);
  note_kernel(KN_REPLAY, "lane_count_kernel<%d, 8>", vt);
  if (vt == VT_I32) hipLaunchKernelGGL((lc::lane_count_kernel<VT_I32, 8>), grid, block, 0, st, a);
  else if (vt == VT_I64) hipLaunchKernelGGL((lc::lane_count_kernel<VT_I64, 8>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((lc::lane_count_kernel<VT_F64, 8>), grid, block, 0, st, a);
  return hipGetLastError();
}

}  // namespace scotty
