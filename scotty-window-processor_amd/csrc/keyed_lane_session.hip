// keyed_lane_session.hip -- one LANE per key for keyed operators with session windows (KeyedScottyWindowOperator over
// SessionWindow, flink-connector/.../KeyedScottyWindowOperator.java:56-86, C/windowType/SessionWindow.java:40-116),
// beside any context-free time windows, on Eager slices.
//
// The wavefront replay (exact_kernels.hip replay_kernel) gives each key a whole wavefront: right for a few keys with
// long micro-batches, but at 10^5-10^6 keys a key brings ~64 tuples per batch and its wavefront spends most of its life
// waiting on that key's cold slice and session lines, one dependent access after another (C4s: 24 ms per 2^26-tuple
// batch at 1 M keys, three wavefronts per SIMD).  Here a lane walks its key's tuples in arrival order with the
// reference's per-tuple state machine as scalar code -- StreamSlicer.determineSlices (S/StreamSlicer.java:36-130),
// SliceManager.processElement / checkSliceEdges / splitSlice (S/SliceManager.java:27-192), SessionContext.updateContext
// (SessionWindow.java:40-98) -- so the 64 keys of a wavefront wait on memory together.  The state layout (XState, slice
// SoA, session columns) is the wavefront replay's, restated operation for operation from exact_op.h's Op with
// sequential loops where Op uses the wavefront's lanes; configurations move freely between the two kernels (scotty_tune
// "keyed_lane_session" 0 runs the wavefront replay instead, the A/B and the parity test's reference).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exact_common.h"
#include "exact_op.h"

namespace scotty {
namespace ls {
using namespace x;

// V: the slice store's view -- XSlices (key-major columns) or XKView (key-interleaved words, COUNT / integer SUM /
// MIN / MAX operators: the lanes of a wavefront touching one field of one slice position read one 512-B run)
template <int VT, class V>
struct LaneS {
  const XCfg* c;
  V q;            // the store's columns (uniform); this key's slice i is element b + i
  int64_t b;
  int64_t sb;     // this key's session base: context k, session i at sb + k * sesscap + i
  XState s;
  int32_t exc;

  __device__ int64_t& TS(int i) const { return q.ts[b + i]; }
  __device__ int64_t& TE(int i) const { return q.te[b + i]; }
  __device__ int64_t& TL(int i) const { return q.tl[b + i]; }
  __device__ int64_t& TF(int i) const { return q.tf[b + i]; }
  __device__ int64_t& CS(int i) const { return q.cs[b + i]; }
  __device__ int64_t& CL(int i) const { return q.cl[b + i]; }
  __device__ int32_t& TY(int i) const { return q.ty[b + i]; }
  __device__ unsigned long long& CNT(int i) const { return q.cnt[b + i]; }
  __device__ unsigned long long& P(int k, int i) const { return q.p[k][b + i]; }
  __device__ int64_t* SSp(const XSess& x, int k) const { return x.start + sb + (int64_t)k * c->sesscap; }

  // ---------------------------------------------------------------- slice list primitives (exact_op.h Op)
  __device__ void copy_slice(int dst, int src) {
    TS(dst) = TS(src); TE(dst) = TE(src); TL(dst) = TL(src); TF(dst) = TF(src);
    CS(dst) = CS(src); CL(dst) = CL(src); TY(dst) = TY(src);
    CNT(dst) = CNT(src); P(0, dst) = P(0, src); P(1, dst) = P(1, src); P(2, dst) = P(2, src);
  }
  __device__ void move_range(int dst, int src, int n) {
    if (n <= 0 || dst == src) return;
    if (dst < src) {
      for (int i = 0; i < n; i++) copy_slice(dst + i, src + i);
    } else {
      for (int i = n - 1; i >= 0; i--) copy_slice(dst + i, src + i);
    }
  }
  __device__ bool ensure_room() {
    if (s.tail < c->sc) return true;
    if (s.head == 0) {
      exc = XERR_SLICE_CAP;
      return false;
    }
    move_range(0, s.head, s.tail - s.head);
    s.tail -= s.head;
    s.head = 0;
    return true;
  }
  __device__ void init_slice(int i, int64_t start, int64_t end, int64_t c_s, int64_t c_l, int32_t type) {
    TS(i) = start; TE(i) = end; TL(i) = start; TF(i) = JMAX; CS(i) = c_s; CL(i) = c_l; TY(i) = type;
    CNT(i) = 0; P(0, i) = 0; P(1, i) = (unsigned long long)ID_MIN; P(2, i) = (unsigned long long)ID_MAX;
  }
  __device__ void note_order(int i) {
    if (i > s.head && TS(i - 1) > TS(i)) s.unsorted |= 1;
    if (i + 1 < s.tail && TS(i) > TS(i + 1)) s.unsorted |= 1;
  }
  __device__ int insert_at(int i) {
    const int rel = i - s.head;
    if (!ensure_room()) return -1;
    i = s.head + rel;
    move_range(i + 1, i, s.tail - i);
    s.tail++;
    return i;
  }
  __device__ void remove_at(int i) {
    move_range(i, i + 1, s.tail - i - 1);
    s.tail--;
  }
  __device__ bool valid(int i) {
    if (i < s.head || i >= s.tail) {
      exc = XERR_INDEX;
      return false;
    }
    return true;
  }
  // LazyAggregateStore.findSliceIndexByTimestamp (:29-37): last slice with tStart <= t, -1 if none.  A sorted list is
  // searched by galloping down from the tail (an out-of-order tuple mostly lands in one of the last slices: one or
  // two loads instead of a bisection's chain); an unsorted one backwards, as the reference's loop runs
  __device__ int find_ts(int64_t t) const {
    if (s.tail <= s.head) return -1;
    if (!(s.unsorted & 1)) {
      int hi = s.tail - 1;
      if (TS(hi) <= t) return hi;
      int step = 1, lo;
      for (;;) {  // TS(hi) > t
        const int nx = hi - step;
        if (nx <= s.head) {
          if (TS(s.head) > t) return -1;
          lo = s.head;
          break;
        }
        if (TS(nx) <= t) {
          lo = nx;
          break;
        }
        hi = nx;
        step <<= 1;
      }
      while (hi - lo > 1) {  // TS(lo) <= t < TS(hi)
        const int m = (lo + hi) >> 1;
        if (TS(m) <= t) lo = m; else hi = m;
      }
      return lo;
    }
    for (int i = s.tail - 1; i >= s.head; i--)
      if (TS(i) <= t) return i;
    return -1;
  }
  // LazyAggregateStore.findSliceByEnd (:127-135)
  __device__ int find_end(int64_t e) const {
    for (int i = s.tail - 1; i >= s.head; i--)
      if (TE(i) == e) return i;
    return -1;
  }
  // AbstractSlice.addElement + AggregateState.addElement (one tuple, exact)
  __device__ void add_element(int i, int64_t t, int64_t vbits) {
    TL(i) = max(TL(i), t);
    TF(i) = min(TF(i), t);
    CL(i) = jadd(CL(i), 1);
    CNT(i) = CNT(i) + 1;
    const Lift l = lift(VT, vbits);
    if (c->need & NEED_SUM) {
      if (VT == VT_F64)
        P(0, i) = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)P(0, i)) +
                                                           __longlong_as_double((long long)l.sum));
      else
        P(0, i) = P(0, i) + l.sum;
    }
    if (c->need & NEED_MIN) P(1, i) = (unsigned long long)min((int64_t)P(1, i), l.mn);
    if (c->need & NEED_MAX) P(2, i) = (unsigned long long)max((int64_t)P(2, i), l.mx);
  }
  // SliceManager.appendSlice (S/SliceManager.java:27-38)
  __device__ void append_slice(int64_t start, int32_t type) {
    if (s.tail > s.head) {
      const int k = s.tail - 1;
      TE(k) = start;
      TY(k) = type;
    }
    if (!ensure_room()) return;
    const int i = s.tail;
    init_slice(i, start, JMAX, s.currentCount, s.currentCount, 1);
    s.tail++;
    if (i > s.head && TS(i - 1) > start) s.unsorted |= 1;
  }
  // SliceManager.splitSlice (S/SliceManager.java:168-192); Eager slices move no tuples
  __device__ void split_slice(int idx, int64_t timestamp) {
    if (!valid(idx)) return;
    int a = idx;
    int bpos;
    if (timestamp < TE(a)) {
      bpos = a + 1;
    } else if (idx + 1 < s.tail) {
      a = idx + 1;
      bpos = idx + 2;
    } else {
      return;
    }
    const int64_t a_end = TE(a), a_cs = CS(a), a_cl = CL(a);
    const int32_t a_ty = TY(a);
    const int rel_a = a - s.head;
    bpos = insert_at(bpos);
    if (bpos < 0) return;
    a = s.head + rel_a;
    init_slice(bpos, timestamp, a_end, a_cs, a_cl, ty_kind(a_ty));
    TE(a) = timestamp;
    TY(a) = 1;
    note_order(bpos);
  }
  // AbstractSlice.merge + LazyAggregateStore.mergeSlice (:119-124)
  __device__ void merge_slice(int idx) {
    if (!valid(idx) || !valid(idx + 1)) return;
    const int q = idx + 1;
    TL(idx) = max(TL(idx), TL(q));
    TF(idx) = min(TF(idx), TF(q));
    TE(idx) = max(TE(idx), TE(q));
    CNT(idx) = CNT(idx) + CNT(q);
    if (VT == VT_F64)
      P(0, idx) = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)P(0, idx)) +
                                                           __longlong_as_double((long long)P(0, q)));
    else
      P(0, idx) = P(0, idx) + P(0, q);
    P(1, idx) = (unsigned long long)min((int64_t)P(1, idx), (int64_t)P(1, q));
    P(2, idx) = (unsigned long long)max((int64_t)P(2, idx), (int64_t)P(2, q));
    remove_at(q);
  }
  // SliceManager.checkSliceEdges (S/SliceManager.java:89-166), modifications in insertion order
  __device__ void check_slice_edges(const Mod* mods, int nm) {
    for (int k = 0; k < nm && !exc; k++) {
      const Mod m = mods[k];
      if (m.kind == 0) {  // ShiftModification
        const int si = find_end(m.pre);
        if (si == -1) continue;
        const int32_t st = TY(si);
        if (ty_movable(st)) {
          if (!valid(si + 1)) return;
          TE(si) = m.post;
          TS(si + 1) = m.post;
          s.unsorted |= 2;
          note_order(si + 1);
        } else {
          if (!ty_fixed(st)) TY(si) = ty_flex(st - 1);
          split_slice(si, m.post);
        }
      } else if (m.kind == 1) {  // DeleteModification
        const int si = find_end(m.pre);
        if (si >= 0) {
          const int32_t st = TY(si);
          if (ty_movable(st)) {
            if (!valid(si + 1)) return;
            merge_slice(si);
          } else if (!ty_fixed(st)) {
            TY(si) = ty_flex(st - 1);
          }
        }
      } else {  // AddModification
        const int si = find_ts(m.post);
        if (!valid(si)) return;
        if (TS(si) != m.post && TE(si) != m.post) split_slice(si, m.post);
      }
    }
  }

  // ---------------------------------------------------------------- SessionContext (SessionWindow.java:40-116)
  __device__ void add_window(const XSess& x, int k, int i, int64_t start, int64_t end, Mod* mods, int& nm) {
    const int n = s.ns(k);  // WindowContext :19-25
    if (i < 0 || i > n) {
      exc = XERR_INDEX;
      return;
    }
    if (n >= c->sesscap) {
      exc = XERR_SESS_CAP;
      return;
    }
    int64_t* st = SSp(x, k);
    int64_t* en = x.end + (st - x.start);
    for (int q = n; q > i; q--) {
      st[q] = st[q - 1];
      en[q] = en[q - 1];
    }
    st[i] = start;
    en[i] = end;
    s.set_ns(k, n + 1);
    if (mods && nm + 2 <= XMAXMODS) {
      mods[nm++] = Mod{2, 0, start};
      mods[nm++] = Mod{2, 0, end};
    }
  }
  __device__ void remove_window(const XSess& x, int k, int i, Mod* mods, int& nm) {  // :48-52
    const int n = s.ns(k);
    if (i < 0 || i >= n) {
      exc = XERR_INDEX;
      return;
    }
    int64_t* st = SSp(x, k);
    int64_t* en = x.end + (st - x.start);
    if (mods && nm + 2 <= XMAXMODS) {
      mods[nm++] = Mod{1, st[i], 0};
      mods[nm++] = Mod{1, en[i], 0};
    }
    for (int q = i; q < n - 1; q++) {
      st[q] = st[q + 1];
      en[q] = en[q + 1];
    }
    s.set_ns(k, n - 1);
  }
  __device__ void merge_with_pre(const XSess& x, int k, int idx, Mod* mods, int& nm) {  // :39-46
    if (idx < 0 || idx >= s.ns(k) || idx - 1 < 0) {
      exc = XERR_INDEX;
      return;
    }
    int64_t* en = x.end + (SSp(x, k) - x.start);
    en[idx - 1] = en[idx];  // shiftEnd records no modification
    remove_window(x, k, idx, mods, nm);
  }
  __device__ int get_session(const XSess& x, int k, int64_t pos) const {  // :89-101
    const int64_t gap = c->gap[k];
    const int n = s.ns(k);
    const int64_t* st = SSp(x, k);
    const int64_t* en = x.end + (st - x.start);
    int i = 0;
    for (; i < n; i++) {
      const int64_t a = st[i], e = en[i];
      if (jsub(a, gap) <= pos && jadd(e, gap) >= pos) return i;
      if (jsub(a, gap) > pos) return i - 1;
    }
    return i - 1;
  }
  __device__ void session_update(const XSess& x, int k, int64_t pos, Mod* mods, int& nm) {  // :42-87
    const int64_t gap = c->gap[k];
    const int n = s.ns(k);
    if (n == 0) {  // hasActiveWindows() returns isEmpty() (WindowContext.java:15-17)
      add_window(x, k, 0, pos, pos, mods, nm);
      return;
    }
    int64_t* st = SSp(x, k);
    int64_t* en = x.end + (st - x.start);
    // a position at or past the last session's end: getSession returns the last session (every earlier one ends more
    // than a gap before the last one starts), so only the shiftEnd / new-session branches can apply
    const int64_t le = en[n - 1];
    int si;
    if (pos >= le && pos >= st[n - 1]) {
      si = n - 1;
    } else {
      si = get_session(x, k, pos);
      if (si == -1) {
        add_window(x, k, 0, pos, pos, mods, nm);
        return;
      }
    }
    const int64_t a = st[si], e = en[si];
    if (jsub(a, gap) > pos) {
      add_window(x, k, si, pos, pos, mods, nm);
    } else if (a > pos && jsub(a, gap) < pos) {
      if (mods && nm < XMAXMODS) mods[nm++] = Mod{0, a, pos};  // shiftStart
      st[si] = pos;
      if (si > 0) {
        if (jadd(en[si - 1], gap) >= st[si]) merge_with_pre(x, k, si, mods, nm);
      }
    } else if (e < pos && jadd(e, gap) >= pos) {
      en[si] = pos;  // shiftEnd
      if (si < s.ns(k) - 1) {
        if (jadd(en[si], gap) >= st[si + 1]) merge_with_pre(x, k, si + 1, mods, nm);
      }
    } else if (jadd(e, gap) < pos) {
      add_window(x, k, si + 1, pos, pos, mods, nm);
    }
  }

  // ---------------------------------------------------------------- StreamSlicer (S/StreamSlicer.java:36-130)
  __device__ int64_t next_fixed_edge(int64_t te_) const {  // calculateNextFixedEdge (:103-116)
    const int64_t cur = s.nextEdgeTs == JMIN ? JMAX : s.nextEdgeTs;
    const int64_t t_c = max(jsub(te_, c->max_lateness), cur);
    int64_t e = JMAX;
    for (int w = 0; w < c->n_cf; w++) {
      if (c->cf_measure[w] != 0) continue;
      const int kd = c->cf_kind[w];
      const int64_t wa = c->cf_a[w], wb = c->cf_b[w];
      int64_t r;
      if (kd == 0) r = jsub(jadd(t_c, wa), jmod(t_c, wa));
      else if (kd == 1) r = jsub(jadd(t_c, wb), jmod(t_c, wb));
      else if (t_c == JMAX || t_c < wa) r = wa;
      else if (t_c >= wa && t_c < jadd(wa, wb)) r = jadd(wa, wb);
      else r = JMAX;
      e = min(e, r);
    }
    return e;
  }
  __device__ int flex_count(int64_t te_) const {  // calculateNextFlexEdge (:118-130)
    const int64_t t_c = max(s.maxEventTime, s.nextEdgeTs);
    int flex = 0;
    for (int k = 0; k < c->n_ctx; k++)
      if (te_ >= jadd(t_c, c->gap[k])) flex++;
    return flex;
  }
  __device__ void determine_slices(int64_t te_) {  // :36-86 (time measure only: no count windows here)
    if (te_ >= s.maxEventTime) {
      if (c->has_fixed && s.nextEdgeTs == JMIN) s.nextEdgeTs = next_fixed_edge(te_);
      const int flex = flex_count(te_);
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
      } else if (flex > 0) {
        append_slice(te_, ty_flex(flex));
        if (exc) return;
      }
    }
    s.currentCount = jadd(s.currentCount, 1);  // WindowManager.incrementCount (:196-198)
    s.maxEventTime = max(te_, s.maxEventTime);
  }
  // SliceManager.processElement (S/SliceManager.java:47-87)
  __device__ void manager_process(const XSess& x, int64_t t, int64_t vbits) {
    if (s.tail <= s.head) append_slice(0, 1);
    if (exc) return;
    s.started = 1;
    const int cur = s.tail - 1;
    if (t >= TL(cur)) {
      add_element(cur, t, vbits);
      for (int k = 0; k < c->n_ctx && !exc; k++) {
        int nd = 0;
        session_update(x, k, t, nullptr, nd);  // modifications are dropped (:59-62)
      }
      return;
    }
    for (int k = 0; k < c->n_ctx && !exc; k++) {
      Mod mods[XMAXMODS];
      int nm = 0;
      session_update(x, k, t, mods, nm);
      if (exc) return;
      check_slice_edges(mods, nm);
    }
    if (exc) return;
    const int idx = find_ts(t);
    if (!valid(idx)) return;
    add_element(idx, t, vbits);
  }
};

// One tuple through the general restatement (everything the fast path below does not take: flexible edges, session
// edits that move, split or merge slices, new sessions before the last, several session contexts, capacity edges).
// Out of line: its state lives in the caller's LaneS, in scratch memory, which only these rare tuples pay for.
template <int VT, class V>
__device__ __noinline__ void general_tuple(LaneS<VT, V>& L, const XSess x, int64_t t, int64_t vb) {
  L.exc = 0;
  L.determine_slices(t);
  if (!L.exc) L.manager_process(x, t, vb);
  if (xerr_tuple_failed(L.exc)) {
    L.s.dropped++;
    L.exc = 0;
  } else if (L.exc) {
    L.s.err = L.exc;
  }
}

// PK: the batch comes as packed 8-byte records (a.rec_stride 8, int32 values; a compile-time choice, so the record
// loads of the ring below keep one code path and no branch join waits on them)
template <int VT, int OCC, class V, bool PK = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void lane_session_kernel(XBatchArgs a) {
  const XCfg* cfg = a.cfg;
  const int64_t op = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (op >= a.n_ops) return;
  const int64_t b0 = a.seg_begin[op], b1 = a.seg_end[op];
  if (b1 <= b0) return;
  XState* sp = a.st + op;
  if (sp->err) return;
  if (a.retry && !sp->pending) return;
  const unsigned char* rec = (const unsigned char*)a.ts;
  // an int32 batch may come as packed 8-byte records {key << pk_bits | ts - pk_base, value} (keyed_kernels.hip Rec<8>)
  constexpr bool packed = VT == VT_I32 && PK;
  const uint32_t pk_mask = (1u << a.pk_bits) - 1u;
  const int64_t pk_base = a.pk_base;
  auto load = [&](int64_t i, int64_t& t, int64_t& vb) {
    if constexpr (packed) {
      const uint2 w = *(const uint2*)(rec + i * 8);
      t = pk_base + (int64_t)(w.x & pk_mask);
      vb = (int64_t)(int32_t)w.y;
      return;
    }
    const unsigned char* r = rec + i * a.rec_stride;
    t = *(const int64_t*)r;
    if constexpr (VT == VT_I32) vb = (int64_t)*(const int32_t*)(r + 8);
    else vb = *(const int64_t*)(r + 8);
  };
  XState s0 = *sp;
  // capacity pre-check (the wavefront replay's bound): a key that might overflow its slice or session capacity is
  // deferred untouched, the host grows the capacities and relaunches the deferred keys (retry).  The bound needs the
  // span of event time the key's tuples can add slices over: for a started key that span lies within [maxEventTime,
  // the batch's largest timestamp], so when that wider span already fits, the key's tuples are not read for it;
  // otherwise they are, eight records per round (eight scattered loads in flight)
  {
    const int64_t seglen = b1 - b0;
    int need_x = 0;
    for (int k = 0; k < cfg->n_ctx; k++) need_x = max(need_x, s0.ns(k));
    const int64_t need_ss = (int64_t)need_x + seglen + 1;
    auto need_slices = [&](double span) {
      double bound = 0.0;
      for (int w = 0; w < cfg->n_cf; w++) {
        const int k = cfg->cf_kind[w];
        const double step = k == 0 ? (double)cfg->cf_a[w] : (double)cfg->cf_b[w];
        if (k == 2) bound += 2.0;
        else bound += span / step + 2.0;
      }
      bound += 3.0 * (double)seglen;  // session edits: a flexible edge, a split and a shift per tuple at most
      return (double)(s0.tail - s0.head) + bound + 2.0;
    };
    bool fits = false;
    if (s0.started && a.ts_max_b) {
      const int64_t tmax_b = (int64_t)(*a.ts_max_b ^ 0x8000000000000000ull);
      const double span = tmax_b > s0.maxEventTime ? (double)tmax_b - (double)s0.maxEventTime : 0.0;
      fits = need_slices(span) <= (double)cfg->sc && need_ss <= cfg->sesscap;
    }
    if (!fits) {
      int64_t tmin = JMAX, tmax = JMIN;
      int64_t i = b0;
      for (; i + 8 <= b1; i += 8) {
        int64_t tt[8], v_;
#pragma unroll
        for (int u = 0; u < 8; u++) load(i + u, tt[u], v_);
#pragma unroll
        for (int u = 0; u < 8; u++) {
          tmin = min(tmin, tt[u]);
          tmax = max(tmax, tt[u]);
        }
      }
      for (; i < b1; i++) {
        int64_t t, v_;
        load(i, t, v_);
        tmin = min(tmin, t);
        tmax = max(tmax, t);
      }
      int64_t from = s0.started ? max(s0.maxEventTime, jsub(tmin, cfg->max_lateness)) : jsub(tmin, cfg->max_lateness);
      if (from > tmax) from = tmax;
      const double need_s = need_slices((double)tmax - (double)from);
      if (need_s > (double)cfg->sc || need_ss > cfg->sesscap) {
        atomicMax(&a.need[0], (unsigned long long)min(need_s, 1e15) + 2ull);
        atomicMax(&a.need[1], (unsigned long long)need_ss);
        sp->pending = 1;
        return;
      }
    }
  }
  s0.pending = 0;

  // ---- fast path state, in registers: the StreamSlicer / store scalars, the one session context's last session, and
  //      the current (last) slice's fields.  It takes the steady-state tuples of one session context: in-order tuples
  //      that cross fixed edges, extend the last session or open a new one behind it without a flexible edge, and
  //      out-of-order tuples inside the last session -- the same transitions the general code makes for them.
  // the store's columns as a local view (a reference into the kernel argument would keep the argument block in
  // scratch memory and reload a pointer from it on every access)
  const V q = xview<V>(a.sl);
  const auto Q_ts = q.ts;
  const auto Q_te = q.te;
  const auto Q_tl = q.tl;
  const auto Q_tf = q.tf;
  const auto Q_cs = q.cs;
  const auto Q_cl = q.cl;
  const auto Q_ty = q.ty;
  const auto Q_cnt = q.cnt;
  const auto Q_p0 = q.p[0];
  const auto Q_p1 = q.p[1];
  const auto Q_p2 = q.p[2];
  // lowest slice position whose partials this batch changes: the lane watermark's running prefixes and MIN / MAX
  // block summaries (keyed_lane.hip, XState.pvalid) are valid below it only
  int32_t minmod = INT32_MAX;
  const int64_t bb = op * (int64_t)cfg->sc;
  const int64_t sbase = op * cfg->ctx_alloc * (int64_t)cfg->sesscap;
  int64_t* const sst = a.ss.start + sbase;  // context 0
  int64_t* const sen = a.ss.end + sbase;
  const bool one_ctx = cfg->n_ctx == 1;
  const int64_t gap = cfg->gap[0];
  const int32_t sc = cfg->sc;
  int64_t mx = s0.maxEventTime, ne = s0.nextEdgeTs, cc = s0.currentCount;
  int32_t head = s0.head, tail = s0.tail, uns = s0.unsorted, started = s0.started, ns = s0.nsess[0];
  uint64_t dropped = s0.dropped;
  int32_t err = s0.err;
  int64_t st_l = JMIN, en_l = JMIN;
  // the current (last) slice ci and the one before it pv (the late tuples' usual target), in registers; c_ts / p_ts
  // their tStart.  en_l is written back to the session list at flush_cur
  int32_t ci = -1, pv = -1;
  int64_t c_ts = 0, c_tl = 0, c_tf = 0, c_cl = 0, c_p1 = 0, c_p2 = 0;
  uint64_t c_cnt = 0, c_p0 = 0;
  int64_t p_ts = 0, p_tl = 0, p_tf = 0, p_cl = 0, p_p1 = 0, p_p2 = 0;
  uint64_t p_cnt = 0, p_p0 = 0;
  auto load_fast = [&]() {  // session tail and the last two slices from memory
    if (one_ctx && ns > 0) {
      st_l = sst[ns - 1];
      en_l = sen[ns - 1];
    }
    ci = tail > head ? tail - 1 : -1;
    pv = tail - 1 > head ? tail - 2 : -1;
    if (ci >= 0) {
      const int64_t j = bb + ci;
      c_ts = Q_ts[j]; c_tl = Q_tl[j]; c_tf = Q_tf[j]; c_cl = Q_cl[j]; c_cnt = Q_cnt[j];
      c_p0 = Q_p0[j]; c_p1 = (int64_t)Q_p1[j]; c_p2 = (int64_t)Q_p2[j];
    }
    if (pv >= 0) {
      const int64_t j = bb + pv;
      p_ts = Q_ts[j]; p_tl = Q_tl[j]; p_tf = Q_tf[j]; p_cl = Q_cl[j]; p_cnt = Q_cnt[j];
      p_p0 = Q_p0[j]; p_p1 = (int64_t)Q_p1[j]; p_p2 = (int64_t)Q_p2[j];
    }
  };
  auto flush_prev = [&]() {
    if (pv < 0) return;
    const int64_t j = bb + pv;
    Q_tl[j] = p_tl; Q_tf[j] = p_tf; Q_cl[j] = p_cl; Q_cnt[j] = p_cnt;
    Q_p0[j] = p_p0; Q_p1[j] = (unsigned long long)p_p1; Q_p2[j] = (unsigned long long)p_p2;
  };
  auto flush_cur = [&]() {
    if (one_ctx && ns > 0) sen[ns - 1] = en_l;
    flush_prev();
    if (ci < 0) return;
    const int64_t j = bb + ci;
    Q_tl[j] = c_tl; Q_tf[j] = c_tf; Q_cl[j] = c_cl; Q_cnt[j] = c_cnt;
    Q_p0[j] = c_p0; Q_p1[j] = (unsigned long long)c_p1; Q_p2[j] = (unsigned long long)c_p2;
  };
  auto fold = [&](int64_t& tl, int64_t& tf, int64_t& cl, uint64_t& cnt, uint64_t& p0, int64_t& p1, int64_t& p2,
                  int64_t t, int64_t vb) {
    tl = max(tl, t);
    tf = min(tf, t);
    cl = jadd(cl, 1);
    cnt++;
    const Lift l = lift(VT, vb);
    if (cfg->need & NEED_SUM) {
      if (VT == VT_F64)
        p0 = (uint64_t)__double_as_longlong(__longlong_as_double((long long)p0) + __longlong_as_double((long long)l.sum));
      else
        p0 += l.sum;
    }
    if (cfg->need & NEED_MIN) p1 = min(p1, l.mn);
    if (cfg->need & NEED_MAX) p2 = max(p2, l.mx);
  };
  auto add_cur = [&](int64_t t, int64_t vb) {
    fold(c_tl, c_tf, c_cl, c_cnt, c_p0, c_p1, c_p2, t, vb);
    minmod = min(minmod, ci);
  };
  auto add_prev = [&](int64_t t, int64_t vb) {
    fold(p_tl, p_tf, p_cl, p_cnt, p_p0, p_p1, p_p2, t, vb);
    minmod = min(minmod, pv);
  };
  auto add_mem = [&](int i, int64_t t, int64_t vb) {  // an older slice, in memory
    minmod = min(minmod, i);
    const int64_t j = bb + i;
    Q_tl[j] = max(Q_tl[j], t);
    Q_tf[j] = min(Q_tf[j], t);
    Q_cl[j] = jadd(Q_cl[j], 1);
    Q_cnt[j] = Q_cnt[j] + 1;
    const Lift l = lift(VT, vb);
    if (cfg->need & NEED_SUM) {
      if (VT == VT_F64)
        Q_p0[j] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)Q_p0[j]) +
                                                             __longlong_as_double((long long)l.sum));
      else
        Q_p0[j] = Q_p0[j] + l.sum;
    }
    if (cfg->need & NEED_MIN) Q_p1[j] = (unsigned long long)min((int64_t)Q_p1[j], l.mn);
    if (cfg->need & NEED_MAX) Q_p2[j] = (unsigned long long)max((int64_t)Q_p2[j], l.mx);
  };
  // calculateNextFixedEdge (S/StreamSlicer.java:103-116) from the pending edge cur
  auto next_edge = [&](int64_t te_, int64_t cur) {
    const int64_t cur_ = cur == JMIN ? JMAX : cur, lt_ = jsub(te_, cfg->max_lateness);
    const int64_t t_c = lt_ > cur_ ? lt_ : cur_;
    int64_t e = JMAX;
    for (int w = 0; w < cfg->n_cf; w++) {
      if (cfg->cf_measure[w] != 0) continue;
      const int kd = cfg->cf_kind[w];
      const int64_t wa = cfg->cf_a[w], wb = cfg->cf_b[w];
      int64_t r;
      if (kd == 0) r = jsub(jadd(t_c, wa), jmod(t_c, wa));
      else if (kd == 1) r = jsub(jadd(t_c, wb), jmod(t_c, wb));
      else if (t_c == JMAX || t_c < wa) r = wa;
      else if (t_c >= wa && t_c < jadd(wa, wb)) r = jadd(wa, wb);
      else r = JMAX;
      e = min(e, r);
    }
    return e;
  };
  // SliceManager.appendSlice (S/SliceManager.java:27-38) of an edge of type ety (fixed, or a flexible edge's counter),
  // the current slice in registers (its fields move to the previous-slice registers, the old previous slice goes to
  // memory)
  auto append_edge = [&](int64_t start, int32_t ety) {
    if (ci >= 0) {
      flush_prev();
      Q_te[bb + ci] = start;
      Q_ty[bb + ci] = ety;
      pv = ci; p_ts = c_ts; p_tl = c_tl; p_tf = c_tf; p_cl = c_cl; p_cnt = c_cnt;
      p_p0 = c_p0; p_p1 = c_p1; p_p2 = c_p2;
      if (c_ts > start) uns |= 1;
    }
    const int64_t j = bb + tail;
    Q_ts[j] = start; Q_te[j] = JMAX; Q_cs[j] = cc; Q_ty[j] = 1;
    minmod = min(minmod, tail);
    ci = tail;
    tail++;
    c_ts = start; c_tl = start; c_tf = JMAX; c_cl = cc; c_cnt = 0; c_p0 = 0; c_p1 = ID_MIN; c_p2 = ID_MAX;
  };
  // last slice with tStart <= t on a sorted list, galloping down from the tail (out-of-order tuples land near it)
  auto find_sorted = [&](int64_t t) -> int {
    int hi = tail - 1;
    if (c_ts <= t) return hi;
    if (pv >= 0 && p_ts <= t) return pv;
    if (pv >= 0) hi = pv;
    int step = 1, lo;
    for (;;) {
      const int nx = hi - step;
      if (nx <= head) {
        if (Q_ts[bb + head] > t) return -1;
        lo = head;
        break;
      }
      if (Q_ts[bb + nx] <= t) {
        lo = nx;
        break;
      }
      hi = nx;
      step <<= 1;
    }
    while (hi - lo > 1) {
      const int m = (lo + hi) >> 1;
      if (Q_ts[bb + m] <= t) lo = m; else hi = m;
    }
    return lo;
  };
  const XSess xs{a.ss.start, a.ss.end};  // (by value: no reference may point into the argument block)
  LaneS<VT, V> L;  // the general path's state (scratch; only rare tuples touch it)
  L.c = cfg;
  L.q = q;
  L.b = bb;
  L.sb = sbase;
  load_fast();
  // the key's records go through a per-lane ring of 8 in LDS: the next 8 are loaded (one 128-B line of 16-B records,
  // half of one of packed 8-B records) while the current 8 are processed, so the tuple loop does not wait on a load
  // every iteration (the loads are unconditional, the index clamped, so no branch join waits for them)
  __shared__ int64_t R_t[8][256], R_v[8][256];
  const int tid = threadIdx.x;
  int64_t pt[8], pw[8];
  auto fetch8 = [&](int64_t c) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int64_t i = min(c + u, b1 - 1);
      if constexpr (VT == VT_I32) {
        if constexpr (packed) {
          const uint2 w = *(const uint2*)(rec + i * 8);
          pt[u] = pk_base + (int64_t)(w.x & pk_mask);
          pw[u] = (int64_t)(int32_t)w.y;
        } else {
          const uint4 w = *(const uint4*)(rec + i * 16);
          pt[u] = (int64_t)(((uint64_t)w.y << 32) | w.x);
          pw[u] = (int64_t)(int32_t)w.z;
        }
      } else {
        load(i, pt[u], pw[u]);
      }
    }
  };
  auto stage8 = [&]() {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      R_t[u][tid] = pt[u];
      R_v[u][tid] = pw[u];
    }
  };
  uint32_t n_gen = 0, n_in = 0, n_late = 0, n_late_mem = 0;  // path counters (a.dbg)
  fetch8(b0);
  stage8();
  for (int64_t c0 = b0; c0 < b1 && !err; c0 += 8) {
  fetch8(c0 + 8);
  const int m_ = (int)min((int64_t)8, b1 - c0);
  for (int u_ = 0; u_ < m_ && !err; u_++) {
    const int64_t t = R_t[u_][tid], vb = R_v[u_][tid];
    bool fast = one_ctx && ns > 0 && ci >= 0 && started;
    bool shift = false, flexe = false;
    int edit = 0;  // 1: the movable edge below the previous slice moves; 2: the previous slice splits
    int n_app = 0;
    int why = 0;  // debugging aid (a.dbg[4 + why]): why a tuple left the fast path
    if (fast) {
      if (t >= mx) {  // in-order: a first pending edge, room for the fixed edges it crosses and a flexible one
        const int64_t t_c = max(mx, ne);
        flexe = t >= jadd(t_c, gap);  // StreamSlicer.calculateNextFlexEdge (:118-130), one session context
        if (cfg->has_fixed == 0) {
          // session windows only: no fixed edge is ever pending (min_next_edge_ts stays Long.MIN_VALUE, :52-54), so
          // the only edge is the flexible one; te == Long.MIN_VALUE would meet the `min_next_edge_ts == te` branch
          n_app = flexe ? 1 : 0;
          if (t == JMIN) {
            fast = false;
            why = 1;
          } else if (tail + n_app > sc) {
            fast = false;
            why = 3;
          }
        } else if (ne == JMIN) {
          fast = false;
          why = 1;
        } else {
          int64_t e = ne;
          if (t >= ne) {
            while (t > e && n_app <= 8) {
              if (e >= 0) n_app++;
              const int64_t nx = next_edge(t, e);
              if (nx == JMIN || nx <= e) {  // the reference's hang / overflow: the general path reports it
                n_app = 99;
                break;
              }
              e = nx;
            }
          }
          if (e == t) n_app++;
          else if (flexe) n_app++;
          if (n_app > 8 || tail + n_app > sc) {
            fast = false;
            why = n_app > 8 ? 2 : 3;
          }
        }
        // the session: extended, unchanged, or a new one behind the last (t >= maxEventTime >= its end)
        if (fast && jadd(en_l, gap) < t && ns >= cfg->sesscap) {
          fast = false;
          why = 4;
        }
      } else if (t >= st_l && t <= en_l) {
        // out-of-order inside the last session: updateContext changes nothing, no modification
      } else if (t < st_l && t < c_tl && c_ts == st_l && pv >= 0 && jsub(st_l, gap) < t) {
        // out-of-order below the last session's start, within its gap: shiftStart (SessionWindow.java:56-66) when no
        // earlier session reaches t (getSession returns the last one, no merge follows), and checkSliceEdges moves the
        // movable edge between the previous slice and the current one -- which starts at the session start -- down to
        // t (S/SliceManager.java:89-125)
        const bool alone = ns < 2 || t > jadd(sen[ns - 2], gap);
        const int32_t ty0 = Q_ty[bb + pv];
        shift = alone && ty_movable(ty0);
        if (!shift) {
          // the edge below the current slice cannot move (a fixed grid edge, or a flexible edge of several contexts):
          // checkSliceEdges splits the previous slice at t instead (S/SliceManager.java:140-150, splitSlice :168-192),
          // room permitting without a compaction, the previous slice starting below t
          if (alone && tail < sc && p_ts < t && Q_te[bb + pv] == st_l) {
            edit = 2;
          } else {
            fast = false;
            why = alone ? 5 : 6;
          }
        }
      } else if (t < st_l && t < c_tl && c_ts != st_l && p_ts == st_l && pv - 1 >= head && jsub(st_l, gap) < t &&
                 (ns < 2 || t > jadd(sen[ns - 2], gap)) && Q_te[bb + pv - 1] == st_l &&
                 ty_movable(Q_ty[bb + pv - 1])) {
        // the last session starts at the previous slice (after a split above): shiftStart, and checkSliceEdges moves
        // the movable edge below the previous slice down to t
        edit = 1;
      } else {
        fast = false;
        why = t < st_l ? (c_ts != st_l ? 7 : 8) : 9;
      }
    }
    if (fast) {
      if (t >= mx) {
        // StreamSlicer.determineSlices, in-order branch (:51-86). The pending edge advances whenever t passes it, also
        // when every edge crossed is negative and none is appended (:65-69), so the next calculateNextFlexEdge sees it
        if (cfg->has_fixed == 0) {
          if (flexe) append_edge(t, ty_flex(1));  // calculateNextFlexEdge: the session gap reached (one context)
        } else if (n_app > 0 || t > ne) {
          while (t > ne) {
            if (ne >= 0) append_edge(ne, XTYPE_FIXED);
            ne = next_edge(t, ne);
          }
          if (ne == t) {
            append_edge(t, XTYPE_FIXED);
            ne = next_edge(t, ne);
          } else if (flexe) {
            append_edge(t, ty_flex(1));  // calculateNextFlexEdge: the session gap reached (one context)
          }
        }
        cc = jadd(cc, 1);
        mx = t;
        n_in++;
        // SliceManager.processElement in-order branch (:56-63): the current slice, then updateContext whose
        // modifications are dropped -- shiftEnd of the last session, or a new session at the end
        add_cur(t, vb);
        if (t != en_l) {
          if (t <= jadd(en_l, gap)) {
            en_l = t;
          } else {
            sen[ns - 1] = en_l;
            sst[ns] = t;
            sen[ns] = t;
            ns++;
            st_l = t;
            en_l = t;
          }
        }
      } else {
        cc = jadd(cc, 1);  // determineSlices: out of order, WindowManager.incrementCount only
        n_late++;
        if (shift) {  // the session start and the edge below the current slice move down to t
          Q_te[bb + pv] = t;
          Q_ts[bb + ci] = t;
          c_ts = t;
          uns |= 2;
          if (p_ts > t) uns |= 1;  // note_order of the moved slice
          st_l = t;
          sst[ns - 1] = t;
        } else if (edit == 1) {  // the session start and the edge below the previous slice move down to t
          const int64_t pp_ts = Q_ts[bb + pv - 1];
          Q_te[bb + pv - 1] = t;
          Q_ts[bb + pv] = t;
          p_ts = t;
          uns |= 2;
          if (pp_ts > t || t > c_ts) uns |= 1;  // note_order of the moved slice
          st_l = t;
          sst[ns - 1] = t;
        } else if (edit == 2) {
          // splitSlice(pv, t): the previous slice ends at t (a flexible edge), a new slice [t, session start) takes
          // the old edge's kind, the current slice moves up one position (insert_at; tail < sc: no compaction)
          const int32_t ty0 = Q_ty[bb + pv];
          const int32_t ty1 = ty_fixed(ty0) ? ty0 : ty_flex(ty0 - 1);
          const int64_t a_cs = Q_cs[bb + pv], a_cl = p_cl;
          flush_prev();
          Q_te[bb + pv] = t;
          Q_ty[bb + pv] = 1;
          const int nc = ci + 1;
          Q_ts[bb + nc] = c_ts;
          Q_te[bb + nc] = Q_te[bb + ci];
          Q_cs[bb + nc] = Q_cs[bb + ci];
          Q_ty[bb + nc] = Q_ty[bb + ci];
          Q_ts[bb + ci] = t;
          Q_te[bb + ci] = st_l;
          Q_cs[bb + ci] = a_cs;
          Q_ty[bb + ci] = ty_kind(ty1);
          pv = ci;
          p_ts = t; p_tl = t; p_tf = JMAX; p_cl = a_cl; p_cnt = 0; p_p0 = 0; p_p1 = ID_MIN; p_p2 = ID_MAX;
          minmod = min(minmod, ci);
          ci = nc;
          tail++;
          st_l = t;
          sst[ns - 1] = t;
        }
        // the in-order branch of processElement (t >= the current slice's tLast), else findSliceIndexByTimestamp:
        // its first two probes from the tail are the current and the previous slice (registers), on a sorted list
        // and on an unsorted one alike (the reference's loop runs backwards from the tail)
        if (t >= c_tl || c_ts <= t) {
          add_cur(t, vb);
        } else if (pv >= 0 && p_ts <= t) {
          add_prev(t, vb);
        } else {
          n_late_mem++;
          int idx;
          if (uns & 1) {  // an unsorted list: the rest of the reference's backward scan
            int k = pv >= 0 ? pv - 1 : tail - 2;
            while (k >= head && Q_ts[bb + k] > t) k--;
            idx = k >= head ? k : -1;
          } else {
            idx = find_sorted(t);
          }
          if (idx < 0) dropped++;  // IndexOutOfBoundsException: the tuple is lost
          else add_mem(idx, t, vb);
        }
      }
      continue;
    }
    // ---- the general path for this tuple
    n_gen++;
    if (a.dbg) atomicAdd(&a.dbg[4 + why], 1ull);
    flush_cur();
    L.s = s0;
    L.s.maxEventTime = mx; L.s.nextEdgeTs = ne; L.s.currentCount = cc;
    L.s.head = head; L.s.tail = tail; L.s.unsorted = uns; L.s.started = started; L.s.nsess[0] = ns;
    L.s.dropped = dropped; L.s.err = err;
    general_tuple<VT, V>(L, xs, t, vb);
    minmod = 0;  // (session edits move, split and merge slices; a compaction moves them all)
    s0 = L.s;
    mx = s0.maxEventTime; ne = s0.nextEdgeTs; cc = s0.currentCount;
    head = s0.head; tail = s0.tail; uns = s0.unsorted; started = s0.started; ns = s0.nsess[0];
    dropped = s0.dropped; err = s0.err;
    load_fast();
  }
  stage8();
  }
  flush_cur();
  s0.maxEventTime = mx; s0.nextEdgeTs = ne; s0.currentCount = cc;
  s0.head = head; s0.tail = tail; s0.unsorted = uns; s0.started = started; s0.nsess[0] = ns;
  s0.dropped = dropped; s0.err = err;
  if (minmod < s0.pvalid) s0.pvalid = minmod;
  *sp = s0;
  if (a.dbg) {  // (lanes that returned early count nothing; the atomics below are per lane -- a debugging aid)
    atomicAdd(&a.dbg[0], (unsigned long long)n_gen);
    atomicAdd(&a.dbg[1], (unsigned long long)n_in);
    atomicAdd(&a.dbg[2], (unsigned long long)n_late);
    atomicAdd(&a.dbg[3], (unsigned long long)n_late_mem);
  }
}

}  // namespace ls

// Eligible: keyed, one or more time-measured session windows beside context-free time windows, Eager slices (no count
// windows, no LazySlice record sets) -- exact_engine.cpp lane_session_mode()
hipError_t launch_lane_session(const XBatchArgs& a, int vt, int occ, hipStream_t st) {
  if (a.n_ops <= 0) return hipSuccess;
  const dim3 grid((unsigned)((a.n_ops + 255) / 256)), block(256);
#define SCOTTY_LS(VT_, OCC_, V_) hipLaunchKernelGGL((ls::lane_session_kernel<VT_, OCC_, V_>), grid, block, 0, st, a)
  // the rocprofv3 name of the instance (scotty_debug_kernel_name): <VT, OCC, store view, packed records>
  note_kernel(KN_LANE_SESSION, a.rec_stride == 8 ? "lane_session_kernel<%d, %d, XKView, true>"
                               : a.sl.kw          ? "lane_session_kernel<%d, %d, XKView, false>"
                                                  : "lane_session_kernel<%d, %d, XSlices, false>",
              vt, occ == 2 ? 2 : 3);
  if (a.rec_stride == 8) {  // packed records: int32 values, key-interleaved store only (exact_engine.cpp)
    if (vt != VT_I32 || !a.sl.kw) return hipErrorInvalidValue;
    if (occ == 2) hipLaunchKernelGGL((ls::lane_session_kernel<VT_I32, 2, XKView, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((ls::lane_session_kernel<VT_I32, 3, XKView, true>), grid, block, 0, st, a);
    return hipGetLastError();
  }
  if (a.sl.kw) {  // key-interleaved store: integer values
    if (occ == 2) {
      if (vt == VT_I32) SCOTTY_LS(VT_I32, 2, XKView); else SCOTTY_LS(VT_I64, 2, XKView);
    } else {
      if (vt == VT_I32) SCOTTY_LS(VT_I32, 3, XKView); else SCOTTY_LS(VT_I64, 3, XKView);
    }
  } else if (occ == 2) {
    if (vt == VT_I32) SCOTTY_LS(VT_I32, 2, XSlices);
    else if (vt == VT_I64) SCOTTY_LS(VT_I64, 2, XSlices);
    else SCOTTY_LS(VT_F64, 2, XSlices);
  } else {
    if (vt == VT_I32) SCOTTY_LS(VT_I32, 3, XSlices);
    else if (vt == VT_I64) SCOTTY_LS(VT_I64, 3, XSlices);
    else SCOTTY_LS(VT_F64, 3, XSlices);
  }
#undef SCOTTY_LS
  return hipGetLastError();
}

}  // namespace scotty
