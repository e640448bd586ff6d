// exact_kernels.hip -- gfx950 kernels of the exact ("replay") engine (see exact_common.h).
//
// One wavefront owns one operator.  It walks the operator's micro-batch in arrival order, 64 tuples per
// step.  For every still-unprocessed tuple j of the step, each lane decides from the operator state at
// the start of the step, plus exclusive prefix maxima over the earlier lanes, whether the tuple is
// "simple": it creates no slice edge (S/StreamSlicer.java:36-86), needs no count shift
// (S/SliceManager.java:77-85) and its SessionContext.updateContext (C/windowType/SessionWindow.java:42-87)
// is a no-op or extends the last session's end.  The simple prefix up to the first non-simple tuple is
// applied with one segmented wave reduction per touched slice (AbstractSlice.addElement +
// AggregateValueState.addElement, S/slice/AbstractSlice.java:27-31, S/state/AggregateValueState.java:23-31);
// the non-simple tuple ("event") then runs the reference logic exactly, wave-uniformly (every lane
// computes the same scalars; lane-parallel only for scans and moves).  Then the step continues after it.
//
// Watermarks (S/WindowManager.java:41-95) run in three launches: per-op trigger counting, per-op window
// emission + GC (one wave per op), and aggregation (one wave per emitted window).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exact_common.h"

namespace scotty {
namespace x {

constexpr int64_t JMAX = INT64_MAX, JMIN = INT64_MIN;
constexpr int64_t ID_MIN = INT64_MAX;  // identity of the min partial
constexpr int64_t ID_MAX = INT64_MIN;  // identity of the max partial

__device__ __forceinline__ int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
__device__ __forceinline__ int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
__device__ __forceinline__ int64_t jmod(int64_t a, int64_t b) { return b == -1 ? 0 : a % b; }

__device__ __forceinline__ int64_t rl64(int64_t v, int lane) {
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)(uint64_t)v, lane);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t wmax(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (int64_t)__shfl_xor((long long)v, o));
  return v;
}
__device__ __forceinline__ int64_t wmin(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (int64_t)__shfl_xor((long long)v, o));
  return v;
}
__device__ __forceinline__ uint64_t wsum(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, o);
  return v;
}
__device__ __forceinline__ double wsumf(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// exclusive prefix max over lanes (lane 0 gets JMIN)
__device__ __forceinline__ int64_t excl_pmax(int64_t v, int lane) {
  int64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int64_t u = (int64_t)__shfl_up((long long)inc, o);
    if (lane >= o) inc = max(inc, u);
  }
  int64_t ex = (int64_t)__shfl_up((long long)inc, 1);
  return lane == 0 ? JMIN : ex;
}

// Ordered int64 keys for Java Math.min/Math.max on double (same encoding as slicing_kernels.hip)
__device__ __forceinline__ int64_t f64_key(double d) {
  int64_t b = __double_as_longlong(d);
  return b ^ ((b >> 63) & 0x7FFFFFFFFFFFFFFFLL);
}

// lifted contributions of one tuple (value already in the op's value type, stored as 64-bit pattern)
struct Lift {
  uint64_t sum;   // u64 wrap sum (ints) or double bits (f64)
  int64_t mn, mx;
};
__device__ __forceinline__ Lift lift(int vt, int64_t vbits) {
  Lift l;
  if (vt == VT_F64) {
    double d = __longlong_as_double(vbits);
    l.sum = (uint64_t)vbits;
    l.mn = d != d ? INT64_MIN : f64_key(d);
    l.mx = d != d ? INT64_MAX : f64_key(d);
  } else {
    l.sum = (uint64_t)vbits;
    l.mn = vbits;
    l.mx = vbits;
  }
  return l;
}

__device__ __forceinline__ bool ty_fixed(int32_t t) { return t == XTYPE_FIXED || (t & XTYPE_FIXED) != 0; }
__device__ __forceinline__ bool ty_lazy(int32_t t) { return (t & XTYPE_LAZY) != 0; }
__device__ __forceinline__ int32_t ty_kind(int32_t t) { return ty_fixed(t) ? XTYPE_FIXED : (t & ~XTYPE_LAZY); }
// Slice.Flexible.isMovable: counter == 1 (S/slice/Slice.java:117-120)
__device__ __forceinline__ bool ty_movable(int32_t t) { return !ty_fixed(t) && (t & ~XTYPE_LAZY) == 1; }
__device__ __forceinline__ int32_t ty_flex(int32_t counter) { return counter & ~XTYPE_LAZY & ~XTYPE_FIXED; }

__device__ __forceinline__ double key_to_f64(int64_t kk) {
  return __longlong_as_double(kk ^ ((kk >> 63) & 0x7FFFFFFFFFFFFFFFLL));
}
// AggregateFunction.lower of the recognised kinds; int32 kinds are wrapped to int32 (Integer arithmetic)
__device__ __forceinline__ int64_t lower_value(int kind, uint64_t cnt, uint64_t sw, int64_t mn, int64_t mx) {
  switch (kind) {
    case 0: return (int64_t)(int32_t)(uint32_t)sw;                        // SUM_I32
    case 1: return (int64_t)(int32_t)(uint32_t)cnt;                       // COUNT
    case 2: case 5: return mn;                                            // MIN_I32 / MIN_I64
    case 3: case 6: return mx;                                            // MAX_I32 / MAX_I64
    case 4: case 7: return (int64_t)sw;                                   // SUM_I64 / SUM_F64 (double bits)
    case 8: return __double_as_longlong(mn == INT64_MIN ? __builtin_nan("") : key_to_f64(mn));
    case 9: return __double_as_longlong(mx == INT64_MAX ? __builtin_nan("") : key_to_f64(mx));
  }
  return 0;
}

struct Mod {  // C/windowType/windowContext/{Shift,Delete,Add}Modification.java
  int32_t kind;   // 0 shift, 1 delete, 2 add
  int64_t pre, post;
};

// ======================================================================== one operator, wave-uniform
struct Op {
  const XCfg* cfg;
  // slice arrays of this op (already offset by op * sc)
  int64_t *ts, *te, *tl, *tf, *cs, *cl;
  int32_t* ty;
  unsigned long long *cnt, *p0, *p1, *p2;
  int64_t* ss[XMAXCTX];
  int64_t* se[XMAXCTX];
  XState s;
  int32_t exc;
  int lane;

  __device__ void bind(const XCfg* c, const XSlices& sl, const XSess& sx, int64_t op, int ln) {
    cfg = c;
    const int64_t b = op * (int64_t)c->sc;
    ts = sl.ts + b; te = sl.te + b; tl = sl.tl + b; tf = sl.tf + b; cs = sl.cs + b; cl = sl.cl + b;
    ty = sl.ty + b; cnt = sl.cnt + b; p0 = sl.p[0] + b; p1 = sl.p[1] + b; p2 = sl.p[2] + b;
    for (int c2 = 0; c2 < XMAXCTX; c2++) {
      const int64_t sb = (op * c->ctx_alloc + min(c2, max(c->ctx_alloc - 1, 0))) * (int64_t)c->sesscap;
      ss[c2] = sx.start + sb;
      se[c2] = sx.end + sb;
    }
    exc = 0;
    lane = ln;
  }

  // ---------------------------------------------------------------- slice list primitives
  __device__ void copy_slice(int dst, int src) {
    ts[dst] = ts[src]; te[dst] = te[src]; tl[dst] = tl[src]; tf[dst] = tf[src];
    cs[dst] = cs[src]; cl[dst] = cl[src]; ty[dst] = ty[src];
    cnt[dst] = cnt[src]; p0[dst] = p0[src]; p1[dst] = p1[src]; p2[dst] = p2[src];
  }
  // lane-parallel move of n slices from src to dst (dst < src: forward chunks; dst > src: backward chunks)
  __device__ void move_range(int dst, int src, int n) {
    if (n <= 0 || dst == src) return;
    if (dst < src) {
      for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        int64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0;
        int32_t a6 = 0;
        unsigned long long a7 = 0, a8 = 0, a9 = 0, a10 = 0;
        if (i < n) {
          a0 = ts[src + i]; a1 = te[src + i]; a2 = tl[src + i]; a3 = tf[src + i]; a4 = cs[src + i];
          a5 = cl[src + i]; a6 = ty[src + i]; a7 = cnt[src + i]; a8 = p0[src + i]; a9 = p1[src + i];
          a10 = p2[src + i];
        }
        __builtin_amdgcn_wave_barrier();
        if (i < n) {
          ts[dst + i] = a0; te[dst + i] = a1; tl[dst + i] = a2; tf[dst + i] = a3; cs[dst + i] = a4;
          cl[dst + i] = a5; ty[dst + i] = a6; cnt[dst + i] = a7; p0[dst + i] = a8; p1[dst + i] = a9;
          p2[dst + i] = a10;
        }
        __builtin_amdgcn_wave_barrier();
      }
    } else {
      for (int b = n; b > 0; b -= 64) {
        const int i = b - 1 - lane;
        int64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0;
        int32_t a6 = 0;
        unsigned long long a7 = 0, a8 = 0, a9 = 0, a10 = 0;
        if (i >= 0) {
          a0 = ts[src + i]; a1 = te[src + i]; a2 = tl[src + i]; a3 = tf[src + i]; a4 = cs[src + i];
          a5 = cl[src + i]; a6 = ty[src + i]; a7 = cnt[src + i]; a8 = p0[src + i]; a9 = p1[src + i];
          a10 = p2[src + i];
        }
        __builtin_amdgcn_wave_barrier();
        if (i >= 0) {
          ts[dst + i] = a0; te[dst + i] = a1; tl[dst + i] = a2; tf[dst + i] = a3; cs[dst + i] = a4;
          cl[dst + i] = a5; ty[dst + i] = a6; cnt[dst + i] = a7; p0[dst + i] = a8; p1[dst + i] = a9;
          p2[dst + i] = a10;
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    __threadfence_block();
  }
  // make room for one more slice at the end (compacts [head, tail) to the front when needed)
  __device__ bool ensure_room() {
    if (s.tail < cfg->sc) return true;
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
    ts[i] = start; te[i] = end; tl[i] = start; tf[i] = JMAX; cs[i] = c_s; cl[i] = c_l; ty[i] = type;
    cnt[i] = 0; p0[i] = 0; p1[i] = (unsigned long long)ID_MIN; p2[i] = (unsigned long long)ID_MAX;
  }
  __device__ int32_t new_lazy_bit() const { return cfg->lazy ? XTYPE_LAZY : 0; }
  __device__ void note_order(int i) {
    if (i > s.head && ts[i - 1] > ts[i]) s.unsorted |= 1;
    if (i + 1 < s.tail && ts[i] > ts[i + 1]) s.unsorted |= 1;
  }
  // insert an uninitialised slot at index i (shifts [i, tail) up); returns the (possibly moved) index
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

  // LazyAggregateStore.findSliceIndexByTimestamp (:29-37): last slice with tStart <= t, -1 if none
  __device__ int find_ts(int64_t t) {
    if (s.tail <= s.head) return -1;
    if (!(s.unsorted & 1)) {
      int lo = s.head, hi = s.tail;  // count of tStart <= t in [head, tail)
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (ts[mid] <= t) lo = mid + 1; else hi = mid;
      }
      return lo - 1 >= s.head ? lo - 1 : -1;
    }
    for (int b = s.tail - 1; b >= s.head; b -= 64) {
      const int i = b - lane;
      const bool hit = i >= s.head && ts[i] <= t;
      const unsigned long long m = __ballot(hit);
      if (m) return b - (__ffsll((long long)m) - 1);
    }
    return -1;
  }
  // LazyAggregateStore.findSliceIndexByCount (:41-49)
  __device__ int find_count(int64_t c) {
    for (int b = s.tail - 1; b >= s.head; b -= 64) {
      const int i = b - lane;
      const bool hit = i >= s.head && cs[i] <= c;
      const unsigned long long m = __ballot(hit);
      if (m) return b - (__ffsll((long long)m) - 1);
    }
    return -1;
  }
  // LazyAggregateStore.findSliceByEnd (:127-135)
  __device__ int find_end(int64_t e) {
    for (int b = s.tail - 1; b >= s.head; b -= 64) {
      const int i = b - lane;
      const bool hit = i >= s.head && te[i] == e;
      const unsigned long long m = __ballot(hit);
      if (m) return b - (__ffsll((long long)m) - 1);
    }
    return -1;
  }

  // AbstractSlice.addElement + AggregateState.addElement (one tuple, exact)
  __device__ void add_element(int i, int64_t t, int64_t vbits) {
    tl[i] = max(tl[i], t);
    tf[i] = min(tf[i], t);
    cl[i] = jadd(cl[i], 1);
    cnt[i] = cnt[i] + 1;
    const Lift l = lift(cfg->vt, vbits);
    if (cfg->need & NEED_SUM) {
      if (cfg->vt == VT_F64)
        p0[i] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)p0[i]) +
                                                         __longlong_as_double((long long)l.sum));
      else
        p0[i] = p0[i] + l.sum;
    }
    if (cfg->need & NEED_MIN) p1[i] = (unsigned long long)min((int64_t)p1[i], l.mn);
    if (cfg->need & NEED_MAX) p2[i] = (unsigned long long)max((int64_t)p2[i], l.mx);
  }

  // SliceManager.appendSlice (S/SliceManager.java:27-38)
  __device__ void append_slice(int64_t start, int32_t type) {
    if (s.tail > s.head) {
      const int c = s.tail - 1;
      te[c] = start;
      ty[c] = type | (ty[c] & XTYPE_LAZY);
    }
    if (!ensure_room()) return;
    const int i = s.tail;
    init_slice(i, start, JMAX, s.currentCount, s.currentCount, 1 | new_lazy_bit());
    s.tail++;
    if (i > s.head && ts[i - 1] > start) s.unsorted |= 1;
  }

  // SliceManager.splitSlice (S/SliceManager.java:168-192); EagerSlices never move tuples
  __device__ void split_slice(int idx, int64_t timestamp) {
    if (!valid(idx)) return;
    int a = idx;
    int bpos;
    if (timestamp < te[a]) {
      bpos = a + 1;
    } else if (idx + 1 < s.tail) {
      a = idx + 1;
      bpos = idx + 2;
    } else {
      return;
    }
    const int64_t a_end = te[a], a_cs = cs[a], a_cl = cl[a];
    const int32_t a_ty = ty[a];
    const int rel_a = a - s.head;
    bpos = insert_at(bpos);
    if (bpos < 0) return;
    a = s.head + rel_a;
    init_slice(bpos, timestamp, a_end, a_cs, a_cl, ty_kind(a_ty) | new_lazy_bit());
    te[a] = timestamp;
    ty[a] = 1 | (a_ty & XTYPE_LAZY);
    note_order(bpos);
    if (ty_lazy(a_ty) && tl[a] >= timestamp) exc = XERR_UNSUPPORTED;  // LazySlice record movement
  }

  // AbstractSlice.merge + LazyAggregateStore.mergeSlice (:119-124)
  __device__ void merge_slice(int idx) {
    if (!valid(idx) || !valid(idx + 1)) return;
    const int b = idx + 1;
    tl[idx] = max(tl[idx], tl[b]);
    tf[idx] = min(tf[idx], tf[b]);
    te[idx] = max(te[idx], te[b]);
    cnt[idx] = cnt[idx] + cnt[b];
    if (cfg->vt == VT_F64)
      p0[idx] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)p0[idx]) +
                                                         __longlong_as_double((long long)p0[b]));
    else
      p0[idx] = p0[idx] + p0[b];
    p1[idx] = (unsigned long long)min((int64_t)p1[idx], (int64_t)p1[b]);
    p2[idx] = (unsigned long long)max((int64_t)p2[idx], (int64_t)p2[b]);
    remove_at(b);
  }

  // SliceManager.checkSliceEdges (S/SliceManager.java:89-166), modifications in insertion order
  __device__ void check_slice_edges(const Mod* mods, int nm) {
    for (int k = 0; k < nm && !exc; k++) {
      const Mod m = mods[k];
      if (m.kind == 0) {  // ShiftModification
        const int si = find_end(m.pre);
        if (si == -1) continue;
        const int32_t st = ty[si];
        if (ty_movable(st)) {
          if (!valid(si + 1)) return;
          const int nx = si + 1;
          te[si] = m.post;
          ts[nx] = m.post;
          s.unsorted |= 2;
          note_order(nx);
          if (ty_lazy(st)) {
            if (m.post < m.pre) {
              if (tf[si] < tl[si] && tl[si] >= m.post) exc = XERR_UNSUPPORTED;
            } else {
              if (tf[nx] < tl[nx] && tf[nx] < m.post) exc = XERR_UNSUPPORTED;
            }
          }
        } else {
          if (!ty_fixed(st)) ty[si] = ty_flex((st & ~XTYPE_LAZY) - 1) | (st & XTYPE_LAZY);
          split_slice(si, m.post);
        }
      } else if (m.kind == 1) {  // DeleteModification
        const int si = find_end(m.pre);
        if (si >= 0) {
          const int32_t st = ty[si];
          if (ty_movable(st)) {
            if (!valid(si + 1)) return;
            if (ty_lazy(ty[si + 1]) && cl[si + 1] > 0) {
              exc = XERR_UNSUPPORTED;
              return;
            }
            merge_slice(si);
          } else if (!ty_fixed(st)) {
            ty[si] = ty_flex((st & ~XTYPE_LAZY) - 1) | (st & XTYPE_LAZY);
          }
        }
      } else {  // AddModification
        const int si = find_ts(m.post);
        if (!valid(si)) return;
        if (ts[si] != m.post && te[si] != m.post) split_slice(si, m.post);
      }
    }
  }

  // ---------------------------------------------------------------- SessionContext (SessionWindow.java:40-116)
  __device__ void add_window(int c, int i, int64_t start, int64_t end, Mod* mods, int& nm) {  // WindowContext :19-25
    const int n = s.nsess[c];
    if (i < 0 || i > n) {
      exc = XERR_INDEX;
      return;
    }
    if (n >= cfg->sesscap) {
      exc = XERR_SESS_CAP;
      return;
    }
    for (int k = n; k > i; k--) {
      ss[c][k] = ss[c][k - 1];
      se[c][k] = se[c][k - 1];
    }
    ss[c][i] = start;
    se[c][i] = end;
    s.nsess[c] = n + 1;
    if (mods && nm + 2 <= XMAXMODS) {
      mods[nm++] = Mod{2, 0, start};
      mods[nm++] = Mod{2, 0, end};
    }
  }
  __device__ void remove_window(int c, int i, Mod* mods, int& nm) {  // :48-52
    const int n = s.nsess[c];
    if (i < 0 || i >= n) {
      exc = XERR_INDEX;
      return;
    }
    if (mods && nm + 2 <= XMAXMODS) {
      mods[nm++] = Mod{1, ss[c][i], 0};
      mods[nm++] = Mod{1, se[c][i], 0};
    }
    for (int k = i; k < n - 1; k++) {
      ss[c][k] = ss[c][k + 1];
      se[c][k] = se[c][k + 1];
    }
    s.nsess[c] = n - 1;
  }
  __device__ void merge_with_pre(int c, int idx, Mod* mods, int& nm) {  // :39-46
    if (idx < 0 || idx >= s.nsess[c] || idx - 1 < 0) {
      exc = XERR_INDEX;
      return;
    }
    se[c][idx - 1] = se[c][idx];  // shiftEnd records no modification
    remove_window(c, idx, mods, nm);
  }
  __device__ int get_session(int c, int64_t pos) {  // :89-101
    const int64_t gap = cfg->gap[c];
    const int n = s.nsess[c];
    int i = 0;
    for (; i < n; i++) {
      const int64_t st = ss[c][i], en = se[c][i];
      if (jsub(st, gap) <= pos && jadd(en, gap) >= pos) return i;
      if (jsub(st, gap) > pos) return i - 1;
    }
    return i - 1;
  }
  __device__ void session_update(int c, int64_t pos, Mod* mods, int& nm) {  // :42-87
    const int64_t gap = cfg->gap[c];
    if (s.nsess[c] == 0) {  // hasActiveWindows() returns isEmpty() (WindowContext.java:15-17)
      add_window(c, 0, pos, pos, mods, nm);
      return;
    }
    const int si = get_session(c, pos);
    if (si == -1) {
      add_window(c, 0, pos, pos, mods, nm);
      return;
    }
    const int64_t st = ss[c][si], en = se[c][si];
    if (jsub(st, gap) > pos) {
      add_window(c, si, pos, pos, mods, nm);
    } else if (st > pos && jsub(st, gap) < pos) {
      if (mods && nm < XMAXMODS) mods[nm++] = Mod{0, st, pos};  // shiftStart
      ss[c][si] = pos;
      if (si > 0) {
        if (jadd(se[c][si - 1], gap) >= ss[c][si]) merge_with_pre(c, si, mods, nm);
      }
    } else if (en < pos && jadd(en, gap) >= pos) {
      se[c][si] = pos;  // shiftEnd
      if (si < s.nsess[c] - 1) {
        if (jadd(se[c][si], gap) >= ss[c][si + 1]) merge_with_pre(c, si + 1, mods, nm);
      }
    } else if (jadd(en, gap) < pos) {
      add_window(c, si + 1, pos, pos, mods, nm);
    }
  }

  // ---------------------------------------------------------------- StreamSlicer (S/StreamSlicer.java:36-141)
  // calculateNextFixedEdge (:103-116): lane-parallel min over the time-measure context-free windows
  __device__ int64_t next_fixed_edge(int64_t te_) {
    const int64_t cur = s.nextEdgeTs == JMIN ? JMAX : s.nextEdgeTs;
    const int64_t t_c = max(jsub(te_, cfg->max_lateness), cur);
    int64_t e = JMAX;
    for (int w = lane; w < cfg->n_cf; w += 64) {
      if (cfg->cf_measure[w] != SCOTTY_MEASURE_TIME_) continue;
      e = min(e, assign_next(w, t_c));
    }
    return wmin(e);
  }
  // calculateNextFixedEdgeCount (:88-101)
  __device__ int64_t next_count_edge() {
    const int64_t cur = s.nextEdgeCount == JMIN ? 0 : s.nextEdgeCount;
    const int64_t t_c = max(s.currentCount, cur);
    int64_t e = JMAX;
    for (int w = lane; w < cfg->n_cf; w += 64) {
      if (cfg->cf_measure[w] != SCOTTY_MEASURE_COUNT_) continue;
      e = min(e, assign_next(w, t_c));
    }
    return wmin(e);
  }
  static constexpr int SCOTTY_MEASURE_TIME_ = 0, SCOTTY_MEASURE_COUNT_ = 1;
  // assignNextWindowStart: TumblingWindow.java:29-31, SlidingWindow.java:41-43, FixedBandWindow.java:37-48
  __device__ int64_t assign_next(int w, int64_t t) const {
    const int k = cfg->cf_kind[w];
    const int64_t a = cfg->cf_a[w], b = cfg->cf_b[w];
    if (k == 0) return jsub(jadd(t, a), jmod(t, a));
    if (k == 1) return jsub(jadd(t, b), jmod(t, b));
    if (t == JMAX || t < a) return a;
    if (t >= a && t < jadd(a, b)) return jadd(a, b);
    return JMAX;
  }
  // calculateNextFlexEdge (:118-130)
  __device__ int flex_count(int64_t te_) const {
    const int64_t t_c = max(s.maxEventTime, s.nextEdgeTs);
    int flex = 0;
    for (int c = 0; c < cfg->n_ctx; c++)
      if (te_ >= jadd(t_c, cfg->gap[c])) flex++;
    return flex;
  }
  __device__ void determine_slices(int64_t te_) {  // :36-86
    if (cfg->has_count) {
      if (s.nextEdgeCount == JMIN || s.currentCount == s.nextEdgeCount) {
        if (s.maxEventTime == JMIN) s.maxEventTime = te_;
        append_slice(s.maxEventTime, XTYPE_FIXED);
        if (exc) return;
        s.nextEdgeCount = next_count_edge();
      }
    }
    if (cfg->has_time) {
      const bool in_order = te_ >= s.maxEventTime;
      if (in_order) {
        if (cfg->has_fixed && s.nextEdgeTs == JMIN) s.nextEdgeTs = next_fixed_edge(te_);
        const int flex = cfg->has_ctx ? flex_count(te_) : 0;
        while (cfg->has_fixed && te_ > s.nextEdgeTs) {
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
    }
    s.currentCount = jadd(s.currentCount, 1);  // WindowManager.incrementCount (:196-198)
    s.maxEventTime = max(te_, s.maxEventTime);
  }

  // SliceManager.processElement (S/SliceManager.java:47-87)
  __device__ void manager_process(int64_t t, int64_t vbits) {
    if (s.tail <= s.head) append_slice(0, 1);
    if (exc) return;
    s.started = 1;
    const int cur = s.tail - 1;
    if (t >= tl[cur]) {
      add_element(cur, t, vbits);
      for (int c = 0; c < cfg->n_ctx && !exc; c++) {
        Mod discard[XMAXMODS];
        int nd = 0;
        session_update(c, t, discard, nd);  // modifications are dropped (:59-62)
      }
      return;
    }
    for (int c = 0; c < cfg->n_ctx && !exc; c++) {
      Mod mods[XMAXMODS];
      int nm = 0;
      session_update(c, t, mods, nm);
      if (exc) return;
      check_slice_edges(mods, nm);
    }
    if (exc) return;
    const int idx = find_ts(t);
    if (!valid(idx)) return;
    add_element(idx, t, vbits);
    if (cfg->has_count && idx <= s.tail - 2) exc = XERR_UNSUPPORTED;  // LazySlice count shift (:77-85)
  }
};

// ======================================================================== replay kernel
// Exactly how one simple tuple and the event processing interact is documented in exact_common.h.
template <int VT>
__device__ __forceinline__ void load_tuple(const XBatchArgs& a, int64_t i, int64_t& t, int64_t& vb) {
  if (a.rec_stride > 0) {
    const unsigned char* r = (const unsigned char*)a.ts + i * a.rec_stride;
    t = *(const int64_t*)r;
    if constexpr (VT == VT_I32) vb = (int64_t)*(const int32_t*)(r + 8);
    else vb = *(const int64_t*)(r + 8);
  } else {
    t = a.ts[i];
    if constexpr (VT == VT_I32) vb = (int64_t)((const int32_t*)a.val)[i];
    else vb = ((const int64_t*)a.val)[i];
  }
}

template <int VT>
__global__ __launch_bounds__(256) void replay_kernel(XBatchArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const XCfg* cfg = a.cfg;
  for (int64_t op = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); op < a.n_ops; op += nwaves) {
    int64_t b0 = 0, b1 = a.n;
    if (a.seg_begin) {
      b0 = a.seg_begin[op];
      b1 = a.seg_end[op];
    }
    if (b1 <= b0) continue;
    Op o;
    o.bind(cfg, a.sl, a.ss, op, lane);
    o.s = a.st[op];
    if (o.s.err) continue;
    if (a.retry && !o.s.pending) continue;
    o.s.pending = 0;
    if (a.need) {
      // capacity pre-check: an upper bound of the slices / sessions this segment can add.  Ops that might
      // overflow are deferred untouched; the host grows the capacities and relaunches them (retry).
      int64_t tmin = JMAX, tmax = JMIN;
      for (int64_t i = b0 + lane; i < b1; i += 64) {
        int64_t t_, v_;
        load_tuple<VT>(a, i, t_, v_);
        tmin = min(tmin, t_);
        tmax = max(tmax, t_);
      }
      tmin = wmin(tmin);
      tmax = wmax(tmax);
      const int64_t seglen = b1 - b0;
      int64_t from = o.s.started ? max(o.s.maxEventTime, jsub(tmin, cfg->max_lateness)) : jsub(tmin, cfg->max_lateness);
      if (from > tmax) from = tmax;
      const double span = (double)tmax - (double)from;
      double bound = 0.0;
      for (int w = lane; w < cfg->n_cf; w += 64) {
        const int k = cfg->cf_kind[w];
        const double step = k == 0 ? (double)cfg->cf_a[w] : (double)cfg->cf_b[w];
        if (k == 2) bound += 2.0;
        else if (cfg->cf_measure[w] == 1) bound += (double)seglen / step + 2.0;
        else bound += span / step + 2.0;
      }
      for (int o2 = 32; o2 > 0; o2 >>= 1) bound += __shfl_xor(bound, o2);
      if (cfg->n_ctx > 0) bound += 3.0 * (double)seglen;
      const double need_s = (double)(o.s.tail - o.s.head) + bound + 2.0;
      int need_x = 0;
      for (int c = 0; c < cfg->n_ctx; c++) need_x = max(need_x, o.s.nsess[c]);
      const int64_t need_ss = cfg->n_ctx > 0 ? (int64_t)need_x + seglen + 1 : 0;
      if (need_s > (double)cfg->sc || need_ss > cfg->sesscap) {
        if (lane == 0) {
          atomicMax(&a.need[0], (unsigned long long)min(need_s, 1e15) + 2ull);
          atomicMax(&a.need[1], (unsigned long long)need_ss);
          o.s.pending = 1;
          a.st[op] = o.s;
        }
        continue;
      }
    }
    for (int64_t c0 = b0; c0 < b1 && !o.s.err; c0 += 64) {
      const int n = (int)min((int64_t)64, b1 - c0);
      int64_t t = JMAX, vb = 0;
      if (lane < n) load_tuple<VT>(a, c0 + lane, t, vb);
      int j0 = 0;
      while (j0 < n) {
        // ---- classify lanes [j0, n) against the state at j0 (+ prefix effects of the simple lanes before)
        const bool mine = lane >= j0 && lane < n;
        const int64_t q = excl_pmax(mine ? t : JMIN, lane);  // max ts of lanes [j0, lane)
        bool simple = mine && o.s.tail > o.s.head;
        const int cur = o.s.tail - 1;
        int64_t cur_start = 0, cur_tl = 0;
        if (o.s.tail > o.s.head) {
          cur_start = o.ts[cur];
          cur_tl = o.tl[cur];
        }
        if (cfg->has_count) {
          const int64_t cj = jadd(o.s.currentCount, lane - j0);
          if (o.s.nextEdgeCount == JMIN || cj == o.s.nextEdgeCount) simple = false;
        }
        const int64_t pj = max(o.s.maxEventTime, q);
        if (cfg->has_time && t >= pj) {
          if (cfg->has_fixed) {
            if (o.s.nextEdgeTs == JMIN || t >= o.s.nextEdgeTs) simple = false;
          } else if (t == o.s.nextEdgeTs) {
            simple = false;
          }
          if (cfg->has_ctx) {
            const int64_t tc = max(pj, o.s.nextEdgeTs);
            for (int c = 0; c < cfg->n_ctx; c++)
              if (t >= jadd(tc, cfg->gap[c])) simple = false;
          }
        }
        const int64_t tl_j = max(cur_tl, q);  // the max earlier simple lane always lands in cur
        const bool in_order_m = t >= tl_j;
        int ext_mask = 0;
        for (int c = 0; c < cfg->n_ctx; c++) {
          const int ns = o.s.nsess[c];
          const int64_t gap = cfg->gap[c];
          if (ns == 0) {
            simple = false;
            continue;
          }
          int64_t lim = JMIN;
          for (int k = 0; k < ns - 1; k++) lim = max(lim, jadd(o.se[c][k], gap));
          const int64_t last_s = o.ss[c][ns - 1], last_e0 = o.se[c][ns - 1];
          const int64_t e_j = max(last_e0, q);
          if (t > lim) {
            if (t >= last_s && t <= e_j) ext_mask |= 1 << c;
            else if (t > e_j && t <= jadd(e_j, gap)) ext_mask |= 1 << c;
            else simple = false;
          } else if (simple) {
            // first session in the reach of t (getSession) must contain t
            bool ok = false;
            for (int k = 0; k < ns; k++) {
              const int64_t st = o.ss[c][k], en = k == ns - 1 ? e_j : o.se[c][k];
              if (jsub(st, gap) <= t && jadd(en, gap) >= t) {
                ok = st <= t && t <= en;
                break;
              }
              if (jsub(st, gap) > t) break;
            }
            if (!ok) simple = false;
          }
        }
        if (!in_order_m && simple) {
          if (t < cur_start) {
            if (cfg->has_count || (o.s.unsorted & 1) || t < o.ts[o.s.head]) simple = false;
          }
        }
        const unsigned long long ev = __ballot(mine && !simple);
        const int jstar = ev ? (__ffsll((long long)ev) - 1) : n;
        // ---- apply the simple prefix [j0, jstar)
        if (jstar > j0) {
          const bool act = lane >= j0 && lane < jstar;
          int sidx = -1;
          if (act) {
            if (in_order_m || t >= cur_start) {
              sidx = cur;
            } else {
              int lo = o.s.head, hi = o.s.tail;
              while (lo < hi) {
                int mid = (lo + hi) >> 1;
                if (o.ts[mid] <= t) lo = mid + 1; else hi = mid;
              }
              sidx = lo - 1;
            }
          }
          const Lift lf = lift(VT, vb);
          unsigned long long pend = __ballot(act);
          while (pend) {
            const int leader = __ffsll((long long)pend) - 1;
            const int si = __builtin_amdgcn_readlane(sidx, leader);
            const bool in = act && sidx == si;
            const unsigned long long m = __ballot(in);
            const uint64_t c_ = (uint64_t)__popcll(m);
            const int64_t tmx = wmax(in ? t : JMIN);
            const int64_t tmn = wmin(in ? t : JMAX);
            uint64_t sw = 0;
            if (cfg->need & NEED_SUM) {
              if constexpr (VT == VT_F64) sw = (uint64_t)__double_as_longlong(wsumf(in ? __longlong_as_double(vb) : 0.0));
              else sw = wsum(in ? lf.sum : 0);
            }
            const int64_t mn = (cfg->need & NEED_MIN) ? wmin(in ? lf.mn : ID_MIN) : ID_MIN;
            const int64_t mx = (cfg->need & NEED_MAX) ? wmax(in ? lf.mx : ID_MAX) : ID_MAX;
            o.tl[si] = max(o.tl[si], tmx);
            o.tf[si] = min(o.tf[si], tmn);
            o.cl[si] = jadd(o.cl[si], (int64_t)c_);
            o.cnt[si] = o.cnt[si] + c_;
            if (cfg->need & NEED_SUM) {
              if constexpr (VT == VT_F64)
                o.p0[si] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)o.p0[si]) +
                                                                    __longlong_as_double((long long)sw));
              else
                o.p0[si] = o.p0[si] + sw;
            }
            if (cfg->need & NEED_MIN) o.p1[si] = (unsigned long long)min((int64_t)o.p1[si], mn);
            if (cfg->need & NEED_MAX) o.p2[si] = (unsigned long long)max((int64_t)o.p2[si], mx);
            pend &= ~m;
          }
          const int64_t pmax = wmax(act ? t : JMIN);
          o.s.maxEventTime = max(o.s.maxEventTime, pmax);
          o.s.currentCount = jadd(o.s.currentCount, jstar - j0);
          for (int c = 0; c < cfg->n_ctx; c++) {
            const int ns = o.s.nsess[c];
            const int64_t emax = wmax(act && ((ext_mask >> c) & 1) ? t : JMIN);
            if (ns > 0 && emax != JMIN && emax > o.se[c][ns - 1]) o.se[c][ns - 1] = emax;
          }
          __threadfence_block();
        }
        if (jstar >= n) break;
        // ---- the event: the reference logic, exactly (wave-uniform)
        {
          const int64_t et = rl64(t, jstar), ev_b = rl64(vb, jstar);
          o.exc = 0;
          o.determine_slices(et);
          if (!o.exc) o.manager_process(et, ev_b);
          if (o.exc == XERR_INDEX) {
            o.s.dropped++;
            o.exc = 0;
          } else if (o.exc) {
            o.s.err = o.exc;
          }
          __threadfence_block();
        }
        j0 = jstar + 1;
      }
    }
    if (lane == 0) a.st[op] = o.s;
  }
}

// ======================================================================== watermark
// Triggered windows of one op in the reference's order (S/WindowManager.java:98-118): context-free windows
// in registration order, then context-aware windows.  DRY: count only, no state change.
template <bool DRY>
__device__ int64_t wm_triggers(Op& o, int64_t wm, int64_t* w_start, int64_t* w_end, int32_t* w_meas,
                               int32_t* w_op, int64_t off, int32_t opid) {
  const XCfg* cfg = o.cfg;
  int64_t k = 0;
  auto emit = [&](int64_t st, int64_t en, int32_t meas) {
    if (!DRY && o.lane == 0) {
      w_start[off + k] = st;
      w_end[off + k] = en;
      w_meas[off + k] = meas;
      w_op[off + k] = opid;
    }
    k++;
  };
  const int64_t last = o.s.lastWatermark;
  for (int w = 0; w < cfg->n_cf; w++) {
    const int kind = cfg->cf_kind[w], meas = cfg->cf_measure[w];
    const int64_t a = cfg->cf_a[w], b = cfg->cf_b[w];
    int64_t lo = last, hi = wm;
    if (meas == 1) {  // count measure: trigger up to the cLast of the slice holding wm (:109-115)
      int idx = o.find_ts(wm);
      if (idx < 0) {
        o.exc = XERR_WM_INDEX;
        return k;
      }
      if (o.tl[idx] >= wm && idx > o.s.head) idx--;
      lo = o.s.lastCount;
      hi = jadd(o.cl[idx], 1);
    }
    if (kind == 0) {  // TumblingWindow.triggerWindows :34-39
      const int64_t ls = jsub(lo, jmod(jadd(lo, a), a));
      for (int64_t ws = ls; jadd(ws, a) <= hi; ws = jadd(ws, a)) emit(ws, jadd(ws, a), meas);
    } else if (kind == 1) {  // SlidingWindow.triggerWindows :50-57
      const int64_t ls = jsub(hi, jmod(jadd(hi, b), b));
      for (int64_t ws = ls; jadd(ws, a) > lo; ws = jsub(ws, b))
        if (ws >= 0 && jadd(ws, a) <= jadd(hi, 1)) emit(ws, jadd(ws, a), meas);
    } else {  // FixedBandWindow.triggerWindows :51-57
      const int64_t e = jadd(a, b);
      if (lo <= e && e <= hi) emit(a, e, meas);
    }
  }
  for (int c = 0; c < cfg->n_ctx; c++) {  // SessionContext.triggerWindows (SessionWindow.java:108-119)
    const int64_t gap = cfg->gap[c];
    const int ns = o.s.nsess[c];
    if (ns == 0) {
      o.exc = XERR_WM_INDEX;  // getWindow(0) on an empty context
      return k;
    }
    int i = 0;
    while (i < ns && jadd(o.se[c][i], gap) < wm) {
      emit(o.ss[c][i], jadd(o.se[c][i], gap), cfg->ctx_measure[c]);
      i++;
    }
    if (!DRY && i > 0) {
      for (int j = i; j < ns; j++) {
        o.ss[c][j - i] = o.ss[c][j];
        o.se[c][j - i] = o.se[c][j];
      }
      o.s.nsess[c] = ns - i;
    }
  }
  return k;
}

__device__ __forceinline__ void wm_prologue(Op& o, int64_t wm) {
  // S/WindowManager.java:43-55
  if (o.s.lastWatermark == -1) o.s.lastWatermark = max((int64_t)0, jsub(wm, o.cfg->max_lateness));
}

__global__ __launch_bounds__(256) void wm_count_kernel(XWmArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t op = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (op >= a.n_ops) return;
  Op o;
  o.bind(a.cfg, a.sl, a.ss, op, lane);
  o.s = a.st[op];
  int64_t k = 0;
  if (lane == 0) {
    if (o.s.dropped) atomicAdd(a.dropped_total, (unsigned long long)o.s.dropped);
    if (o.s.err) atomicOr(a.op_err, 1 << o.s.err);
  }
  if (!o.s.err && o.s.tail > o.s.head) {
    wm_prologue(o, a.wm);
    const int64_t oldest = o.ts[o.s.head];
    if (o.s.lastWatermark < oldest) o.s.lastWatermark = oldest;
    k = wm_triggers<true>(o, a.wm, nullptr, nullptr, nullptr, nullptr, 0, 0);
    if (o.exc && lane == 0) atomicOr(a.err_flag, 1);
  }
  if (lane == 0) a.wcount[op] = k;
}

// emits the rows, computes the aggregation scan range and runs the watermark's state changes + GC
__global__ __launch_bounds__(256) void wm_emit_kernel(XWmArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t op = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (op >= a.n_ops) return;
  Op o;
  o.bind(a.cfg, a.sl, a.ss, op, lane);
  o.s = a.st[op];
  const XCfg* cfg = a.cfg;
  if (o.s.err) return;
  if (o.s.tail <= o.s.head) {  // empty store: lastWatermark := wm (:43-49)
    wm_prologue(o, a.wm);
    o.s.lastWatermark = a.wm;
    if (lane == 0) a.st[op] = o.s;
    return;
  }
  wm_prologue(o, a.wm);
  const int64_t oldest = o.ts[o.s.head];
  if (o.s.lastWatermark < oldest) o.s.lastWatermark = oldest;
  const int64_t off = a.woff[op];
  const int64_t k = wm_triggers<false>(o, a.wm, a.w_start, a.w_end, a.w_meas, a.w_op, off, (int32_t)op);
  // aggregate range of LazyAggregateStore.aggregate (:83-90)
  int64_t minTs = JMAX, maxTs = 0, minCount = o.s.currentCount, maxCount = 0;
  __threadfence_block();
  for (int64_t i = lane; i < k; i += 64) {
    const int64_t st = a.w_start[off + i], en = a.w_end[off + i];
    if (a.w_meas[off + i] == 0) {
      minTs = min(minTs, st);
      maxTs = max(maxTs, en);
    } else {
      minCount = min(minCount, st);
      maxCount = max(maxCount, en);
    }
  }
  minTs = wmin(minTs);
  maxTs = wmax(maxTs);
  minCount = wmin(minCount);
  maxCount = wmax(maxCount);
  if (k > 0) {
    const int S = o.s.tail - o.s.head;
    auto rel = [&](int i) { return i < 0 ? -1 : i - o.s.head; };
    int si = max(rel(o.find_ts(minTs)), 0);
    si = min(si, rel(o.find_count(minCount)));
    int ei = min(S - 1, rel(o.find_ts(maxTs)));
    ei = max(ei, rel(o.find_count(maxCount)));
    if (si < 0 && si <= ei) {  // getSlice(-1): IndexOutOfBoundsException in the reference
      if (lane == 0) atomicOr(a.err_flag, 2);
      si = 0;
    }
    o.s.wlo = o.s.head + si;       // absolute; slices stay in place until the next push
    o.s.whi = o.s.head + ei + 1;   // exclusive
  } else {
    o.s.wlo = o.s.whi = o.s.head;
  }
  o.s.lastWatermark = a.wm;
  o.s.lastCount = o.s.currentCount;
  // clearAfterWatermark (:82-95)
  const int64_t cw = jsub(a.wm, cfg->max_lateness);
  int64_t first = cw;
  for (int c = 0; c < cfg->n_ctx; c++)
    for (int i = 0; i < o.s.nsess[c]; i++) first = min(first, o.ss[c][i]);
  const int64_t t = min(jsub(cw, cfg->max_fixed), first);
  const int idx = o.find_ts(t);
  if (idx > o.s.head) o.s.head = idx;
  if (lane == 0) a.st[op] = o.s;
}

// one wave per emitted window: AggregateWindowState.containsSlice/addState over the op's scan range
__global__ __launch_bounds__(256) void wm_agg_kernel(XWmArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wi >= a.n_rows) return;
  const int64_t op = a.w_op[wi];
  const XState& st = a.st[op];
  const int64_t base = op * (int64_t)a.cfg->sc;
  const int64_t ws = a.w_start[wi], we = a.w_end[wi];
  const bool tmeas = a.w_meas[wi] == 0;
  int64_t lo = st.wlo, hi = st.whi;
  if (lo < 0) lo = 0;
  const int64_t* key = tmeas ? a.sl.ts + base : a.sl.cs + base;
  if (!(st.unsorted & 3) || !tmeas) {  // narrow to start keys in [ws, we] (contained slices satisfy it)
    int64_t l = lo, h = hi;
    while (l < h) {
      int64_t m = (l + h) >> 1;
      if (key[m] < ws) l = m + 1; else h = m;
    }
    const int64_t nlo = l;
    l = nlo; h = hi;
    while (l < h) {
      int64_t m = (l + h) >> 1;
      if (key[m] <= we) l = m + 1; else h = m;
    }
    lo = nlo;
    hi = l;
  }
  const int need = a.cfg->need, vt = a.cfg->vt;
  uint64_t cnt = 0, sw = 0;
  double sf = 0.0;
  int64_t mn = ID_MIN, mx = ID_MAX;
  for (int64_t i = lo + lane; i < hi; i += 64) {
    const int64_t s = base + i;
    const bool contains = tmeas ? (ws <= a.sl.ts[s] && we > a.sl.tl[s]) : (ws <= a.sl.cs[s] && we >= a.sl.cl[s]);
    if (!contains) continue;
    const uint64_t c = a.sl.cnt[s];
    if (c == 0) continue;
    cnt += c;
    if (need & NEED_SUM) {
      if (vt == VT_F64) sf += __longlong_as_double((long long)a.sl.p[0][s]);
      else sw += a.sl.p[0][s];
    }
    if (need & NEED_MIN) mn = min(mn, (int64_t)a.sl.p[1][s]);
    if (need & NEED_MAX) mx = max(mx, (int64_t)a.sl.p[2][s]);
  }
  cnt = wsum(cnt);
  if (vt == VT_F64) sf = wsumf(sf);
  else sw = wsum(sw);
  mn = wmin(mn);
  mx = wmax(mx);
  if (lane == 0) {
    a.has_value[wi] = cnt ? 1 : 0;
    if (a.w_key) a.w_key[wi] = a.slot_key ? a.slot_key[op] : (uint32_t)op;
    const uint64_t sword = vt == VT_F64 ? (uint64_t)__double_as_longlong(sf) : sw;
    for (int k = 0; k < a.cfg->n_aggs; k++)
      a.values[k][wi] = cnt ? lower_value(a.cfg->agg_kind[k], cnt, sword, mn, mx) : 0;
  }
}

__global__ void xstate_init_kernel(XState* st, int64_t from, int64_t to, const uint32_t* slot_key) {
  for (int64_t i = from + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < to; i += (int64_t)gridDim.x * blockDim.x) {
    XState s{};
    s.maxEventTime = JMIN;
    s.nextEdgeTs = JMIN;
    s.nextEdgeCount = JMIN;
    s.lastWatermark = -1;
    s.key = slot_key ? (int32_t)slot_key[i] : 0;
    st[i] = s;
  }
}

}  // namespace x

// ---------------------------------------------------------------- launch wrappers
hipError_t launch_replay(const XBatchArgs& a, int vt, hipStream_t st) {
  if (a.n_ops <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((a.n_ops + 3) / 4, 65536);
  if (vt == VT_I32) hipLaunchKernelGGL(x::replay_kernel<VT_I32>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (vt == VT_I64) hipLaunchKernelGGL(x::replay_kernel<VT_I64>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(x::replay_kernel<VT_F64>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_wm_count(const XWmArgs& a, hipStream_t st) {
  if (a.n_ops <= 0) return hipSuccess;
  hipLaunchKernelGGL(x::wm_count_kernel, dim3((unsigned)((a.n_ops + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_wm_emit(const XWmArgs& a, hipStream_t st) {
  if (a.n_ops <= 0) return hipSuccess;
  hipLaunchKernelGGL(x::wm_emit_kernel, dim3((unsigned)((a.n_ops + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_xstate_init(XState* st_, int64_t from, int64_t to, const uint32_t* slot_key, hipStream_t st) {
  if (to <= from) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((to - from + 255) / 256, 4096);
  hipLaunchKernelGGL(x::xstate_init_kernel, dim3((unsigned)blocks), dim3(256), 0, st, st_, from, to, slot_key);
  return hipGetLastError();
}
hipError_t launch_wm_agg(const XWmArgs& a, hipStream_t st) {
  if (a.n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(x::wm_agg_kernel, dim3((unsigned)((a.n_rows + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace scotty
