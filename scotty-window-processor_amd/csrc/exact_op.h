// exact_op.h -- the reference operator's per-tuple state machine as wave-uniform device code, shared by
// the keyed replay kernel (exact_kernels.hip) and the batch-parallel non-keyed path (exact_batch.hip).
#pragma once
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
// Full-wave reductions over DPP row shifts / broadcasts (no LDS crossbar): the gfx9 inclusive-scan sequence
// (row_shr 1-3 of the lane's own value, row_shr 4 / 8 within the row, row_bcast 15 / 31 across rows) leaves the
// total in lane 63, which is broadcast.  Every lane of the wave must be active at the call.
template <int CTRL, int ROW, int BANK>
__device__ __forceinline__ uint64_t dpp64(uint64_t id, uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)id, (int)(uint32_t)v, CTRL, ROW, BANK, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(id >> 32), (int)(uint32_t)(v >> 32), CTRL, ROW, BANK, false);
  return ((uint64_t)hi << 32) | lo;
}
template <class F>
__device__ __forceinline__ uint64_t dpp_reduce(uint64_t x, uint64_t id, F f) {
  uint64_t v = f(x, dpp64<0x111, 0xF, 0xF>(id, x));  // row_shr:1
  v = f(v, dpp64<0x112, 0xF, 0xF>(id, x));           // row_shr:2 (of the lane's own value)
  v = f(v, dpp64<0x113, 0xF, 0xF>(id, x));           // row_shr:3
  v = f(v, dpp64<0x114, 0xF, 0xE>(id, v));           // row_shr:4, banks 1-3
  v = f(v, dpp64<0x118, 0xF, 0xC>(id, v));           // row_shr:8, banks 2-3
  v = f(v, dpp64<0x142, 0xA, 0xF>(id, v));           // row_bcast:15 into rows 1, 3
  v = f(v, dpp64<0x143, 0xC, 0xF>(id, v));           // row_bcast:31 into rows 2, 3
  return (uint64_t)rl64((int64_t)v, 63);
}
__device__ __forceinline__ int64_t fmax64(int64_t v) {
  return (int64_t)dpp_reduce((uint64_t)v, (uint64_t)JMIN,
                             [](uint64_t p, uint64_t q) { return (uint64_t)max((int64_t)p, (int64_t)q); });
}
__device__ __forceinline__ int64_t fmin64(int64_t v) {
  return (int64_t)dpp_reduce((uint64_t)v, (uint64_t)JMAX,
                             [](uint64_t p, uint64_t q) { return (uint64_t)min((int64_t)p, (int64_t)q); });
}
__device__ __forceinline__ uint64_t fsum64(uint64_t v) {
  return dpp_reduce(v, 0ull, [](uint64_t p, uint64_t q) { return p + q; });
}
__device__ __forceinline__ double fsumf(double v) {
  return __longlong_as_double((long long)dpp_reduce((uint64_t)__double_as_longlong(v), (uint64_t)__double_as_longlong(0.0),
                                                    [](uint64_t p, uint64_t q) {
                                                      return (uint64_t)__double_as_longlong(
                                                          __longlong_as_double((long long)p) +
                                                          __longlong_as_double((long long)q));
                                                    }));
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
#define LANE_ID ((int)__lane_id())

// Slice-list searches run by a whole wavefront (wave-uniform arguments and result).
// wave_first: first i in [lo, hi) with pred(i), for pred false...false true...true over the range; hi if none.  A
// 64-ary search, one probe per lane per round (two rounds for up to 4096 slices) instead of a chain of ~12 dependent
// loads.
template <typename P>
__device__ __forceinline__ int wave_first(int lo, int hi, P pred) {
  const int lane = LANE_ID;
  while (hi - lo > 64) {
    const int stride = (hi - lo + 63) >> 6;
    const int p = lo + lane * stride;
    const unsigned long long bal = __ballot(p < hi && pred(p));
    if (bal == 0) {
      lo = lo + ((hi - 1 - lo) / stride) * stride + 1;  // past the last probe
    } else {
      const int f = __ffsll((long long)bal) - 1;
      if (f == 0) return lo;
      const int pf = lo + f * stride;  // answer in (pf - stride, pf]
      lo = pf - stride + 1;
      hi = pf;
    }
  }
  const int p = lo + lane;
  const unsigned long long bal = __ballot(p < hi && pred(p));
  return bal ? lo + __ffsll((long long)bal) - 1 : hi;
}
// wave_last: last i in [lo, hi) with pred(i), -1 if none (no order assumed): a backward scan, four 64-slice chunks per
// round so their loads are in flight together
template <typename P>
__device__ __forceinline__ int wave_last(int lo, int hi, P pred) {
  for (int b = hi - 1; b >= lo; b -= 256) {
    unsigned long long m[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int i = b - j * 64 - LANE_ID;
      m[j] = __ballot(i >= lo && pred(i));
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (m[j]) return b - j * 64 - (__ffsll((long long)m[j]) - 1);
  }
  return -1;
}
struct Op {
  const XCfg* cfg;
  // slice arrays of this op (already offset by op * sc)
  int64_t *ts, *te, *tl, *tf, *cs, *cl;
  int32_t* ty;
  unsigned long long *cnt, *p0, *p1, *p2;
  // session columns of context c: ss[c][i] / se[c][i] (start / end of session i), computed from one base pointer
  // (an array of per-context pointers indexed by a loop variable was kept in scratch memory, adding a dependent
  // scratch load to every session access)
  struct SessCol {
    int64_t* base;
    int64_t stride;
    int cmax;
    __device__ __forceinline__ int64_t* operator[](int c) const { return base + (int64_t)min(c, cmax) * stride; }
  };
  SessCol ss, se;
  // records mode: per-slice record ranges, non-null flags, the op's record arena
  int64_t *rlo, *rhi, *rts, *rv;
  int32_t* nn;
  XState s;
  int32_t exc;
  // the lane index is read from the hardware, not stored: an Op may live in LDS, shared by its wave's lanes

  __device__ void bind(const XCfg* c, const XSlices& sl, const XSess& sx, int64_t op, int ln) {
    cfg = c;
    const int64_t b = op * (int64_t)c->sc;
    ts = sl.ts + b; te = sl.te + b; tl = sl.tl + b; tf = sl.tf + b; cs = sl.cs + b; cl = sl.cl + b;
    ty = sl.ty + b; cnt = sl.cnt + b; p0 = sl.p[0] + b; p1 = sl.p[1] + b; p2 = sl.p[2] + b;
    if (c->records) {
      rlo = sl.rlo + b; rhi = sl.rhi + b; nn = sl.nn + b;
      rts = sl.rts + op * c->rcap; rv = sl.rv + op * c->rcap;
    } else {
      rlo = rhi = rts = rv = nullptr;
      nn = nullptr;
    }
    const int64_t sb = op * c->ctx_alloc * (int64_t)c->sesscap;
    ss = SessCol{sx.start + sb, (int64_t)c->sesscap, max(c->ctx_alloc - 1, 0)};
    se = SessCol{sx.end + sb, (int64_t)c->sesscap, max(c->ctx_alloc - 1, 0)};
    exc = 0;
    (void)ln;
  }

  // ---------------------------------------------------------------- slice list primitives
  __device__ void copy_slice(int dst, int src) {
    ts[dst] = ts[src]; te[dst] = te[src]; tl[dst] = tl[src]; tf[dst] = tf[src];
    cs[dst] = cs[src]; cl[dst] = cl[src]; ty[dst] = ty[src];
    cnt[dst] = cnt[src]; p0[dst] = p0[src]; p1[dst] = p1[src]; p2[dst] = p2[src];
    if (cfg->records) {
      rlo[dst] = rlo[src]; rhi[dst] = rhi[src]; nn[dst] = nn[src];
    }
  }
  // lane-parallel move of n slices from src to dst (dst < src: forward chunks; dst > src: backward chunks)
  __device__ void move_range(int dst, int src, int n) {
    if (n <= 0 || dst == src) return;
    const bool rec = cfg->records != 0;
    if (dst < src) {
      for (int b = 0; b < n; b += 64) {
        const int i = b + LANE_ID;
        int64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, r0 = 0, r1 = 0;
        int32_t a6 = 0, r2 = 0;
        unsigned long long a7 = 0, a8 = 0, a9 = 0, a10 = 0;
        if (i < n) {
          a0 = ts[src + i]; a1 = te[src + i]; a2 = tl[src + i]; a3 = tf[src + i]; a4 = cs[src + i];
          a5 = cl[src + i]; a6 = ty[src + i]; a7 = cnt[src + i]; a8 = p0[src + i]; a9 = p1[src + i];
          a10 = p2[src + i];
          if (rec) { r0 = rlo[src + i]; r1 = rhi[src + i]; r2 = nn[src + i]; }
        }
        __builtin_amdgcn_wave_barrier();
        if (i < n) {
          ts[dst + i] = a0; te[dst + i] = a1; tl[dst + i] = a2; tf[dst + i] = a3; cs[dst + i] = a4;
          cl[dst + i] = a5; ty[dst + i] = a6; cnt[dst + i] = a7; p0[dst + i] = a8; p1[dst + i] = a9;
          p2[dst + i] = a10;
          if (rec) { rlo[dst + i] = r0; rhi[dst + i] = r1; nn[dst + i] = r2; }
        }
        __builtin_amdgcn_wave_barrier();
      }
    } else {
      for (int b = n; b > 0; b -= 64) {
        const int i = b - 1 - LANE_ID;
        int64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, r0 = 0, r1 = 0;
        int32_t a6 = 0, r2 = 0;
        unsigned long long a7 = 0, a8 = 0, a9 = 0, a10 = 0;
        if (i >= 0) {
          a0 = ts[src + i]; a1 = te[src + i]; a2 = tl[src + i]; a3 = tf[src + i]; a4 = cs[src + i];
          a5 = cl[src + i]; a6 = ty[src + i]; a7 = cnt[src + i]; a8 = p0[src + i]; a9 = p1[src + i];
          a10 = p2[src + i];
          if (rec) { r0 = rlo[src + i]; r1 = rhi[src + i]; r2 = nn[src + i]; }
        }
        __builtin_amdgcn_wave_barrier();
        if (i >= 0) {
          ts[dst + i] = a0; te[dst + i] = a1; tl[dst + i] = a2; tf[dst + i] = a3; cs[dst + i] = a4;
          cl[dst + i] = a5; ty[dst + i] = a6; cnt[dst + i] = a7; p0[dst + i] = a8; p1[dst + i] = a9;
          p2[dst + i] = a10;
          if (rec) { rlo[dst + i] = r0; rhi[dst + i] = r1; nn[dst + i] = r2; }
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
  // rpos: where the slice's (empty) record range starts (records mode)
  __device__ void init_slice(int i, int64_t start, int64_t end, int64_t c_s, int64_t c_l, int32_t type,
                             int64_t rpos = 0) {
    ts[i] = start; te[i] = end; tl[i] = start; tf[i] = JMAX; cs[i] = c_s; cl[i] = c_l; ty[i] = type;
    cnt[i] = 0; p0[i] = 0; p1[i] = (unsigned long long)ID_MIN; p2[i] = (unsigned long long)ID_MAX;
    if (cfg->records) {
      rlo[i] = rpos; rhi[i] = rpos; nn[i] = 0;
    }
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
    if (!(s.unsorted & 1)) {  // count of tStart <= t in [head, tail)
      const int lo = wave_first(s.head, s.tail, [&](int i) { return ts[i] > t; });
      return lo - 1 >= s.head ? lo - 1 : -1;
    }
    return wave_last(s.head, s.tail, [&](int i) { return ts[i] <= t; });
  }
  // LazyAggregateStore.findSliceIndexByCount (:41-49)
  __device__ int find_count(int64_t c) {
    return wave_last(s.head, s.tail, [&](int i) { return cs[i] <= c; });
  }
  // LazyAggregateStore.findSliceByEnd (:127-135)
  __device__ int find_end(int64_t e) {
    return wave_last(s.head, s.tail, [&](int i) { return te[i] == e; });
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
    if (cfg->records) {
      nn[i] = 1;
      if (ty_lazy(ty[i])) rec_insert(i, t, vbits);  // LazySlice.addElement: records.add (:23-27)
    }
  }

  // ---------------------------------------------------------------- LazySlice record sets (records mode)
  // lane-parallel move of n records from src to dst in the op's arena (either direction, overlap-safe)
  __device__ void rec_move(int64_t dst, int64_t src, int64_t n) {
    if (n <= 0 || dst == src) return;
    if (dst < src) {
      for (int64_t b = 0; b < n; b += 64) {
        const int64_t i = b + LANE_ID;
        int64_t a = 0, v = 0;
        if (i < n) { a = rts[src + i]; v = rv[src + i]; }
        __builtin_amdgcn_wave_barrier();
        if (i < n) { rts[dst + i] = a; rv[dst + i] = v; }
        __builtin_amdgcn_wave_barrier();
      }
    } else {
      for (int64_t b = n; b > 0; b -= 64) {
        const int64_t i = b - 1 - LANE_ID;
        int64_t a = 0, v = 0;
        if (i >= 0) { a = rts[src + i]; v = rv[src + i]; }
        __builtin_amdgcn_wave_barrier();
        if (i >= 0) { rts[dst + i] = a; rv[dst + i] = v; }
        __builtin_amdgcn_wave_barrier();
      }
    }
    __threadfence_block();
  }
  // record ranges of slices [from, tail) move by d
  __device__ void rec_adjust(int from, int64_t d) {
    for (int i = from + LANE_ID; i < s.tail; i += 64) {
      rlo[i] += d;
      rhi[i] += d;
    }
    __threadfence_block();
  }
  // first p in [lo, hi) with rts[p] >= t (hi if none): wavefront-cooperative, 64 probes per round
  __device__ int64_t rec_lb(int64_t lo, int64_t hi, int64_t t) {
    while (hi - lo > 64) {
      const int64_t stride = (hi - lo + 63) >> 6;
      const int64_t p = lo + (int64_t)LANE_ID * stride;
      const unsigned long long bal = __ballot(p < hi && rts[p] >= t);
      if (bal == 0) {
        lo = lo + ((hi - 1 - lo) / stride) * stride + 1;
      } else {
        const int f = __ffsll((long long)bal) - 1;
        if (f == 0) return lo;
        const int64_t pf = lo + (int64_t)f * stride;
        lo = pf - stride + 1;
        hi = pf;
      }
    }
    const int64_t p = lo + LANE_ID;
    const unsigned long long bal = __ballot(p < hi && rts[p] >= t);
    return bal ? lo + __ffsll((long long)bal) - 1 : hi;
  }
  // TreeSet.add: insert (t, v) into slice i's sorted set unless a record with ts t exists (S/slice/StreamRecord.java:25-27)
  __device__ void rec_insert(int i, int64_t t, int64_t vbits) {
    const int64_t p = rec_lb(rlo[i], rhi[i], t);
    if (p < rhi[i] && rts[p] == t) return;
    if (s.rend >= cfg->rcap) {
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
  // remove the arena record at p owned by slice i
  __device__ void rec_delete(int i, int64_t p) {
    rec_move(p, p + 1, s.rend - p - 1);
    rhi[i] -= 1;
    rec_adjust(i + 1, -1);
    s.rend--;
  }
  // AggregateValueState.recompute over the slice's record set (S/state/AggregateValueState.java:43-49)
  __device__ void rec_recompute(int i) {
    uint64_t c = 0, sw = 0;
    double sf = 0.0;
    int64_t mn = ID_MIN, mx = ID_MAX;
    for (int64_t p = rlo[i] + LANE_ID; p < rhi[i]; p += 64) {
      const Lift l = lift(cfg->vt, rv[p]);
      c++;
      if (cfg->vt == VT_F64) sf += __longlong_as_double((long long)l.sum);
      else sw += l.sum;
      mn = min(mn, l.mn);
      mx = max(mx, l.mx);
    }
    c = wsum(c);
    if (cfg->vt == VT_F64) sw = (uint64_t)__double_as_longlong(wsumf(sf));
    else sw = wsum(sw);
    mn = wmin(mn);
    mx = wmax(mx);
    cnt[i] = c;
    p0[i] = sw;
    p1[i] = (unsigned long long)mn;
    p2[i] = (unsigned long long)mx;
    nn[i] = c != 0;  // clear() then addElement per record: null when the set is empty
  }
  // AggregateState.removeElement (S/state/AggregateValueState.java:33-41): liftAndInvert of every (invertible)
  // function, else recompute from the records.  have == false: the record is Java null.
  __device__ void part_remove(int i, bool have, int64_t vbits) {
    if (cfg->invertible) {
      if (!have) {  // liftAndInvert(partial, null.record)
        exc = XERR_NPE;
        return;
      }
      const Lift l = lift(cfg->vt, vbits);
      cnt[i] = cnt[i] - 1;
      if (cfg->vt == VT_F64)
        p0[i] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)p0[i]) -
                                                         __longlong_as_double((long long)l.sum));
      else
        p0[i] = p0[i] - l.sum;
    } else {
      rec_recompute(i);
    }
  }
  // AbstractSlice.addElement + AggregateState.addElement of a moved record (LazySlice.prependElement :29-33), the
  // record itself placed by the caller
  __device__ void part_add(int i, int64_t t, int64_t vbits) {
    tl[i] = max(tl[i], t);
    tf[i] = min(tf[i], t);
    cl[i] = jadd(cl[i], 1);
    cnt[i] = cnt[i] + 1;
    nn[i] = 1;
    const Lift l = lift(cfg->vt, vbits);
    if (cfg->vt == VT_F64)
      p0[i] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)p0[i]) +
                                                       __longlong_as_double((long long)l.sum));
    else
      p0[i] = p0[i] + l.sum;
    p1[i] = (unsigned long long)min((int64_t)p1[i], l.mn);
    p2[i] = (unsigned long long)max((int64_t)p2[i], l.mx);
  }
  // slice(i).dropLastElement() -> slice(i+1).prependElement(record) (LazySlice.java:29-44).  The two record sets
  // are adjacent in the arena: the record changes owner by moving the boundary, then takes its sorted place in
  // slice i+1 (a rotation; a duplicate ts is dropped -- TreeSet.add of an equal element).
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
      __threadfence_block();
    }
  }
  // slice(j).dropFirstElement() -> slice(j-1).prependElement(record) (LazySlice.java:29-33, :46-53)
  __device__ void move_first_to_prev(int j) {
    const int i = j - 1;
    const bool have = rhi[j] > rlo[j];
    int64_t t = 0, v = 0;
    if (have) {
      t = rts[rlo[j]];
      v = rv[rlo[j]];
      rlo[j] += 1;
      rhi[i] += 1;
    }
    if (rhi[j] <= rlo[j]) {  // records.getFirst() on the emptied set
      if (have) rec_delete(i, rhi[i] - 1);
      exc = XERR_NOELEM;
      return;
    }
    cl[j] = jsub(cl[j], 1);
    tf[j] = rts[rlo[j]];
    part_remove(j, have, v);
    if (exc) {
      if (have) rec_delete(i, rhi[i] - 1);
      return;
    }
    part_add(i, t, v);
    const int64_t e = rhi[i] - 1;  // the new record, last in slice i's range
    const int64_t p = rec_lb(rlo[i], e, t);
    if (p < e && rts[p] == t) {
      rec_delete(i, e);
    } else if (p < e) {
      rec_move(p + 1, p, e - p);
      rts[p] = t;
      rv[p] = v;
      __threadfence_block();
    }
  }
  // slice(j).dropLastElement() -> slice(j-1).prependElement(record) (DeleteModification, S/SliceManager.java:141-146):
  // slice j's last record is rotated to the front of j's range, then moved like move_first_to_prev
  __device__ void move_last_of_next_to_prev(int j) {
    const int i = j - 1;
    const bool have = rhi[j] > rlo[j];
    int64_t t = 0, v = 0;
    if (have) {
      t = rts[rhi[j] - 1];
      v = rv[rhi[j] - 1];
      rec_move(rlo[j] + 1, rlo[j], rhi[j] - 1 - rlo[j]);
      rts[rlo[j]] = t;
      rv[rlo[j]] = v;
      __threadfence_block();
      rlo[j] += 1;
      rhi[i] += 1;
    }
    cl[j] = jsub(cl[j], 1);
    if (rhi[j] > rlo[j]) tl[j] = rts[rhi[j] - 1];
    part_remove(j, have, v);
    if (exc) {
      if (have) rec_delete(i, rhi[i] - 1);
      return;
    }
    if (!have) {
      exc = XERR_NPE;
      return;
    }
    part_add(i, t, v);
    const int64_t e = rhi[i] - 1;
    const int64_t p = rec_lb(rlo[i], e, t);
    if (p < e && rts[p] == t) {
      rec_delete(i, e);
    } else if (p < e) {
      rec_move(p + 1, p, e - p);
      rts[p] = t;
      rv[p] = v;
      __threadfence_block();
    }
  }
  // arena compaction: live records [rlo[head], rend) move to the arena start
  __device__ void rec_compact() {
    if (!cfg->records || s.tail <= s.head) {
      if (cfg->records && s.tail <= s.head) s.rend = 0;
      return;
    }
    const int64_t base = rlo[s.head];
    if (base <= 0) return;
    rec_move(0, base, s.rend - base);
    for (int i = s.head + LANE_ID; i < s.tail; i += 64) {
      rlo[i] -= base;
      rhi[i] -= base;
    }
    __threadfence_block();
    s.rend -= base;
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
    init_slice(i, start, JMAX, s.currentCount, s.currentCount, 1 | new_lazy_bit(), s.rend);
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
    init_slice(bpos, timestamp, a_end, a_cs, a_cl, ty_kind(a_ty) | new_lazy_bit(), cfg->records ? rhi[a] : 0);
    te[a] = timestamp;
    ty[a] = 1 | (a_ty & XTYPE_LAZY);
    note_order(bpos);
    if (ty_lazy(a_ty) && tl[a] >= timestamp) {  // move records to the new slice (:186-191)
      if (!cfg->records || !ty_lazy(ty[bpos])) {
        exc = XERR_UNSUPPORTED;
        return;
      }
      while (!exc && tl[a] >= timestamp) move_last_to_next(a);
    }
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
    if (cfg->records) {
      nn[idx] = nn[idx] | nn[b];
      // AbstractSlice.merge does not move records: slice b's remaining set is dropped with the slice
      while (rhi[b] > rlo[b]) rec_delete(b, rhi[b] - 1);
    }
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
          if (ty_lazy(st)) {  // move tuples across the moved edge (:106-125)
            if (m.post < m.pre) {
              if (tf[si] < tl[si] && tl[si] >= m.post) {
                if (!cfg->records) exc = XERR_UNSUPPORTED;
                while (!exc && tf[si] < tl[si] && tl[si] >= m.post) move_last_to_next(si);
              }
            } else {
              if (tf[nx] < tl[nx] && tf[nx] < m.post) {
                if (!cfg->records) exc = XERR_UNSUPPORTED;
                while (!exc && tf[nx] < tl[nx] && tf[nx] < m.post) move_first_to_prev(nx);
              }
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
            if (ty_lazy(ty[si + 1]) && cl[si + 1] > 0) {  // move records to the new slice (:141-146)
              if (!cfg->records) {
                exc = XERR_UNSUPPORTED;
                return;
              }
              while (!exc && cl[si + 1] > 0) move_last_of_next_to_prev(si + 1);
              if (exc) return;
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
    const int n = s.ns(c);
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
    s.set_ns(c, n + 1);
    if (mods && nm + 2 <= XMAXMODS) {
      mods[nm++] = Mod{2, 0, start};
      mods[nm++] = Mod{2, 0, end};
    }
  }
  __device__ void remove_window(int c, int i, Mod* mods, int& nm) {  // :48-52
    const int n = s.ns(c);
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
    s.set_ns(c, n - 1);
  }
  __device__ void merge_with_pre(int c, int idx, Mod* mods, int& nm) {  // :39-46
    if (idx < 0 || idx >= s.ns(c) || idx - 1 < 0) {
      exc = XERR_INDEX;
      return;
    }
    se[c][idx - 1] = se[c][idx];  // shiftEnd records no modification
    remove_window(c, idx, mods, nm);
  }
  __device__ int get_session(int c, int64_t pos) {  // :89-101
    const int64_t gap = cfg->gap[c];
    const int n = s.ns(c);
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
    if (s.ns(c) == 0) {  // hasActiveWindows() returns isEmpty() (WindowContext.java:15-17)
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
      if (si < s.ns(c) - 1) {
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
    for (int w = LANE_ID; w < cfg->n_cf; w += 64) {
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
    for (int w = LANE_ID; w < cfg->n_cf; w += 64) {
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
    if (exc) return;
    if (cfg->has_count && idx <= s.tail - 2) {  // shift count in slices: each later slice's last record (:77-85)
      if (!cfg->records) {
        exc = XERR_UNSUPPORTED;
        return;
      }
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

}  // namespace x
}  // namespace scotty
