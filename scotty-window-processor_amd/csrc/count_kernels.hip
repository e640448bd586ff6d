// count_kernels.hip -- gfx950 kernels of the count-window path (layout and derivation: count_common.h).
//
// One micro-batch:
//   1. count_mark_kernel     edge bitmap over the batch's counts: the union grid of the windows'
//                            assignNextWindowStart in count space from the pending edge on
//                            (StreamSlicer.determineSlices / calculateNextFixedEdgeCount, S/StreamSlicer.java:36-44,
//                            :88-101); one thread per grid point.
//   2. count_stepc_kernel    edges per 256-tuple step (popcount) -> exclusive scan = cell of each step's start.
//   3. count_ingest_kernel   the HBM pass (12 B/tuple): SliceManager.processElement + LazySlice.addElement +
//                            AggregateValueState.addElement (S/SliceManager.java:47-87, S/slice/LazySlice.java:23-27);
//                            a tuple's cell = edges at or before its index; register accumulators for the wave's
//                            current cell, global atomics only in steps that contain an edge; step maxima of ts.
//   4. count_edges_kernel    tStart of every new slice = max ts before its edge (S/StreamSlicer.java:39-41, :83):
//                            prefix max over step maxima + an in-step wave scan; one wave per step with edges.
//   5. count_append_kernel   SliceManager.appendSlice (S/SliceManager.java:27-38) for every edge, partials folded
//                            into the open slice; the out-of-order check (a tuple older than its own slice).
//   6. count_finish_kernel   StreamSlicer.maxEventTime, store tail.
// Watermark (WindowManager.processWatermark, S/WindowManager.java:41-80):
//   count_wm_find_kernel     the count trigger's cend (S/WindowManager.java:109-115) and the oldest slice start,
//   count_wm_range_kernel    LazyAggregateStore.aggregate's scan range (S/aggregationstore/LazyAggregateStore.java:83-90),
//   count_wm_agg_kernel<G>   AggregateWindowState.containsSlice/addState (S/state/AggregateWindowState.java:25-53)
//                            per window: prefix-sum difference for invertible integer aggregates, else a G-lane scan,
//   count_gc_kernel          clearAfterWatermark / removeSlices (S/WindowManager.java:82-95).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/scotty_mi355x.h"
#include "count_common.h"
#include "exact_op.h"

namespace scotty {
namespace ck {

constexpr int64_t JMAX = INT64_MAX, JMIN = INT64_MIN;
constexpr int64_t ID_MIN = INT64_MAX;  // identity of min partials
constexpr int64_t ID_MAX = INT64_MIN;  // identity of max partials

template <typename T, typename F>
__device__ __forceinline__ T wred(T v, F f) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = f(v, (T)__shfl_xor(v, o));
  return v;
}
// full-wave DPP reductions (x::dpp_reduce; every lane active): the ingest kernel's flushes and edge steps
__device__ __forceinline__ uint64_t rsum(uint64_t v) { return x::fsum64(v); }
__device__ __forceinline__ int64_t rmax(int64_t v) { return x::fmax64(v); }
__device__ __forceinline__ int64_t rmin(int64_t v) { return x::fmin64(v); }
__device__ __forceinline__ double rsumf(double v) { return x::fsumf(v); }
__device__ __forceinline__ int64_t uni(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// First index in [l, h) where pred is false (pred true on a prefix of the range), h if there is none; searched by the
// G lanes (lane = 0 .. G-1) of an aligned lane group together, G probes per round.  l, h group-uniform.
template <int G, class P>
__device__ __forceinline__ int64_t group_first_false(int64_t l, int64_t h, int lane, P pred) {
  const int sh = (int)(threadIdx.x & 63) & ~(G - 1);
  const unsigned long long gm = G == 64 ? ~0ull : ((1ull << G) - 1);
  while (h - l > G) {
    const int64_t stride = (h - l + G - 1) / G;
    const int64_t p = l + (int64_t)lane * stride;
    const bool t = p < h && pred(p);
    const int c = __popcll((__ballot(t) >> sh) & gm);  // probes p_0 .. p_{c-1} true, p_c (if < h) false
    if (c == 0) return l;
    const int64_t pc = l + (int64_t)c * stride;
    l = l + (int64_t)(c - 1) * stride + 1;
    h = min(h, pc);
  }
  const int64_t p = l + lane;
  const bool t = p < h && pred(p);
  return l + __popcll((__ballot(t) >> sh) & gm);
}

// ---------------------------------------------------------------- 1. edge bitmap
// blockIdx.y = window.  Points of window w in [lo, hi): tumbling multiples of size, sliding multiples of slide
// (assignNextWindowStart, C/windowType/TumblingWindow.java:29-31, SlidingWindow.java:41-43), fixed band
// start and start+size (FixedBandWindow.java:37-48).  0 is only an edge as the stream's first tuple.
__global__ __launch_bounds__(256) void count_mark_kernel(CPushArgs a) {
  const int w = blockIdx.y;
  const CWin win = a.wins[w];
  const int64_t lo = max(a.C, a.mark_from), hi = a.C + a.n;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  auto set = [&](int64_t c) {
    const int64_t i = c - a.C;
    atomicOr(&a.bits[i >> 5], 1u << (i & 31));
  };
  if (g == 0 && w == 0 && a.extra_point >= a.C && a.extra_point < hi) set(a.extra_point);
  if (lo >= hi) return;
  if (win.kind == SCOTTY_WIN_FIXED_BAND) {
    if (g == 0) {
      if (win.a >= lo && win.a < hi && win.a > 0) set(win.a);
      const int64_t e = win.a + win.b;
      if (e >= lo && e < hi && e > 0) set(e);
    }
    return;
  }
  const int64_t step = win.kind == SCOTTY_WIN_TUMBLING ? win.a : win.b;
  const int64_t first = lo <= 0 ? step : ((lo + step - 1) / step) * step;
  for (int64_t m = first + g * step; m < hi; m += (int64_t)gridDim.x * blockDim.x * step) set(m);
}

// first time edge with batch position >= x
// First index in [lo, hi) with key >= g (key nondecreasing), hi if none, searched from a guess p: a galloping search
// outwards from p, then bisection inside the bracket -- O(log distance) dependent loads, 1-2 when the guess is close
// (event times and edge positions of a batch are near-uniform; a bisection from scratch took log2(n))
__device__ __forceinline__ int64_t lb_from(const int64_t* key, int64_t lo, int64_t hi, int64_t g, int64_t p) {
  p = p < lo ? lo : (p > hi ? hi : p);
  int64_t l, h;  // the answer lies in [l, h]
  if (p < hi && key[p] < g) {
    l = p + 1;
    h = hi;
    for (int64_t d = 1;; d <<= 1) {
      const int64_t q = p + d;
      if (q >= hi) break;
      if (key[q] >= g) {
        h = q;
        break;
      }
      l = q + 1;
    }
  } else {
    l = lo;
    h = p;
    for (int64_t d = 1;; d <<= 1) {
      const int64_t q = p - d;
      if (q < lo) break;
      if (key[q] < g) {
        l = q + 1;
        break;
      }
      h = q;
    }
  }
  while (l < h) {
    const int64_t m = (l + h) >> 1;
    if (key[m] < g) l = m + 1; else h = m;
  }
  return l;
}
// time edges before batch position x; guess: edges spread evenly over the batch
__device__ __forceinline__ int64_t te_lb(const CPushArgs& a, int64_t x) {
  const int64_t guess = a.n > 0 ? (int64_t)((double)x / (double)a.n * (double)a.n_te) : 0;
  return lb_from(a.te_pos, 0, a.n_te, x, guess);
}

// ---------------------------------------------------------------- 1b. time edges (time windows, in-order stream)
// Candidate k: the first tuple at or above cand[k] decides it (commit_kernel's rule, per candidate).
__global__ void count_tcand_kernel(CTimeArgs a) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.n_cand) return;
  const int64_t g = a.step ? a.cand0 + k * a.step : a.cand[k];
  // the first tuple >= g: a galloping search from the position the batch's first and last timestamps interpolate
  // (lane groups searching together -- 8 or 64 lanes per candidate -- issued more loads than they saved latency,
  // profiles/r06/ab/count_ingest/)
  const int64_t t0 = a.ts[a.start], t1 = a.ts[a.n - 1];
  double r = t1 > t0 ? ((double)g - (double)t0) / ((double)t1 - (double)t0) : 0.0;  // (no int64 wrap)
  r = r > 0.0 ? (r < 1.0 ? r : 1.0) : 0.0;                                            // (NaN -> 0)
  const int64_t guess = a.start + (int64_t)(r * (double)(a.n - 1 - a.start));
  const int64_t p = lb_from(a.ts, a.start, a.n, g, guess);
  // p < n: the host enumerates candidates up to the batch's last (= max) ts
  const int64_t e = a.ts[p];
  const int64_t m = p > a.start ? a.ts[p - 1] : a.prev_max;
  // the pending edge is appended once crossed; a later grid point iff the running max before its first tuple
  // reached the point before it, or that tuple lies within maxLateness of it (edges further back are skipped,
  // calculateNextFixedEdge's max(te - maxLateness, edge)); `while (te > edge)` appends only edges >= 0
  const int64_t gp = k == 0 ? 0 : (a.step ? g - a.step : a.cand[k - 1]);
  bool edge = k == 0 || gp <= m || (int64_t)((uint64_t)e - (uint64_t)g) < a.lateness;
  edge = edge && (g >= 0 || e == g);
  a.flag[k] = edge ? 1 : 0;
  a.pos[k] = p;
}

// order-preserving compaction of the decided candidates (offsets: exclusive scan of the flags)
__global__ void count_tscatter_kernel(CTimeArgs a) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.n_cand) return;
  if (k == a.n_cand - 1) *a.n_te = (unsigned long long)(a.off[k] + a.flag[k]);
  if (!a.flag[k]) return;
  const int64_t j = a.off[k];
  a.te_pos[j] = a.pos[k];
  a.te_g[j] = a.step ? a.cand0 + k * a.step : a.cand[k];
}

// ---------------------------------------------------------------- 2. edges per step
__global__ void count_stepc_kernel(CPushArgs a) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.nsteps) return;
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int64_t wi = s * 8 + k;
    if (wi < a.nwords) c += __popc(a.bits[wi]);
  }
  if (a.n_te > 0) {
    const int64_t lo = te_lb(a, s * CSTEP), hi = te_lb(a, (s + 1) * CSTEP);
    c += hi - lo;
    a.stepte[s] = lo;
    if (s == a.nsteps - 1) a.stepte[a.nsteps] = a.n_te;
    // up to 3 time edges of the step as packed in-step offsets (count | o0 << 8 | o1 << 16 | o2 << 24), else 255
    uint32_t pk = 255u;
    if (hi - lo <= 3) {
      pk = (uint32_t)(hi - lo);
      for (int64_t k = lo; k < hi; k++) pk |= (uint32_t)(a.te_pos[k] - s * CSTEP) << (8 * (1 + (k - lo)));
    }
    a.steptp[s] = pk;
  }
  a.stepc[s] = c;
}

__global__ void count_cells_init_kernel(CCells c, int64_t n) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    c.cnt[j] = 0;
    c.tl[j] = JMIN;
    c.tf[j] = JMAX;
    c.p[0][j] = 0;
    c.p[1][j] = (unsigned long long)ID_MIN;
    c.p[2][j] = (unsigned long long)ID_MAX;
  }
}

// ---------------------------------------------------------------- 3. ingest
template <int VT>
struct Lifted {
  uint64_t sw;
  double sf;
  int64_t mn, mx;
};
template <int VT>
__device__ __forceinline__ void lift(int64_t vb, uint64_t& sw, int64_t& mn, int64_t& mx) {
  if constexpr (VT == VT_F64) {
    const double d = __longlong_as_double(vb);
    sw = (uint64_t)vb;
    mn = d != d ? INT64_MIN : x::f64_key(d);
    mx = d != d ? INT64_MAX : x::f64_key(d);
  } else {
    sw = (uint64_t)vb;
    mn = vb;
    mx = vb;
  }
}

template <int VT, int NEED>
__device__ __forceinline__ void cell_add(const CCells& c, int64_t j, uint64_t n, int64_t tmax, int64_t tmin,
                                         uint64_t sw, double sf, int64_t mn, int64_t mx) {
  atomicAdd(&c.cnt[j], (unsigned long long)n);
  atomicMax(&c.tl[j], (long long)tmax);
  atomicMin(&c.tf[j], (long long)tmin);
  if constexpr ((NEED & NEED_SUM) != 0) {
    if constexpr (VT == VT_F64) atomicAdd((double*)&c.p[0][j], sf);
    else atomicAdd(&c.p[0][j], (unsigned long long)sw);
  }
  if constexpr ((NEED & NEED_MIN) != 0) atomicMin((long long*)&c.p[1][j], (long long)mn);
  if constexpr ((NEED & NEED_MAX) != 0) atomicMax((long long*)&c.p[2][j], (long long)mx);
}

// One wave per run of per_wave consecutive steps (256 tuples each, 4 per lane: offsets 2l, 2l+1, 128+2l, 129+2l).
// Steps without an edge only accumulate into the wave's current cell (per-lane registers, no cross-lane work); a
// step with edges reduces each of its cells once (masked wave reduction) and writes the count edges' records.
// The max ts before a count edge: in-order batches take the previous tuple's ts; otherwise the wave's running max
// plus the in-step prefix here, completed across waves by count_efix_kernel (wavemax -> wavepre).
template <int VT, int NEED>
__global__ __launch_bounds__(256) void count_ingest_kernel(CPushArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t s0 = wave * a.per_wave;
  const int64_t s1 = min(a.nsteps, s0 + a.per_wave);
  if (s0 >= s1) return;
  const int64_t first_start = uni(a.meta->first_start);
  // per-lane accumulator of the wave's current cell
  uint64_t cnt = 0, sw = 0;
  double sf = 0.0;
  int64_t tmax = JMIN, tmin = JMAX, mn = ID_MIN, mx = ID_MAX;
  int64_t cur = -1;
  uint32_t n_late = 0;
  int64_t lmax = JMIN;  // running max of this lane's tuples in the wave (dropped ones too)
  auto flush = [&]() {
    const uint64_t c = rsum(cnt);
    if (c != 0) {
      const int64_t tm = rmax(tmax);
      const int64_t tn = rmin(tmin);
      uint64_t s = 0;
      double f = 0.0;
      if constexpr ((NEED & NEED_SUM) != 0) {
        if constexpr (VT == VT_F64) f = rsumf(sf);
        else s = rsum(sw);
      }
      int64_t m1 = ID_MIN, m2 = ID_MAX;
      if constexpr ((NEED & NEED_MIN) != 0) m1 = rmin(mn);
      if constexpr ((NEED & NEED_MAX) != 0) m2 = rmax(mx);
      if (lane == 0) cell_add<VT, NEED>(a.cells, cur, c, tm, tn, s, f, m1, m2);
    }
    cnt = 0; sw = 0; sf = 0.0; tmax = JMIN; tmin = JMAX; mn = ID_MIN; mx = ID_MAX;
  };
  auto add = [&](int64_t t, int64_t vb) {
    uint64_t w;
    int64_t l, h;
    lift<VT>(vb, w, l, h);
    cnt++;
    tmax = max(tmax, t);
    tmin = min(tmin, t);
    if constexpr ((NEED & NEED_SUM) != 0) {
      if constexpr (VT == VT_F64) sf += __longlong_as_double((long long)w);
      else sw += w;
    }
    if constexpr ((NEED & NEED_MIN) != 0) mn = min(mn, l);
    if constexpr ((NEED & NEED_MAX) != 0) mx = max(mx, h);
  };
  typedef long long v2i64 __attribute__((ext_vector_type(2)));
  typedef int v2i32 __attribute__((ext_vector_type(2)));
  using VV = typename std::conditional<VT == VT_I32, v2i32, v2i64>::type;
  using VE = typename std::conditional<VT == VT_I32, int32_t, int64_t>::type;
  // A full step's loads, kept as loaded (vectors, no conversion: a conversion at the load would wait for the data
  // there) -- the step's edge-bitmap word (lanes 0-7), slice base and packed time edges first, then its tuples, so
  // the scalars of the next step can be read while later steps' tuples are still in flight.  Two steps are in
  // flight ahead of the one being combined (one was not enough: a wave waited a full HBM round trip per step).
  struct CStep {
    uint32_t bw, tp;
    int64_t sb;
    v2i64 ta, tb;
    VV va, vb;
  };
  const int64_t nfull = a.n / CSTEP;        // steps with CSTEP tuples
  const int64_t e1 = min(s1, nfull);        // the wave's full steps [s0, e1); a ragged last step after them
  auto ld_full = [&](int64_t s, CStep& st) {  // s < nfull: every load unconditional, every value as loaded
    const int64_t base = s * CSTEP;
    st.bw = a.bits[min(s * 8 + lane, a.nwords - 1)];  // (lanes 0-7 hold the step's words; masked at use)
    st.sb = a.stepbase[s];
    st.tp = a.steptp[s];  // (meaningful when a.n_te > 0; masked at use)
    const int64_t i0 = base + 2 * lane, i1 = base + 128 + 2 * lane;
    st.ta = __builtin_nontemporal_load((const v2i64*)(a.ts + i0));
    st.tb = __builtin_nontemporal_load((const v2i64*)(a.ts + i1));
    st.va = __builtin_nontemporal_load((const VV*)((const VE*)a.val + i0));
    st.vb = __builtin_nontemporal_load((const VV*)((const VE*)a.val + i1));
  };
  auto unpack = [&](const CStep& st, int64_t* t, int64_t* v) {
    t[0] = st.ta.x; t[1] = st.ta.y; t[2] = st.tb.x; t[3] = st.tb.y;
    v[0] = (int64_t)st.va.x; v[1] = (int64_t)st.va.y; v[2] = (int64_t)st.vb.x; v[3] = (int64_t)st.vb.y;
  };
  // in-order batches: the ts before the wave's first tuple (a count edge's slice start)
  int64_t prev_last = JMIN;
  if (a.check_sorted) prev_last = s0 > 0 ? a.ts[s0 * CSTEP - 1] : (a.shard ? JMIN : (int64_t)a.meta->prev_max);
  // one step: t/v/ok its tuples, bw_ its bitmap word (lanes 0-7), sb_ / tp_ its slice base and packed time edges
  auto step = [&](int64_t s, const int64_t (&t)[4], const int64_t (&v)[4], const bool (&ok)[4], uint32_t bw_,
                  int64_t sb_, uint32_t tp_) {
    const int64_t base = s * CSTEP;
    const int64_t i0 = base + 2 * lane, i1 = base + 128 + 2 * lane;
    const uint32_t bw = lane < 8 && s * 8 + lane < a.nwords ? bw_ : 0u;
    const uint32_t tp = a.n_te > 0 ? __builtin_amdgcn_readfirstlane(tp_) : 0u;
    const int64_t sb = uni(sb_);
    int64_t before_step = JMIN;  // ts of the tuple before this step (in-order batches)
    if (a.check_sorted) {
      before_step = prev_last;
      prev_last = (int64_t)__shfl((long long)t[3], 63);
      // the time-edge search (count_tcand_kernel) assumes a nondecreasing batch: every adjacent pair inside the step,
      // and the pair across the step's start (the tuple before it: the previous step's last, or the one before the
      // wave's range) -- so no step needs the next step's tuples
      const int64_t n0 = (int64_t)__shfl_down((long long)t[0], 1), n2 = (int64_t)__shfl_down((long long)t[2], 1);
      const int64_t l2 = (int64_t)__shfl((long long)t[2], 0);
      const int64_t s1_ = lane < 63 ? n0 : l2;  // successor of i0 + 1
      const bool bad = (i0 + 1 < a.n && t[1] < t[0]) || (i0 + 2 < a.n && s1_ < t[1]) ||
                       (i1 + 1 < a.n && t[3] < t[2]) || (lane < 63 && i1 + 2 < a.n && n2 < t[3]) ||
                       (lane == 0 && base > 0 && base < a.n && t[0] < before_step);
      if (bad) atomicOr((unsigned long long*)&a.meta->err, 8ull);
    }
    // edge words of the step (wave-uniform) and its time edges
    uint32_t wd[8];
#pragma unroll
    for (int k = 0; k < 8; k++) wd[k] = __builtin_amdgcn_readlane(bw, k);
    uint32_t any = wd[0] | wd[1] | wd[2] | wd[3] | wd[4] | wd[5] | wd[6] | wd[7];
    // packed in-step offsets (count_stepc_kernel), or the [t0, t1) range of te_pos when > 3
    int64_t t0 = 0, t1 = 0;
    const bool tpacked = (tp & 255u) != 255u;
    if (a.n_te > 0) {
      if (!tpacked) {
        t0 = uni(a.stepte[s]);
        t1 = uni(a.stepte[s + 1]);
      } else {
        t1 = tp & 255u;
      }
      if (t1 > t0) any |= 1u;
    }
    if (any == 0) {
      if (sb != cur) {
        if (cur >= 0) flush();
        cur = sb;
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if (!ok[j]) continue;
        lmax = max(lmax, t[j]);
        if (t[j] < first_start) n_late++;
        else add(t[j], v[j]);
      }
      return;
    }
    // time edges at in-step offsets <= o (le) or < o
    auto tcount = [&](int o, bool le) -> int64_t {
      int64_t c = 0;
      if (tpacked) {
        const int tn = (int)(tp & 255u);
#pragma unroll
        for (int i = 0; i < 3; i++) {
          const int oi = (int)((tp >> (8 * (i + 1))) & 255u);
          c += (i < tn && (le ? oi <= o : oi < o)) ? 1 : 0;
        }
      } else {
        for (int64_t k = t0; k < t1; k++) c += (le ? a.te_pos[k] <= base + o : a.te_pos[k] < base + o) ? 1 : 0;
      }
      return c;
    };
    // a step with edges: cell of every tuple (count edge before the time edges at one position)
    int pre[9];
    pre[0] = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) pre[k + 1] = pre[k] + __popc(wd[k]);
    const int64_t last = sb + pre[8] + (t1 - t0);
    const int off[4] = {2 * lane, 2 * lane + 1, 128 + 2 * lane, 129 + 2 * lane};
    int64_t cell[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int o = off[j], q = o >> 5, b = o & 31;
      const uint32_t mask = (uint32_t)((2ull << b) - 1);
      // time edges at or before this tuple (the tuple lands in the last slice appended)
      cell[j] = sb + pre[q] + __popc(wd[q] & mask) + tcount(o, true);
    }
    // count edges: batch position and the max ts of every tuple before them
    if (pre[8] != 0) {
      int64_t prv[4];
      if (a.check_sorted) {  // in-order: the previous tuple's ts
        const int64_t p1 = (int64_t)__shfl_up((long long)t[1], 1), p3 = (int64_t)__shfl_up((long long)t[3], 1);
        const int64_t l63 = (int64_t)__shfl((long long)t[1], 63);
        prv[0] = lane == 0 ? before_step : p1;
        prv[1] = t[0];
        prv[2] = lane == 0 ? l63 : p3;
        prv[3] = t[2];
      } else {  // the wave's running max before the step, then the in-step exclusive prefix max
        const int64_t W = rmax(lmax);
        int64_t ia = max(t[0], t[1]), ib = max(t[2], t[3]);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int64_t ua = (int64_t)__shfl_up((long long)ia, o), ub = (int64_t)__shfl_up((long long)ib, o);
          if (lane >= o) {
            ia = max(ia, ua);
            ib = max(ib, ub);
          }
        }
        const int64_t tot_a = (int64_t)__shfl((long long)ia, 63);
        int64_t ea = (int64_t)__shfl_up((long long)ia, 1), eb = (int64_t)__shfl_up((long long)ib, 1);
        if (lane == 0) ea = eb = JMIN;
        prv[0] = max(W, ea);
        prv[1] = max(prv[0], t[0]);
        prv[2] = max(max(W, tot_a), eb);
        prv[3] = max(prv[2], t[2]);
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int o = off[j], q = o >> 5, b = o & 31;
        if (!ok[j] || !((wd[q] >> b) & 1u)) continue;
        // edges strictly before o: count edges, then the time edges of earlier tuples
        const int64_t e = sb + pre[q] + __popc(wd[q] & ((1u << b) - 1u)) + tcount(o, false);
        a.cells.e_pos[e] = base + o;
        // in-order: final (the stream's first tuple sets maxEventTime to its own ts, S/StreamSlicer.java:39-40);
        // otherwise a partial completed by count_efix_kernel
        a.cells.e_ts[e] = (a.check_sorted && prv[j] == JMIN && !a.shard) ? t[j] : prv[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (ok[j]) lmax = max(lmax, t[j]);
    int64_t c_lo = JMAX;
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (ok[j]) c_lo = min(c_lo, cell[j]);
    c_lo = rmin(c_lo);
    if (last - c_lo <= 8) {
      // few cells: one masked wave reduction per cell before the last; the last stays in registers
      for (int64_t c = c_lo; c < last; c++) {
        uint64_t kc = 0, kw = 0;
        double kf = 0.0;
        int64_t kt = JMIN, kn = JMAX, km = ID_MIN, kx = ID_MAX;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (!ok[j] || cell[j] != c || t[j] < first_start) continue;
          uint64_t w;
          int64_t l, h;
          lift<VT>(v[j], w, l, h);
          kc++;
          kt = max(kt, t[j]);
          kn = min(kn, t[j]);
          if constexpr ((NEED & NEED_SUM) != 0) {
            if constexpr (VT == VT_F64) kf += __longlong_as_double((long long)w);
            else kw += w;
          }
          if constexpr ((NEED & NEED_MIN) != 0) km = min(km, l);
          if constexpr ((NEED & NEED_MAX) != 0) kx = max(kx, h);
        }
        if (c == cur) {  // the slice carried over from the previous step: registers
          cnt += kc;
          tmax = max(tmax, kt);
          tmin = min(tmin, kn);
          sw += kw;
          sf += kf;
          mn = min(mn, km);
          mx = max(mx, kx);
          continue;
        }
        const uint64_t rc = rsum(kc);
        if (rc == 0) continue;
        const int64_t rt = rmax(kt);
        const int64_t rn = rmin(kn);
        uint64_t rw = 0;
        double rf = 0.0;
        if constexpr ((NEED & NEED_SUM) != 0) {
          if constexpr (VT == VT_F64) rf = rsumf(kf);
          else rw = rsum(kw);
        }
        int64_t rm = ID_MIN, rx = ID_MAX;
        if constexpr ((NEED & NEED_MIN) != 0) rm = rmin(km);
        if constexpr ((NEED & NEED_MAX) != 0) rx = rmax(kx);
        if (lane == 0) cell_add<VT, NEED>(a.cells, c, rc, rt, rn, rw, rf, rm, rx);
      }
      if (last != cur) {
        if (cur >= 0) flush();
        cur = last;
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if (!ok[j]) continue;
        if (t[j] < first_start) n_late++;
        else if (cell[j] == last) add(t[j], v[j]);
      }
      return;
    }
    // many edges in the step: the last cell in registers, other tuples straight to their cell
    if (last != cur) {
      if (cur >= 0) flush();
      cur = last;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (!ok[j]) continue;
      if (t[j] < first_start) {
        n_late++;
        continue;
      }
      if (cell[j] == cur) {
        add(t[j], v[j]);
      } else {
        uint64_t w;
        int64_t l, h;
        lift<VT>(v[j], w, l, h);
        cell_add<VT, NEED>(a.cells, cell[j], 1, t[j], t[j], w, __longlong_as_double((long long)w), l, h);
      }
    }
  };
  // full steps, two in flight ahead of the one combined: buffers a_ / b_ take turns (no register copies: a copy of
  // a buffer whose loads are in flight waits for them); the loads of step s + 2 are clamped to the wave's last full
  // step (unconditional: nothing waits for them before their use)
  if (s0 < e1) {
    CStep a_, b_;
    ld_full(s0, a_);
    ld_full(min(s0 + 1, e1 - 1), b_);
    const bool all_ok[4] = {true, true, true, true};
    auto run = [&](int64_t s, CStep& buf, int64_t reload) {
      int64_t t[4], v[4];
      unpack(buf, t, v);
      const uint32_t bw = buf.bw, tp = buf.tp;
      const int64_t sb = buf.sb;
      step(s, t, v, all_ok, bw, sb, tp);
      ld_full(min(reload, e1 - 1), buf);
    };
    const int64_t npair = (e1 - s0) / 2;
    for (int64_t k = 0; k < npair; k++) {
      const int64_t s = s0 + 2 * k;
      run(s, a_, s + 2);
      run(s + 1, b_, s + 3);
    }
    if ((e1 - s0) & 1) run(e1 - 1, a_, e1 - 1);
  }
  if (e1 < s1) {  // the batch's ragged last step (s = nfull, fewer than CSTEP tuples)
    const int64_t s = e1;
    const int64_t base = s * CSTEP;
    const int64_t i0 = base + 2 * lane, i1 = base + 128 + 2 * lane;
    const int64_t idx[4] = {i0, i0 + 1, i1, i1 + 1};
    int64_t t[4], v[4];
    bool ok[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      ok[j] = idx[j] < a.n;
      t[j] = ok[j] ? a.ts[idx[j]] : JMIN;
      if constexpr (VT == VT_I32) v[j] = ok[j] ? (int64_t)((const int32_t*)a.val)[idx[j]] : 0;
      else v[j] = ok[j] ? ((const int64_t*)a.val)[idx[j]] : 0;
    }
    const int64_t wi = s * 8 + lane;
    const uint32_t bw = lane < 8 && wi < a.nwords ? a.bits[wi] : 0u;
    const uint32_t tp = a.n_te > 0 ? a.steptp[s] : 0u;
    step(s, t, v, ok, bw, a.stepbase[s], tp);
  }
  if (cur >= 0) flush();
  const uint32_t nl = wred(n_late, [](uint32_t p, uint32_t q) { return p + q; });
  if (lane == 0 && nl) atomicAdd((unsigned long long*)&a.meta->late_push, (unsigned long long)nl);
  const int64_t wm = rmax(lmax);
  if (lane == 0) a.stepmax[wave] = wm;  // per-wave max (the prefix over waves: count_premax_*)
}

// count edges of unsorted batches: complete the max ts before each edge with the waves before its own
__global__ void count_efix_kernel(CPushArgs a) {
  const int64_t E = a.meta->n_edges;
  const int64_t span = a.per_wave * CSTEP;
  const long long prev = a.shard ? JMIN : a.meta->prev_max;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = a.cells.e_pos[e], w = p / span;
    int64_t m = max((int64_t)prev, a.cells.e_ts[e]);
    if (w > 0) m = max(m, (int64_t)a.steppre[w - 1]);
    // the stream's first tuple sets maxEventTime to its own ts (S/StreamSlicer.java:39-40)
    a.cells.e_ts[e] = (m == JMIN && !a.shard) ? a.ts[p] : m;
  }
}

// ---------------------------------------------------------------- 4. edge positions and slice starts
// prefix max over step maxima (inclusive, single pass per 1024-step block + block carry)
__global__ __launch_bounds__(1024) void count_premax_block_kernel(const long long* in, long long* out, int64_t n,
                                                                  long long* bsum) {
  __shared__ long long wt[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t i = (int64_t)blockIdx.x * 1024 + tid;
  long long v = i < n ? in[i] : JMIN;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long u = __shfl_up(v, o);
    if (lane >= o) v = max(v, u);
  }
  if (lane == 63) wt[wid] = v;
  __syncthreads();
  long long add = JMIN;
  for (int w = 0; w < wid; w++) add = max(add, wt[w]);
  v = max(v, add);
  if (i < n) out[i] = v;
  if (tid == 1023) bsum[blockIdx.x] = v;
}
__global__ void count_premax_carry_kernel(long long* out, int64_t n, const long long* bsum_incl) {
  const int64_t b = blockIdx.x;
  if (b == 0) return;
  const long long c = bsum_incl[b - 1];
  const int64_t i = b * 1024 + threadIdx.x;
  if (i < n) out[i] = max(out[i], c);
}

// index, position and tStart (the edge itself, SliceManager.appendSlice(min_next_edge_ts)) of every time edge
__global__ void count_tedges_kernel(CPushArgs a) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.n_te) return;
  const int64_t p = a.te_pos[j], s = p / CSTEP, o = p - s * CSTEP;
  int64_t cb = 0;  // count edges of the step at or before this tuple
  for (int k = 0; k < 8; k++) {
    const int64_t wi = s * 8 + k;
    if (wi >= a.nwords) break;
    const uint32_t w = a.bits[wi];
    const int lo = k * 32;
    if (o >= lo + 31) cb += __popc(w);
    else if (o >= lo) cb += __popc(w & (uint32_t)((2ull << (o - lo)) - 1));
  }
  const int64_t e = a.stepbase[s] + cb + (j - te_lb(a, s * CSTEP));
  a.cells.e_pos[e] = a.shard ? ~p : p;  // shard records mark time edges (their tStart is the edge itself)
  a.cells.e_ts[e] = a.te_g[j];
}

// ---------------------------------------------------------------- 5. append
template <int VT>
__global__ __launch_bounds__(256) void count_append_kernel(CPushArgs a) {
  const CMeta& m = *a.meta;
  const int64_t E = m.n_edges;
  const int64_t head = m.head, tail = m.tail;
  const CCells& c = a.cells;
  const CSlices& sl = a.sl;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= E; j += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t n = c.cnt[j];
    if (j == 0) {  // the slice open before the batch
      if (n == 0) continue;
      const int64_t k = tail - 1;
      if (k < head) {
        atomicOr((unsigned long long*)&a.meta->err, 2ull);  // internal: tuples without a slice
        continue;
      }
      if (c.tf[0] < sl.ts[k]) atomicOr((unsigned long long*)&a.meta->err, 1ull);
      sl.cnt[k] += n;
      sl.tl[k] = max(sl.tl[k], (int64_t)c.tl[0]);
      if (VT == VT_F64)
        sl.p[0][k] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)sl.p[0][k]) +
                                                             __longlong_as_double((long long)c.p[0][0]));
      else
        sl.p[0][k] += c.p[0][0];
      sl.p[1][k] = (unsigned long long)min((int64_t)sl.p[1][k], (int64_t)c.p[1][0]);
      sl.p[2][k] = (unsigned long long)max((int64_t)sl.p[2][k], (int64_t)c.p[2][0]);
      continue;
    }
    const int64_t k = tail + j - 1;
    const int64_t st = c.e_ts[j - 1];
    if (n != 0 && c.tf[j] < st) atomicOr((unsigned long long*)&a.meta->err, 1ull);
    sl.ts[k] = st;
    sl.tl[k] = max(st, (int64_t)c.tl[j]);  // tLast starts at tStart (S/slice/AbstractSlice.java:15-23)
    sl.cs[k] = a.C + c.e_pos[j - 1];
    sl.cnt[k] = n;
    sl.p[0][k] = c.p[0][j];
    sl.p[1][k] = c.p[1][j];
    sl.p[2][k] = c.p[2][j];
  }
}

// cells to identity, plus (block 0, thread 0) the batch's edge count and the first-push scalars: one launch for what were
// three (count_nedges_kernel + count_cells_init_kernel + count_first_start_kernel, kept below for reference)
__global__ void count_prep_kernel(CPushArgs a) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t last = a.nsteps - 1;
    CMeta& m = *a.meta;
    m.n_edges = a.stepbase[last] + a.stepc[last];
    m.first_start = m.tail > m.head ? a.sl.ts[m.head] : (a.shard ? a.ts0 : a.ts[0]);
    m.late_push = 0;
  }
  const CCells& c = a.cells;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.cell_cap; j += (int64_t)gridDim.x * blockDim.x) {
    c.cnt[j] = 0;
    c.tl[j] = JMIN;
    c.tf[j] = JMAX;
    c.p[0][j] = 0;
    c.p[1][j] = (unsigned long long)ID_MIN;
    c.p[2][j] = (unsigned long long)ID_MAX;
  }
}
__global__ void count_nedges_kernel(CPushArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int64_t last = a.nsteps - 1;
  a.meta->n_edges = a.stepbase[last] + a.stepc[last];
}

__global__ void count_finish_kernel(CPushArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  CMeta& m = *a.meta;
  m.tail += m.n_edges;
  m.prev_max = max(m.prev_max, (int64_t)a.steppre[a.nwaves - 1]);
  m.late_total += m.late_push;
}

// first push of the stream: the oldest slice will be the one the first tuple opens (tStart = its ts)
__global__ void count_first_start_kernel(CPushArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  CMeta& m = *a.meta;
  m.first_start = m.tail > m.head ? a.sl.ts[m.head] : (a.shard ? a.ts0 : a.ts[0]);
  m.late_push = 0;
}

// ---------------------------------------------------------------- watermark
__device__ __forceinline__ int64_t last_le(const int64_t* key, int64_t lo, int64_t hi, int64_t x) {
  // last index in [lo, hi) with key <= x (key nondecreasing), lo - 1 if none
  int64_t l = lo, h = hi;
  while (l < h) {
    const int64_t mid = (l + h) >> 1;
    if (key[mid] <= x) l = mid + 1; else h = mid;
  }
  return l - 1;
}

__global__ void count_wm_find_kernel(CWmArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  CMeta& m = *a.meta;
  const int64_t head = m.head, tail = m.tail;
  m.range_err = 0;
  if (tail <= head) {
    m.wm_status = 1;
    return;
  }
  m.oldest = a.sl.ts[head];
  int64_t idx = last_le(a.sl.ts, head, tail, a.wm);  // findSliceIndexByTimestamp(wm)
  if (idx < head) {
    m.wm_status = 2;  // getSlice(-1)
    return;
  }
  if (a.sl.tl[idx] >= a.wm && idx > head) idx--;
  m.cend = a.sl.cs[idx] + (int64_t)a.sl.cnt[idx];  // cLast
  m.wm_status = 0;
}

// LazyAggregateStore.aggregate start/end index (S/aggregationstore/LazyAggregateStore.java:83-90; with no time
// windows minTs = MAX, maxTs = 0)
__global__ void count_wm_range_kernel(CWmArgs a) {
  if (blockIdx.x != 0) return;
  const int lane = threadIdx.x;
  CMeta& m = *a.meta;
  const int64_t head = m.head, tail = m.tail, S = tail - head;
  auto rel = [&](int64_t i) { return i < head ? (int64_t)-1 : i - head; };
  // cLast is not stored; cStart is nondecreasing, findSliceIndexByCount = last slice with cStart <= c.  The four
  // searches are independent: lanes 0-3 run one each (one chain of dependent loads instead of four in a row)
  int64_t r = 0;
  if (lane < 4) {
    const int64_t* key = (lane & 1) ? a.sl.cs : a.sl.ts;
    const int64_t x = lane == 0 ? a.min_ts : lane == 1 ? a.min_count : lane == 2 ? a.max_ts : a.max_count;
    r = rel(last_le(key, head, tail, x));
  }
  const int64_t r_ts_lo = (int64_t)__shfl((long long)r, 0), r_c_lo = (int64_t)__shfl((long long)r, 1);
  const int64_t r_ts_hi = (int64_t)__shfl((long long)r, 2), r_c_hi = (int64_t)__shfl((long long)r, 3);
  if (lane != 0) return;
  int64_t si = max(r_ts_lo, (int64_t)0);
  si = min(si, r_c_lo);
  int64_t ei = min(S - 1, r_ts_hi);
  ei = max(ei, r_c_hi);
  if (si < 0 && si <= ei) {
    m.range_err = 1;
    si = 0;
  }
  m.r_lo = head + si;
  m.r_hi = head + ei + 1;
}

// exclusive prefix sums of cnt and sum over [r_lo, r_hi): single-block chunks + carry (sizes here are the
// retained slices a watermark touches)
__global__ __launch_bounds__(1024) void count_pre_block_kernel(CWmArgs a, unsigned long long* bsum) {
  __shared__ unsigned long long wt[2][16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t lo = a.meta->r_lo, hi = a.meta->r_hi, n = hi - lo;
  const int64_t i = (int64_t)blockIdx.x * 1024 + tid;
  unsigned long long vc = i < n ? a.sl.cnt[lo + i] : 0, vs = i < n ? a.sl.p[0][lo + i] : 0;
  unsigned long long ic = vc, is = vs;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long uc = __shfl_up(ic, o), us = __shfl_up(is, o);
    if (lane >= o) {
      ic += uc;
      is += us;
    }
  }
  if (lane == 63) {
    wt[0][wid] = ic;
    wt[1][wid] = is;
  }
  __syncthreads();
  unsigned long long ac = 0, as = 0;
  for (int w = 0; w < wid; w++) {
    ac += wt[0][w];
    as += wt[1][w];
  }
  if (i < n) {
    a.pre_cnt[i] = ic - vc + ac;
    a.pre_sum[i] = is - vs + as;
  }
  if (tid == 1023) {
    bsum[2 * blockIdx.x] = ic + ac;
    bsum[2 * blockIdx.x + 1] = is + as;
  }
}
// exclusive scan of the block sums (one workgroup, 1024 blocks per round) and the range total at index n
__global__ __launch_bounds__(1024) void count_pre_bscan_kernel(CWmArgs a, unsigned long long* bsum, int64_t nblocks) {
  __shared__ unsigned long long wt[2][16];
  __shared__ unsigned long long carry[2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t n = a.meta->r_hi - a.meta->r_lo;
  if (tid == 0) carry[0] = carry[1] = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < nblocks; b0 += 1024) {
    const int64_t b = b0 + tid;
    const unsigned long long vc = b < nblocks ? bsum[2 * b] : 0, vs = b < nblocks ? bsum[2 * b + 1] : 0;
    unsigned long long ic = vc, is = vs;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long uc = __shfl_up(ic, o), us = __shfl_up(is, o);
      if (lane >= o) {
        ic += uc;
        is += us;
      }
    }
    if (lane == 63) {
      wt[0][wid] = ic;
      wt[1][wid] = is;
    }
    __syncthreads();
    unsigned long long ac = carry[0], as = carry[1];
    for (int w = 0; w < wid; w++) {
      ac += wt[0][w];
      as += wt[1][w];
    }
    if (b < nblocks) {
      bsum[2 * b] = ic - vc + ac;  // exclusive
      bsum[2 * b + 1] = is - vs + as;
    }
    __syncthreads();
    if (tid == 1023) {
      carry[0] = ic + ac;
      carry[1] = is + as;
    }
    __syncthreads();
  }
  if (tid == 0 && n >= 0) {
    a.pre_cnt[n] = carry[0];
    a.pre_sum[n] = carry[1];
  }
}
// the same exclusive prefix sums (and the range totals at index n) in one workgroup, 8 slices per thread per round:
// one launch instead of three for the few thousand slices a watermark usually scans
__global__ __launch_bounds__(1024) void count_pre_one_kernel(CWmArgs a) {
  constexpr int PER = 8;
  __shared__ unsigned long long wt[2][16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t lo = a.meta->r_lo, n = a.meta->r_hi - lo;
  unsigned long long cc = 0, cs = 0;  // running totals before the round
  for (int64_t base = 0; base < n; base += 1024 * PER) {
    unsigned long long vc[PER], vs[PER];
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const int64_t i = base + (int64_t)tid * PER + j;
      vc[j] = i < n ? a.sl.cnt[lo + i] : 0;
      vs[j] = i < n ? a.sl.p[0][lo + i] : 0;
    }
    unsigned long long tc = 0, ts_ = 0;
#pragma unroll
    for (int j = 0; j < PER; j++) {
      tc += vc[j];
      ts_ += vs[j];
    }
    unsigned long long ic = tc, is = ts_;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long uc = __shfl_up(ic, o), us = __shfl_up(is, o);
      if (lane >= o) {
        ic += uc;
        is += us;
      }
    }
    if (lane == 63) {
      wt[0][wid] = ic;
      wt[1][wid] = is;
    }
    __syncthreads();
    unsigned long long bc = cc, bs = cs, totc = cc, tots = cs;
    for (int w = 0; w < 16; w++) {
      if (w < wid) {
        bc += wt[0][w];
        bs += wt[1][w];
      }
      totc += wt[0][w];
      tots += wt[1][w];
    }
    unsigned long long rc = bc + ic - tc, rs = bs + is - ts_;  // exclusive prefix of this thread's first slice
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const int64_t i = base + (int64_t)tid * PER + j;
      if (i < n) {
        a.pre_cnt[i] = rc;
        a.pre_sum[i] = rs;
      }
      rc += vc[j];
      rs += vs[j];
    }
    cc = totc;
    cs = tots;
    __syncthreads();
  }
  if (tid == 0 && n >= 0) {
    a.pre_cnt[n] = cc;
    a.pre_sum[n] = cs;
  }
}
__global__ __launch_bounds__(1024) void count_pre_add_kernel(CWmArgs a, const unsigned long long* bsum) {
  const int64_t n = a.meta->r_hi - a.meta->r_lo;
  const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  if (blockIdx.x == 0 || i >= n) return;
  a.pre_cnt[i] += bsum[2 * blockIdx.x];
  a.pre_sum[i] += bsum[2 * blockIdx.x + 1];
}

template <int G>
__global__ __launch_bounds__(256) void count_wm_agg_kernel(CWmArgs a) {
  const int lane = threadIdx.x & (G - 1);
  const int64_t wi = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  if (wi >= a.nw) return;
  const int64_t ws = a.w_start[wi], we = a.w_end[wi];
  const bool tmeas = a.w_meas && a.w_meas[wi] == SCOTTY_MEASURE_TIME;
  const int64_t r_lo = a.meta->r_lo, r_hi = a.meta->r_hi;
  // contained slices (AggregateWindowState.containsSlice, S/state/AggregateWindowState.java:25-35): count
  // measure ws <= cStart && we >= cLast, cStart >= ws a suffix and cLast = cStart + cnt <= we a prefix; time
  // measure ws <= tStart && we > tLast, both nondecreasing on an in-order stream's slices
  int64_t lo, hi;
  if (!tmeas) {
    // count measure: cStart and cLast are nondecreasing on the count path's slices, so the window's G lanes search
    // together, G probes per round (log_G instead of log_2 rounds of dependent loads)
    lo = group_first_false<G>(r_lo, r_hi, lane, [&](int64_t i) { return a.sl.cs[i] < ws; });
    hi = group_first_false<G>(lo, r_hi, lane,
                              [&](int64_t i) { return a.sl.cs[i] + (int64_t)a.sl.cnt[i] <= we; });
  } else if (r_lo >= a.ts_sorted_from) {  // time measure over slices past the first tuple's: tStart / tLast sorted
    lo = group_first_false<G>(r_lo, r_hi, lane, [&](int64_t i) { return a.sl.ts[i] < ws; });
    hi = group_first_false<G>(lo, r_hi, lane, [&](int64_t i) { return a.sl.tl[i] < we; });
  } else {
    int64_t l = r_lo, h = r_hi;
    while (l < h) {
      const int64_t mid = (l + h) >> 1;
      if (a.sl.ts[mid] < ws) l = mid + 1; else h = mid;
    }
    lo = l;
    l = lo;
    h = r_hi;
    while (l < h) {
      const int64_t mid = (l + h) >> 1;
      if (a.sl.tl[mid] < we) l = mid + 1; else h = mid;
    }
    hi = l;
  }
  uint64_t cnt = 0, sw = 0;
  double sf = 0.0;
  int64_t mn = ID_MIN, mx = ID_MAX;
  if (a.prefix) {
    if (lane == 0 && hi > lo) {
      cnt = a.pre_cnt[hi - r_lo] - a.pre_cnt[lo - r_lo];
      sw = a.pre_sum[hi - r_lo] - a.pre_sum[lo - r_lo];
    }
  } else {
    for (int64_t k = lo + lane; k < hi; k += G) {
      const uint64_t c = a.sl.cnt[k];
      if (c == 0) continue;
      cnt += c;
      if (a.need & NEED_SUM) {
        if (a.vt == VT_F64) sf += __longlong_as_double((long long)a.sl.p[0][k]);
        else sw += a.sl.p[0][k];
      }
      if (a.need & NEED_MIN) mn = min(mn, (int64_t)a.sl.p[1][k]);
      if (a.need & NEED_MAX) mx = max(mx, (int64_t)a.sl.p[2][k]);
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
      cnt += (uint64_t)__shfl_xor((unsigned long long)cnt, o);
      sw += (uint64_t)__shfl_xor((unsigned long long)sw, o);
      sf += __shfl_xor(sf, o);
      mn = min(mn, (int64_t)__shfl_xor((long long)mn, o));
      mx = max(mx, (int64_t)__shfl_xor((long long)mx, o));
    }
  }
  if (lane == 0) {
    a.has_value[wi] = cnt ? 1 : 0;
    const uint64_t sword = a.vt == VT_F64 && !a.prefix ? (uint64_t)__double_as_longlong(sf) : sw;
    for (int k = 0; k < a.n_aggs; k++) a.values[k][wi] = cnt ? x::lower_value(a.agg_kind[k], cnt, sword, mn, mx) : 0;
  }
}

// rows of the triggered windows from per-window arithmetic runs (seg_off: exclusive prefix of the run lengths)
__global__ void count_rows_kernel(const CRowSeg* segs, const int64_t* seg_off, int nseg, int64_t* w_start,
                                  int64_t* w_end, int32_t* w_meas, int64_t nw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nw) return;
  int l = 0, h = nseg - 1;  // last run with seg_off <= i
  while (l < h) {
    const int m = (l + h + 1) >> 1;
    if (seg_off[m] <= i) l = m; else h = m - 1;
  }
  const CRowSeg g = segs[l];
  const int64_t st = g.first + (i - seg_off[l]) * g.step;
  w_start[i] = st;
  w_end[i] = st + g.size;
  w_meas[i] = (int32_t)g.meas;
}

__global__ void count_gc_kernel(CWmArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  CMeta& m = *a.meta;
  // the aggregation threw (getSlice(-1)): the reference leaves processWatermark before clearAfterWatermark, so the
  // store stays as it is (the host reports the exception after its one synchronisation)
  if (a.nw > 0 && m.range_err) return;
  if (m.tail <= m.head) return;
  const int64_t idx = last_le(a.sl.ts, m.head, m.tail, a.gc_before);  // LazyAggregateStore.removeSlices
  if (idx > m.head) m.head = idx;
}

// ---------------------------------------------------------------- sharding (count_common.h, CSHARD_HDR)
__global__ __launch_bounds__(256) void count_export_kernel(CPushArgs a, int64_t* rec, int64_t cap) {
  const CMeta& m = *a.meta;
  const int64_t E = m.n_edges;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g == 0) {
    rec[0] = a.steppre[a.nwaves - 1];
    rec[1] = (int64_t)m.late_push;
    rec[2] = E;
    rec[3] = a.n;
    rec[4] = a.C;
    rec[5] = E + 1 > cap ? 1 : 0;
  }
  int64_t* cells = rec + CSHARD_HDR;
  int64_t* edges = cells + 6 * cap;
  for (int64_t j = g; j < cap; j += (int64_t)gridDim.x * blockDim.x) {
    if (j <= E) {
      int64_t* c = cells + 6 * j;
      c[0] = (int64_t)a.cells.cnt[j];
      c[1] = a.cells.tl[j];
      c[2] = a.cells.tf[j];
      c[3] = (int64_t)a.cells.p[0][j];
      c[4] = (int64_t)a.cells.p[1][j];
      c[5] = (int64_t)a.cells.p[2][j];
    }
    if (j < E) {  // time edges: count word ~(global count)
      const int64_t p = a.cells.e_pos[j];
      edges[2 * j] = p >= 0 ? a.C + p : ~(a.C + ~p);
      edges[2 * j + 1] = a.cells.e_ts[j];
    }
  }
}

// rank offsets into the slice list and the stream's max ts before each rank's chunk
__global__ void count_shard_plan_kernel(CShardArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  CMeta& m = *a.meta;
  const int64_t words = cshard_words(a.cap);
  int64_t off = m.tail;
  long long pm = m.prev_max;
  for (int r = 0; r < a.world; r++) {
    const int64_t* h = a.gathered + r * words;
    if (h[5]) atomicOr((unsigned long long*)&m.err, 4ull);  // exchange capacity exceeded
    a.plan[2 * r] = off;
    a.plan[2 * r + 1] = pm;
    off += h[5] ? 0 : h[2];
    pm = max(pm, (long long)h[0]);
  }
}

__global__ __launch_bounds__(256) void count_shard_append_kernel(CShardArgs a) {
  const int r = blockIdx.y;
  const int64_t words = cshard_words(a.cap);
  const int64_t* rec = a.gathered + r * words;
  if (rec[5]) return;
  const int64_t E = rec[2];
  const int64_t* cells = rec + CSHARD_HDR;
  const int64_t* edges = cells + 6 * a.cap;
  const int64_t off = a.plan[2 * r];
  const int64_t pm = a.plan[2 * r + 1];
  for (int64_t j = 1 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= E; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t* c = cells + 6 * j;
    const int64_t ec = edges[2 * (j - 1)];
    int64_t st = edges[2 * (j - 1) + 1];  // time edge: the grid point itself
    if (ec >= 0) {  // count edge: maxEventTime before its tuple
      st = max(pm, st);
      if (st == JMIN) st = a.ts0;  // the stream's first tuple sets maxEventTime to its own ts (S/StreamSlicer.java:39-40)
    }
    const int64_t k = off + j - 1;
    if (c[0] != 0 && c[2] < st) atomicOr((unsigned long long*)&a.meta->err, 1ull);
    a.sl.ts[k] = st;
    a.sl.tl[k] = max(st, c[1]);
    a.sl.cs[k] = ec >= 0 ? ec : ~ec;
    a.sl.cnt[k] = (unsigned long long)c[0];
    a.sl.p[0][k] = (unsigned long long)c[3];
    a.sl.p[1][k] = (unsigned long long)c[4];
    a.sl.p[2][k] = (unsigned long long)c[5];
  }
}

// cell 0 of every rank folds into the slice open when its chunk began, in rank (= arrival) order
__global__ void count_shard_merge_kernel(CShardArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  CMeta& m = *a.meta;
  const int64_t words = cshard_words(a.cap);
  int64_t edges_total = 0;
  long long pm = m.prev_max;
  uint64_t late = 0;
  for (int r = 0; r < a.world; r++) {
    const int64_t* rec = a.gathered + r * words;
    late += (uint64_t)rec[1];
    pm = max(pm, (long long)rec[0]);
    if (rec[5]) continue;
    edges_total += rec[2];
    const int64_t* c = rec + CSHARD_HDR;
    if (c[0] == 0) continue;
    const int64_t k = a.plan[2 * r] - 1;
    if (k < m.head) {
      atomicOr((unsigned long long*)&m.err, 2ull);
      continue;
    }
    if (c[2] < a.sl.ts[k]) atomicOr((unsigned long long*)&m.err, 1ull);
    a.sl.cnt[k] += (unsigned long long)c[0];
    a.sl.tl[k] = max(a.sl.tl[k], c[1]);
    if (a.vt == VT_F64)
      a.sl.p[0][k] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)a.sl.p[0][k]) +
                                                             __longlong_as_double((long long)c[3]));
    else
      a.sl.p[0][k] += (unsigned long long)c[3];
    a.sl.p[1][k] = (unsigned long long)min((int64_t)a.sl.p[1][k], c[4]);
    a.sl.p[2][k] = (unsigned long long)max((int64_t)a.sl.p[2][k], c[5]);
  }
  m.tail += edges_total;
  m.prev_max = pm;
  m.late_total += late;
}

}  // namespace ck

// ---------------------------------------------------------------- launch wrappers
hipError_t launch_scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t st);
// e0 / e1 (nullable): timing events the dispatch stamps with its own start / end (hipExtLaunchKernel), as the grid
// path's ingest does -- marker events recorded around the launch also held the marker-to-dispatch gaps
template <int VT, int NEED>
static void launch_ingest_cn(const CPushArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const int64_t waves = (a.nsteps + a.per_wave - 1) / a.per_wave;
  note_kernel(KN_COUNT_INGEST, "count_ingest_kernel<%d, %d>", VT, NEED);
  const dim3 g((unsigned)((waves + 3) / 4));
  if (e0 || e1) hipExtLaunchKernelGGL((ck::count_ingest_kernel<VT, NEED>), g, dim3(256), 0, st, e0, e1, 0, a);
  else hipLaunchKernelGGL((ck::count_ingest_kernel<VT, NEED>), g, dim3(256), 0, st, a);
}
template <int VT>
static void launch_ingest_cv(const CPushArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  switch (a.need) {
    case 0: launch_ingest_cn<VT, 0>(a, st, e0, e1); break;
    case 1: launch_ingest_cn<VT, 1>(a, st, e0, e1); break;
    case 2: launch_ingest_cn<VT, 2>(a, st, e0, e1); break;
    case 3: launch_ingest_cn<VT, 3>(a, st, e0, e1); break;
    case 4: launch_ingest_cn<VT, 4>(a, st, e0, e1); break;
    case 5: launch_ingest_cn<VT, 5>(a, st, e0, e1); break;
    case 6: launch_ingest_cn<VT, 6>(a, st, e0, e1); break;
    default: launch_ingest_cn<VT, 7>(a, st, e0, e1); break;
  }
}

// everything of one push after the bitmap was cleared; premax_tmp: >= nsteps/1024 + 2 words
hipError_t launch_count_push(const CPushArgs& a, int64_t max_points_per_window, int64_t* scan_tmp,
                             long long* premax_tmp, hipStream_t st, hipEvent_t ingest_start,
                             hipEvent_t ingest_end) {
  if (a.n <= 0) return hipSuccess;
  {
    const int64_t th = std::max<int64_t>(1, std::min<int64_t>(max_points_per_window, 1 << 16));
    const unsigned bx = (unsigned)((th + 255) / 256);
    hipLaunchKernelGGL(ck::count_mark_kernel, dim3(bx, (unsigned)std::max(1, a.n_wins)), dim3(256), 0, st, a);
  }
  hipLaunchKernelGGL(ck::count_stepc_kernel, dim3((unsigned)((a.nsteps + 255) / 256)), dim3(256), 0, st, a);
  hipError_t e = launch_scan_i64(a.stepc, a.stepbase, a.nsteps, scan_tmp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ck::count_prep_kernel, dim3((unsigned)std::min<int64_t>((a.cell_cap + 255) / 256, 4096)), dim3(256),
                     0, st, a);
  if (a.vt == VT_I32) launch_ingest_cv<VT_I32>(a, st, ingest_start, ingest_end);
  else if (a.vt == VT_I64) launch_ingest_cv<VT_I64>(a, st, ingest_start, ingest_end);
  else launch_ingest_cv<VT_F64>(a, st, ingest_start, ingest_end);
  // prefix max over the wave maxima (a one-workgroup variant, count_premax_one_kernel, measured no faster: its
  // 16-values-per-thread loads do not coalesce)
  const int64_t nb = (a.nwaves + 1023) / 1024;
  hipLaunchKernelGGL(ck::count_premax_block_kernel, dim3((unsigned)nb), dim3(1024), 0, st, a.stepmax, a.steppre,
                     a.nwaves, premax_tmp);
  if (nb > 1) {
    hipLaunchKernelGGL(ck::count_premax_block_kernel, dim3((unsigned)((nb + 1023) / 1024)), dim3(1024), 0, st,
                       premax_tmp, premax_tmp, nb, premax_tmp + nb);
    if (nb > 1024) return hipErrorInvalidValue;  // > 2^20 waves per push: split the push
    hipLaunchKernelGGL(ck::count_premax_carry_kernel, dim3((unsigned)nb), dim3(1024), 0, st, a.steppre, a.nwaves,
                       premax_tmp);
  }
  if (!a.check_sorted)  // unsorted batches: complete the count edges' slice starts
    hipLaunchKernelGGL(ck::count_efix_kernel, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((a.cell_cap + 255) / 256, 4096))),
                       dim3(256), 0, st, a);
  if (a.n_te > 0)
    hipLaunchKernelGGL(ck::count_tedges_kernel, dim3((unsigned)((a.n_te + 255) / 256)), dim3(256), 0, st, a);
  if (a.shard) return hipGetLastError();  // the caller exports (launch_count_export) instead of appending
  const unsigned ab = (unsigned)std::min<int64_t>((a.cell_cap + 255) / 256, 8192);
  if (a.vt == VT_F64) hipLaunchKernelGGL(ck::count_append_kernel<VT_F64>, dim3(ab), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ck::count_append_kernel<VT_I32>, dim3(ab), dim3(256), 0, st, a);
  hipLaunchKernelGGL(ck::count_finish_kernel, dim3(1), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_count_time_edges(const CTimeArgs& a, int64_t* scan_tmp, hipStream_t st) {
  if (a.n_cand <= 0) return hipSuccess;
  const unsigned nb = (unsigned)((a.n_cand + 255) / 256);
  hipLaunchKernelGGL(ck::count_tcand_kernel, dim3(nb), dim3(256), 0, st, a);
  hipError_t e = launch_scan_i64(a.flag, a.off, a.n_cand, scan_tmp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ck::count_tscatter_kernel, dim3(nb), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_count_export(const CPushArgs& a, int64_t* rec, int64_t cap, hipStream_t st) {
  hipLaunchKernelGGL(ck::count_export_kernel, dim3((unsigned)std::min<int64_t>((cap + 255) / 256, 4096)), dim3(256), 0,
                     st, a, rec, cap);
  return hipGetLastError();
}

hipError_t launch_count_shard_commit(const CShardArgs& a, int64_t max_edges, hipStream_t st) {
  hipLaunchKernelGGL(ck::count_shard_plan_kernel, dim3(1), dim3(64), 0, st, a);
  const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((max_edges + 255) / 256, 4096));
  hipLaunchKernelGGL(ck::count_shard_append_kernel, dim3(bx, (unsigned)a.world), dim3(256), 0, st, a);
  hipLaunchKernelGGL(ck::count_shard_merge_kernel, dim3(1), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_count_rows(const CRowSeg* segs, const int64_t* seg_off, int nseg, int64_t* w_start, int64_t* w_end,
                             int32_t* w_meas, int64_t nw, hipStream_t st) {
  if (nw <= 0) return hipSuccess;
  hipLaunchKernelGGL(ck::count_rows_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, segs, seg_off, nseg,
                     w_start, w_end, w_meas, nw);
  return hipGetLastError();
}

hipError_t launch_count_wm_find(const CWmArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(ck::count_wm_find_kernel, dim3(1), dim3(64), 0, st, a);
  return hipGetLastError();
}

// range + (prefix sums) + per-window aggregation + GC; range_blocks = upper bound of (r_hi - r_lo + 1) / 1024
hipError_t launch_count_wm_agg(const CWmArgs& a, int64_t range_blocks, unsigned long long* bsum, hipStream_t st,
                               bool one_wg) {
  hipLaunchKernelGGL(ck::count_wm_range_kernel, dim3(1), dim3(64), 0, st, a);
  if (a.nw > 0) {
    if (a.prefix && one_wg && range_blocks <= 64) {  // (<= 2^16 slices in range: one workgroup)
      hipLaunchKernelGGL(ck::count_pre_one_kernel, dim3(1), dim3(1024), 0, st, a);
    } else if (a.prefix) {
      hipLaunchKernelGGL(ck::count_pre_block_kernel, dim3((unsigned)std::max<int64_t>(1, range_blocks)), dim3(1024), 0,
                         st, a, bsum);
      hipLaunchKernelGGL(ck::count_pre_bscan_kernel, dim3(1), dim3(1024), 0, st, a, bsum,
                         std::max<int64_t>(1, range_blocks));
      hipLaunchKernelGGL(ck::count_pre_add_kernel, dim3((unsigned)std::max<int64_t>(1, range_blocks)), dim3(1024), 0,
                         st, a, bsum);
    }
    hipLaunchKernelGGL(ck::count_wm_agg_kernel<16>, dim3((unsigned)((a.nw + 15) / 16)), dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t launch_count_gc(const CWmArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(ck::count_gc_kernel, dim3(1), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace scotty
