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

#include <algorithm>

#include "exact_op.h"

namespace scotty {
namespace x {

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
  __shared__ Op o_lds[4];
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
    Op& o = o_lds[threadIdx.x >> 6];  // per-wave operator state in LDS (a private Op sat in scratch)
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
      for (int c = 0; c < cfg->n_ctx; c++) need_x = max(need_x, o.s.ns(c));
      const int64_t need_ss = cfg->n_ctx > 0 ? (int64_t)need_x + seglen + 1 : 0;
      // records: every tuple adds at most one record; the live arena range is compacted first when needed
      int64_t need_r = 0;
      if (cfg->records) {
        const int64_t live = o.s.tail > o.s.head ? o.s.rend - o.rlo[o.s.head] : 0;
        need_r = live + seglen + 64;
      }
      if (need_s > (double)cfg->sc || need_ss > cfg->sesscap || need_r > cfg->rcap) {
        if (lane == 0) {
          atomicMax(&a.need[0], (unsigned long long)min(need_s, 1e15) + 2ull);
          atomicMax(&a.need[1], (unsigned long long)need_ss);
          atomicMax(&a.need[2], (unsigned long long)need_r);
          o.s.pending = 1;
          a.st[op] = o.s;
        }
        continue;
      }
      if (cfg->records && o.s.rend + seglen + 64 > cfg->rcap) o.rec_compact();
    } else if (cfg->records && o.s.rend + (b1 - b0) + 64 > cfg->rcap) {
      o.rec_compact();
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
          const int ns = o.s.ns(c);
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
          // records: a tuple inside the current slice but not after its last record takes a sorted insert
          if (cfg->records) simple = false;
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
          if (cfg->records) {
            // every simple lane landed in the current slice in ts order: append its record unless an earlier
            // record of the slice has the same ts (TreeSet.add, S/slice/LazySlice.java:23-27)
            o.nn[cur] = 1;
            if (ty_lazy(o.ty[cur])) {
              const int64_t lastrec = o.rhi[cur] > o.rlo[cur] ? o.rts[o.rhi[cur] - 1] : JMIN;
              const bool nr = act && t > max(lastrec, q);
              const unsigned long long m = __ballot(nr);
              if (nr) {
                const int64_t pos = o.s.rend + __popcll(m & ((1ull << lane) - 1));
                o.rts[pos] = t;
                o.rv[pos] = vb;
              }
              const int64_t k = __popcll(m);
              o.rhi[cur] += k;
              o.s.rend += k;
            }
          }
          const int64_t pmax = wmax(act ? t : JMIN);
          o.s.maxEventTime = max(o.s.maxEventTime, pmax);
          o.s.currentCount = jadd(o.s.currentCount, jstar - j0);
          for (int c = 0; c < cfg->n_ctx; c++) {
            const int ns = o.s.ns(c);
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
          if (xerr_tuple_failed(o.exc)) {
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
    if (!DRY && __lane_id() == 0) {
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
    constexpr int64_t LIM = (int64_t)1 << 61;
    const bool arith = kind <= 1 && lo > -LIM && lo < LIM && hi > -LIM && hi < LIM && a < LIM && b < LIM;
    if (arith) {  // the trigger loops below as one arithmetic run: ws = first + i * step, i < cnt (lanes split it)
      int64_t first, step, cnt;
      if (kind == 0) {
        const int64_t ls = lo - jmod(lo + a, a);
        first = ls;
        step = a;
        cnt = hi - ls - a >= 0 ? (hi - ls - a) / a + 1 : 0;
      } else {
        const int64_t ls = hi - jmod(hi + b, b);
        const int64_t k_end = ls + a > lo ? (ls + a - lo + b - 1) / b : 0;
        const int64_t k_lo = ls + a - hi - 1 > 0 ? (ls + a - hi - 1 + b - 1) / b : 0;
        const int64_t k_hi = min(k_end - 1, ls >= 0 ? ls / b : (int64_t)-1);
        first = ls - k_lo * b;
        step = -b;
        cnt = max((int64_t)0, k_hi - k_lo + 1);
      }
      if (!DRY)
        for (int64_t i = __lane_id(); i < cnt; i += 64) {
          const int64_t ws = first + i * step;
          w_start[off + k + i] = ws;
          w_end[off + k + i] = ws + a;
          w_meas[off + k + i] = meas;
          w_op[off + k + i] = opid;
        }
      k += cnt;
    } else if (kind == 0) {  // TumblingWindow.triggerWindows :34-39
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
    const int ns = o.s.ns(c);
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
      o.s.set_ns(c, ns - i);
    }
  }
  return k;
}

__device__ __forceinline__ void wm_prologue(Op& o, int64_t wm) {
  // S/WindowManager.java:43-55
  if (o.s.lastWatermark == -1) o.s.lastWatermark = max((int64_t)0, jsub(wm, o.cfg->max_lateness));
}

__global__ __launch_bounds__(256) void wm_count_kernel(XWmArgs a) {
  __shared__ Op o_lds[4];
  const int lane = threadIdx.x & 63;
  const int64_t op = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (op >= a.n_ops) return;
  Op& o = o_lds[threadIdx.x >> 6];  // per-wave operator state in LDS (a private Op sat in scratch)
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
  __shared__ Op o_lds[4];
  const int lane = threadIdx.x & 63;
  const int64_t op = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (op >= a.n_ops) return;
  Op& o = o_lds[threadIdx.x >> 6];  // per-wave operator state in LDS (a private Op sat in scratch)
  o.bind(a.cfg, a.sl, a.ss, op, lane);
  o.s = a.st[op];
  const XCfg* cfg = a.cfg;
  if (a.single && lane == 0) {  // the count pass's accounting (single mode has none)
    if (a.zero4) {  // the control words (flags, dropped, op error, row count) start at 0: the one wave of op 0 writes them
      a.zero4[0] = 0;
      a.zero4[1] = 0;
      a.zero4[2] = 0;
      a.zero4[3] = 0;
    }
    if (o.s.dropped) atomicAdd(a.dropped_total, (unsigned long long)o.s.dropped);
    if (o.s.err) atomicOr(a.op_err, 1 << o.s.err);
  }
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
  if (a.single) {  // the count pass's checks, before any state changes: an exception leaves the operator as it was
    const int64_t kd = wm_triggers<true>(o, a.wm, nullptr, nullptr, nullptr, nullptr, 0, 0);
    if (o.exc || kd > a.n_rows) {
      if (lane == 0) atomicOr(a.err_flag, o.exc ? 1 : 4);
      return;
    }
  }
  const int64_t off = a.single ? 0 : a.woff[op];
  const int64_t k = wm_triggers<false>(o, a.wm, a.w_start, a.w_end, a.w_meas, a.w_op, off, (int32_t)op);
  if (a.single && lane == 0) *a.row_count = (unsigned long long)k;
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
    // min(si, findSliceIndexByCount(minCount)) and max(ei, findSliceIndexByCount(maxCount)) look only where the last
    // slice with cStart <= x can change the bound: a hit at or after si leaves si (searched first, from the tail), a
    // hit at or before ei leaves ei (only (ei, tail) is searched) -- not the whole list from the tail
    int si = max(rel(o.find_ts(minTs)), 0);
    {
      const int h = o.s.head + si;
      if (wave_last(h, o.s.tail, [&](int i) { return o.cs[i] <= minCount; }) < 0)
        si = min(si, rel(wave_last(o.s.head, h, [&](int i) { return o.cs[i] <= minCount; })));
    }
    int ei = min(S - 1, rel(o.find_ts(maxTs)));
    {
      const int j = wave_last(o.s.head + ei + 1, o.s.tail, [&](int i) { return o.cs[i] <= maxCount; });
      if (j >= 0) ei = max(ei, rel(j));
    }
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
    for (int i = 0; i < o.s.ns(c); i++) first = min(first, o.ss[c][i]);
  const int64_t t = min(jsub(cw, cfg->max_fixed), first);
  const int idx = o.find_ts(t);
  if (idx > o.s.head) o.s.head = idx;
  if (lane == 0) a.st[op] = o.s;
}

// G lanes per emitted window (G = 64: one wavefront; G = 16: four windows per wavefront, for the many short
// scan ranges of keyed operators): AggregateWindowState.containsSlice/addState over the op's scan range
template <int G, typename T, typename F>
__device__ __forceinline__ T greduce(T v, F f) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v = f(v, (T)__shfl_xor(v, o));
  return v;
}
// first m in [lo, hi) with pred(m) (pred monotone false -> true), hi if none: G-ary search by a group of G lanes
// (lane = index in the group; every lane of the group runs it with the same arguments)
template <int G, typename P>
__device__ __forceinline__ int64_t group_first(int64_t lo, int64_t hi, int lane, P pred) {
  const int gsh = (int)(__lane_id() & (64 - G));  // the group's first bit in the wave's ballot
  auto gbal = [&](bool b) -> unsigned long long {
    const unsigned long long m = __ballot(b);
    return G == 64 ? m : (m >> gsh) & ((1ull << G) - 1);
  };
  while (hi - lo > G) {
    const int64_t stride = (hi - lo + G - 1) / G;
    const int64_t p = lo + (int64_t)lane * stride;
    const unsigned long long bal = gbal(p < hi && pred(p));
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
  const int64_t p = lo + lane;
  const unsigned long long bal = gbal(p < hi && pred(p));
  return bal ? lo + __ffsll((long long)bal) - 1 : hi;
}

template <int G>
__device__ __forceinline__ void agg_row(const XWmArgs& a, int64_t wi, int lane);

// Block summaries of the single operator's scan range (a wavefront per 64-slice block): what a window containing the
// whole block adds (AggregateWindowState.addState over its slices, S/state/AggregateWindowState.java:33-39), and
// the block's smallest tStart / largest tLast, so containment (:25-31) of the whole block is one test.
__global__ __launch_bounds__(256) void wm_blocks_kernel(XWmArgs a) {
  const int lane = threadIdx.x & 63;
  const XState& st = a.st[0];
  if (st.err || (st.unsorted & 3) || a.cfg->records) return;
  const int64_t wlo = max((int64_t)st.wlo, (int64_t)0), whi = st.whi;
  if (whi <= wlo) return;
  const int need = a.cfg->need;
  const bool f64 = a.cfg->vt == VT_F64;
  const int64_t b_first = wlo / XB_BLK, b_last = (whi - 1) / XB_BLK;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t b = b_first + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b <= b_last; b += nw) {
    if (b - b_first >= a.blk.nbcap) break;
    const int64_t s = b * XB_BLK + lane;
    const bool in = s >= wlo && s < whi;
    uint64_t c = 0, sw = 0;
    double sf = 0.0;
    int64_t mn = ID_MIN, mx = ID_MAX, t0 = JMAX, t1 = JMIN;
    if (in) {
      c = a.sl.cnt[s];
      t0 = a.sl.ts[s];
      t1 = a.sl.tl[s];
      if (need & NEED_SUM) {
        if (f64) sf = __longlong_as_double((long long)a.sl.p[0][s]);
        else sw = a.sl.p[0][s];
      }
      if (need & NEED_MIN) mn = (int64_t)a.sl.p[1][s];
      if (need & NEED_MAX) mx = (int64_t)a.sl.p[2][s];
    }
    c = greduce<64>((unsigned long long)c, [](unsigned long long x, unsigned long long y) { return x + y; });
    if (need & NEED_SUM) {
      if (f64) sf = greduce<64>(sf, [](double x, double y) { return x + y; });
      else sw = greduce<64>((unsigned long long)sw, [](unsigned long long x, unsigned long long y) { return x + y; });
    }
    mn = greduce<64>((long long)mn, [](long long x, long long y) { return x < y ? x : y; });
    mx = greduce<64>((long long)mx, [](long long x, long long y) { return x > y ? x : y; });
    t0 = greduce<64>((long long)t0, [](long long x, long long y) { return x < y ? x : y; });
    t1 = greduce<64>((long long)t1, [](long long x, long long y) { return x > y ? x : y; });
    const bool whole = b * XB_BLK >= wlo && (b + 1) * XB_BLK <= whi;
    if (lane == 0) {
      const int64_t i = b - b_first;  // indexed from the scan range's first block
      a.blk.cnt[i] = c;
      a.blk.sum[i] = f64 ? (unsigned long long)__double_as_longlong(sf) : sw;
      a.blk.mn[i] = mn;
      a.blk.mx[i] = mx;
      a.blk.ts_min[i] = whole ? t0 : JMIN;
      a.blk.tl_max[i] = t1;
    }
  }
}

// rows: n_rows, or (single mode) the count the emit kernel wrote; groups stride over them
template <int G>
__global__ __launch_bounds__(256) void wm_agg_kernel(XWmArgs a) {
  const int lane = threadIdx.x & (G - 1);
  const int64_t nrows = a.single ? (int64_t)*a.row_count : a.n_rows;
  const int64_t stride = (int64_t)gridDim.x * (256 / G);
  for (int64_t wi = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G; wi < nrows; wi += stride) agg_row<G>(a, wi, lane);
}

template <int G>
__device__ __forceinline__ void agg_row(const XWmArgs& a, int64_t wi, int lane) {
  const int64_t op = a.w_op[wi];
  const XState& st = a.st[op];
  const int64_t base = op * (int64_t)a.cfg->sc;
  const int64_t ws = a.w_start[wi], we = a.w_end[wi];
  const bool tmeas = a.w_meas[wi] == 0;
  int64_t lo = st.wlo, hi = st.whi;
  if (lo < 0) lo = 0;
  const int64_t* key = tmeas ? a.sl.ts + base : a.sl.cs + base;
  // narrow to start keys in [ws, we] (contained slices satisfy it) by a G-ary search of the group (one probe per
  // lane per round; a bisection is a chain of dependent loads); a range of a few group widths is scanned as is
  if ((!(st.unsorted & 3) || !tmeas) && hi - lo > 4 * G) {
    const int64_t nlo = group_first<G>(lo, hi, lane, [&](int64_t m) { return key[m] >= ws; });
    // contained slices start no later than the window's end -- except with LazySlice record moves, which can
    // leave a slice's tLast (cLast) below its tStart (cStart): then only the lower bound narrows
    if (!a.cfg->records) hi = group_first<G>(nlo, hi, lane, [&](int64_t m) { return key[m] > we; });
    lo = nlo;
  }
  const int need = a.cfg->need, vt = a.cfg->vt;
  const bool recs = a.cfg->records != 0;
  uint64_t cnt = 0, sw = 0, present = 0;
  double sf = 0.0;
  int64_t mn = ID_MIN, mx = ID_MAX;
  // one slice: AggregateWindowState.containsSlice + addState (S/state/AggregateWindowState.java:25-39)
  auto add_slice = [&](int64_t i) {
    const int64_t s = base + i;
    const int64_t k0 = tmeas ? a.sl.ts[s] : a.sl.cs[s];
    const int64_t k1 = tmeas ? a.sl.tl[s] : a.sl.cl[s];
    const uint64_t c = a.sl.cnt[s];
    const bool contains = tmeas ? (ws <= k0 && we > k1) : (ws <= k0 && we >= k1);
    if (!(contains && (recs ? a.sl.nn[s] != 0 : c != 0))) return;
    present = 1;
    cnt += c;
    if (need & NEED_SUM) {
      if (vt == VT_F64) sf += __longlong_as_double((long long)a.sl.p[0][s]);
      else sw += a.sl.p[0][s];
    }
    if (need & NEED_MIN) mn = min(mn, (int64_t)a.sl.p[1][s]);
    if (need & NEED_MAX) mx = max(mx, (int64_t)a.sl.p[2][s]);
  };
  // One operator with block summaries (wm_blocks_kernel, time windows on a sorted list): a lane per 64-slice block;
  // a block the window contains whole adds its summary, the others (at most the two at the run's ends, usually) are
  // scanned slice by slice by the wavefront -- the window costs its blocks, not its slices (north_star: window
  // assembly from slice summaries; LazyAggregateStore.aggregate, S/aggregationstore/LazyAggregateStore.java:83-111)
  const bool blocks = G == 64 && a.blk.cnt != nullptr && tmeas && !recs && !(st.unsorted & 3) && hi > lo &&
                      lo >= st.wlo && hi <= st.whi;
  if (blocks) {
    const int64_t bf = st.wlo / XB_BLK;
    for (int64_t b0 = lo / XB_BLK; b0 <= (hi - 1) / XB_BLK; b0 += G) {
      const int64_t b = b0 + lane;
      bool whole = false;
      if (b <= (hi - 1) / XB_BLK && b - bf < a.blk.nbcap) {
        const int64_t i = b - bf;
        whole = a.blk.ts_min[i] >= ws && a.blk.tl_max[i] < we;  // every slice of the block contained
        if (whole && a.blk.cnt[i] != 0) {
          present = 1;
          cnt += a.blk.cnt[i];
          if (need & NEED_SUM) {
            if (vt == VT_F64) sf += __longlong_as_double((long long)a.blk.sum[i]);
            else sw += a.blk.sum[i];
          }
          if (need & NEED_MIN) mn = min(mn, (int64_t)a.blk.mn[i]);
          if (need & NEED_MAX) mx = max(mx, (int64_t)a.blk.mx[i]);
        }
      }
      unsigned long long part = __ballot(b <= (hi - 1) / XB_BLK && !whole);
      while (part) {  // blocks in part: the wavefront tests each slice
        const int j = __ffsll((long long)part) - 1;
        part &= part - 1;
        const int64_t i = (b0 + j) * XB_BLK + lane;
        if (i >= lo && i < hi) add_slice(i);
      }
    }
  }
  // two slices per lane per round, every load issued before the containment tests (no early continue)
  for (int64_t i0 = lo + lane; !blocks && i0 < hi; i0 += 2 * G) {
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int64_t i = i0 + u * G;
      const bool in = i < hi;
      const int64_t s = base + (in ? i : lo);
      const int64_t k0 = tmeas ? a.sl.ts[s] : a.sl.cs[s];
      const int64_t k1 = tmeas ? a.sl.tl[s] : a.sl.cl[s];
      const uint64_t c = a.sl.cnt[s];
      const bool nonnull = recs ? a.sl.nn[s] != 0 : c != 0;
      const uint64_t p0 = (need & NEED_SUM) ? a.sl.p[0][s] : 0;
      const int64_t p1 = (need & NEED_MIN) ? (int64_t)a.sl.p[1][s] : ID_MIN;
      const int64_t p2 = (need & NEED_MAX) ? (int64_t)a.sl.p[2][s] : ID_MAX;
      const bool contains = tmeas ? (ws <= k0 && we > k1) : (ws <= k0 && we >= k1);
      // a partial is present when non-null: count > 0, or (records mode) kept after liftAndInvert
      if (!(in && contains && nonnull)) continue;
      present = 1;
      cnt += c;
      if (need & NEED_SUM) {
        if (vt == VT_F64) sf += __longlong_as_double((long long)p0);
        else sw += p0;
      }
      if (need & NEED_MIN) mn = min(mn, p1);
      if (need & NEED_MAX) mx = max(mx, p2);
    }
  }
  auto add_u = [](unsigned long long x, unsigned long long y) { return x + y; };
  auto min_i = [](long long x, long long y) { return x < y ? x : y; };
  auto max_i = [](long long x, long long y) { return x > y ? x : y; };
  cnt = greduce<G>((unsigned long long)cnt, add_u);
  present = greduce<G>((unsigned long long)present, add_u);
  if (need & NEED_SUM) {
    if (vt == VT_F64) sf = greduce<G>(sf, [](double x, double y) { return x + y; });
    else sw = greduce<G>((unsigned long long)sw, add_u);
  }
  if (need & NEED_MIN) mn = greduce<G>((long long)mn, min_i);
  if (need & NEED_MAX) mx = greduce<G>((long long)mx, max_i);
  if (lane == 0) {
    a.has_value[wi] = present ? 1 : 0;
    if (a.w_key) a.w_key[wi] = a.slot_key ? a.slot_key[op] : (uint32_t)op;
    const uint64_t sword = vt == VT_F64 ? (uint64_t)__double_as_longlong(sf) : sw;
    for (int k = 0; k < a.cfg->n_aggs; k++)
      a.values[k][wi] = present ? lower_value(a.cfg->agg_kind[k], cnt, sword, mn, mx) : 0;
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
  note_kernel(KN_REPLAY, "replay_kernel<%d>", vt);
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
hipError_t launch_wm_blocks(const XWmArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(x::wm_blocks_kernel, dim3(64), dim3(256), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_wm_agg(const XWmArgs& a, hipStream_t st, int group) {
  if (a.n_rows <= 0) return hipSuccess;
  // single mode: n_rows is the capacity (the device holds the count): at most 256 workgroups stride over the rows
  const int64_t cap = a.single ? 256 : INT32_MAX;
  if (group == 16)
    hipLaunchKernelGGL(x::wm_agg_kernel<16>, dim3((unsigned)std::min<int64_t>((a.n_rows + 15) / 16, cap)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(x::wm_agg_kernel<64>, dim3((unsigned)std::min<int64_t>((a.n_rows + 3) / 4, cap)), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace scotty
