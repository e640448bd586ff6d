// exact_batch.hip -- batch-parallel exact path of a NON-keyed operator with session / count windows.
//
// The reference processes tuple after tuple (S/SlicingWindowOperator.java:41-44).  A micro-batch of one
// operator is split into "simple" tuples, whose effect on the operator commutes, and "events", in three
// steps over the whole chip:
//
//  classification (tiles of 4096 arrival-ordered tuples, all CUs) -- from the exclusive prefix max P of
//  the batch (StreamSlicer.maxEventTime before each tuple) and the operator state at batch start:
//   * in-order tuples (t >= P) are events iff they may cross the pending fixed edge (the pending edge after
//     any processed in-order tuple te is nextGrid(te) = min_w assignNextWindowStart_w(te),
//     S/StreamSlicer.java:55-84, :103-116), may open a flexible edge or a new session (the last session of
//     every SessionContext always ends at maxEventTime: only in-order tuples extend it or start a newer
//     one, C/windowType/SessionWindow.java:42-87), or hit a count edge (:37-44, :88-101);
//   * out-of-order tuples are events unless they fall inside a session of every context (then
//     updateContext is a no-op and checkSliceEdges gets no modification).  Sessions only grow or merge
//     inside a micro-batch, so "inside" stays true whatever earlier events do.  The in-batch sessions form
//     a chain of jumps of the running max by more than the gap; it is compacted per context.
//  event pass (one wavefront, exact reference logic, exact_op.h) -- walks the compacted events in order.
//   Before each event it re-applies the effect of the simple tuples since the previous event, all of which
//   is a max (M = max ts in between): maxEventTime, the current slice's tLast and the last session's end.
//   An out-of-order event of an operator with sessions may split / shift / merge older slices, so it ends a
//   "segment": the simple tuples before it are applied first.
//  apply (all CUs) -- simple tuples of a segment are lifted and combined into their slice: the last slice
//   present at their arrival when t >= its tStart (slices appended later start above the running max), else
//   the last slice with tStart <= t (LazyAggregateStore.findSliceIndexByTimestamp, :29-37).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "exact_batch.h"
#include "exact_op.h"

namespace scotty {

constexpr int XB_THREADS = 256;
constexpr int XB_ITEMS = 16;
constexpr int XB_TILE = XB_THREADS * XB_ITEMS;  // 4096 tuples per tile

// batch-start snapshot of the operator, built by xb_prep_kernel (1 wave)
struct XSnap {
  int64_t p_start;         // maxEventTime (JMIN if no tuple yet)
  int64_t n0;              // nextEdgeTs
  int64_t nc0;             // nextEdgeCount
  int64_t c0;              // currentCount
  int64_t oldest;          // tStart of the oldest retained slice
  int32_t started, unsorted, head, tail;
  int64_t min_gap;
  int32_t inv[XMAXCTX];    // last session ends at maxEventTime
  int32_t ns[XMAXCTX];     // sessions per context
  int64_t last_start[XMAXCTX], stored_end[XMAXCTX], lim[XMAXCTX];
};

// control block of the event pass / apply segments
struct XBCtl {
  int64_t ev_total;        // events of the batch
  int64_t ev_next;         // next event to process
  int64_t seg_start;       // first tuple of the current segment
  int64_t seg_end;         // end of the segment to apply
  int64_t ep_count;        // epoch entries of the current segment
  int32_t stopped, done;
  int32_t resume;          // the next event is the stop event of the previous segment
  int32_t pad;
  int64_t m_tail;          // max ts after the batch's last event (JMIN if none)
  int32_t retry;           // the round outgrew the event / new-session buffers: nothing was applied, the host
                           // grows them (ev_total, ns_tot) and runs the round again
  int32_t pad2;
};


namespace xb {
using namespace x;

__device__ __forceinline__ int64_t load_v(const XBArgs& a, int64_t i) {
  if (a.vt == VT_I32) return (int64_t)((const int32_t*)a.val)[i];
  return ((const int64_t*)a.val)[i];
}

// block-wide exclusive max over 256 threads (4 waves); wtot: LDS [4]
__device__ __forceinline__ int64_t block_excl_max(int64_t v, long long* wtot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = (int64_t)__shfl_up((long long)inc, o);
    if (lane >= o) inc = max(inc, u);
  }
  if (lane == 63) wtot[wid] = inc;
  __syncthreads();
  int64_t before = JMIN;
  for (int w = 0; w < wid; w++) before = max(before, (int64_t)wtot[w]);
  int64_t ex = (int64_t)__shfl_up((long long)inc, 1);
  if (lane == 0) ex = JMIN;
  __syncthreads();
  return max(before, ex);
}
__device__ __forceinline__ int64_t block_excl_sum(int64_t v, long long* wtot, int64_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = (int64_t)__shfl_up((long long)inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wtot[wid] = inc;
  __syncthreads();
  int64_t before = 0, tot = 0;
  for (int w = 0; w < 4; w++) {
    if (w < wid) before += wtot[w];
    tot += wtot[w];
  }
  __syncthreads();
  if (total) *total = tot;
  return before + inc - v;
}

// min over time-measure context-free windows of assignNextWindowStart(x) (lanes split the windows)
__device__ __forceinline__ int64_t next_grid(const XCfg* c, int64_t xv) {
  const int lane = threadIdx.x & 63;
  int64_t e = JMAX;
  for (int w = lane; w < c->n_cf; w += 64) {
    if (c->cf_measure[w] != 0) continue;
    const int k = c->cf_kind[w];
    const int64_t a = c->cf_a[w], b = c->cf_b[w];
    int64_t r;
    if (k == 0) r = jsub(jadd(xv, a), jmod(xv, a));
    else if (k == 1) r = jsub(jadd(xv, b), jmod(xv, b));
    else if (xv == JMAX || xv < a) r = a;
    else if (xv < jadd(a, b)) r = jadd(a, b);
    else r = JMAX;
    e = min(e, r);
  }
  return wmin(e);
}
__device__ __forceinline__ bool on_count_grid(const XCfg* c, int64_t cnt) {
  for (int w = 0; w < c->n_cf; w++) {
    if (c->cf_measure[w] != 1) continue;
    const int k = c->cf_kind[w];
    const int64_t a = c->cf_a[w], b = c->cf_b[w];
    if (k == 0 && jmod(cnt, a) == 0) return true;
    if (k == 1 && jmod(cnt, b) == 0) return true;
    if (k == 2 && (cnt == a || cnt == jadd(a, b))) return true;
  }
  return false;
}

// Per-thread view of one tile: 16 contiguous tuples staged in LDS (row of this thread) and the exclusive prefix
// max P before the first of them.  P and nextGrid(P) of later items are produced in order by TileWalk, so no
// per-item arrays live in registers or scratch.
struct TileItems {
  const long long* row;  // tb + thread row: the thread's items in arrival order
  int64_t pre;           // exclusive prefix max before item 0 (incl. carry and p_start)
  int64_t base;          // index of item 0
  int cnt;               // valid items
};

// per-lane nextGrid (serial over the windows): only recomputed when the running max reaches the cached edge
__device__ __forceinline__ int64_t next_grid_lane(const XCfg* c, int64_t xv) {
  int64_t e = JMAX;
  for (int w = 0; w < c->n_cf; w++) {
    if (c->cf_measure[w] != 0) continue;
    const int k = c->cf_kind[w];
    const int64_t a = c->cf_a[w], b = c->cf_b[w];
    int64_t r;
    if (k == 0) r = jsub(jadd(xv, a), jmod(xv, a));
    else if (k == 1) r = jsub(jadd(xv, b), jmod(xv, b));
    else if (xv == JMAX || xv < a) r = a;
    else if (xv < jadd(a, b)) r = jadd(a, b);
    else r = JMAX;
    e = min(e, r);
  }
  return e;
}

constexpr int XB_LDS = XB_TILE / XB_ITEMS * (XB_ITEMS + 1);  // padded: thread rows of 17 words

// coalesced striped loads into LDS, read back as 16 contiguous items per thread (row pad avoids bank conflicts)
__device__ __forceinline__ void stage_tile(const int64_t* src, int64_t n, int64_t tile, long long* tb) {
  const int64_t base = tile * XB_TILE;
#pragma unroll
  for (int r = 0; r < XB_ITEMS; r++) {
    const int e = r * XB_THREADS + threadIdx.x;
    const int64_t i = base + e;
    tb[(e >> 4) * (XB_ITEMS + 1) + (e & 15)] = i < n ? src[i] : JMIN;
  }
  __syncthreads();
}

__device__ __forceinline__ void load_tile(const XBArgs& a, int64_t tile, TileItems& it, long long* wtot,
                                          long long* tb) {
  const XSnap& sn = *a.snap;
  it.base = tile * XB_TILE + (int64_t)threadIdx.x * XB_ITEMS;
  it.cnt = (int)max((int64_t)0, min((int64_t)XB_ITEMS, a.n - it.base));
  stage_tile(a.ts, a.n, tile, tb);
  it.row = tb + threadIdx.x * (XB_ITEMS + 1);
  int64_t run = JMIN;
#pragma unroll
  for (int j = 0; j < XB_ITEMS; j++) run = max(run, (int64_t)it.row[j]);  // padding items are JMIN
  const int64_t before = block_excl_max(run, wtot);
  const int64_t carry = max((int64_t)a.pcarry[tile], sn.p_start);
  it.pre = max(carry, before);
}

// walks a thread's items in order: t, its exclusive prefix max p, and the pending fixed edge g = nextGrid(p)
// (nextGrid(x) is constant on [x, nextGrid(x)) and p is non-decreasing, so it is recomputed only on crossing)
struct TileWalk {
  int64_t p, gcur;
  bool grid;
  __device__ TileWalk(const XBArgs& a, const TileItems& it, bool want_grid)
      : p(it.pre), gcur(JMIN), grid(want_grid && a.cfg->has_fixed && a.cfg->has_time) {}
  __device__ __forceinline__ int64_t g(const XCfg* c) {
    if (!grid) return JMAX;
    if (p < 0) return JMIN;  // assignNextWindowStart bounds the pending edge only for non-negative times (Java %)
    if (gcur == JMIN || p >= gcur) gcur = next_grid_lane(c, p);
    return gcur;
  }
  __device__ __forceinline__ void next(int64_t t) { p = max(p, t); }
};

// The batch snapshot and configuration fields the per-tuple classification reads, loaded once per thread
// (uniform: scalar registers) instead of from global memory at every tuple.
struct XBH {
  int64_t n0, nc0, c0, oldest, min_gap, p_start;
  int32_t started, n_ctx, has_time, has_fixed, has_count, lazy;
  int64_t gap[XMAXCTX], lim[XMAXCTX], last_start[XMAXCTX], stored_end[XMAXCTX];
  int32_t ns[XMAXCTX], inv[XMAXCTX];
};
__device__ __forceinline__ XBH hoist(const XBArgs& a) {
  const XSnap& sn = *a.snap;
  const XCfg* c = a.cfg;
  XBH h;
  h.n0 = sn.n0;
  h.nc0 = sn.nc0;
  h.c0 = sn.c0;
  h.oldest = sn.oldest;
  h.min_gap = sn.min_gap;
  h.p_start = sn.p_start;
  h.started = sn.started;
  h.n_ctx = c->n_ctx;
  h.has_time = c->has_time;
  h.has_fixed = c->has_fixed;
  h.has_count = c->has_count;
  h.lazy = c->lazy;
#pragma unroll
  for (int k = 0; k < XMAXCTX; k++) {
    const bool on = k < h.n_ctx;
    h.gap[k] = on ? c->gap[k] : 0;
    h.lim[k] = on ? sn.lim[k] : JMIN;
    h.last_start[k] = on ? sn.last_start[k] : JMAX;
    h.stored_end[k] = on ? sn.stored_end[k] : JMIN;
    h.ns[k] = on ? sn.ns[k] : 0;
    h.inv[k] = on ? sn.inv[k] : 0;
  }
  return h;
}

// in-order tuple t (t >= p): contexts in which it starts a new session (the chain of in-batch sessions), and
// the end of the session before it
__device__ __forceinline__ int newsess_bits(const XBH& h, int64_t t, int64_t p, int64_t* pb) {
  int nsmask = 0;
#pragma unroll
  for (int k = 0; k < XMAXCTX; k++) {
    if (k >= h.n_ctx) break;
    const int64_t gap = h.gap[k];
    bool nw;
    int64_t before;
    if (!h.inv[k] && p == h.p_start) {
      nw = h.ns[k] == 0 || t > jadd(h.stored_end[k], gap);
      before = h.ns[k] == 0 ? JMIN : h.stored_end[k];
    } else {
      nw = t > jadd(p, gap);
      before = p;
    }
    if (nw) {
      nsmask |= 1 << k;
      pb[k] = before;
    }
  }
  return nsmask;
}
__device__ __forceinline__ int newsess_bits(const XBArgs& a, int64_t t, int64_t p, int64_t* pb) {
  const XBH h = hoist(a);
  return newsess_bits(h, t, p, pb);
}

// in-order classification (depends on P only).  Returns event; sets new-session bits per context (want_ns).
__device__ __forceinline__ bool inorder_event(const XBH& h, const XCfg* c, int64_t t, int64_t p, int64_t g,
                                              int64_t pos, int& nsmask, int64_t* pb, bool want_ns = true) {
  bool ev = false;
  nsmask = 0;
  if (h.has_time) {
    if (h.has_fixed) {
      if ((h.n0 == JMIN && p == h.p_start) || (p < h.n0 && t >= h.n0) || (p >= h.n0 && t >= g)) ev = true;
    }
    if (h.n_ctx > 0) {
      if (t >= jadd(p, h.min_gap)) ev = true;
      // calculateNextFlexEdge (S/StreamSlicer.java:118-130): te >= max(maxEventTime, pending edge) + gap, in
      // Java long arithmetic -- with no time window the pending edge is Long.MAX_VALUE and the sum wraps, so
      // every in-order tuple opens a flexible slice.  Pending edge here: n0 until crossed, then nextGrid(P).
      const int64_t pend = !h.has_fixed ? JMIN : (p < h.n0 ? h.n0 : g);
      const int64_t tc = max(p, pend);
#pragma unroll
      for (int k = 0; k < XMAXCTX; k++)
        if (k < h.n_ctx && t >= jadd(tc, h.gap[k])) ev = true;
    }
  }
#pragma unroll
  for (int k = 0; k < XMAXCTX; k++) {
    if (k >= h.n_ctx) break;
    if (!h.inv[k] && p == h.p_start) ev = true;
    if (t <= h.lim[k]) ev = true;
  }
  if (want_ns) nsmask = newsess_bits(h, t, p, pb);
  if (h.has_count) {
    const int64_t cnt = jadd(h.c0, pos);
    if (h.nc0 == JMIN || cnt == h.nc0 || (cnt > h.nc0 && on_count_grid(c, cnt))) ev = true;
  }
  if (!h.started && pos == 0) ev = true;
  return ev;
}

// ------------------------------------------------------------------------------------------- kernels
__global__ void xb_prep_kernel(XBArgs a) {
  const int lane = threadIdx.x;
  const XCfg* c = a.cfg;
  XState s = *a.st;
  XSnap sn{};
  sn.p_start = s.maxEventTime;
  sn.n0 = s.nextEdgeTs;
  sn.nc0 = s.nextEdgeCount;
  sn.c0 = s.currentCount;
  sn.started = s.tail > s.head;
  sn.unsorted = s.unsorted;
  sn.head = s.head;
  sn.tail = s.tail;
  sn.oldest = JMAX;  // findSliceIndexByTimestamp(t) == -1 <=> t < min tStart (the list may be unsorted)
  for (int i = s.head + lane; i < s.tail; i += 64) sn.oldest = min(sn.oldest, a.sl.ts[i]);
  sn.oldest = wmin(sn.oldest);
  sn.min_gap = JMAX;
  for (int k = 0; k < c->n_ctx; k++) {
    sn.min_gap = min(sn.min_gap, c->gap[k]);
    const int64_t* st_ = a.ss.start + (int64_t)k * c->sesscap;
    const int64_t* en_ = a.ss.end + (int64_t)k * c->sesscap;
    const int ns = s.ns(k);
    sn.ns[k] = ns;
    sn.last_start[k] = ns > 0 ? st_[ns - 1] : JMAX;
    sn.stored_end[k] = ns > 0 ? en_[ns - 1] : JMIN;
    sn.inv[k] = ns > 0 && en_[ns - 1] == s.maxEventTime;
    int64_t lim = JMIN;
    // reach prefix (sequential; sessions per context are few) -- lane 0 writes
    for (int i = 0; i < ns; i++) {
      lim = max(lim, jadd(en_[i], c->gap[k]));
      if (lane == 0) a.reach[(int64_t)k * c->sesscap + i] = lim;
    }
    int64_t lim2 = JMIN;
    for (int i = 0; i < ns - 1; i++) lim2 = max(lim2, jadd(en_[i], c->gap[k]));
    sn.lim[k] = lim2;
  }
  if (lane == 0) *a.snap = sn;
}

// tile maxima; with session windows also the tile's jump flag (tjump).  A tuple after the tile's first one opens a
// session only if it exceeds the running max before it (>= the first ts) by more than a gap, so
// tmax <= first + min_gap rules it out (conservative near the int64 range, where jadd wraps).
__global__ __launch_bounds__(XB_THREADS) void xb_tilemax_kernel(XBArgs a) {
  __shared__ long long wtot[4];
  const int64_t base = (int64_t)blockIdx.x * XB_TILE;
  __shared__ long long wmn[4];
  int64_t m = JMIN, mn = JMAX;
  // unconditional loads (indices past the batch clamp to its last tuple, which lies in this tile when any index
  // does, so the extrema are unchanged): all XB_ITEMS loads are in flight before the first use
  int64_t v[XB_ITEMS];
#pragma unroll
  for (int r = 0; r < XB_ITEMS; r++) v[r] = __builtin_nontemporal_load(a.ts + min(base + r * XB_THREADS + threadIdx.x, a.n - 1));
#pragma unroll
  for (int r = 0; r < XB_ITEMS; r++) {
    m = max(m, v[r]);
    mn = min(mn, v[r]);
  }
  m = wmax(m);
  if (a.cfg_nctx_host > 0) mn = wmin(mn);
  if ((threadIdx.x & 63) == 0) {
    wtot[threadIdx.x >> 6] = m;
    wmn[threadIdx.x >> 6] = mn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t tm = max(max(wtot[0], wtot[1]), max(wtot[2], wtot[3]));
    a.tmax[blockIdx.x] = tm;
    if (a.cfg_nctx_host > 0) {
      a.tmin[blockIdx.x] = min(min(wmn[0], wmn[1]), min(wmn[2], wmn[3]));
      const int64_t gap = a.snap->min_gap, t0 = a.ts[base];
      const bool safe = gap >= 0 && t0 <= JMAX - gap && tm <= JMAX - gap;
      a.tjump[blockIdx.x] = (safe && tm <= t0 + gap) ? 0 : 1;
    }
  }
}

// Single-workgroup exclusive scans over the per-tile values: V is a pair (h, t) combined by op(prev, cur); identity
// id.  Rounds of 8192 values: coalesced loads into LDS, 8 consecutive values per thread scanned in registers, the
// results back through LDS and stored coalesced (strided per-thread global accesses left each wave instruction
// touching 64 cache lines).
struct SPair {
  int64_t h, t;
};
constexpr int SCAN_IT = 8;
constexpr int SCAN_CH = 1024 * SCAN_IT;
template <class Op>
__device__ __forceinline__ SPair wg_scan16(int64_t n, SPair id, SPair carry, Op op, SPair (*ld)(const XBArgs&, int64_t, int),
                                           void (*st)(const XBArgs&, int64_t, int, SPair), const XBArgs& a, int row) {
  __shared__ long long wh[16], wt[16];
  __shared__ long long st_t[SCAN_CH];
  __shared__ int st_h[SCAN_CH];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (n <= 0) return carry;
  for (int64_t c0 = 0; c0 < n; c0 += SCAN_CH) {
    {
      SPair v[SCAN_IT];
#pragma unroll
      for (int j = 0; j < SCAN_IT; j++) v[j] = ld(a, min(c0 + j * 1024 + tid, n - 1), row);
#pragma unroll
      for (int j = 0; j < SCAN_IT; j++) {
        const bool in = c0 + j * 1024 + tid < n;
        st_t[j * 1024 + tid] = in ? v[j].t : id.t;
        st_h[j * 1024 + tid] = (int)(in ? v[j].h : id.h);
      }
    }
    __syncthreads();
    SPair loc[SCAN_IT];
    SPair acc = id;
#pragma unroll
    for (int j = 0; j < SCAN_IT; j++) {
      const SPair v{(int64_t)st_h[tid * SCAN_IT + j], (int64_t)st_t[tid * SCAN_IT + j]};
      loc[j] = acc;
      acc = op(acc, v);
    }
    SPair inc = acc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      SPair u;
      u.h = (int64_t)__shfl_up((long long)inc.h, o);
      u.t = (int64_t)__shfl_up((long long)inc.t, o);
      if (lane >= o) inc = op(u, inc);
    }
    if (lane == 63) {
      wh[wid] = inc.h;
      wt[wid] = inc.t;
    }
    __syncthreads();
    SPair before = carry;
    for (int w = 0; w < wid; w++) before = op(before, SPair{wh[w], wt[w]});
    SPair ex;
    ex.h = (int64_t)__shfl_up((long long)inc.h, 1);
    ex.t = (int64_t)__shfl_up((long long)inc.t, 1);
    if (lane == 0) ex = id;
    const SPair pre = op(before, ex);
#pragma unroll
    for (int j = 0; j < SCAN_IT; j++) {
      const SPair r = op(pre, loc[j]);
      st_t[tid * SCAN_IT + j] = r.t;
      st_h[tid * SCAN_IT + j] = (int)r.h;
    }
    SPair tot = carry;
    for (int w = 0; w < 16; w++) tot = op(tot, SPair{wh[w], wt[w]});
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SCAN_IT; j++) {
      const int64_t k = c0 + j * 1024 + tid;
      if (k < n) st(a, k, row, SPair{(int64_t)st_h[j * 1024 + tid], (int64_t)st_t[j * 1024 + tid]});
    }
    __syncthreads();
    carry = tot;
  }
  return carry;
}

struct OpMax {
  __device__ SPair operator()(SPair p, SPair q) const { return SPair{0, max(p.t, q.t)}; }
};
struct OpSum {
  __device__ SPair operator()(SPair p, SPair q) const { return SPair{0, p.t + q.t}; }
};
struct OpSeg {  // segmented max: a tile with an event resets the running max
  __device__ SPair operator()(SPair p, SPair q) const { return SPair{p.h | q.h, q.h ? q.t : max(p.t, q.t)}; }
};
__device__ SPair ld_tmax(const XBArgs& a, int64_t k, int) { return SPair{0, (int64_t)a.tmax[k]}; }
__device__ void st_pcarry(const XBArgs& a, int64_t k, int, SPair v) { a.pcarry[k] = v.t; }
__device__ SPair ld_seg(const XBArgs& a, int64_t k, int) { return SPair{a.seg_has[k], (int64_t)a.seg_tail[k]}; }
__device__ void st_mcarry(const XBArgs& a, int64_t k, int, SPair v) { a.m_carry[k] = v.t; }

// exclusive carries over tiles (prefix max of tile maxima)
__global__ __launch_bounds__(1024) void xb_carry_kernel(XBArgs a) {
  (void)wg_scan16(a.ntiles, SPair{0, JMIN}, SPair{0, JMIN}, OpMax{}, ld_tmax, st_pcarry, a, 0);
}

// exclusive scan of per-tile counts (rows of length ntiles), totals to tot[row]
__device__ SPair ld_row(const XBArgs& a, int64_t k, int row) { return SPair{0, a.ev_cnt[(int64_t)row * a.ntiles + k]}; }
__device__ void st_row(const XBArgs& a, int64_t k, int row, SPair v) { a.ev_cnt[(int64_t)row * a.ntiles + k] = v.t; }
__global__ __launch_bounds__(1024) void xb_rows_scan_kernel(XBArgs a, int64_t* cnt, int rows, int64_t* tot) {
  XBArgs b = a;
  b.ev_cnt = cnt;  // the rows to scan in place (ev_cnt or ns_cnt)
  for (int r = 0; r < rows; r++) {
    const SPair t = wg_scan16(b.ntiles, SPair{0, 0}, SPair{0, 0}, OpSum{}, ld_row, st_row, b, r);
    if (threadIdx.x == 0 && tot) tot[r] = t.t;
  }
}

// a tile without a jump, once the batch's running max has left p_start (no batch-start special case): only its
// first item can open a session; its new-session bits and the running max before it
__device__ __forceinline__ bool tile_simple(const XBArgs& a, int64_t tile, int& nsm0, int64_t* pb0) {
  const XSnap& sn = *a.snap;
  const int64_t carry = max((int64_t)a.pcarry[tile], sn.p_start);
  if (a.tjump[tile] || carry <= sn.p_start) return false;
  const int64_t t0 = a.ts[tile * XB_TILE];
  nsm0 = t0 >= carry ? newsess_bits(a, t0, carry, pb0) : 0;
  return true;
}

__global__ __launch_bounds__(XB_THREADS) void xb_nscount_kernel(XBArgs a) {
  __shared__ long long wtot[4];
  __shared__ long long tb[XB_LDS];
  {
    int nsm0;
    int64_t pb0[XMAXCTX];
    if (tile_simple(a, blockIdx.x, nsm0, pb0)) {
      if (threadIdx.x == 0)
        for (int k = 0; k < a.cfg->n_ctx; k++) a.ns_cnt[(int64_t)k * a.ntiles + blockIdx.x] = (nsm0 >> k) & 1;
      return;
    }
  }
  TileItems it;
  load_tile(a, blockIdx.x, it, wtot, tb);
  int64_t cnt[XMAXCTX] = {0, 0, 0, 0};
  TileWalk w(a, it, false);
  for (int j = 0; j < it.cnt; j++) {
    const int64_t t = it.row[j];
    if (t >= w.p) {
      int64_t pb[XMAXCTX];
      const int nsm = newsess_bits(a, t, w.p, pb);
#pragma unroll
      for (int k = 0; k < XMAXCTX; k++)
        if (nsm & (1 << k)) cnt[k]++;
    }
    w.next(t);
  }
  for (int k = 0; k < a.cfg->n_ctx; k++) {
    int64_t tot;
    (void)block_excl_sum(cnt[k], wtot, &tot);
    if (threadIdx.x == 0) a.ns_cnt[(int64_t)k * a.ntiles + blockIdx.x] = tot;
  }
}

// pass 2: write the per-context chains of in-batch new sessions (start, end of the previous session)
__global__ __launch_bounds__(XB_THREADS) void xb_nswrite_kernel(XBArgs a) {
  __shared__ long long wtot[4];
  __shared__ long long tb[XB_LDS];
  {
    int nsm0;
    int64_t pb0[XMAXCTX];
    if (tile_simple(a, blockIdx.x, nsm0, pb0)) {
      if (threadIdx.x == 0)
        for (int k = 0; k < a.cfg->n_ctx; k++) {
          if (!((nsm0 >> k) & 1)) continue;
          const int64_t off = a.ns_cnt[(int64_t)k * a.ntiles + blockIdx.x];
          if (off < a.ns_cap) {
            a.ns_start[(int64_t)k * a.ns_cap + off] = a.ts[(int64_t)blockIdx.x * XB_TILE];
            a.ns_pb[(int64_t)k * a.ns_cap + off] = pb0[k];
          }
        }
      return;
    }
  }
  TileItems it;
  load_tile(a, blockIdx.x, it, wtot, tb);
  int64_t cnt[XMAXCTX] = {0, 0, 0, 0};
  uint64_t nsm_all = 0;  // 4 bits per item
  {
    TileWalk w(a, it, false);
    for (int j = 0; j < it.cnt; j++) {
      const int64_t t = it.row[j];
      if (t >= w.p) {
        int64_t pb[XMAXCTX];
        const int nsm = newsess_bits(a, t, w.p, pb);
        nsm_all |= (uint64_t)nsm << (4 * j);
#pragma unroll
        for (int k = 0; k < XMAXCTX; k++)
          if (nsm & (1 << k)) cnt[k]++;
      }
      w.next(t);
    }
  }
  int64_t off[XMAXCTX] = {0, 0, 0, 0};
  for (int k = 0; k < a.cfg->n_ctx; k++)
    off[k] = block_excl_sum(cnt[k], wtot, nullptr) + a.ns_cnt[(int64_t)k * a.ntiles + blockIdx.x];
  if (nsm_all == 0) return;
  TileWalk w(a, it, false);
  for (int j = 0; j < it.cnt; j++) {
    const int64_t t = it.row[j];
    const int nsm = (int)((nsm_all >> (4 * j)) & 15u);
    if (nsm) {
      int64_t pb[XMAXCTX];
      (void)newsess_bits(a, t, w.p, pb);
      for (int k = 0; k < a.cfg->n_ctx; k++) {
        if (!(nsm & (1 << k))) continue;
        if (off[k] < a.ns_cap) {
          a.ns_start[(int64_t)k * a.ns_cap + off[k]] = t;
          a.ns_pb[(int64_t)k * a.ns_cap + off[k]] = pb[k];
        }
        off[k]++;
      }
    }
    w.next(t);
  }
}

// is out-of-order tuple t (before it: m in-batch new sessions of context k, running max p) inside a session
__device__ __forceinline__ bool ooo_inside(const XBArgs& a, const XBH& h, int k, int64_t t, int64_t p, int64_t m) {
  const XCfg* c = a.cfg;
  const int64_t* nss = a.ns_start + (int64_t)k * a.ns_cap;
  const int64_t* nsp = a.ns_pb + (int64_t)k * a.ns_cap;
  m = min(m, a.ns_cap);  // an overflowing round is retried (XBCtl.retry); never read past the buffer
  if (m > 0 && t >= nss[0]) {
    int64_t lo = 0, hi = m;  // last idx < m with nss[idx] <= t
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (nss[mid] <= t) lo = mid; else hi = mid;
    }
    const int64_t end = lo + 1 < m ? nsp[lo + 1] : p;
    return t <= end;
  }
  const int ns = h.ns[k];
  if (ns == 0) return false;
  // the batch-start last session, extended by the in-order tuples
  const int64_t end0 = m > 0 ? nsp[0] : ((h.inv[k] || p > h.p_start) ? p : h.stored_end[k]);
  if (t >= h.last_start[k]) return t <= end0 && t > h.lim[k];
  // settled sessions of the batch start: first session within reach of t must contain it (getSession)
  const int64_t* st_ = a.ss.start + (int64_t)k * c->sesscap;
  const int64_t* en_ = a.ss.end + (int64_t)k * c->sesscap;
  const int64_t* rch = a.reach + (int64_t)k * c->sesscap;
  int lo = 0, hi = ns - 1;  // last settled index with start <= t
  if (hi <= 0 || st_[0] > t) return false;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (st_[mid] <= t) lo = mid; else hi = mid;
  }
  return t <= en_[lo] && (lo == 0 || rch[lo - 1] < t);
}

// out-of-order tuple (t < p): an event unless it falls inside a session of every context
__device__ __forceinline__ bool ooo_event(const XBArgs& a, const XBH& h, int64_t t, int64_t p,
                                          const int64_t* ns_before) {
  if (!h.started) return true;
  if (t < h.oldest || h.has_count) return true;
  if (h.n_ctx > 0) {
    if (h.lazy) return true;
#pragma unroll
    for (int k = 0; k < XMAXCTX; k++) {  // unrolled: h's arrays stay in registers
      if (k >= h.n_ctx) break;
      if (!ooo_inside(a, h, k, t, p, ns_before[k])) return true;
    }
  }
  return false;
}

// pass 3: classify every tuple; event bitmap; per-tile event counts and segmented-max aggregates
// A quiet tile (sessions, no count windows): no tuple after the first can be an event, so only the first is
// classified.  In-order tuples after it: no jump beyond min_gap (strict, tmax < first + min_gap), no grid point in
// (carry, tmax], all above every settled session's reach; out-of-order ones: no in-batch session before the tile
// and tmin at or above every context's last session start and reach and the oldest slice (inside the last
// session, which ends at the running max).  Returns true with *ev0 the first tuple's classification.
__device__ bool quiet_tile(const XBArgs& a, const XBH& h, int64_t tile, bool* ev0) {
  const XCfg* c = a.cfg;
  if (h.n_ctx == 0 || h.has_count || h.lazy || !h.started || a.tjump[tile]) return false;
  const int64_t carry = max((int64_t)a.pcarry[tile], h.p_start);
  if (carry <= h.p_start || carry < 0) return false;
  const int64_t base = tile * XB_TILE, tm = a.tmax[tile], tn = a.tmin[tile], t0 = a.ts[base];
  if (h.min_gap < 0 || t0 > JMAX - h.min_gap || !(tm < t0 + h.min_gap)) return false;
  int64_t nsb[XMAXCTX] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < XMAXCTX; k++) {
    if (k >= h.n_ctx) break;
    nsb[k] = a.ns_cnt[(int64_t)k * a.ntiles + tile];
    if (nsb[k] != 0 || h.ns[k] == 0) return false;
    if (carry <= h.lim[k] || tn <= h.lim[k] || tn < h.last_start[k]) return false;
  }
  if (tn < h.oldest) return false;
  int64_t g = JMAX;
  if (h.has_time && h.has_fixed) {
    g = next_grid_lane(c, carry);
    if (carry < h.n0 ? tm >= h.n0 : tm >= g) return false;
  }
  if (t0 >= carry) {
    int nsm;
    int64_t pb[XMAXCTX];
    *ev0 = inorder_event(h, c, t0, carry, carry < h.n0 ? h.n0 : g, base, nsm, pb, false);
  } else {
    *ev0 = ooo_event(a, h, t0, carry, nsb);
  }
  return true;
}

__global__ __launch_bounds__(XB_THREADS) void xb_classify_kernel(XBArgs a) {
  __shared__ long long wtot[4];
  __shared__ long long tb[XB_LDS];
  const XCfg* c = a.cfg;
  {
    const XBH hq = hoist(a);
    bool ev0 = false;
    if (quiet_tile(a, hq, blockIdx.x, &ev0) && !ev0) {  // no event in the tile: zero bitmap words, no walk
      const int64_t base = (int64_t)blockIdx.x * XB_TILE;
      const int64_t w0 = base >> 5, w1 = min((a.n + 31) >> 5, (base + XB_TILE) >> 5);
      for (int64_t w = w0 + threadIdx.x; w < w1; w += XB_THREADS) a.evbits[w] = 0u;
      if (threadIdx.x == 0) {
        a.ev_cnt[blockIdx.x] = 0;
        a.seg_tail[blockIdx.x] = a.tmax[blockIdx.x];
        a.seg_has[blockIdx.x] = 0;
      }
      return;
    }
  }
  TileItems it;
  load_tile(a, blockIdx.x, it, wtot, tb);
  // new sessions before each item: carry (exclusive offsets of the tile) + local exclusive count
  int64_t nsb[XMAXCTX] = {0, 0, 0, 0};
  int64_t loc[XMAXCTX] = {0, 0, 0, 0};
  uint64_t nsm_all = 0;  // 4 new-session bits per item
  uint32_t io_ev = 0;    // in-order events, evaluated once
  uint32_t io = 0;       // in-order items
  int nsm0 = 0;
  int64_t pb0[XMAXCTX];
  uint32_t bits = 0;
  int64_t nev = 0;
  int64_t tail_m = JMIN;  // max after this thread's last event
  bool has = false;
  auto mark = [&](int j, bool ev, int64_t t) {
    if (ev) {
      bits |= 1u << j;
      nev++;
      has = true;
      tail_m = JMIN;
    } else {
      tail_m = max(tail_m, t);
    }
  };
  const XBH h = hoist(a);
  if (c->n_ctx > 0 && tile_simple(a, blockIdx.x, nsm0, pb0)) {
    // only the tile's first item can open a session: the sessions before each item need no block scan, and one
    // walk classifies in-order and out-of-order items alike
    for (int k = 0; k < c->n_ctx; k++)
      nsb[k] = a.ns_cnt[(int64_t)k * a.ntiles + blockIdx.x] + (threadIdx.x > 0 ? (nsm0 >> k) & 1 : 0);
    TileWalk w(a, it, true);
    for (int j = 0; j < it.cnt; j++) {
      const int64_t t = it.row[j];
      bool ev;
      if (t >= w.p) {
        int64_t pb[XMAXCTX];
        int nsm = 0;
        ev = inorder_event(h, c, t, w.p, w.g(c), it.base + j, nsm, pb, false);
      } else {
        ev = ooo_event(a, h, t, w.p, nsb);
      }
      if (threadIdx.x == 0 && j == 0)
        for (int k = 0; k < c->n_ctx; k++) nsb[k] += (nsm0 >> k) & 1;
      mark(j, ev, t);
      w.next(t);
    }
  } else {
    {
      TileWalk w(a, it, true);
      for (int j = 0; j < it.cnt; j++) {
        const int64_t t = it.row[j];
        if (t >= w.p) {
          io |= 1u << j;
          int64_t pb[XMAXCTX];
          int nsm = 0;
          if (inorder_event(h, c, t, w.p, w.g(c), it.base + j, nsm, pb)) io_ev |= 1u << j;
          nsm_all |= (uint64_t)nsm << (4 * j);
#pragma unroll
          for (int k = 0; k < XMAXCTX; k++)
            if (nsm & (1 << k)) loc[k]++;
        }
        w.next(t);
      }
    }
    for (int k = 0; k < c->n_ctx; k++)
      nsb[k] = block_excl_sum(loc[k], wtot, nullptr) + a.ns_cnt[(int64_t)k * a.ntiles + blockIdx.x];
    TileWalk w(a, it, false);
    for (int j = 0; j < it.cnt; j++) {
      const int64_t t = it.row[j];
      const bool ev = ((io >> j) & 1) ? ((io_ev >> j) & 1) != 0 : ooo_event(a, h, t, w.p, nsb);
      const int nsm = (int)((nsm_all >> (4 * j)) & 15u);
#pragma unroll
      for (int k = 0; k < XMAXCTX; k++)
        if (nsm & (1 << k)) nsb[k]++;
      mark(j, ev, t);
      w.next(t);
    }
  }
  // bitmap: 16 bits per thread, two threads per word
  {
    const uint32_t mine = bits & 0xFFFFu;
    const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1);
    if ((threadIdx.x & 1) == 0 && it.base < a.n) a.evbits[it.base >> 5] = mine | (other << 16);
  }
  int64_t tot;
  (void)block_excl_sum(nev, wtot, &tot);
  // segmented max: the tile's "max after its last event" = max of the tails of the last thread with an event
  // and of every thread after it (two block reductions instead of a serial fold)
  __shared__ long long s_red[8];
  int64_t last_ev = wmax(has ? (int64_t)threadIdx.x : (int64_t)-1);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = last_ev;
  __syncthreads();
  last_ev = max(max((int64_t)s_red[0], (int64_t)s_red[1]), max((int64_t)s_red[2], (int64_t)s_red[3]));
  int64_t m = wmax((int64_t)threadIdx.x >= last_ev ? tail_m : JMIN);
  if ((threadIdx.x & 63) == 0) s_red[4 + (threadIdx.x >> 6)] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = max(max((int64_t)s_red[4], (int64_t)s_red[5]), max((int64_t)s_red[6], (int64_t)s_red[7]));
    a.ev_cnt[blockIdx.x] = tot;
    a.seg_tail[blockIdx.x] = m;
    a.seg_has[blockIdx.x] = last_ev >= 0 ? 1 : 0;
  }
}

// carries of the segmented max over tiles (same operator as in xb_evwrite_kernel)
__global__ __launch_bounds__(1024) void xb_mcarry_kernel(XBArgs a) {
  const SPair t = wg_scan16(a.ntiles, SPair{0, JMIN}, SPair{0, JMIN}, OpSeg{}, ld_seg, st_mcarry, a, 0);
  if (threadIdx.x == 0) a.ctl->m_tail = t.t;
}

// pass 4: write the compacted events (position, ts, value, max ts since the previous event)
__global__ __launch_bounds__(XB_THREADS) void xb_evwrite_kernel(XBArgs a) {
  __shared__ long long wtot[4];
  __shared__ long long s_tail[XB_THREADS];
  __shared__ int s_has[XB_THREADS];
  __shared__ long long tb[XB_LDS];
  {  // a tile without events writes nothing (ev_cnt holds exclusive offsets)
    const int64_t nxt = blockIdx.x + 1 < a.ntiles ? a.ev_cnt[blockIdx.x + 1] : a.ctl->ev_total;
    if (nxt == a.ev_cnt[blockIdx.x]) return;
  }
  stage_tile(a.ts, a.n, blockIdx.x, tb);
  const int64_t base = (int64_t)blockIdx.x * XB_TILE + (int64_t)threadIdx.x * XB_ITEMS;
  const int cnt = (int)max((int64_t)0, min((int64_t)XB_ITEMS, a.n - base));
  uint32_t bits = 0;
  if (base < a.n) bits = (a.evbits[base >> 5] >> ((base & 31))) & 0xFFFFu;
  int64_t t[XB_ITEMS];
  int64_t tail_m = JMIN;
  bool has = false;
  int64_t nev = 0;
  for (int j = 0; j < cnt; j++) {
    t[j] = tb[threadIdx.x * (XB_ITEMS + 1) + j];
    if ((bits >> j) & 1) {
      has = true;
      tail_m = JMIN;
      nev++;
    } else {
      tail_m = max(tail_m, t[j]);
    }
  }
  int64_t off = block_excl_sum(nev, wtot, nullptr) + a.ev_cnt[blockIdx.x];
  // carry into this thread: segmented max over the previous threads of the tile (reset at a thread with an
  // event), seeded with the tile carry -- an exclusive scan with the operator (h1,t1)o(h2,t2) =
  // (h1|h2, h2 ? t2 : max(t1,t2))
  int64_t m;
  {
    const int ln = threadIdx.x & 63, wd = threadIdx.x >> 6;
    int hh = has ? 1 : 0;
    int64_t tt = tail_m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int h2 = __shfl_up(hh, o);
      const int64_t t2 = (int64_t)__shfl_up((long long)tt, o);
      if (ln >= o) {
        tt = hh ? tt : max(t2, tt);
        hh = hh | h2;
      }
    }
    s_tail[threadIdx.x] = tt;  // inclusive within the wave
    s_has[threadIdx.x] = hh;
    __syncthreads();
    // exclusive: previous lane's inclusive, then previous waves, then tile carry
    int hx = ln > 0 ? s_has[threadIdx.x - 1] : 0;
    int64_t tx = ln > 0 ? (int64_t)s_tail[threadIdx.x - 1] : JMIN;
    for (int w = wd - 1; w >= 0 && !hx; w--) {
      const int h2 = s_has[w * 64 + 63];
      const int64_t t2 = s_tail[w * 64 + 63];
      tx = max(tx, t2);
      hx = h2;
    }
    m = hx ? tx : max((int64_t)a.m_carry[blockIdx.x], tx);
  }
  for (int j = 0; j < cnt; j++) {
    if ((bits >> j) & 1) {
      if (off < a.ev_cap) {
        a.ev_pos[off] = base + j;
        a.ev_t[off] = t[j];
        a.ev_v[off] = load_v(a, base + j);
        a.ev_m[off] = m;
      }
      off++;
      m = JMIN;
    } else {
      m = max(m, t[j]);
    }
  }
}

// Effect of the simple tuples since the previous event (or batch start): every part of it is a max of their
// timestamps m -- StreamSlicer.maxEventTime, the current slice's tLast (they land in it iff m >= its tStart)
// and the end of each context's last session (simple in-order tuples only extend it).
__device__ __forceinline__ void reconstruct(Op& o, const XCfg* cfg, int64_t m) {
  if (m == JMIN) return;
  o.s.maxEventTime = max(o.s.maxEventTime, m);
  if (o.s.tail > o.s.head) {
    const int cur = o.s.tail - 1;
    if (m >= o.ts[cur] && m > o.tl[cur]) o.tl[cur] = m;
  }
  for (int c = 0; c < cfg->n_ctx; c++) {
    const int ns = o.s.ns(c);
    if (ns > 0 && m > o.se[c][ns - 1]) o.se[c][ns - 1] = m;
  }
}

// event pass: one wavefront walks the events with the reference logic (exact_op.h)
__global__ __launch_bounds__(64) void xb_events_kernel(XBArgs a) {
  const int lane = threadIdx.x;
  const XCfg* cfg = a.cfg;
  XBCtl ctl = *a.ctl;
  // the operator's state lives in LDS, shared by the wave's lanes (all hold the same values): as a private object it
  // sat in scratch memory, and every step of the event walk paid a scratch round trip
  __shared__ Op o_lds;
  Op& o = o_lds;
  o.bind(cfg, a.sl, a.ss, 0, lane);
  o.s = *a.st;
  if (ctl.done || o.s.err) {
    return;
  }
  long long* dbg = a.dbg;
  int nd = 0;
  auto stamp = [&]() {
    if (dbg && nd < 255) {
      const long long c = (long long)__builtin_amdgcn_s_memtime();
      if (lane == 0) dbg[1 + nd] = c;
      nd++;
    }
  };
  stamp();
  {  // buffers sized from the previous rounds: an overflow changes nothing and is retried by the host
    bool over = ctl.ev_total + 4 > a.ev_cap;
    for (int k = 0; k < cfg->n_ctx; k++) over |= a.ns_tot[k] > a.ns_cap;
    if (over) {
      if (lane == 0) a.ctl->retry = 1;
      return;
    }
  }
  // segment start: compaction is only safe here (slice indices are stable within a segment)
  if (o.s.tail + 64 > cfg->sc && o.s.head > 0) {
    o.move_range(0, o.s.head, o.s.tail - o.s.head);
    o.s.tail -= o.s.head;
    o.s.head = 0;
  }
  stamp();
  int64_t ep = 0;
  if (lane == 0) {
    a.ep_pos[0] = ctl.seg_start - 1;
    a.ep_tail[0] = o.s.tail;
  }
  ep = 1;
  int64_t e = ctl.ev_next;
  bool first = true;
  ctl.stopped = 0;
  // the compacted events are fetched 64 at a time, one per lane, and broadcast: no load round trip per event
  int64_t fb = JMIN;  // first event held in the lanes
  int64_t f_pos = 0, f_t = 0, f_v = 0, f_m = 0;
  for (; e < ctl.ev_total; e++) {
    if (fb == JMIN || e >= fb + 64) {
      fb = e;
      const int64_t k = min(e + lane, ctl.ev_total - 1);
      f_pos = a.ev_pos[k];
      f_t = a.ev_t[k];
      f_v = a.ev_v[k];
      f_m = a.ev_m[k];
    }
    const int src = (int)(e - fb);
    const int64_t pos = (int64_t)__shfl((long long)f_pos, src), t = (int64_t)__shfl((long long)f_t, src);
    const int64_t vb = (int64_t)__shfl((long long)f_v, src), m = (int64_t)__shfl((long long)f_m, src);
    reconstruct(o, cfg, m);
    o.s.currentCount = jadd(a.snap->c0, pos);
    // an out-of-order event of an operator with sessions may split / shift / merge older slices: the simple
    // tuples before it are applied first (segment end).  The stop event itself opens the next segment.
    const bool stop_kind = (cfg->n_ctx > 0 && (t < o.s.maxEventTime || a.snap->min_gap == 0)) ||
                           (!a.snap->started && !first);  // re-classify once the store exists
    const bool cap = o.s.tail + 8 >= cfg->sc || ep + 2 >= a.ep_cap;
    // the stop tuple of the previous round (position 0 of this round) is processed, never deferred again
    if (!(first && ctl.resume && pos == 0) && (stop_kind || cap)) {
      ctl.stopped = 1;
      ctl.seg_end = pos;
      break;
    }
    first = false;
    o.exc = 0;
    stamp();
    o.determine_slices(t);
    stamp();
    if (!o.exc) o.manager_process(t, vb);
    stamp();
    if (xerr_tuple_failed(o.exc)) {
      o.s.dropped++;
      o.exc = 0;
    } else if (o.exc) {
      o.s.err = o.exc;
      e++;
      break;
    }
    __threadfence_block();
    if (lane == 0) {
      a.ep_pos[ep] = pos;
      a.ep_tail[ep] = o.s.tail;
    }
    ep++;
  }
  if (!ctl.stopped) {
    ctl.seg_end = -1;  // host: apply to n
    ctl.done = e >= ctl.ev_total ? 1 : 0;
    ctl.ev_next = e;
    if (ctl.done && !o.s.err) {  // the simple tuples after the last event
      reconstruct(o, cfg, ctl.m_tail);
      o.s.currentCount = jadd(a.snap->c0, a.n);
    }
  } else {
    ctl.ev_next = e;
  }
  ctl.ep_count = ep;
  ctl.resume = 0;
  __threadfence_block();
  stamp();
  if (lane == 0) {
    *a.st = o.s;
    *a.ctl = ctl;
    if (dbg) dbg[0] = nd;
  }
}

// A load on a rarely taken branch whose value is used after the branch: waited for INSIDE the branch (the empty asm
// uses the value there), so the common path past the join carries no wait -- a wait there would be vmcnt(0), draining
// every outstanding prefetch.  Atomic, so the compiler cannot fold it with an LDS load into one flat load either.
template <class T>
__device__ __forceinline__ T gload(const T* p) {
  T v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("" ::"v"(v));
  return v;
}

// apply the simple tuples of [seg_start, seg_end) (all CUs).  Each workgroup streams a contiguous range and
// accumulates into an LDS window over the newest XW slices (LDS atomics), flushed once per touched slice;
// wave-uniform runs (in-order tuples all in the current slice) are reduced in registers first.
constexpr int XW = 256;

template <int VT>
__global__ __launch_bounds__(256) void xb_apply_kernel(XBArgs a) {
  __shared__ unsigned int w_cnt[XW];
  __shared__ long long w_tl[XW], w_tf[XW], w_p1[XW], w_p2[XW];
  __shared__ unsigned long long w_p0[XW];
  const XBCtl& ctl = *a.ctl;
  if (ctl.retry) return;
  const int64_t s0 = ctl.seg_start;
  const int64_t s1 = ctl.seg_end < 0 ? a.n : ctl.seg_end;
  const XCfg* cfg = a.cfg;
  const int need = cfg->need;
  const bool lazy = cfg->lazy != 0;
  const XState& st = *a.st;
  const int head = st.head;
  const int64_t nep = ctl.ep_count;
  // the event pass writes at least the segment's opening epoch entry; it writes none when it returned at once (an
  // operator already failed): nothing to apply, and ep_tail holds nothing of this round
  if (nep <= 0) return;
  const int wtop = a.ep_tail[nep - 1];
  const int wbase = max(head, wtop - XW);
  const int64_t* sk = (st.unsorted & 1) ? a.sufmin : a.sl.ts;
  // LDS copies of the search keys of the window's slices and of the epoch table (binary searches of every
  // out-of-order tuple stay in LDS; only tuples older than the window search HBM)
  constexpr int EPC = 512;
  __shared__ long long w_key[XW];
  __shared__ long long w_ts[XW];
  __shared__ long long e_pos[EPC];
  __shared__ int e_tail[EPC];
  const bool ep_lds = nep <= EPC;
  for (int k = threadIdx.x; k < XW; k += 256) {
    w_cnt[k] = 0;
    w_tl[k] = JMIN;
    w_tf[k] = JMAX;
    w_p0[k] = 0;
    w_p1[k] = ID_MIN;
    w_p2[k] = ID_MAX;
    w_key[k] = wbase + k < wtop ? sk[wbase + k] : JMAX;
    w_ts[k] = wbase + k < wtop ? a.sl.ts[wbase + k] : JMAX;
  }
  if (ep_lds)
    for (int64_t k = threadIdx.x; k < nep; k += 256) {
      e_pos[k] = a.ep_pos[k];
      e_tail[k] = a.ep_tail[k];
    }
  __syncthreads();
  // bucket index over the window's search keys (sorted: tStart, or its suffix minimum on an unsorted list):
  // kidx[b] = keys <= kbase + (b << kshift), so the last key <= t lies between kidx[b] and kidx[b + 1] -- usually one
  // LDS load and at most one compare per out-of-order tuple instead of a bisection of the window
  constexpr int NB = 1024;
  __shared__ unsigned short kidx[NB + 1];
  const int nw = wtop - wbase;
  const int64_t kbase = w_key[0];
  int kshift = 0;
  if (nw > 1) {
    const uint64_t span = (uint64_t)w_key[nw - 1] - (uint64_t)kbase;
    while (kshift < 63 && (span >> kshift) >= (uint64_t)NB) kshift++;
  }
  for (int b = threadIdx.x; b <= NB; b += 256) {
    int c = nw;
    if (b < NB) {
      const uint64_t d = (uint64_t)b << kshift;
      const int64_t x = d > (uint64_t)(JMAX - kbase) ? JMAX : (int64_t)((uint64_t)kbase + d);  // saturating
      int l = 0, h = nw;
      while (l < h) {
        const int mid = (l + h) >> 1;
        if (w_key[mid] <= x) l = mid + 1; else h = mid;
      }
      c = l;
    }
    kidx[b] = (unsigned short)c;
  }
  __syncthreads();
  // the wave's running partial of the slice in-order tuples land in (the last slice present at their arrival);
  // it is reduced and flushed only when that slice changes (an event appended a slice) and at the end
  int s_acc = -1;
  uint32_t acnt = 0;
  int64_t atmx = JMIN, atmn = JMAX, amn = ID_MIN, amx = ID_MAX;
  uint64_t asw = 0;
  double asf = 0.0;
  // one slice update: LDS window when the slice is in it, else the slice arrays
  auto update = [&](int tgt, unsigned int c_, int64_t tmx, int64_t tmn, uint64_t sw, int64_t mn, int64_t mx) {
    if (tgt >= wbase && tgt < wbase + XW) {
      const int k = tgt - wbase;
      atomicAdd(&w_cnt[k], c_);
      atomicMax(&w_tl[k], (long long)tmx);
      if (lazy) atomicMin(&w_tf[k], (long long)tmn);  // tFirst only feeds LazySlice record moves
      if (need & NEED_SUM) {
        if constexpr (VT == VT_F64) atomicAdd((double*)&w_p0[k], __longlong_as_double((long long)sw));
        else atomicAdd(&w_p0[k], (unsigned long long)sw);
      }
      if (need & NEED_MIN) atomicMin(&w_p1[k], (long long)mn);
      if (need & NEED_MAX) atomicMax(&w_p2[k], (long long)mx);
    } else {
      atomicAdd(&a.sl.cnt[tgt], (unsigned long long)c_);
      atomicAdd((unsigned long long*)&a.sl.cl[tgt], (unsigned long long)c_);
      atomicMax((long long*)&a.sl.tl[tgt], (long long)tmx);
      if (lazy) atomicMin((long long*)&a.sl.tf[tgt], (long long)tmn);
      if (need & NEED_SUM) {
        if constexpr (VT == VT_F64) atomicAdd((double*)&a.sl.p[0][tgt], __longlong_as_double((long long)sw));
        else atomicAdd(&a.sl.p[0][tgt], (unsigned long long)sw);
      }
      if (need & NEED_MIN) atomicMin((long long*)&a.sl.p[1][tgt], (long long)mn);
      if (need & NEED_MAX) atomicMax((long long*)&a.sl.p[2][tgt], (long long)mx);
    }
  };
  auto flush_acc = [&]() {  // DPP reductions: every lane of the block is active at the call sites
    if (s_acc < 0) return;
    const uint64_t c_ = fsum64(acnt);
    if (c_ != 0) {
      const int64_t tmx = fmax64(atmx);
      const int64_t tmn = lazy ? fmin64(atmn) : JMAX;
      uint64_t sw = 0;
      if (need & NEED_SUM) {
        if constexpr (VT == VT_F64) sw = (uint64_t)__double_as_longlong(fsumf(asf));
        else sw = fsum64(asw);
      }
      const int64_t mn = (need & NEED_MIN) ? fmin64(amn) : ID_MIN;
      const int64_t mx = (need & NEED_MAX) ? fmax64(amx) : ID_MAX;
      if ((threadIdx.x & 63) == 0) update(s_acc, (unsigned int)c_, tmx, tmn, sw, mn, mx);
    }
    acnt = 0;
    atmx = JMIN;
    atmn = JMAX;
    amn = ID_MIN;
    amx = ID_MAX;
    asw = 0;
    asf = 0.0;
  };
  const int64_t total = s1 - s0;
  int64_t chunk = (total + gridDim.x - 1) / gridDim.x;
  chunk = ((chunk + 255) / 256) * 256;
  const int64_t b0 = s0 + (int64_t)blockIdx.x * chunk;
  const int64_t b1 = min(s1, b0 + chunk);
  // software pipelined XD iterations deep: the tuples and event words of the next XD - 1 iterations are in flight
  // while one is combined (one iteration's loads alone keep too few bytes in flight per CU to approach HBM rate)
  constexpr int XD = 4;
  // unconditional loads (the index clamped into the batch): a load under a branch makes the compiler wait for it at
  // the join, which serialises the pipeline
  const int64_t jmax = max(b1, (int64_t)1) - 1;
  auto ld = [&](int64_t i, int64_t& t, int64_t& vb, uint32_t& wd) {
    const int64_t j = min(i, jmax);
    t = __builtin_nontemporal_load(a.ts + j);
    if constexpr (VT == VT_I32) vb = (int64_t)__builtin_nontemporal_load((const int32_t*)a.val + j);
    else vb = __builtin_nontemporal_load((const int64_t*)a.val + j);
    wd = a.evbits[j >> 5];
  };
  int64_t t_q[XD] = {}, v_q[XD] = {};
  uint32_t wd_q[XD] = {};
#pragma unroll
  for (int d = 0; d < XD; d++) ld(b0 + d * 256 + threadIdx.x, t_q[d], v_q[d], wd_q[d]);
  // epoch cursor of this wave (indices only increase): last epoch entry with pos < the wave's first index
  // LDS-or-HBM reads: the HBM side as an atomic load, so the compiler cannot fold the two into one load through a
  // selected (flat) address -- a flat load waits for every outstanding load and would drain the prefetch pipeline
  auto epos = [&](int64_t k) -> int64_t { return ep_lds ? (int64_t)e_pos[k] : gload(a.ep_pos + k); };
  auto etail = [&](int64_t k) -> int { return ep_lds ? e_tail[k] : gload(a.ep_tail + k); };
  int64_t ecur = 0;
  {
    int64_t lo = 0, hi = nep;
    const int64_t iw = b0 + (threadIdx.x & ~63);
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (epos(mid) < iw) lo = mid; else hi = mid;
    }
    ecur = lo;
  }
  for (int64_t i00 = b0; i00 < b1; i00 += 256 * XD) {
#pragma unroll
    for (int d = 0; d < XD; d++) {
      const int64_t i0 = i00 + d * 256;
      const int64_t i = i0 + threadIdx.x;
      const int64_t t = t_q[d], vb = v_q[d];
      const uint32_t wd = wd_q[d];
      ld(i + 256 * XD, t_q[d], v_q[d], wd_q[d]);
      const int64_t iw = i0 + (int64_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63));
      while (ecur + 1 < nep && epos(ecur + 1) < iw) ecur++;
      // usually no epoch entry falls among the wave's 64 tuples: then every lane's last slice present at arrival is
      // the cursor's, looked up once for the wave
      const bool uni = !(ecur + 1 < nep && epos(ecur + 1) < iw + 63);
      int last_u = -1;
      int64_t tl_u = 0;
      if (uni) {
        last_u = __builtin_amdgcn_readfirstlane(etail(ecur) - 1);
        tl_u = last_u >= wbase ? (int64_t)w_ts[last_u - wbase] : gload(a.sl.ts + last_u);
      }
      bool act = i < b1 && !((wd >> (i & 31)) & 1);
      int si = -1, last = -1;
      if (act) {
        int64_t tl;
        if (uni) {
          last = last_u;
          tl = tl_u;
        } else {
          // last epoch entry with pos < i: the last slice present at arrival (a few steps from the wave cursor)
          int64_t lo = ecur;
          while (lo + 1 < nep && epos(lo + 1) < i) lo++;
          last = etail(lo) - 1;
          tl = last >= wbase ? (int64_t)w_ts[last - wbase] : gload(a.sl.ts + last);
        }
        if (t >= tl) {
          si = last;
        } else if (last > wbase && t >= kbase) {  // in the LDS window: last key <= t in [wbase, last)
          const uint64_t bo = ((uint64_t)t - (uint64_t)kbase) >> kshift;
          const int b = bo < (uint64_t)NB ? (int)bo : NB - 1;
          const int lim = last - wbase;
          int h = min((int)kidx[b + 1], lim);
          int l = min((int)kidx[b], h);
          while (l < h) {
            const int mid = (l + h) >> 1;
            if (w_key[mid] <= t) l = mid + 1; else h = mid;
          }
          si = wbase + l - 1;
        } else {  // last slice in [head, last) with tStart <= t (suffix-min keys on an unsorted list)
          int l = head, h = min(last, wbase);
          while (l < h) {
            const int mid = (l + h) >> 1;
            if (sk[mid] <= t) l = mid + 1; else h = mid;
          }
          si = l - 1;
        }
        if (si < head) {  // cannot happen for a simple tuple (t >= oldest); counted, never silently lost
          atomicAdd((int*)&a.ctl->pad, 1);
          act = false;
        }
      }
      const Lift lf = lift(VT, vb);
      const unsigned long long am = __ballot(act);
      if (!am) continue;
      // the in-order target of the wave's highest active lane; a change flushes the running partial
      const int ref = 63 - __clzll((long long)am);
      const int s_ref = __builtin_amdgcn_readlane(last, ref);
      if (s_ref != s_acc) {
        flush_acc();
        s_acc = s_ref;
      }
      if (act && si == s_acc) {
        acnt++;
        atmx = max(atmx, t);
        atmn = min(atmn, t);
        if (need & NEED_SUM) {
          if constexpr (VT == VT_F64) asf += __longlong_as_double(vb);
          else asw += lf.sum;
        }
        if (need & NEED_MIN) amn = min(amn, lf.mn);
        if (need & NEED_MAX) amx = max(amx, lf.mx);
      } else if (act) {
        update(si, 1u, t, t, lf.sum, lf.mn, lf.mx);
      }
    }
  }
  flush_acc();

  __syncthreads();
  for (int k = threadIdx.x; k < XW; k += 256) {
    const unsigned int c_ = w_cnt[k];
    if (!c_) continue;
    const int s_ = wbase + k;
    atomicAdd(&a.sl.cnt[s_], (unsigned long long)c_);
    atomicAdd((unsigned long long*)&a.sl.cl[s_], (unsigned long long)c_);
    atomicMax((long long*)&a.sl.tl[s_], w_tl[k]);
    if (lazy) atomicMin((long long*)&a.sl.tf[s_], w_tf[k]);
    if (need & NEED_SUM) {
      if constexpr (VT == VT_F64) atomicAdd((double*)&a.sl.p[0][s_], __longlong_as_double((long long)w_p0[k]));
      else atomicAdd(&a.sl.p[0][s_], w_p0[k]);
    }
    if (need & NEED_MIN) atomicMin((long long*)&a.sl.p[1][s_], w_p1[k]);
    if (need & NEED_MAX) atomicMax((long long*)&a.sl.p[2][s_], w_p2[k]);
  }
}

// suffix minimum of tStart over the op's slices (only when the list is unsorted), one workgroup
__global__ __launch_bounds__(1024) void xb_sufmin_kernel(XBArgs a) {
  __shared__ long long wt[16];
  const XState& st = *a.st;
  if (!(st.unsorted & 1)) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int64_t carry = JMAX;
  for (int64_t top = st.tail; top > st.head; top -= 1024) {
    const int64_t i = top - 1 - tid;  // thread 0 = rightmost
    const int64_t v = i >= st.head ? a.sl.ts[i] : JMAX;
    int64_t inc = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t u = (int64_t)__shfl_up((long long)inc, o);
      if (lane >= o) inc = min(inc, u);
    }
    if (lane == 63) wt[wid] = inc;
    __syncthreads();
    int64_t before = carry;
    for (int w = 0; w < wid; w++) before = min(before, (int64_t)wt[w]);
    if (i >= st.head) a.sufmin[i] = min(before, inc);
    int64_t tot = carry;
    for (int w = 0; w < 16; w++) tot = min(tot, (int64_t)wt[w]);
    __syncthreads();
    carry = tot;
  }
}

// after an apply: the next segment starts at the stop event
__global__ void xb_next_segment_kernel(XBArgs a) {
  if (threadIdx.x != 0) return;
  XBCtl c = *a.ctl;
  if (c.retry) return;
  if (c.stopped) {
    c.seg_start = c.seg_end;
    c.resume = 1;
  } else {
    c.seg_start = a.n;
    c.done = 1;
  }
  *a.ctl = c;
}

}  // namespace xb

// ---------------------------------------------------------------- host wrappers
int64_t xb_tile() { return XB_TILE; }
size_t xb_snap_bytes() { return sizeof(XSnap); }
size_t xb_ctl_bytes() { return sizeof(XBCtl); }

hipError_t xb_classify_phase(XBArgs& a, int phase, hipStream_t st) {
  const unsigned nt = (unsigned)a.ntiles;
  switch (phase) {
    case 0:  // snapshot + tile maxima + carries + new-session counts + scan
      hipLaunchKernelGGL(xb::xb_prep_kernel, dim3(1), dim3(64), 0, st, a);
      hipLaunchKernelGGL(xb::xb_tilemax_kernel, dim3(nt), dim3(XB_THREADS), 0, st, a);
      hipLaunchKernelGGL(xb::xb_carry_kernel, dim3(1), dim3(1024), 0, st, a);
      if (a.cfg_nctx_host > 0) {
        hipLaunchKernelGGL(xb::xb_nscount_kernel, dim3(nt), dim3(XB_THREADS), 0, st, a);
        hipLaunchKernelGGL(xb::xb_rows_scan_kernel, dim3(1), dim3(1024), 0, st, a, a.ns_cnt, a.cfg_nctx_host,
                           a.ns_tot);
      }
      break;
    case 1:  // new-session chains, classification, event counts
      if (a.cfg_nctx_host > 0) hipLaunchKernelGGL(xb::xb_nswrite_kernel, dim3(nt), dim3(XB_THREADS), 0, st, a);
      hipLaunchKernelGGL(xb::xb_classify_kernel, dim3(nt), dim3(XB_THREADS), 0, st, a);
      hipLaunchKernelGGL(xb::xb_rows_scan_kernel, dim3(1), dim3(1024), 0, st, a, a.ev_cnt, 1, &a.ctl->ev_total);
      hipLaunchKernelGGL(xb::xb_mcarry_kernel, dim3(1), dim3(1024), 0, st, a);
      break;
    case 2:  // compacted events
      hipLaunchKernelGGL(xb::xb_evwrite_kernel, dim3(nt), dim3(XB_THREADS), 0, st, a);
      break;
  }
  return hipGetLastError();
}

hipError_t xb_events(XBArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(xb::xb_events_kernel, dim3(1), dim3(64), 0, st, a);
  return hipGetLastError();
}
hipError_t xb_apply(XBArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(xb::xb_sufmin_kernel, dim3(1), dim3(1024), 0, st, a);
  static const int64_t max_blocks = [] {
    const char* e = getenv("SCOTTY_XB_APPLY_BLOCKS");  // A/B of the apply grid (flush contention vs occupancy)
    return e ? std::max<int64_t>(64, atoll(e)) : (int64_t)4096;
  }();
  const int64_t blocks = std::min<int64_t>((a.n + 4095) / 4096, max_blocks);
  if (a.vt == VT_I32) hipLaunchKernelGGL(xb::xb_apply_kernel<VT_I32>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (a.vt == VT_I64) hipLaunchKernelGGL(xb::xb_apply_kernel<VT_I64>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(xb::xb_apply_kernel<VT_F64>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  hipLaunchKernelGGL(xb::xb_next_segment_kernel, dim3(1), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace scotty
