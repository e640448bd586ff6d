// exact_quiet.hip -- prep and commit kernels of the one-pass ("quiet batch") path of the non-keyed exact engine
// (exact_quiet.h explains when a batch is quiet and why the grid path's per-cell partials are then exact).
//
// Per micro-batch, on the op's stream:
//   xq_prep_kernel   (1 wave)  -- snapshot of the operator: eligibility, the pending edge's grid index, the lowest
//                                 timestamp an out-of-order tuple may have (last session start of every context, above
//                                 the reach of every earlier session), the ingest's DevMeta view of the slice store
//   cix_build_kernel, ingest_kernel<VT, NEED>   (slicing_kernels.hip, unchanged: one HBM pass over ts + values into
//                                 the cells; cells are scratch, the slice store is not written)
//   xq_commit_kernel (1 workgroup) -- verifies the quiet conditions, then either commits (closed-form edge rule,
//                                 SliceManager.appendSlice, cell fold, StreamSlicer / WindowManager / SessionContext
//                                 scalars) or returns every touched cell to identity for the event-exact path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exact_op.h"
#include "exact_quiet.h"

namespace scotty {
namespace xq {
using namespace x;

// x < y + g without wrapping (Java long arithmetic would wrap near Long.MAX_VALUE and flip the comparison: such
// batches are never quiet)
__device__ __forceinline__ bool lt_plus(int64_t x, int64_t y, int64_t g) { return y <= JMAX - g && x < y + g; }

constexpr int64_t SAFE = (int64_t)1 << 61;  // |values| the quiet path reasons about without wrap arithmetic

__global__ __launch_bounds__(64) void xq_prep_kernel(XQArgs a) {
  const int lane = threadIdx.x;
  const XCfg* c = a.cfg;
  const XState s = *a.st;
  int32_t res = XQ_NONE;
  int64_t why = 0;
  const int64_t P = s.maxEventTime;
  if (!s.started || s.err || s.tail <= s.head || P == JMIN) why |= 32;
  if (P > SAFE) why |= 1024;
  if (why) res = XQ_STATE;
  int64_t j0 = 0, gcount = 0, h_end = JMAX;
  if (res == XQ_NONE && c->has_fixed) {
    const int64_t N = s.nextEdgeTs;  // the pending edge, nextGrid(maxEventTime) (StreamSlicer.java:103-116)
    if (N < 0) {
      res = XQ_STATE;
      why |= 512;
    } else {
      // first grid entry >= N: a 64-ary search (3-4 rounds of one probe per lane over up to 2^20 entries instead of
      // a chain of 20 dependent loads)
      int64_t lo = 0, hi = a.gcount;
      while (hi - lo > 64) {
        const int64_t stride = (hi - lo + 63) >> 6;
        const int64_t p = lo + (int64_t)lane * stride;
        const unsigned long long bal = __ballot(p < hi && a.grid[p] >= N);
        if (bal == 0) {
          lo = lo + ((hi - 1 - lo) / stride) * stride + 1;
        } else {
          const int f = __ffsll((long long)bal) - 1;
          if (f == 0) {
            hi = lo;
            break;
          }
          const int64_t pf = lo + (int64_t)f * stride;
          lo = pf - stride + 1;
          hi = pf;
        }
      }
      if (hi > lo) {
        const int64_t p = lo + lane;
        const unsigned long long bal = __ballot(p < hi && a.grid[p] >= N);
        lo = bal ? lo + __ffsll((long long)bal) - 1 : hi;
      }
      if (lo + 1 >= a.gcount || a.grid[lo] != N) {
        res = XQ_GRID;
      } else {
        j0 = lo;
        gcount = a.gcount;
        h_end = a.grid[gcount - 1];
      }
    }
  }
  int64_t lo_bound = JMIN, min_gap = JMAX;
  int64_t h0 = s.head;  // first slice of the cell view
  int64_t reach0 = JMIN, s_last0 = JMIN;  // context 0: reach of the earlier sessions, last session's start
  if (res == XQ_NONE) {
    for (int k = 0; k < c->n_ctx && res == XQ_NONE; k++) {
      const int64_t gap = c->gap[k];
      min_gap = min(min_gap, gap);
      const int ns = s.ns(k);
      if (ns == 0 || gap <= 0 || gap > SAFE) {
        res = XQ_STATE;
        why |= 128;
        break;
      }
      const int64_t* st_ = a.ss.start + (int64_t)k * c->sesscap;
      const int64_t* en_ = a.ss.end + (int64_t)k * c->sesscap;
      // the last session must end at maxEventTime: in-order tuples then extend it (shiftEnd) and nothing else
      if (en_[ns - 1] != P || st_[ns - 1] < -SAFE) {
        res = XQ_STATE;
        why |= 256;
        break;
      }
      // getSession(t) returns the last session only above the reach (end + gap) of every earlier one
      int64_t reach = JMIN;
      for (int i = lane; i < ns - 1; i += 64) reach = max(reach, en_[i] + gap);
      reach = wmax(reach);
      lo_bound = max(lo_bound, st_[ns - 1]);
      if (reach != JMIN) lo_bound = max(lo_bound, reach + 1);
      if (k == 0) {
        reach0 = reach;
        s_last0 = st_[ns - 1];
      }
    }
  }
  constexpr int64_t SCAN_CAP = 16384;
  constexpr int64_t BAND_NO_EDGE = -2;  // XQCtl.band_si: the start band without a slice edge to move
  // start band (exact_quiet.h): one session context; si = findSliceByEnd(s) (the last slice ending at the last
  // session's start, S/SliceManager.java:94) movable and Eager, si + 1 starting at s, the slices from si + 1 on in
  // tStart order (they become the cell view)
  int64_t band_si = -1, band_lo = JMIN;
  if (res == XQ_NONE && a.band && c->n_ctx == 1) {
    const int64_t S = s_last0, gap = c->gap[0];
    band_lo = S - gap + 1;  // SessionWindow.java:57: start - gap < t (no wrap: |S|, gap <= SAFE)
    if (reach0 != JMIN) band_lo = max(band_lo, reach0 + 1);
    int64_t si = -1;
    for (int64_t b = (int64_t)s.tail - 1; b >= s.head && b > (int64_t)s.tail - 1 - SCAN_CAP && si < 0; b -= 64) {
      const int64_t i = b - lane;
      const unsigned long long hit = __ballot(i >= s.head && a.sl.te[i] == S);
      if (hit) si = b - (__ffsll((long long)hit) - 1);
    }
    const bool lo_ok = band_lo < S && band_lo >= -SAFE;
    bool ok = si >= 0 && si + 1 < s.tail && lo_ok && ty_movable(a.sl.ty[si]) && !ty_lazy(a.sl.ty[si]) &&
              a.sl.ts[si + 1] == S && (int64_t)s.tail - si <= SCAN_CAP;
    for (int64_t i = si + 1 + lane; ok && i + 1 < s.tail; i += 64)
      if (a.sl.ts[i] > a.sl.ts[i + 1]) ok = false;
    ok = __ballot(!ok) == 0;
    if (ok) {
      band_si = si;
    } else if (si < 0 && lo_ok && (int64_t)s.tail - s.head <= SCAN_CAP) {
      // no slice ends at s (StreamSlicer opened the session without a flexible edge: calculateNextFlexEdge compares
      // with the pending fixed edge, S/StreamSlicer.java:118-130): every shiftStart's findSliceByEnd misses and the
      // modification is skipped (S/SliceManager.java:94-96) -- as long as no slice ends anywhere in [band_lo, s], the
      // band's tuples only move the session start, and land where the plain quiet view puts them
      bool none = true;
      for (int64_t i = s.head + lane; i < s.tail; i += 64) {
        const int64_t e = a.sl.te[i];
        if (e >= band_lo && e <= S) none = false;
      }
      if (__ballot(!none) == 0) band_si = BAND_NO_EDGE;
    }
  }
  if (res == XQ_NONE && band_si == BAND_NO_EDGE) lo_bound = band_lo;  // then the plain view below
  if (res == XQ_NONE && band_si >= 0) {
    // the view starts at si + 1 with the band's lower end as its start: every tuple >= band_lo lands where the
    // reference puts it (exact_quiet.h), anything below is refused by the ingest (late) -- which also covers the sorted
    // list's oldest-slice bound
    h0 = band_si + 1;
    lo_bound = band_lo;
  } else if (res == XQ_NONE) {
    if (!(s.unsorted & 1)) {
      // sorted list: the oldest slice bounds every tuple (an older one throws IndexOutOfBounds; the ingest counts it)
      lo_bound = max(lo_bound, a.sl.ts[s.head]);
    } else {
      // a list whose tStart order was broken by session edits: every tuple of a quiet batch is >= lo_bound, and
      // findSliceIndexByTimestamp (the LAST slice with tStart <= t, LazyAggregateStore.java:29-37) then lands in the
      // suffix that starts at the last slice with tStart <= lo_bound -- if that suffix is sorted, it is the view
      int64_t i0 = -1;
      for (int64_t b = (int64_t)s.tail - 1; b >= s.head && b > (int64_t)s.tail - 1 - SCAN_CAP && i0 < 0; b -= 64) {
        const int64_t i = b - lane;
        const unsigned long long hit = __ballot(i >= s.head && a.sl.ts[i] <= lo_bound);
        if (hit) i0 = b - (__ffsll((long long)hit) - 1);
      }
      bool sorted = i0 >= 0;
      for (int64_t i = i0 + lane; sorted && i + 1 < s.tail; i += 64)
        if (a.sl.ts[i] > a.sl.ts[i + 1]) sorted = false;
      sorted = __ballot(!sorted) == 0 && i0 >= 0;
      if (sorted) {
        h0 = i0;
      } else {
        res = XQ_STATE;
        why |= 64;
      }
    }
    if (lo_bound < -SAFE) {
      res = XQ_STATE;
      why |= 1024;
    }
  }
  int64_t jump_pos = -1;
  if (res == XQ_NONE && c->n_ctx > 0 && a.n > 0) {
    // fast refusal: one of the first 64 tuples jumps its running max by a session gap (a new session: the stream
    // resumes after a silence) -- the batch is not quiet, and the ingest pass is skipped
    const int64_t v = lane < a.n ? a.ts[lane] : JMIN;
    int64_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t u = (int64_t)__shfl_up((long long)inc, o);
      if (lane >= o) inc = max(inc, u);
    }
    int64_t ex = (int64_t)__shfl_up((long long)inc, 1);
    ex = lane == 0 ? P : max(P, ex);
    const unsigned long long jb = __ballot(lane < a.n && v != JMIN && !(ex <= JMAX - min_gap && v < ex + min_gap));
    if (jb != 0) {
      res = XQ_NOT_QUIET;
      why |= 4;
      jump_pos = __ffsll((long long)jb) - 1;
    }
  }
  if (res != XQ_NONE) band_si = -1;
  if (lane == 0) {
    DevMeta m{};
    // the band's view: cell 0 (slice band_si + 1) starts at band_lo for the ingest and the cell index; the slice store
    // keeps its start until the commit kernel moves it (nothing is written before the verdict)
    m.view_s0_on = band_si >= 0 ? 1 : 0;
    m.view_s0 = band_si >= 0 ? band_lo : 0;
    m.head = h0;
    m.tail = s.tail;
    m.prev_max = P;
    m.j0 = j0;
    m.gcount = gcount;
    m.overflow = res == XQ_NONE ? 0 : 1;  // the cell-index build and the ingest return at once
    m.cmin = INT64_MAX;
    *a.meta = m;
    XQCtl q{};
    q.result = res;
    q.lo_bound = lo_bound;
    q.min_gap = min_gap;
    q.p_start = P;
    q.c0 = s.currentCount;
    q.pending = s.nextEdgeTs;
    q.h_end = h_end;
    q.why = why;
    q.jump_tile = (why & 4) ? 0 : JMAX;
    q.jump_pos = jump_pos;
    q.band_si = band_si;
    q.band_s = s_last0;
    q.batch_min = JMAX;
    *a.ctl = q;
  }
}

// block-wide (1024 threads) inclusive max scan; wtot: LDS [16] (wtot[15] = the block's max on return)
__device__ __forceinline__ int64_t block_incl_max(int64_t v, long long* wtot, int lane, int wid) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = (int64_t)__shfl_up((long long)v, o);
    if (lane >= o) v = max(v, u);
  }
  if (lane == 63) wtot[wid] = v;
  __syncthreads();
  if (wid == 0) {
    int64_t t = lane < 16 ? (int64_t)wtot[lane] : JMIN;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int64_t u = (int64_t)__shfl_up((long long)t, o);
      if (lane >= o) t = max(t, u);
    }
    if (lane < 16) wtot[lane] = t;
  }
  __syncthreads();
  if (wid > 0) v = max(v, (int64_t)wtot[wid - 1]);
  return v;
}

// ---- scan (1 workgroup): prefix maxima of the ingest's tile maxima, batch max, the candidate grid points
//      g[k] <= batch_max, and the verdict parts that need no pass over the batch
__global__ __launch_bounds__(1024) void xq_scan_kernel(XQArgs a) {
  __shared__ long long s_w[32];
  __shared__ long long s_mn[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const XQCtl q = *a.ctl;
  if (q.result != XQ_NONE) return;  // refused by the prep kernel: no cell was touched
  const DevMeta& m = *a.meta;
  const int64_t j0 = m.j0, gcount = m.gcount;
  const int64_t P = q.p_start;
  int64_t kc = gcount > 0 ? gcount - j0 - 1 : 0;
  if (kc < 0) kc = 0;
  const int64_t* g = a.grid + j0;
  const int64_t nT = (a.n + a.tile - 1) / a.tile;
  // prefix max over the tile maxima (8 consecutive tiles per thread)
  int64_t loc[8];
  int64_t run = JMIN;
  int64_t bmin = JMAX;  // start band: the batch minimum (per-tile minima of the ingest)
  const bool band = q.band_si != -1;  // >= 0: with the movable edge; -2: no edge
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t t = (int64_t)tid * 8 + j;
    run = max(run, t < nT ? (int64_t)a.tilemax[t] : JMIN);
    loc[j] = run;
    if (band && t < nT) bmin = min(bmin, (int64_t)a.tilemin[t]);
  }
  if (band) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bmin = min(bmin, (int64_t)__shfl_xor((long long)bmin, o));
    if (lane == 0) s_mn[wid] = bmin;
  }
  const int64_t incl = block_incl_max(run, s_w, lane, wid);  // (its barriers publish s_mn)
  const int64_t excl_thread = (int64_t)__shfl_up((long long)incl, 1);
  const int64_t carry0 = lane == 0 ? (wid > 0 ? (int64_t)s_w[wid - 1] : JMIN) : excl_thread;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t t = (int64_t)tid * 8 + j;
    if (t < nT) a.pmax[t] = max(carry0, loc[j]);
  }
  const int64_t batch_max = max(P, (int64_t)s_w[15]);
  if (wid != 0) return;
  // candidates: grid points g[k] <= batch_max (k < kc), a 64-ary search
  int64_t lo = 0, hi = kc;  // first k with g[k] > batch_max
  while (hi - lo > 64) {
    const int64_t stride = (hi - lo + 63) >> 6;
    const int64_t p = lo + (int64_t)lane * stride;
    const unsigned long long bal = __ballot(p < hi && g[p] > batch_max);
    if (bal == 0) {
      lo = lo + ((hi - 1 - lo) / stride) * stride + 1;
    } else {
      const int f = __ffsll((long long)bal) - 1;
      if (f == 0) {
        hi = lo;
        break;
      }
      const int64_t pf = lo + (int64_t)f * stride;
      lo = pf - stride + 1;
      hi = pf;
    }
  }
  if (hi > lo) {
    const int64_t p = lo + lane;
    const unsigned long long bal = __ballot(p < hi && g[p] > batch_max);
    lo = bal ? lo + __ffsll((long long)bal) - 1 : hi;
  }
  if (lane == 0) {
    int64_t why = 0;
    if (m.late_push != 0 || m.overflow_push != 0) why |= 1;  // a too-late tuple, or one past the grid horizon
    int64_t bm = JMAX;
    if (band)
      for (int w = 0; w < 16; w++) bm = min(bm, (int64_t)s_mn[w]);
    const int64_t cmin = m.cmin, c_old = m.tail - m.head;
    if (q.band_si == -2) {
      // the no-edge band: the plain view's cells reach below the band (the session opened inside a slice), so the
      // tuples themselves must lie at or above its lower end -- the batch minimum from the ingest's tile minima
      if (bm < q.lo_bound) why |= 2;
    } else if (cmin != INT64_MAX) {  // the lowest cell any tuple landed in must start at or above lo_bound
      const int64_t h_end = gcount > 0 ? a.grid[j0 + kc] : JMAX;
      const int64_t cs0 = cmin == 0 && c_old > 0 && m.view_s0_on ? m.view_s0
                          : cmin < c_old ? a.sl.ts[m.head + cmin] : (cmin - c_old < kc ? g[cmin - c_old] : h_end);
      if (cs0 < q.lo_bound) why |= 2;
    }
    if (batch_max > SAFE) why |= 16;
    XQCtl* o = a.ctl;
    o->batch_max = batch_max;
    o->ncand = lo;
    o->why = why;
    if (band) o->batch_min = bm;
  }
}

constexpr int XE_T = 256;                  // threads per edge workgroup
constexpr int XE_PER = 32;                 // consecutive tuples per thread per chunk
constexpr int XE_CHUNK = XE_T * XE_PER;    // 8192 tuples: one tile of a 2^26-tuple batch in one round of loads
constexpr int XE_GRID = 256;               // edge workgroups
constexpr int XE_LIST = 64;                // slow tiles a workgroup can list (>= its share of NT_MAX tiles)
static_assert((NT_MAX + XE_GRID - 1) / XE_GRID <= XE_LIST, "every tile of a workgroup's share fits its list");

// exclusive max over the threads before this one in a 256-thread block; total = the block's max.  s4: LDS [4]
__device__ __forceinline__ int64_t blk_excl_max(int64_t v, long long* s4, int lane, int wid, int64_t& total) {
  int64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = (int64_t)__shfl_up((long long)inc, o);
    if (lane >= o) inc = max(inc, u);
  }
  if (lane == 63) s4[wid] = inc;
  __syncthreads();
  int64_t before = JMIN;
  total = JMIN;
#pragma unroll
  for (int w = 0; w < XE_T / 64; w++) {
    const int64_t x = s4[w];
    if (w < wid) before = max(before, x);
    total = max(total, x);
  }
  int64_t ex = (int64_t)__shfl_up((long long)inc, 1);
  if (lane == 0) ex = JMIN;
  __syncthreads();  // s4 free again
  return max(before, ex);
}

// this thread's XE_PER consecutive tuples of the chunk at base (JMIN at and past e1)
__device__ __forceinline__ void xe_load(const int64_t* ts, int64_t base, int64_t e1, int tid, int64_t (&v)[XE_PER]) {
  const int64_t i0 = base + (int64_t)tid * XE_PER;
  if (i0 + XE_PER <= e1) {
#pragma unroll
    for (int j = 0; j < XE_PER; j++) v[j] = ts[i0 + j];
  } else {
#pragma unroll
    for (int j = 0; j < XE_PER; j++) v[j] = i0 + j < e1 ? ts[i0 + j] : JMIN;
  }
}

// ---- edges (XE_GRID workgroups): (1) no in-order jump by a session gap -- items after a tile's first are below
//      max(carry, first) + gap, the first below carry + gap (carry = running max before the tile); a tile failing
//      the bound (a slow stream: it spans more than a gap of event time) is checked item by item;
//      (2) per candidate grid point g[k], StreamSlicer.determineSlices (S/StreamSlicer.java:55-84; see commit_kernel
//      of slicing_kernels.hip): the in-order tuple e that first reaches g[k] (running max m before it) makes g[k]
//      an edge iff g[k] == nextGrid(m) or e - g[k] < maxLateness; its arrival index is the new slice's cStart /
//      cLast (WindowManager.getCurrentCount at appendSlice, S/SliceManager.java:36).  One workgroup per candidate
//      reads the candidate's arrival tile in one round of loads (spread over the chip instead of one workgroup's
//      chain of loads per candidate).
__global__ __launch_bounds__(XE_T) void xq_edges_kernel(XQArgs a) {
  __shared__ long long s4[XE_T / 64];
  __shared__ int s_list[XE_LIST];
  __shared__ int s_nl;
  __shared__ int s_i[XE_T / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const XQCtl q = *a.ctl;
  if (q.result != XQ_NONE) return;
  const XCfg* cfg = a.cfg;
  const int64_t P = q.p_start, tile = a.tile, nT = (a.n + tile - 1) / tile;
  const int64_t* g = a.grid + a.meta->j0;
  if (cfg->n_ctx > 0) {
    const int64_t gap = q.min_gap;
    const int64_t per = (nT + gridDim.x - 1) / gridDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * per, t1 = min(nT, t0 + per);
    if (tid == 0) s_nl = 0;
    __syncthreads();
    bool bad = false;
    for (int64_t t = t0 + tid; t < t1; t += XE_T) {
      const int64_t carry = t > 0 ? max(P, (int64_t)a.pmax[t - 1]) : P;
      const int64_t f0 = a.ts[t * tile], tm = a.tilemax[t];
      if (!lt_plus(f0, carry, gap)) {
        if (!bad) atomicMin((long long*)&a.ctl->jump_tile, (long long)t);  // t ascends: the thread's first
        bad = true;
      } else if (!lt_plus(tm, max(carry, f0), gap)) {
        s_list[atomicAdd(&s_nl, 1)] = (int)t;
      }
    }
    if (bad) atomicOr((unsigned long long*)&a.ctl->why, 4ull);
    __syncthreads();
    const int nl = s_nl;
    for (int li = 0; li < nl; li++) {
      const int64_t t = s_list[li];
      int64_t r = t > 0 ? max(P, (int64_t)a.pmax[t - 1]) : P;
      const int64_t e1 = min(a.n, (t + 1) * tile);
      bool badi = false;
      for (int64_t base = t * tile; base < e1; base += XE_CHUNK) {
        int64_t v[XE_PER];
        xe_load(a.ts, base, e1, tid, v);
        int64_t tmx = JMIN;
#pragma unroll
        for (int j = 0; j < XE_PER; j++) tmx = max(tmx, v[j]);
        int64_t total;
        int64_t run = max(r, blk_excl_max(tmx, s4, lane, wid, total));
        const int64_t i0 = base + (int64_t)tid * XE_PER;
#pragma unroll
        for (int j = 0; j < XE_PER; j++) {
          if (i0 + j < e1 && !lt_plus(v[j], run, gap)) badi = true;
          run = max(run, v[j]);
        }
        r = max(r, total);
      }
      if (__syncthreads_or(badi) && tid == 0) {
        atomicOr((unsigned long long*)&a.ctl->why, 8ull);
        atomicMin((long long*)&a.ctl->jump_tile, (long long)t);
      }
    }
  }
  const int64_t ncand = a.ctl->ncand;
  const int64_t L = cfg->max_lateness;
  for (int64_t k = blockIdx.x; k < ncand; k += gridDim.x) {
    const int64_t gk = g[k];
    // arrival tile of the first tuple >= gk: the number of tiles whose prefix max is below gk
    int cb = 0;
#pragma unroll 8
    for (int64_t t = tid; t < nT; t += XE_T) cb += a.pmax[t] < gk ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cb += __shfl_xor(cb, o);
    if (lane == 0) s_i[wid] = cb;
    __syncthreads();
    int64_t tk = 0;
#pragma unroll
    for (int w = 0; w < XE_T / 64; w++) tk += s_i[w];
    __syncthreads();
    bool found = false;
    if (tk < nT) {
      int64_t r = tk > 0 ? max(P, (int64_t)a.pmax[tk - 1]) : P;
      const int64_t e1 = min(a.n, (tk + 1) * tile);
      for (int64_t base = tk * tile; base < e1; base += XE_CHUNK) {
        int64_t v[XE_PER];
        xe_load(a.ts, base, e1, tid, v);
        int hit = -1;
        int64_t hv = JMIN, before = JMIN, tmx = JMIN;
#pragma unroll
        for (int j = 0; j < XE_PER; j++) {
          if (hit < 0 && v[j] >= gk) {
            hit = j;
            hv = v[j];
            before = tmx;
          }
          tmx = max(tmx, v[j]);
        }
        int64_t total;
        const int64_t ex = blk_excl_max(tmx, s4, lane, wid, total);
        const unsigned long long bal = __ballot(hit >= 0);
        if (lane == 0) s_i[wid] = bal ? wid * 64 + __ffsll((long long)bal) - 1 : XE_T;
        __syncthreads();
        int win = XE_T;
#pragma unroll
        for (int w = 0; w < XE_T / 64; w++) win = min(win, s_i[w]);
        __syncthreads();
        if (win < XE_T) {
          if (tid == win) {
            const int64_t mm = max(max(r, ex), before);
            const bool emit = k == 0 || g[k - 1] <= mm || (int64_t)((uint64_t)hv - (uint64_t)gk) < L;
            a.flag[k] = emit ? 1 : 0;
            a.epos[k] = base + (int64_t)tid * XE_PER + hit;
          }
          found = true;
          break;
        }
        r = max(r, total);
      }
    }
    if (!found && tid == 0) {  // unreachable: g[k] <= batch_max is reached inside the batch
      a.flag[k] = k == 0 ? 1 : 0;
      a.epos[k] = -1;
    }
  }
}

// ---- commit (1 workgroup): verdict, slice appends, cell fold, operator scalars
__global__ __launch_bounds__(1024) void xq_commit_kernel(XQArgs a) {
  __shared__ long long s_w[32];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  auto stamp = [&](int k) {
    if (a.dbg && tid == 0) a.dbg[k] = (long long)__builtin_amdgcn_s_memtime();
  };
  stamp(0);
  const XQCtl q = *a.ctl;
  if (q.result != XQ_NONE) return;  // refused by the prep kernel: no cell was touched
  const XCfg* cfg = a.cfg;
  const DevMeta& m = *a.meta;
  const int64_t head = m.head, tail = m.tail, j0 = m.j0, gcount = m.gcount, cmin = m.cmin;
  const int64_t c_old = tail - head;
  int64_t kc = gcount > 0 ? gcount - j0 - 1 : 0;
  if (kc < 0) kc = 0;
  const int64_t h_end = gcount > 0 ? a.grid[j0 + kc] : JMAX;
  const int64_t* g = a.grid + j0;
  const int need = cfg->need, vt = cfg->vt;
  const int64_t batch_max = q.batch_max;
  const int64_t ncand = q.ncand;
  const bool fail = q.why != 0;

  // ---- rank = inclusive prefix count of emitted edges
  int64_t n_emit = 0;
  {
    int64_t base_cnt = 0;
    for (int64_t base = 0; base < (fail ? 0 : ncand); base += 1024) {
      const int64_t k = base + tid;
      const bool f = k < ncand && a.flag[k] == 1;
      const unsigned long long bal = __ballot(f);
      const int in_wave = __popcll(bal & ((2ull << lane) - 1));
      if (lane == 0) s_w[wid] = __popcll(bal);
      __syncthreads();
      int64_t before = 0, tot = 0;
      for (int w = 0; w < 16; w++) {
        if (w < wid) before += s_w[w];
        tot += s_w[w];
      }
      if (k < ncand) {
        const int32_t rk = (int32_t)(base_cnt + before + in_wave);
        a.rank[k] = rk;
        if (f) {
          a.eg[rk - 1] = g[k];
          a.epos[ncand + rk - 1] = a.epos[k];  // by rank, behind the per-candidate entries
        }
      }
      base_cnt += tot;
      __syncthreads();
    }
    n_emit = base_cnt;
  }
  int32_t result = XQ_COMMITTED;
  stamp(1);
  if (fail) result = XQ_NOT_QUIET;
  else if (tail + n_emit > cfg->sc) result = XQ_CAPACITY;
  __syncthreads();

  const int64_t ncell = c_old + (result == XQ_COMMITTED ? ncand : kc);
  const int64_t cfirst = min(max(cmin, (int64_t)0), ncell);
  if (result != XQ_COMMITTED) {
    // nothing is committed: every touched cell back to identity; the host runs the event-exact path
    for (int64_t c = cfirst + tid; c < ncell; c += 1024) {
      if (a.c_cnt[c] == 0) continue;
      a.c_cnt[c] = 0;
      a.c_tmax[c] = JMIN;
      a.c_part[0][c] = 0;
      a.c_part[1][c] = (unsigned long long)ID_MIN;
      a.c_part[2][c] = (unsigned long long)ID_MAX;
    }
    if (tid == 0) a.ctl->result = result;
    return;
  }

  // ---- SliceManager.appendSlice (S/SliceManager.java:27-38) for every emitted edge, in order
  const XSlices& sl = a.sl;
  const int64_t c0 = q.c0;
  for (int64_t r = tid; r < n_emit; r += 1024) {
    const int64_t s = tail + r;
    const int64_t e = a.eg[r];
    sl.ts[s] = e;
    sl.te[s] = r + 1 < n_emit ? a.eg[r + 1] : JMAX;
    sl.tl[s] = e;
    sl.tf[s] = JMAX;
    sl.cs[s] = jadd(c0, a.epos[ncand + r]);
    sl.cl[s] = sl.cs[s];
    sl.ty[s] = r + 1 < n_emit ? XTYPE_FIXED : 1;  // the newest slice stays Flexible() until the next append
    sl.cnt[s] = 0;
    sl.p[0][s] = 0;
    sl.p[1][s] = (unsigned long long)ID_MIN;
    sl.p[2][s] = (unsigned long long)ID_MAX;
  }
  if (tid == 0 && n_emit > 0) {
    const int64_t pv = tail - 1;
    sl.te[pv] = a.eg[0];
    sl.ty[pv] = XTYPE_FIXED | (sl.ty[pv] & XTYPE_LAZY);
  }
  __syncthreads();
  stamp(2);
  // ---- cells into slices (AbstractSlice.addElement + AggregateState.addElement), cells back to identity
  for (int64_t c = cfirst + tid; c < ncell; c += 1024) {
    const unsigned long long cnt = a.c_cnt[c];
    if (cnt == 0) continue;
    int64_t s;
    if (c < c_old) {
      s = head + c;
    } else {
      const int32_t rk = a.rank[c - c_old];
      s = rk > 0 ? tail + rk - 1 : tail - 1;
    }
    atomicAdd(&sl.cnt[s], cnt);
    atomicAdd((unsigned long long*)&sl.cl[s], cnt);
    atomicMax((long long*)&sl.tl[s], a.c_tmax[c]);
    if (need & NEED_SUM) {
      if (vt == VT_F64) atomicAdd((double*)&sl.p[0][s], __longlong_as_double((long long)a.c_part[0][c]));
      else atomicAdd(&sl.p[0][s], a.c_part[0][c]);
    }
    if (need & NEED_MIN) atomicMin((long long*)&sl.p[1][s], (long long)a.c_part[1][c]);
    if (need & NEED_MAX) atomicMax((long long*)&sl.p[2][s], (long long)a.c_part[2][c]);
    a.c_cnt[c] = 0;
    a.c_tmax[c] = JMIN;
    a.c_part[0][c] = 0;
    a.c_part[1][c] = (unsigned long long)ID_MIN;
    a.c_part[2][c] = (unsigned long long)ID_MAX;
  }
  stamp(3);
  // ---- scalars: StreamSlicer.maxEventTime / min_next_edge_ts, WindowManager.currentCount, and the last session of
  //      every context extended to the batch max (every in-order tuple is within a gap of it: shiftEnd)
  if (tid == 0) {
    XState s = *a.st;
    s.maxEventTime = batch_max;
    if (cfg->has_fixed) s.nextEdgeTs = g[ncand];
    s.currentCount = jadd(c0, a.n);
    s.tail = (int32_t)(tail + n_emit);
    int64_t band_to = JMAX;
    if (q.band_si >= 0) {
      // start band: the record-low chain of shiftStart modifications in one step (exact_quiet.h) -- the last session
      // starts at the batch minimum, the movable edge between si and si + 1 follows (S/SliceManager.java:101-105),
      // and the order bits as SliceManager.note_order would leave them (exact_op.h check_slice_edges)
      const int64_t si = q.band_si, bm = q.batch_min;
      if (bm < q.band_s) {
        sl.ts[si + 1] = bm;
        sl.te[si] = bm;
        s.unsorted |= 2;
        if (sl.ts[si] > bm) s.unsorted |= 1;
        band_to = bm;
      }
    } else if (q.band_si == -2 && q.batch_min < q.band_s) {
      band_to = q.batch_min;  // no slice edge at the session start: only the start moves
    }
    *a.st = s;
    for (int k = 0; k < cfg->n_ctx; k++) {
      const int ns = s.ns(k);
      int64_t* en_ = a.ss.end + (int64_t)k * cfg->sesscap;
      en_[ns - 1] = max(en_[ns - 1], batch_max);
      if (k == 0 && band_to != JMAX) a.ss.start[ns - 1] = band_to;
    }
    XQCtl* o = a.ctl;
    o->n_emit = n_emit;
    o->rebuild = cfg->has_fixed && (kc - ncand < 1024 || (h_end != JMAX && h_end - batch_max < a.margin)) ? 1 : 0;
    o->result = XQ_COMMITTED;
  }
}

}  // namespace xq

hipError_t launch_xq_prep(const XQArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(xq::xq_prep_kernel, dim3(1), dim3(64), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_xq_commit(const XQArgs& a, hipStream_t st) {
  if ((a.n + a.tile - 1) / a.tile > NT_MAX) return hipErrorInvalidValue;  // the scan holds 8 tiles per thread
  hipLaunchKernelGGL(xq::xq_scan_kernel, dim3(1), dim3(1024), 0, st, a);
  hipLaunchKernelGGL(xq::xq_edges_kernel, dim3(xq::XE_GRID), dim3(xq::XE_T), 0, st, a);
  hipLaunchKernelGGL(xq::xq_commit_kernel, dim3(1), dim3(1024), 0, st, a);
  return hipGetLastError();
}

}  // namespace scotty
