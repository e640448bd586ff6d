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
      int64_t lo = 0, hi = a.gcount;  // first grid entry >= N
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.grid[mid] < N) lo = mid + 1; else hi = mid;
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
    }
  }
  if (res == XQ_NONE) {
    if (!(s.unsorted & 1)) {
      // sorted list: the oldest slice bounds every tuple (an older one throws IndexOutOfBounds; the ingest counts it)
      lo_bound = max(lo_bound, a.sl.ts[s.head]);
    } else {
      // a list whose tStart order was broken by session edits: every tuple of a quiet batch is >= lo_bound, and
      // findSliceIndexByTimestamp (the LAST slice with tStart <= t, LazyAggregateStore.java:29-37) then lands in the
      // suffix that starts at the last slice with tStart <= lo_bound -- if that suffix is sorted, it is the view
      constexpr int64_t SCAN_CAP = 16384;
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
    if (__ballot(lane < a.n && v != JMIN && !(ex <= JMAX - min_gap && v < ex + min_gap)) != 0) {
      res = XQ_NOT_QUIET;
      why |= 4;
    }
  }
  if (lane == 0) {
    DevMeta m{};
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
    *a.ctl = q;
  }
}

__device__ __forceinline__ int64_t lower_bound_lds(const long long* p, int64_t n, int64_t x) {  // first p[i] >= x
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (p[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// block-wide (1024 threads) inclusive max scan; wtot: LDS [16]
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

__global__ __launch_bounds__(1024) void xq_commit_kernel(XQArgs a) {
  __shared__ long long s_p[NT_MAX];  // tile maxima -> prefix maxima (arrival order)
  __shared__ long long s_w[32];
  __shared__ int64_t sc[8];
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
  const int64_t P = q.p_start;
  const int64_t c_old = tail - head;
  int64_t kc = gcount > 0 ? gcount - j0 - 1 : 0;
  if (kc < 0) kc = 0;
  const int64_t h_end = gcount > 0 ? a.grid[j0 + kc] : JMAX;
  const int64_t* g = a.grid + j0;
  const int64_t L = cfg->max_lateness;
  const int64_t tile = a.tile;
  const int64_t nT = (a.n + tile - 1) / tile;
  const int need = cfg->need, vt = cfg->vt;

  // ---- prefix max over the tile maxima (8 consecutive tiles per thread)
  int64_t loc[8];
  int64_t run = JMIN;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t t = (int64_t)tid * 8 + j;
    run = max(run, t < nT ? (int64_t)a.tilemax[t] : JMIN);
    loc[j] = run;
  }
  const int64_t incl = block_incl_max(run, s_w, lane, wid);
  const int64_t excl_thread = (int64_t)__shfl_up((long long)incl, 1);
  const int64_t carry0 = lane == 0 ? (wid > 0 ? (int64_t)s_w[wid - 1] : JMIN) : excl_thread;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t t = (int64_t)tid * 8 + j;
    if (t < nT) s_p[t] = max(carry0, loc[j]);
  }
  __syncthreads();
  const int64_t batch_max = max(P, nT > 0 ? (int64_t)s_p[nT - 1] : JMIN);
  stamp(1);

  // ---- quiet verdict
  bool fail = false;
  __shared__ int s_why;
  if (tid == 0) {
    int why = 0;
    if (m.late_push != 0 || m.overflow_push != 0) why |= 1;  // a too-late tuple, or one past the grid horizon
    if (cmin != INT64_MAX) {  // the lowest cell any tuple landed in must start at or above lo_bound
      const int64_t cs0 = cmin < c_old ? a.sl.ts[head + cmin] : (cmin - c_old < kc ? g[cmin - c_old] : h_end);
      if (cs0 < q.lo_bound) why |= 2;
    }
    if (batch_max > SAFE) why |= 16;
    s_why = why;
    fail = why != 0;
  }
  __shared__ int s_nscan;
  __shared__ int s_scan[64];
  if (tid == 0) s_nscan = 0;
  __syncthreads();
  if (cfg->n_ctx > 0) {
    // no in-order jump by a gap: items after a tile's first are below max(carry, first) + gap; the first is below
    // carry + gap (carry = running max before the tile).  A tile failing this bound (a slow stream: the tile spans
    // more than a gap of event time) is checked item by item below.
    for (int64_t t = tid; t < nT; t += 1024) {
      const int64_t carry = t > 0 ? max(P, (int64_t)s_p[t - 1]) : P;
      const int64_t t0 = a.ts[t * tile], tm = a.tilemax[t];
      if (!lt_plus(t0, carry, q.min_gap)) {
        fail = true;
        atomicOr(&s_why, 4);
      } else if (!lt_plus(tm, max(carry, t0), q.min_gap)) {
        const int i = atomicAdd(&s_nscan, 1);
        if (i < 64) s_scan[i] = (int)t;
        else {
          fail = true;
          atomicOr(&s_why, 8);
        }
      }
    }
  }
  fail = __syncthreads_or(fail);
  if (!fail && s_nscan > 0) {
    // exact test of the listed tiles: every item below (running max before it) + gap, one wave per tile
    const int nscan = s_nscan;
    for (int i = wid; i < nscan; i += 16) {
      const int64_t t = s_scan[i];
      int64_t run_ = t > 0 ? max(P, (int64_t)s_p[t - 1]) : P;
      const int64_t e0 = t * tile, e1 = min(a.n, e0 + tile);
      bool bad = false;
      for (int64_t base = e0; base < e1 && !bad; base += 64) {
        const int64_t idx = base + lane;
        const int64_t v = idx < e1 ? a.ts[idx] : JMIN;
        int64_t inc = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int64_t u = (int64_t)__shfl_up((long long)inc, o);
          if (lane >= o) inc = max(inc, u);
        }
        int64_t ex = (int64_t)__shfl_up((long long)inc, 1);
        if (lane == 0) ex = JMIN;
        ex = max(ex, run_);
        bad = __ballot(idx < e1 && !lt_plus(v, ex, q.min_gap)) != 0;
        run_ = max(run_, rl64(inc, 63));
      }
      if (bad) {
        fail = true;
        atomicOr(&s_why, 8);
      }
    }
    fail = __syncthreads_or(fail);
  }

  stamp(2);
  // ---- candidates: grid points g[k] <= batch_max (k < kc)
  if (wid == 0) {
    int64_t lo = 0, hi = fail ? 0 : kc;  // first k with g[k] > batch_max
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
    if (lane == 0) sc[0] = lo;
  }
  __syncthreads();
  const int64_t ncand = sc[0];
  stamp(3);

  // ---- edge decision (StreamSlicer.determineSlices, S/StreamSlicer.java:55-84; see commit_kernel): a grid point g
  //      first reached by the in-order tuple e (running max m before it) becomes an edge iff g == nextGrid(m) or
  //      e - g < maxLateness.  Every candidate's first-reaching tuple is located in its tile by one wave (its arrival
  //      index is the new slice's cStart / cLast: WindowManager.getCurrentCount at appendSlice, S/SliceManager.java:36).
  for (int64_t k = wid; k < ncand; k += 16) {
    const int64_t gk = g[k];
    const int64_t ts_ = lower_bound_lds(s_p, nT, gk);
    int64_t r = ts_ > 0 ? max(P, (int64_t)s_p[ts_ - 1]) : P;
    const int64_t e0 = ts_ * tile, e1 = min(a.n, e0 + tile);
    int64_t e = JMIN, mm = JMIN, pos = -1;
    constexpr int B = 16;
    for (int64_t base = e0; base < e1 && pos < 0; base += 64 * B) {
      int64_t v[B];
#pragma unroll
      for (int j = 0; j < B; j++) {
        const int64_t i = base + j * 64 + lane;
        v[j] = i < e1 ? a.ts[i] : JMIN;
      }
      int jf = -1;  // first of the B rows holding a tuple >= gk (wave-uniform)
      unsigned long long hf = 0;
      int64_t vf = JMIN;
#pragma unroll
      for (int j = 0; j < B; j++) {
        const unsigned long long hit = __ballot(v[j] >= gk);
        if (jf < 0) {
          if (hit) {
            jf = j;
            hf = hit;
            vf = v[j];
          } else {
            r = max(r, wmax(v[j]));
          }
        }
      }
      if (jf >= 0) {
        const int f = __ffsll((long long)hf) - 1;
        e = rl64(vf, f);
        mm = max(r, wmax(lane < f ? vf : JMIN));
        pos = base + jf * 64 + f;
      }
    }
    if (lane == 0) {
      const bool emit = k == 0 || g[k - 1] <= mm || (int64_t)((uint64_t)e - (uint64_t)gk) < L;
      a.flag[k] = emit ? 1 : 0;
      a.epos[k] = pos;
    }
  }
  __syncthreads();

  stamp(4);
  // ---- rank = inclusive prefix count of emitted edges
  int64_t n_emit = 0;
  {
    int64_t base_cnt = 0;
    for (int64_t base = 0; base < ncand; base += 1024) {
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
  stamp(5);
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
    if (tid == 0) {
      a.ctl->result = result;
      a.ctl->why = s_why;
    }
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
  stamp(6);
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
  stamp(7);
  // ---- scalars: StreamSlicer.maxEventTime / min_next_edge_ts, WindowManager.currentCount, and the last session of
  //      every context extended to the batch max (every in-order tuple is within a gap of it: shiftEnd)
  if (tid == 0) {
    XState s = *a.st;
    s.maxEventTime = batch_max;
    if (cfg->has_fixed) s.nextEdgeTs = g[ncand];
    s.currentCount = jadd(c0, a.n);
    s.tail = (int32_t)(tail + n_emit);
    *a.st = s;
    for (int k = 0; k < cfg->n_ctx; k++) {
      const int ns = s.ns(k);
      int64_t* en_ = a.ss.end + (int64_t)k * cfg->sesscap;
      en_[ns - 1] = max(en_[ns - 1], batch_max);
    }
    XQCtl* o = a.ctl;
    o->n_emit = n_emit;
    o->batch_max = batch_max;
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
  hipLaunchKernelGGL(xq::xq_commit_kernel, dim3(1), dim3(1024), 0, st, a);
  return hipGetLastError();
}

}  // namespace scotty
