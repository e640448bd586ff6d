// count_engine.cpp -- host side of the count-window path (count_common.h).  The host tracks the count and the
// pending count edge exactly (edges are a function of counts), launches one push as a chain of kernels without
// synchronising, and synchronises once per watermark (count trigger) plus once for the results.
#include "count_engine.h"
#include "host_copy.h"

#include <algorithm>
#include <chrono>
#include <cstring>

namespace scotty {

hipError_t launch_count_push(const CPushArgs& a, int64_t max_points_per_window, int64_t* scan_tmp,
                             long long* premax_tmp, hipStream_t st, hipEvent_t ingest_start, hipEvent_t ingest_end);
hipError_t launch_count_wm_find(const CWmArgs& a, hipStream_t st);
hipError_t launch_count_export(const CPushArgs& a, int64_t* rec, int64_t cap, hipStream_t st);
hipError_t launch_count_shard_commit(const CShardArgs& a, int64_t max_edges, hipStream_t st);
hipError_t launch_count_wm_agg(const CWmArgs& a, int64_t range_blocks, unsigned long long* bsum, hipStream_t st,
                               bool one_wg);
hipError_t launch_count_gc(const CWmArgs& a, hipStream_t st);
hipError_t launch_count_time_edges(const CTimeArgs& a, int64_t* scan_tmp, hipStream_t st);
hipError_t launch_count_rows(const CRowSeg* segs, const int64_t* seg_off, int nseg, int64_t* w_start, int64_t* w_end,
                             int32_t* w_meas, int64_t nw, hipStream_t st);

#define CCHK(x)                                                      \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      err = std::string("HIP: ") + hipGetErrorString(e_) + " at " #x; \
      failed = true;                                                 \
      return SCOTTY_ERR_HIP;                                         \
    }                                                                \
  } while (0)

namespace {
constexpr int64_t JMAX = INT64_MAX, JMIN = INT64_MIN;
constexpr int64_t MAX_PUSH = (int64_t)1 << 28;       // tuples per launch chain (step prefix max: 2 levels)
constexpr int64_t MAX_EDGES_PER_PUSH = (int64_t)1 << 26;
int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
int64_t jmod(int64_t a, int64_t b) { return b == -1 ? 0 : a % b; }
template <typename T>
hipError_t dalloc(T** p, int64_t n) {
  return dev_malloc((void**)p, (size_t)std::max<int64_t>(n, 1) * sizeof(T));  // poisoned under SCOTTY_ALLOC_POISON
}
void dfree(void* p) {
  if (p) (void)hipFree(p);
}
// assignNextWindowStart of a count window (C/windowType/TumblingWindow.java:29-31, SlidingWindow.java:41-43,
// FixedBandWindow.java:37-48): smallest grid point > t
int64_t assign_next(const CWin& w, int64_t t) {
  if (w.kind == SCOTTY_WIN_TUMBLING) return jsub(jadd(t, w.a), jmod(t, w.a));
  if (w.kind == SCOTTY_WIN_SLIDING) return jsub(jadd(t, w.b), jmod(t, w.b));
  if (t == JMAX || t < w.a) return w.a;
  if (t >= w.a && t < jadd(w.a, w.b)) return jadd(w.a, w.b);
  return JMAX;
}
// grid points of w in [lo, hi) (as marked by count_mark_kernel)
int64_t points_in(const CWin& w, int64_t lo, int64_t hi) {
  if (lo >= hi) return 0;
  if (w.kind == SCOTTY_WIN_FIXED_BAND) {
    int64_t c = 0;
    if (w.a > 0 && w.a >= lo && w.a < hi) c++;
    const int64_t e = jadd(w.a, w.b);
    if (e > 0 && e >= lo && e < hi) c++;
    return c;
  }
  const int64_t step = w.kind == SCOTTY_WIN_TUMBLING ? w.a : w.b;
  const int64_t first = lo <= 0 ? step : ((lo + step - 1) / step) * step;
  if (first >= hi) return 0;
  return (hi - 1 - first) / step + 1;
}
}  // namespace

CEngine::~CEngine() {
  (void)hipSetDevice(device);
  if (stream) (void)hipStreamSynchronize(stream);
  dfree(d_meta);
  if (h_meta) (void)hipHostFree(h_meta);
  dfree(d_wins);
  dfree(sl.ts); dfree(sl.tl); dfree(sl.cs); dfree(sl.cnt);
  for (int k = 0; k < NPART; k++) dfree(sl.p[k]);
  if (h_segs) (void)hipHostFree(h_segs);
  dfree(d_segbuf);
  dfree(spare.ts); dfree(spare.tl); dfree(spare.cs); dfree(spare.cnt);
  for (int k = 0; k < NPART; k++) dfree(spare.p[k]);
  dfree(cells.cnt); dfree(cells.tl); dfree(cells.tf); dfree(cells.e_pos); dfree(cells.e_ts);
  for (int k = 0; k < NPART; k++) dfree(cells.p[k]);
  dfree(d_bits); dfree(d_stepc); dfree(d_stepbase); dfree(d_scan); dfree(d_stepmax); dfree(d_steppre);
  dfree(d_stepte); dfree(d_steptp);
  dfree(d_premax);
  dfree(d_wstart); dfree(d_wend); dfree(d_meas); dfree(d_has);
  for (int k = 0; k < SCOTTY_MAX_AGGS; k++) dfree(d_vals[k]);
  dfree(d_pre_cnt); dfree(d_pre_sum); dfree(d_bsum);
  dfree(d_plan);
  dfree(d_cand); dfree(d_cpos); dfree(d_te_pos); dfree(d_te_g); dfree(d_cflag); dfree(d_nte);
  dfree(d_coff); dfree(d_cscan);
  if (h_tmp) (void)hipHostFree(h_tmp);
}

int CEngine::init(int dev, hipStream_t st, int vt_, std::string& e) {
  device = dev;
  stream = st;
  vt = vt_;
  if (dev_malloc((void**)&d_meta, sizeof(CMeta)) != hipSuccess ||
      mapped_host_alloc((void**)&h_meta, (void**)&h_meta_dev, sizeof(CMeta)) != hipSuccess ||
      hipHostMalloc((void**)&h_tmp, 8 * sizeof(int64_t), hipHostMallocDefault) != hipSuccess ||
      dev_malloc((void**)&d_nte, sizeof(unsigned long long)) != hipSuccess) {
    e = "count engine: out of memory";
    return SCOTTY_ERR_NOMEM;
  }
  CMeta m{};
  m.prev_max = JMIN;
  *h_meta = m;
  if (hipMemcpy(d_meta, &m, sizeof(CMeta), hipMemcpyHostToDevice) != hipSuccess) {
    e = "count engine: HIP error";
    return SCOTTY_ERR_HIP;
  }
  return SCOTTY_OK;
}

int CEngine::configure(const std::vector<XWinDef>& ws, const std::vector<int>& ag, int64_t lateness) {
  std::vector<CWin> nw, tw, all;
  int64_t mf = 0;
  for (const XWinDef& w : ws) {
    if (w.kind == SCOTTY_WIN_SESSION)
      return fail(SCOTTY_ERR_UNSUPPORTED, "count path: only context-free windows");
    CWin c{};
    c.kind = w.kind;
    c.measure = w.measure;
    c.a = w.a;
    c.b = w.b;
    (w.measure == SCOTTY_MEASURE_COUNT ? nw : tw).push_back(c);
    all.push_back(c);
    mf = std::max(mf, w.kind == SCOTTY_WIN_FIXED_BAND ? w.b : w.a);  // clearDelay (C/windowType/*.java)
  }
  if (started && tw.size() != twins.size())
    return fail(SCOTTY_ERR_UNSUPPORTED, "count path: time windows added after the first tuple");
  // mid-stream additions: the pending edge keeps its value (StreamSlicer recomputes it only at the next edge)
  wins = nw;
  twins = tw;
  reg = all;
  tstep = 0;  // one common period of every time window (tumbling size / sliding slide), else 0
  for (const CWin& w : tw) {
    const int64_t p = w.kind == SCOTTY_WIN_TUMBLING ? w.a : w.kind == SCOTTY_WIN_SLIDING ? w.b : -1;
    if (p <= 0 || (tstep != 0 && p != tstep)) {
      tstep = 0;
      break;
    }
    tstep = p;
  }
  max_fixed = mf;
  aggs = ag;
  max_lateness = lateness;
  need = 0;
  prefix = !aggs.empty();
  for (int k : aggs) {
    if (k == SCOTTY_AGG_SUM_I32 || k == SCOTTY_AGG_SUM_I64 || k == SCOTTY_AGG_SUM_F64) need |= NEED_SUM;
    if (k == SCOTTY_AGG_MIN_I32 || k == SCOTTY_AGG_MIN_I64 || k == SCOTTY_AGG_MIN_F64) need |= NEED_MIN;
    if (k == SCOTTY_AGG_MAX_I32 || k == SCOTTY_AGG_MAX_I64 || k == SCOTTY_AGG_MAX_F64) need |= NEED_MAX;
    if (k != SCOTTY_AGG_SUM_I32 && k != SCOTTY_AGG_SUM_I64 && k != SCOTTY_AGG_COUNT) prefix = false;
  }
  dfree(d_wins);
  d_wins = nullptr;
  CCHK(dalloc(&d_wins, (int64_t)wins.size()));
  if (!wins.empty())
    CCHK(hipMemcpyAsync(d_wins, wins.data(), wins.size() * sizeof(CWin), hipMemcpyHostToDevice, stream));
  CCHK(hipStreamSynchronize(stream));
  return SCOTTY_OK;
}

int64_t CEngine::next_time_point(int64_t x) const {
  int64_t e = JMAX;
  for (const CWin& w : twins) e = std::min(e, assign_next(w, x));
  return e;
}

// Time edges of an in-order push (StreamSlicer.determineSlices' time branch, S/StreamSlicer.java:46-83): the
// stream's first tuple walks calculateNextFixedEdge as the reference does (Long.MAX_VALUE start, edges < 0 not
// appended, :103-116); after it every union grid point from the pending edge up to the batch max is a candidate
// decided on the device by the first tuple reaching it.  Fills a.te_* (edges in position order).
// Sharded (sh != nullptr): this chunk's part of a global micro-batch.  With maxLateness >= 0 the pending edge after
// a tuple is the first grid point above it, so the first grid point above the max ts before the chunk
// (sh->ts_before) is an edge wherever it is first reached, and the chunk decides exactly the grid points in
// (ts before, chunk max]; the pending edge, maxEventTime and the batch's candidate count (the commit's slice bound)
// are computed identically on every rank from the batch max (sh->ts_last).
int CEngine::time_edges(const int64_t* d_ts, int64_t n, CPushArgs& a, const ShardTime* sh) {
  a.te_pos = nullptr;
  a.te_g = nullptr;
  a.n_te = 0;
  shard_te_bound = 0;
  if (twins.empty() || (sh ? sh->n_total : n) <= 0) return SCOTTY_OK;
  if (max_lateness < 0)
    return fail(SCOTTY_ERR_UNSUPPORTED, "count path with time windows: negative maxLateness");
  int64_t t_first = JMAX, t_last = JMIN;
  if (n > 0) {
    CCHK(hipMemcpyAsync(h_tmp, d_ts, 8, hipMemcpyDeviceToHost, stream));
    CCHK(hipMemcpyAsync(h_tmp + 1, d_ts + n - 1, 8, hipMemcpyDeviceToHost, stream));
    CCHK(hipStreamSynchronize(stream));
    t_first = h_tmp[0];
    t_last = h_tmp[1];
  }
  const int64_t before = sh ? sh->ts_before : JMIN;       // max ts of the batch's tuples before this chunk
  const int64_t batch_last = sh ? sh->ts_last : t_last;  // max ts of the whole batch
  const int64_t stream_first = sh ? sh->ts0 : t_first;   // the stream's first tuple (first batch only)
  const bool first_here = !started && (sh ? sh->n_before == 0 : true) && n > 0;
  if (n > 0 && (t_last < t_first || (started && t_first < h_prev_max) || t_first < before))
    return fail(SCOTTY_ERR_UNSUPPORTED, "count path with time windows: the stream must be in timestamp order "
                                        "(scotty_tune \"count_path\" 1 promises it)");
  std::vector<int64_t> first;  // edges the stream's first tuple appends (position 0)
  int64_t start = 0, prev = std::max(h_prev_max, before);
  int64_t N = t_pending;
  if (!started) {  // every rank replays the first tuple's walk: its pending edge is the batch's first candidate
    const int64_t te = stream_first, L = max_lateness;
    auto calc = [&](int64_t cur_edge) {  // calculateNextFixedEdge(te)
      const int64_t cur = cur_edge == JMIN ? JMAX : cur_edge;
      return next_time_point(std::max(jsub(te, L), cur));
    };
    N = calc(JMIN);
    int guard = 0;
    while (te > N) {
      if (N >= 0) first.push_back(N);
      N = calc(N);
      if (++guard > (1 << 22) || N == JMIN)
        return fail(SCOTTY_ERR_UNSUPPORTED, "the reference StreamSlicer loops forever on this configuration "
                                            "(calculateNextFixedEdge, S/StreamSlicer.java:103-116)");
    }
    if (N == te) {
      first.push_back(N);
      N = calc(N);
    }
    if (first_here) start = 1;
    prev = std::max(prev, te);
  }
  const int64_t nf_all = (int64_t)first.size();
  if (!started) ts_sorted_from = 1 + nf_all;
  if (!first_here) first.clear();
  // union grid from the pending edge up to the batch max: the chunk's candidates are the points in (prev, t_last]
  std::vector<int64_t> cand;
  int64_t n_all = 0, g = N, c0 = 0, nc = 0;
  const int64_t P = tstep;
  const bool arith = P > 0 && N >= 0 && N % P == 0 && batch_last < JMAX - P;
  if (arith) {  // one period (the grid is N + kP): candidates are generated on the device (CTimeArgs.step)
    n_all = batch_last >= N ? (batch_last - N) / P + 1 : 0;
    g = N + n_all * P;
    if (start < n && t_last >= N) {
      const int64_t k_lo = prev >= N ? (prev - N) / P + 1 : 0, k_hi = (t_last - N) / P;
      c0 = N + k_lo * P;
      nc = std::max<int64_t>(0, k_hi - k_lo + 1);
    }
  } else {
    for (; g <= batch_last; g = next_time_point(g)) {
      if (++n_all > ((int64_t)1 << 22))
        return fail(SCOTTY_ERR_UNSUPPORTED, "count path: more than 2^22 time grid points in one micro-batch");
      if (g > prev && start < n && g <= t_last) cand.push_back(g);
      if (next_time_point(g) <= g) {  // JMAX / overflow: no further grid point
        g = next_time_point(g);
        break;
      }
    }
    nc = (int64_t)cand.size();
  }
  if (nc > ((int64_t)1 << 26))
    return fail(SCOTTY_ERR_UNSUPPORTED, "count path: more than 2^26 time grid points in one micro-batch");
  // the pending edge after the batch: the first grid point above its last (maximum) timestamp
  t_pending = n_all > 0 ? g : N;
  h_prev_max = std::max(h_prev_max, batch_last);
  shard_te_bound = nf_all + n_all;
  const int64_t nf = (int64_t)first.size();
  if (nc > tcap) {
    dfree(d_cand); dfree(d_cpos); dfree(d_cflag); dfree(d_coff); dfree(d_cscan);
    tcap = nc + nc / 2 + 1024;
    CCHK(dalloc(&d_cand, tcap));
    CCHK(dalloc(&d_cpos, tcap));
    CCHK(dalloc(&d_cflag, tcap));
    CCHK(dalloc(&d_coff, tcap));
    CCHK(dalloc(&d_cscan, tcap / 512 + 64));
  }
  if (nc + nf > tecap) {
    dfree(d_te_pos); dfree(d_te_g);
    tecap = nc + nf + (nc + nf) / 2 + 1024;
    CCHK(dalloc(&d_te_pos, tecap));
    CCHK(dalloc(&d_te_g, tecap));
  }
  if (nf > 0) {  // (member buffers: the copies may still read them after this call returns)
    h_first_pos.assign(nf, 0);
    h_first_g.assign(first.begin(), first.end());
    CCHK(hipMemcpyAsync(d_te_pos, h_first_pos.data(), nf * 8, hipMemcpyHostToDevice, stream));
    CCHK(hipMemcpyAsync(d_te_g, h_first_g.data(), nf * 8, hipMemcpyHostToDevice, stream));
  }
  int64_t nte = nf;
  if (nc > 0) {
    if (!arith) CCHK(hipMemcpyAsync(d_cand, cand.data(), nc * 8, hipMemcpyHostToDevice, stream));
    CTimeArgs t{};
    t.step = arith ? P : 0;
    t.cand0 = c0;
    t.ts = d_ts;
    t.n = n;
    t.start = start;
    t.prev_max = prev;
    t.lateness = max_lateness;
    t.cand = d_cand;
    t.n_cand = nc;
    t.prev0 = JMIN;
    t.te_pos = d_te_pos + nf;
    t.te_g = d_te_g + nf;
    t.n_te = d_nte;
    t.flag = d_cflag;
    t.off = d_coff;
    t.pos = d_cpos;
    CCHK(launch_count_time_edges(t, d_cscan, stream));
    CCHK(hipMemcpyAsync(h_tmp + 2, d_nte, 8, hipMemcpyDeviceToHost, stream));
    CCHK(hipStreamSynchronize(stream));
    nte += h_tmp[2];
  }
  a.te_pos = d_te_pos;
  a.te_g = d_te_g;
  a.n_te = nte;
  last_nte = nte;
  return SCOTTY_OK;
}

int64_t CEngine::next_point(int64_t x) const {
  int64_t e = JMAX;
  for (const CWin& w : wins) e = std::min(e, assign_next(w, x - 1));
  return e;
}

// slices: keep [head, tail) and room for `need` more; reallocates and moves the retained range to index 0
int CEngine::grow_slices(int64_t need_more) {
  CCHK(hipMemcpyAsync(h_meta, d_meta, sizeof(CMeta), hipMemcpyDeviceToHost, stream));
  CCHK(hipStreamSynchronize(stream));
  const int64_t head = h_meta->head, tail = h_meta->tail, S = tail - head;
  if (tail + need_more <= scap) {
    tail_ub = tail;
    head_lb = head;
    return SCOTTY_OK;
  }
  // steady state: the retained range moves between two buffer sets of the same capacity (no allocation); room
  // for ~8 micro-batches of slices between moves
  int64_t ncap = std::max<int64_t>({(S + need_more) * 8, scap, 4096});
  CSlices n{};
  if (spare_cap >= S + need_more) {
    n = spare;
    ncap = spare_cap;
  } else {
    if (spare_cap) {
      if (h_segs) (void)hipHostFree(h_segs);
  dfree(d_segbuf);
  dfree(spare.ts); dfree(spare.tl); dfree(spare.cs); dfree(spare.cnt);
      for (int k = 0; k < NPART; k++) dfree(spare.p[k]);
    }
    CCHK(dalloc(&n.ts, ncap));
    CCHK(dalloc(&n.tl, ncap));
    CCHK(dalloc(&n.cs, ncap));
    CCHK(dalloc(&n.cnt, ncap));
    for (int k = 0; k < NPART; k++) CCHK(dalloc(&n.p[k], ncap));
  }
  spare = CSlices{};
  spare_cap = 0;
  if (S > 0) {
    CCHK(hipMemcpyAsync(n.ts, sl.ts + head, S * 8, hipMemcpyDeviceToDevice, stream));
    CCHK(hipMemcpyAsync(n.tl, sl.tl + head, S * 8, hipMemcpyDeviceToDevice, stream));
    CCHK(hipMemcpyAsync(n.cs, sl.cs + head, S * 8, hipMemcpyDeviceToDevice, stream));
    CCHK(hipMemcpyAsync(n.cnt, sl.cnt + head, S * 8, hipMemcpyDeviceToDevice, stream));
    for (int k = 0; k < NPART; k++)
      CCHK(hipMemcpyAsync(n.p[k], sl.p[k] + head, S * 8, hipMemcpyDeviceToDevice, stream));
  }
  h_meta->head = 0;
  h_meta->tail = S;
  CCHK(hipMemcpyAsync(d_meta, h_meta, sizeof(CMeta), hipMemcpyHostToDevice, stream));
  CCHK(hipStreamSynchronize(stream));
  if (scap >= ncap / 2 && sl.ts) {  // keep the old set as the next move's target
    spare = sl;
    spare_cap = scap;
  } else {
    dfree(sl.ts); dfree(sl.tl); dfree(sl.cs); dfree(sl.cnt);
    for (int k = 0; k < NPART; k++) dfree(sl.p[k]);
  }
  sl = n;
  scap = ncap;
  tail_ub = S;
  head_lb = 0;
  ts_sorted_from = std::max<int64_t>(0, ts_sorted_from - head);
  return SCOTTY_OK;
}

// edges of counts [lo_count, hi_count) of the stream: the pending edge and every union grid point after it
int64_t CEngine::batch_edges_bound(int64_t lo_count, int64_t hi_count) const {
  int64_t mark_from, b = 0;
  if (pending == JMIN) {
    if (count >= lo_count && count < hi_count) b = 1;
    mark_from = next_point(count + 1);
  } else {
    mark_from = pending;
  }
  const int64_t lo = std::max(lo_count, mark_from);
  for (const CWin& w : wins) b += points_in(w, lo, hi_count);
  return b;
}

// buffers and launch arguments for ingesting counts [C, C + n) (the whole stream's batch or a rank's chunk)
int CEngine::prepare(int64_t C, int64_t n, int64_t range_lo, int64_t range_hi, CPushArgs& a, int64_t& ebound,
                     int64_t& maxp, int64_t n_te) {
  (void)range_lo;
  (void)range_hi;
  int64_t mark_from, extra = -1;
  if (pending == JMIN) {  // the stream's first tuple appends the first slice (S/StreamSlicer.java:37-43)
    extra = count;
    mark_from = next_point(count + 1);
  } else {
    mark_from = pending;
  }
  const int64_t lo = std::max(C, mark_from), hi = C + n;
  ebound = ((extra >= C && extra < hi) ? 1 : 0) + n_te;
  maxp = 0;
  for (const CWin& w : wins) {
    const int64_t p = points_in(w, lo, hi);
    ebound += p;
    maxp = std::max(maxp, p);
  }
  if (ebound > MAX_EDGES_PER_PUSH)
    return fail(SCOTTY_ERR_UNSUPPORTED, "count windows create more than 2^26 slices in one micro-batch");
  const int64_t nwords = (n + 31) / 32, nsteps = (n + CSTEP - 1) / CSTEP;
  if (nwords > bcap) {
    dfree(d_bits);
    bcap = nwords + nwords / 4 + 64;
    CCHK(dalloc(&d_bits, bcap));
  }
  if (nsteps > stcap) {
    dfree(d_stepc); dfree(d_stepbase); dfree(d_scan); dfree(d_stepmax); dfree(d_steppre); dfree(d_premax);
    dfree(d_stepte); dfree(d_steptp);
    stcap = nsteps + nsteps / 4 + 64;
    CCHK(dalloc(&d_stepc, stcap));
    CCHK(dalloc(&d_stepbase, stcap));
    CCHK(dalloc(&d_stepte, stcap + 1));
    CCHK(dalloc(&d_steptp, stcap));
    CCHK(dalloc(&d_scan, stcap / 512 + 64));
    CCHK(dalloc(&d_stepmax, stcap));
    CCHK(dalloc(&d_steppre, stcap));
    CCHK(dalloc(&d_premax, stcap / 1024 + 64));
  }
  if (ebound + 1 > ccap) {
    dfree(cells.cnt); dfree(cells.tl); dfree(cells.tf); dfree(cells.e_pos); dfree(cells.e_ts);
    for (int k = 0; k < NPART; k++) dfree(cells.p[k]);
    ccap = ebound + 1 + (ebound + 1) / 4 + 64;
    CCHK(dalloc(&cells.cnt, ccap));
    CCHK(dalloc(&cells.tl, ccap));
    CCHK(dalloc(&cells.tf, ccap));
    CCHK(dalloc(&cells.e_pos, ccap));
    CCHK(dalloc(&cells.e_ts, ccap));
    for (int k = 0; k < NPART; k++) CCHK(dalloc(&cells.p[k], ccap));
  }
  CCHK(hipMemsetAsync(d_bits, 0, nwords * 4, stream));
  a = CPushArgs{};
  a.n = n;
  a.bits = d_bits;
  a.nwords = nwords;
  a.C = C;
  a.mark_from = mark_from;
  a.extra_point = extra;
  a.wins = d_wins;
  a.n_wins = (int32_t)wins.size();
  a.need = need;
  a.vt = vt;
  a.stepc = d_stepc;
  a.stepbase = d_stepbase;
  a.stepte = d_stepte;
  a.steptp = d_steptp;
  a.stepmax = d_stepmax;
  a.steppre = d_steppre;
  a.nsteps = nsteps;
  a.per_wave = std::max<int64_t>(1, (nsteps + 16383) / 16384);  // ~4096 workgroups of 4 waves
  a.nwaves = (nsteps + a.per_wave - 1) / a.per_wave;
  a.cells = cells;
  a.cell_cap = ebound + 1;
  a.sl = sl;
  a.meta = d_meta;
  return SCOTTY_OK;
}

int CEngine::push(const int64_t* d_ts, const void* d_val, int64_t n, hipEvent_t ev0, hipEvent_t ev1) {
  if (failed) return SCOTTY_ERR_STATE;
  const size_t vb = vt == VT_I32 ? 4 : 8;
  while (n > MAX_PUSH) {  // keep one launch chain within the step prefix-max depth
    int rc = push(d_ts, d_val, MAX_PUSH, nullptr, nullptr);
    if (rc) return rc;
    d_ts += MAX_PUSH;
    d_val = (const unsigned char*)d_val + MAX_PUSH * vb;
    n -= MAX_PUSH;
  }
  if (n <= 0) return SCOTTY_OK;
  CPushArgs ta{};
  const auto h0 = std::chrono::steady_clock::now();
  int rc = time_edges(d_ts, n, ta, nullptr);
  if (rc) return rc;
  last_te_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
  CPushArgs a;
  int64_t ebound = 0, maxp = 0;
  rc = prepare(count, n, count, count + n, a, ebound, maxp, ta.n_te);
  if (rc) return rc;
  a.te_pos = ta.te_pos;
  a.te_g = ta.te_g;
  a.n_te = ta.n_te;
  a.check_sorted = twins.empty() ? 0 : 1;
  if (tail_ub + ebound > scap) {
    rc = grow_slices(ebound);
    if (rc) return rc;
    a.sl = sl;
  }
  a.ts = d_ts;
  a.val = d_val;
  CCHK(launch_count_push(a, maxp, d_scan, d_premax, stream, ev0, ev1));
  count += n;
  pending = (pending != JMIN && pending >= count) ? pending : next_point(count);
  tail_ub += ebound;
  started = true;
  return SCOTTY_OK;
}

int CEngine::shard_push(const int64_t* d_ts, const void* d_val, int64_t n, int64_t ts0, int64_t n_before,
                        int64_t n_total, int64_t ts_before, int64_t ts_last, int64_t* d_rec) {
  if (failed) return SCOTTY_ERR_STATE;
  if (n_total > MAX_PUSH || n < 0 || n_before < 0 || n_before + n > n_total)
    return fail(SCOTTY_ERR_ARG, "shard chunk outside its micro-batch (or micro-batch above 2^28 tuples)");
  shard_total = n_total;
  if (pending == JMIN) shard_ts0 = ts0;
  ShardTime sh{ts0, n_before, n_total, ts_before, ts_last};
  CPushArgs ta{};
  int rc = time_edges(d_ts, n, ta, &sh);
  if (rc) return rc;
  CPushArgs a;
  int64_t ebound = 0, maxp = 0;
  rc = prepare(count + n_before, std::max<int64_t>(n, 1), count, count + n_total, a, ebound, maxp, ta.n_te);
  if (rc) return rc;
  a.te_pos = ta.te_pos;
  a.te_g = ta.te_g;
  a.n_te = ta.n_te;
  a.check_sorted = twins.empty() ? 0 : 1;
  a.n = n;
  a.ts = d_ts;
  a.val = d_val;
  a.shard = 1;
  a.ts0 = shard_ts0;
  if (n > 0) {
    CCHK(launch_count_push(a, maxp, d_scan, d_premax, stream, nullptr, nullptr));
    CCHK(launch_count_export(a, d_rec, shard_cap, stream));
  } else {  // an empty chunk: no tuples, no edges, prefix max -inf
    CCHK(hipStreamSynchronize(stream));  // the previous header copy has read h_shard_hdr
    h_shard_hdr.assign(CSHARD_HDR, 0);
    h_shard_hdr[0] = JMIN;
    h_shard_hdr[4] = a.C;
    CCHK(hipMemsetAsync(d_rec, 0, shard_words() * 8, stream));
    CCHK(hipMemcpyAsync(d_rec, h_shard_hdr.data(), CSHARD_HDR * 8, hipMemcpyHostToDevice, stream));
  }
  if (!shard_async) CCHK(hipStreamSynchronize(stream));  // the record is read by the collective on another stream
  return SCOTTY_OK;
}

int CEngine::shard_commit(const int64_t* d_gathered, int world) {
  if (failed) return SCOTTY_ERR_STATE;
  const int64_t eb = batch_edges_bound(count, count + shard_total) + shard_te_bound;
  if (tail_ub + eb > scap) {
    int rc = grow_slices(eb);
    if (rc) return rc;
  }
  if (world > plan_cap) {
    dfree(d_plan);
    plan_cap = world;
    CCHK(dalloc(&d_plan, 2 * (int64_t)world));
  }
  CShardArgs a{};
  a.gathered = d_gathered;
  a.world = world;
  a.cap = shard_cap;
  a.ts0 = shard_ts0;
  a.vt = vt;
  a.plan = d_plan;
  a.sl = sl;
  a.meta = d_meta;
  CCHK(launch_count_shard_commit(a, std::min(eb, shard_cap), stream));
  count += shard_total;
  pending = (pending != JMIN && pending >= count) ? pending : next_point(count);
  tail_ub += eb;
  started = started || shard_total > 0;
  return SCOTTY_OK;
}

// ContextFreeWindow.triggerWindows of every window in registration order: count windows with (lastCount, cend + 1),
// time windows with (lastWatermark, watermark) (S/WindowManager.java:104-118; C/windowType/TumblingWindow.java:34-39, SlidingWindow.java:50-57,
// FixedBandWindow.java:51-57)
void CEngine::trigger(int64_t last_c, int64_t cur_c, int64_t last_t, int64_t cur_t) {
  rows.clear();
  for (const CWin& w : reg) {
    const bool tm = w.measure == SCOTTY_MEASURE_TIME;
    const int64_t last = tm ? last_t : last_c, cur = tm ? cur_t : cur_c;
    const int32_t ms = w.measure;
    if (w.kind == SCOTTY_WIN_TUMBLING) {
      const int64_t size = w.a;
      const int64_t ls = jsub(last, jmod(jadd(last, size), size));
      for (int64_t s = ls; jadd(s, size) <= cur; s = jadd(s, size)) rows.push_back({s, jadd(s, size), ms});
    } else if (w.kind == SCOTTY_WIN_SLIDING) {
      const int64_t size = w.a, slide = w.b;
      const int64_t ls = jsub(cur, jmod(jadd(cur, slide), slide));
      for (int64_t s = ls; jadd(s, size) > last; s = jsub(s, slide))
        if (s >= 0 && jadd(s, size) <= jadd(cur, 1)) rows.push_back({s, jadd(s, size), ms});
    } else {
      const int64_t e = jadd(w.a, w.b);
      if (last <= e && e <= cur) rows.push_back({w.a, e, ms});
    }
  }
}

// trigger() as arithmetic runs, one per window (rows stay in registration order); false when a bound is too close
// to the int64 range for plain arithmetic (the loop in trigger() then reproduces Java's wrap-around)
bool CEngine::trigger_segs(int64_t last_c, int64_t cur_c, int64_t last_t, int64_t cur_t) {
  constexpr int64_t LIM = (int64_t)1 << 61;
  auto ok = [&](int64_t x) { return x > -LIM && x < LIM; };
  auto cdiv = [](int64_t p, int64_t q) { return (p + q - 1) / q; };  // p > 0, q > 0
  std::vector<CRowSeg> segs;
  segs.reserve(reg.size());
  for (const CWin& w : reg) {
    const bool tm = w.measure == SCOTTY_MEASURE_TIME;
    const int64_t last = tm ? last_t : last_c, cur = tm ? cur_t : cur_c;
    if (!ok(last) || !ok(cur) || !ok(w.a) || !ok(w.b)) return false;
    CRowSeg g{0, 0, 0, 0, w.measure};
    if (w.kind == SCOTTY_WIN_TUMBLING) {  // s = ls + k size while s + size <= cur
      const int64_t size = w.a, ls = last - jmod(last + size, size);
      g.first = ls;
      g.step = size;
      g.size = size;
      g.count = cur - ls - size >= 0 ? (cur - ls - size) / size + 1 : 0;
    } else if (w.kind == SCOTTY_WIN_SLIDING) {  // s = ls - k slide while s + size > last; s >= 0, s + size <= cur + 1
      const int64_t size = w.a, slide = w.b, ls = cur - jmod(cur + slide, slide);
      const int64_t k_end = ls + size > last ? cdiv(ls + size - last, slide) : 0;
      const int64_t k_lo = ls + size - cur - 1 > 0 ? cdiv(ls + size - cur - 1, slide) : 0;
      const int64_t k_hi = std::min(k_end - 1, ls >= 0 ? ls / slide : (int64_t)-1);
      g.first = ls - k_lo * slide;
      g.step = -slide;
      g.size = size;
      g.count = std::max<int64_t>(0, k_hi - k_lo + 1);
    } else {
      const int64_t e = w.a + w.b;
      g.first = w.a;
      g.size = w.b;
      g.count = (last <= e && e <= cur) ? 1 : 0;
    }
    segs.push_back(g);
  }
  nseg = (int)segs.size();
  if (nseg + (nseg + 1) > segcap) {
    if (h_segs) (void)hipHostFree(h_segs);
    dfree(d_segbuf);
    h_segs = nullptr;
    d_segbuf = nullptr;
    segcap = 2 * nseg + 64;
    if (hipHostMalloc((void**)&h_segs, segcap * sizeof(CRowSeg), hipHostMallocDefault) != hipSuccess ||
        dev_malloc(&d_segbuf, segcap * sizeof(CRowSeg)) != hipSuccess) {
      segcap = 0;
      return false;
    }
  }
  (void)hipStreamSynchronize(stream);  // the pinned runs of the previous watermark were read
  int64_t* off = (int64_t*)(h_segs + nseg);
  int64_t o = 0;
  for (int i = 0; i < nseg; i++) {
    h_segs[i] = segs[i];
    off[i] = o;
    o += segs[i].count;
  }
  off[nseg] = o;
  return true;
}

int CEngine::watermark(int64_t wm, XResult& r, bool to_host) {
  r.n = 0;
  r.clear_cols(aggs.size());
  if (failed) return SCOTTY_ERR_STATE;
  // WindowManager.processWatermark (S/WindowManager.java:41-80)
  if (last_wm == -1) last_wm = std::max<int64_t>(0, jsub(wm, max_lateness));
  if (!started) {
    last_wm = wm;
    r.dropped = dropped_;
    return SCOTTY_OK;
  }
  CWmArgs a{};
  a.sl = sl;
  a.meta = d_meta;
  a.wm = wm;
  CCHK(launch_count_wm_find(a, stream));
  CCHK(launch_copy_to_host(d_meta, h_meta_dev, sizeof(CMeta), stream));
  CCHK(hipStreamSynchronize(stream));
  dropped_ = h_meta->late_total;
  r.dropped = dropped_;
  if (h_meta->err & 1)
    return fail(SCOTTY_ERR_UNSUPPORTED,
                "a tuple older than its count slice would be inserted into an earlier LazySlice and shift records "
                "(S/SliceManager.java:64-85): not implemented on the MI355X count path");
  if (h_meta->err & 8)
    return fail(SCOTTY_ERR_UNSUPPORTED, "count path with time windows: a micro-batch was not in timestamp order "
                                        "(scotty_tune \"count_path\" 1 promises an in-order stream)");
  if (h_meta->err & 4)
    return fail(SCOTTY_ERR_NOMEM, "count-path shard record capacity exceeded (scotty_tune \"shard_count_cells\")");
  if (h_meta->err)
    return fail(SCOTTY_ERR_STATE, "internal: count path lost tuples");
  tail_ub = h_meta->tail;
  head_lb = h_meta->head;
  if (h_meta->wm_status == 1) {
    last_wm = wm;
    return SCOTTY_OK;
  }
  if (last_wm < h_meta->oldest) last_wm = h_meta->oldest;
  if (h_meta->wm_status == 2) {
    err = "processWatermark threw IndexOutOfBoundsException (count trigger: watermark before the oldest slice, "
          "S/WindowManager.java:109-112)";
    return SCOTTY_ERR_INDEX;
  }
  const bool segs = trigger_segs(last_count, jadd(h_meta->cend, 1), last_wm, wm);
  if (!segs) trigger(last_count, jadd(h_meta->cend, 1), last_wm, wm);
  int64_t nw = 0;
  int64_t min_c = count, max_c = 0, min_t = JMAX, max_t = 0;  // S/WindowManager.java:61-71
  auto bound = [&](int32_t meas, int64_t st, int64_t en) {
    if (meas == SCOTTY_MEASURE_TIME) {
      min_t = std::min(min_t, st);
      max_t = std::max(max_t, en);
    } else {
      min_c = std::min(min_c, st);
      max_c = std::max(max_c, en);
    }
  };
  if (segs) {
    for (int i = 0; i < nseg; i++) {
      const CRowSeg& g = h_segs[i];
      if (g.count == 0) continue;
      const int64_t s_a = g.first, s_b = g.first + (g.count - 1) * g.step;
      bound((int32_t)g.meas, std::min(s_a, s_b), std::max(s_a, s_b) + g.size);
    }
    nw = ((int64_t*)(h_segs + nseg))[nseg];
  } else {
    for (const Row& w : rows) bound(w.meas, w.start, w.end);
    nw = (int64_t)rows.size();
  }
  if (nw > wcap) {
    dfree(d_wstart); dfree(d_wend); dfree(d_meas); dfree(d_has);
    for (int k = 0; k < SCOTTY_MAX_AGGS; k++) {
      dfree(d_vals[k]);
      d_vals[k] = nullptr;
    }
    wcap = nw + nw / 2 + 1024;
    CCHK(dalloc(&d_wstart, wcap));
    CCHK(dalloc(&d_wend, wcap));
    CCHK(dalloc(&d_meas, wcap));
    CCHK(dalloc(&d_has, wcap));
    for (size_t k = 0; k < aggs.size(); k++) CCHK(dalloc(&d_vals[k], wcap));
  }
  const int64_t S_ub = tail_ub - head_lb + 2;
  if (prefix && S_ub > pcap) {
    dfree(d_pre_cnt); dfree(d_pre_sum); dfree(d_bsum);
    pcap = S_ub + S_ub / 2 + 1024;
    CCHK(dalloc(&d_pre_cnt, pcap));
    CCHK(dalloc(&d_pre_sum, pcap));
    CCHK(dalloc(&d_bsum, 2 * (pcap / 1024 + 2)));
  }
  if (segs) {  // rows generated on the device from the runs
    if (nw > 0) {
      CCHK(hipMemcpyAsync(d_segbuf, h_segs, nseg * sizeof(CRowSeg) + (nseg + 1) * 8, hipMemcpyHostToDevice, stream));
      CCHK(launch_count_rows((const CRowSeg*)d_segbuf, (const int64_t*)((CRowSeg*)d_segbuf + nseg), nseg, d_wstart,
                             d_wend, d_meas, nw, stream));
    }
  } else {
    h_start.resize(nw);
    h_end.resize(nw);
    h_meas.resize(nw);
    for (int64_t i = 0; i < nw; i++) {
      h_start[i] = rows[i].start;
      h_end[i] = rows[i].end;
      h_meas[i] = rows[i].meas;
    }
    if (nw > 0) {
      CCHK(hipMemcpyAsync(d_wstart, h_start.data(), nw * 8, hipMemcpyHostToDevice, stream));
      CCHK(hipMemcpyAsync(d_wend, h_end.data(), nw * 8, hipMemcpyHostToDevice, stream));
      CCHK(hipMemcpyAsync(d_meas, h_meas.data(), nw * 4, hipMemcpyHostToDevice, stream));
    }
  }
  a.min_count = min_c;
  a.max_count = max_c;
  a.min_ts = min_t;
  a.max_ts = max_t;
  a.ts_sorted_from = ts_sorted_from;
  a.w_meas = d_meas;
  a.gc_before = jsub(jsub(wm, max_lateness), max_fixed);
  a.w_start = d_wstart;
  a.w_end = d_wend;
  a.nw = nw;
  a.need = need;
  a.vt = vt;
  a.n_aggs = (int32_t)aggs.size();
  a.prefix = prefix ? 1 : 0;
  for (size_t k = 0; k < aggs.size(); k++) {
    a.agg_kind[k] = aggs[k];
    a.values[k] = d_vals[k];
  }
  a.pre_cnt = d_pre_cnt;
  a.pre_sum = d_pre_sum;
  a.has_value = d_has;
  // LazyAggregateStore.aggregate runs only with windows (S/WindowManager.java:73-75), then clearAfterWatermark(wm -
  // maxLateness) (:82-95) -- which the GC kernel skips when the aggregation's range check threw; the host learns
  // that at the one synchronisation below, with the result copies
  if (nw > 0) CCHK(launch_count_wm_agg(a, (S_ub + 1023) / 1024 + 1, d_bsum, stream, prefix_one));
  CCHK(launch_count_gc(a, stream));
  if (nw > 0) CCHK(launch_copy_to_host(d_meta, h_meta_dev, sizeof(CMeta), stream));
  r.n = nw;
  r.d_start = d_wstart;
  r.d_end = d_wend;
  r.d_meas = d_meas;
  r.d_key = nullptr;
  r.d_has = d_has;
  for (size_t k = 0; k < aggs.size(); k++) r.d_vals[k] = d_vals[k];
  if (to_host && nw > 0) {
    if (segs) {
      r.start.resize(nw);
      r.end.resize(nw);
      r.meas.resize(nw);
      CCHK(hipMemcpyAsync(r.start.data(), d_wstart, nw * 8, hipMemcpyDeviceToHost, stream));
      CCHK(hipMemcpyAsync(r.end.data(), d_wend, nw * 8, hipMemcpyDeviceToHost, stream));
      CCHK(hipMemcpyAsync(r.meas.data(), d_meas, nw * 4, hipMemcpyDeviceToHost, stream));
    } else {
      r.start.assign(h_start.begin(), h_start.end());
      r.end.assign(h_end.begin(), h_end.end());
      r.meas.assign(h_meas.begin(), h_meas.end());
    }
    r.has.resize(nw);
    for (size_t k = 0; k < aggs.size(); k++) r.vals[k].resize(nw);
    CCHK(hipMemcpyAsync(r.has.data(), d_has, nw, hipMemcpyDeviceToHost, stream));
    for (size_t k = 0; k < aggs.size(); k++)
      CCHK(hipMemcpyAsync(r.vals[k].data(), d_vals[k], nw * 8, hipMemcpyDeviceToHost, stream));
  }
  CCHK(hipStreamSynchronize(stream));
  if (nw > 0 && h_meta->range_err) {
    r.n = 0;
    err = "processWatermark threw IndexOutOfBoundsException (LazyAggregateStore.aggregate: a window starts before "
          "the oldest retained slice, S/aggregationstore/LazyAggregateStore.java:83-90)";
    return SCOTTY_ERR_INDEX;
  }
  last_wm = wm;
  last_count = count;
  return SCOTTY_OK;
}

int64_t CEngine::slice_count() {
  if (hipMemcpyAsync(h_meta, d_meta, sizeof(CMeta), hipMemcpyDeviceToHost, stream) != hipSuccess) return -1;
  if (hipStreamSynchronize(stream) != hipSuccess) return -1;
  return h_meta->tail - h_meta->head;
}

}  // namespace scotty
