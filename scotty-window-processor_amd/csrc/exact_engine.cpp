// exact_engine.cpp -- host side of the exact ("replay") engine: operator table, keyed batching, watermark
// result assembly.  Per-tuple work runs only in gfx950 kernels (exact_kernels.hip, keyed_kernels.hip);
// the host sequences launches on the op's stream and owns the window/function configuration, like the
// reference's WindowManager registration (S/WindowManager.java:121-151).
#include "exact_batch.h"
#include "exact_engine.h"
#include "dev_alloc.h"
#include "exact_quiet.h"
#include "host_copy.h"
#include "keyed_grid.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstddef>
#include <cstring>
#include <queue>

namespace scotty {
hipError_t launch_replay(const XBatchArgs& a, int vt, hipStream_t st);
hipError_t launch_wm_count(const XWmArgs& a, hipStream_t st);
hipError_t launch_wm_emit(const XWmArgs& a, hipStream_t st);
hipError_t launch_wm_agg(const XWmArgs& a, hipStream_t st, int group);
hipError_t launch_wm_blocks(const XWmArgs& a, hipStream_t st);
hipError_t launch_lane_replay(const XBatchArgs& a, const XCfg& host_cfg, hipStream_t st);
hipError_t launch_lane_session(const XBatchArgs& a, int vt, int occ, hipStream_t st);
hipError_t launch_lane_count(const XBatchArgs& a, int vt, hipStream_t st);  // keyed_lane_count.hip
hipError_t launch_lane_wm_count(const XWmArgs& a, hipStream_t st);
hipError_t launch_lane_wm_emit(const XWmArgs& a, bool agg, hipStream_t st);
hipError_t launch_xstate_init(XState* st_, int64_t from, int64_t to, const uint32_t* slot_key, hipStream_t st);
hipError_t launch_scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t st);
hipError_t launch_key_insert(const uint32_t* keys, int64_t n, unsigned long long* table, uint64_t mask,
                             uint32_t* new_pos, unsigned long long* new_count, int32_t* full, uint32_t* slot,
                             hipStream_t st);
hipError_t launch_key_assign(unsigned long long* table, const uint32_t* new_pos, int64_t n_new, int64_t base,
                             uint32_t* slot_key, hipStream_t st);
hipError_t launch_rehash(const unsigned long long* old_t, uint64_t old_n, unsigned long long* nt, uint64_t mask, int drop_new,
                         hipStream_t st);
hipError_t launch_slot(const uint32_t* keys, int64_t n, const unsigned long long* table, uint64_t mask,
                       uint32_t* slot, bool fixup, hipStream_t st);
hipError_t launch_sort_by_slot(int rec, const int64_t* ts, const void* val, const uint32_t* slot, int64_t n,
                               int slot_bits, void* bufA, void* bufB, int32_t* hist, int32_t* hist10,
                               int32_t* scan_tmp, void** result, hipStream_t st, int64_t tbase, int tb, bool hist0,
                               int digit10);
hipError_t launch_range_hist(const uint32_t* keys, const int64_t* ts, int64_t n, int32_t* hist, int32_t* hist10,
                             unsigned long long* part, unsigned long long* range, hipStream_t st);
int64_t seg_tiles(int64_t n);
hipError_t launch_seg_count(int rec, const void* recs, int64_t n, int32_t* cnt, long long* tmax_tile,
                            unsigned long long* tmax_b, hipStream_t st, int64_t tbase, int tb);
hipError_t launch_seg_write(int rec, const void* recs, int64_t n, const int32_t* off, uint32_t* ukey, int64_t* ubeg,
                            hipStream_t st, int64_t tbase, int tb);
hipError_t launch_seg_fill(const int64_t* ubeg, const uint32_t* uslot, int64_t u_n, int64_t n, int64_t* seg_begin,
                           int64_t* seg_end, hipStream_t st);
int64_t sort_tile();
hipError_t launch_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* tmp, hipStream_t st);
hipError_t launch_kg_build(const uint32_t* slot_key, int64_t n_ops, unsigned long long* tab, uint64_t mask,
                           hipStream_t st);
hipError_t launch_kg_partition(const KgArgs& a, int vt, hipStream_t st);
hipError_t launch_kg_scatter(const KgArgs& a, int vt, hipStream_t st);
hipError_t launch_kg_bucket(const KgArgs& a, int vt, bool mm, int64_t n_ops, hipStream_t st, int which);
hipError_t launch_kg_mark_deferred(const KgArgs& a, hipStream_t st);
int kg_tile(int vt, int64_t nbk, int variant);
int kg_cells(bool mm);
hipError_t launch_kg_bounds(const int64_t* ts, int64_t n, const XCfg* cfg, int kmax, int64_t* gpts, int64_t* out,
                            hipStream_t st);
hipError_t launch_kg_dcount(const uint8_t* mark, int64_t n, int32_t* blk, hipStream_t st);
hipError_t launch_cix_build(const IngestArgs& a, hipStream_t st);
hipError_t launch_ingest(const IngestArgs& a, int vt, int need, int64_t nblocks, hipStream_t st, int mode);
int ingest_wgs_per_cu(int vt, int need);
hipError_t launch_fill_u64(unsigned long long* p, int64_t n, unsigned long long v, hipStream_t st);
hipError_t launch_kg_dgather(const uint32_t* key, const int64_t* ts, const void* val, uint8_t* mark, int64_t n,
                             const int32_t* blk_off, uint32_t* okey, int64_t* ots, void* oval, int vt,
                             hipStream_t st);
}  // namespace scotty


namespace scotty {

#define XCHK(expr)                                                         \
  do {                                                                     \
    hipError_t _e = (expr);                                                \
    if (_e != hipSuccess) {                                                \
      err = std::string(#expr ": ") + hipGetErrorString(_e);               \
      failed = true;                                                       \
      return SCOTTY_ERR_HIP;                                               \
    }                                                                      \
  } while (0)

namespace {
// device allocation.  Every buffer is written by the engine before any kernel reads it (state explicitly
// initialised, scratch written by the producing kernel of the same launch chain); the zero fill is defence in
// depth only.  SCOTTY_ALLOC_POISON (dev_alloc.h) replaces it by a poison byte to check exactly that.
template <typename T>
hipError_t dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void**)p, count * sizeof(T));
  if (e != hipSuccess) return e;
  const int pb = alloc_poison();
  return dev_fill_sync(*p, pb >= 0 ? pb : 0, count * sizeof(T));
}
void dfree(void* p) {
  if (p) (void)hipFree(p);
}
int agg_need(int kind) {
  switch (kind) {
    case SCOTTY_AGG_SUM_I32: case SCOTTY_AGG_SUM_I64: case SCOTTY_AGG_SUM_F64: return NEED_SUM;
    case SCOTTY_AGG_MIN_I32: case SCOTTY_AGG_MIN_I64: case SCOTTY_AGG_MIN_F64: return NEED_MIN;
    case SCOTTY_AGG_MAX_I32: case SCOTTY_AGG_MAX_I64: case SCOTTY_AGG_MAX_F64: return NEED_MAX;
    default: return 0;
  }
}
int bits_for(int64_t n) {  // bits to represent n-1
  int b = 0;
  while (b < 40 && ((int64_t)1 << b) < n) b++;
  return b;
}
}  // namespace

XEngine::~XEngine() { release(); }

void XEngine::release() {
  dfree(d_cfg); dfree(d_cf_kind); dfree(d_cf_meas); dfree(d_cf_a); dfree(d_cf_b);
  dfree(d_st);
  dfree(sl.ts); dfree(sl.te); dfree(sl.tl); dfree(sl.tf); dfree(sl.cs); dfree(sl.cl); dfree(sl.ty); dfree(sl.cnt);
  dfree(sl.pc); dfree(sl.ps); dfree(sl.kw);
  for (int k = 0; k < NPART; k++) dfree(sl.p[k]);
  dfree(sl.rlo); dfree(sl.rhi); dfree(sl.nn); dfree(sl.rts); dfree(sl.rv);
  dfree(ss.start); dfree(ss.end);
  dfree(d_lsdbg);
  dfree(d_need); dfree(d_table); dfree(d_newpos); dfree(d_newcnt); dfree(d_full); dfree(d_slot_key);
  dfree(d_slot); dfree(d_recA); dfree(d_recB); dfree(d_hist); dfree(d_scan32); dfree(d_seg_b); dfree(d_seg_e);
  dfree(d_rpart);
  dfree(d_ukey); dfree(d_ubeg); dfree(d_segcnt); dfree(d_segoff); dfree(d_segscan); dfree(d_tmaxt); dfree(d_kmax);
  dfree(d_wcount); dfree(d_woff); dfree(d_scan64); dfree(d_misc);
  dfree(d_w_start); dfree(d_w_end); dfree(d_w_meas); dfree(d_w_op); dfree(d_w_key); dfree(d_has);
  for (int k = 0; k < SCOTTY_MAX_AGGS; k++) dfree(d_vals[k]);
  if (h_misc) (void)hipHostFree(h_misc);
  dfree(xb_snap); dfree(xb_ctl); dfree(xb_reach); dfree(xb_tmax); dfree(xb_pcarry); dfree(xb_segtail);
  dfree(xb_tjump); dfree(xb_tmin);
  dfree(xb_mcarry); dfree(xb_nscnt); dfree(xb_nstot); dfree(xb_nsstart); dfree(xb_nspb); dfree(xb_evcnt);
  dfree(xb_seghas); dfree(xb_bits); dfree(xb_evpos); dfree(xb_evt); dfree(xb_evv); dfree(xb_eppos);
  dfree(xb_evm); dfree(xb_eptail); dfree(xb_sufmin);
  dfree(d_xq_grid); dfree(d_xq_ccnt); dfree(d_xq_ctmax); dfree(d_xq_tilemax); dfree(d_xq_tilemin); dfree(d_xq_pmax); dfree(d_xq_rank); dfree(d_xq_flag);
  for (int k = 0; k < NPART; k++) dfree(d_xq_cpart[k]);
  dfree(d_xq_eg); dfree(d_xq_epos); dfree(d_xq_meta); dfree(d_xq_cix); dfree(d_xq_cixmeta); dfree(d_xq_ctl);
  dfree(d_dbg);
  d_dbg = nullptr;
  dfree(xblk.cnt); dfree(xblk.sum); dfree(xblk.mn); dfree(xblk.mx); dfree(xblk.ts_min); dfree(xblk.tl_max);
  xblk = XBlocks{};
  xblk_cap = 0;
  for (auto& e : ev_pending) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
  for (auto& e : ev_pool) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
  ev_pending.clear();
  ev_pool.clear();
  dfree(d_kgtab); dfree(d_kghist); dfree(d_kgscan); dfree(d_kgblk); dfree(d_kgrec); dfree(d_kgmark); dfree(d_kgctl);
  dfree(d_kgkey); dfree(d_kgts); dfree(d_kgval); dfree(d_kggpts); dfree(d_kgpos); dfree(d_kgpart); dfree(d_kgdflag);
  if (h_kgctl) (void)hipHostFree(h_kgctl);
  h_kgctl = nullptr;
  d_cfg = nullptr;
  d_st = nullptr;
  h_misc = nullptr;
}

int XEngine::init(int dev, hipStream_t st, int value_type, bool is_keyed, std::string& e_out) {
  device = dev;
  stream = st;
  vt = value_type;
  keyed = is_keyed;
  (void)e_out;
  XCHK(dalloc(&d_cfg, 1));
  XCHK(dalloc(&d_misc, 8));
  XCHK(mapped_host_alloc((void**)&h_misc, (void**)&h_misc_dev, 16 * sizeof(int64_t)));
  XCHK(dalloc(&d_newcnt, 1));
  XCHK(dalloc(&d_full, 1));
  XCHK(dalloc(&d_need, 4));
  return SCOTTY_OK;
}

// WindowManager.addWindowAssigner / addAggregation / setMaxLateness (S/WindowManager.java:121-202)
int XEngine::configure(const std::vector<XWinDef>& wins, const std::vector<int>& aggs, int64_t max_lateness,
                       const std::vector<int>& agg_inv) {
  h_wins = wins;
  XCfg c{};
  std::vector<int32_t> kind, meas;
  std::vector<int64_t> a, b;
  int nctx = 0;
  bool has_ctx = false, session_case = false;
  int64_t max_fixed = 0;
  for (const XWinDef& w : wins) {
    if (w.kind == SCOTTY_WIN_SESSION) {
      if (nctx >= XMAXCTX) {
        err = "more than 4 session windows per operator are not supported on the MI355X path";
        return SCOTTY_ERR_UNSUPPORTED;
      }
      session_case = !has_ctx || session_case;
      has_ctx = true;
      c.gap[nctx] = w.a;
      c.ctx_measure[nctx] = w.measure;
      nctx++;
    } else {
      kind.push_back(w.kind);
      meas.push_back(w.measure);
      a.push_back(w.a);
      b.push_back(w.b);
      max_fixed = std::max(max_fixed, w.kind == SCOTTY_WIN_FIXED_BAND ? w.b : w.a);  // clearDelay
    }
    if (w.measure == SCOTTY_MEASURE_COUNT) c.has_count = 1;
    else c.has_time = 1;
  }
  c.n_cf = (int32_t)kind.size();
  c.n_ctx = nctx;
  c.has_fixed = c.n_cf > 0;
  c.has_ctx = has_ctx;
  c.session_case = session_case;
  c.max_lateness = max_lateness;
  c.max_fixed = max_fixed;
  // SliceFactory.createSlice (S/slice/SliceFactory.java:17-22)
  c.lazy = !(!c.has_count && (!has_ctx || session_case) && max_lateness > 0);
  // LazySlice record sets, kept from the first configuration with Lazy slices on (a later lateness change keeps them)
  records = records || c.lazy;
  c.records = records ? 1 : 0;
  int n_inv = 0;
  for (size_t i = 0; i < aggs.size(); i++) n_inv += (i < agg_inv.size() && agg_inv[i]) ? 1 : 0;
  c.invertible = (!aggs.empty() && n_inv == (int)aggs.size()) ? 1 : 0;
  if (records && n_inv != 0 && n_inv != (int)aggs.size()) {
    err = "LazySlice record removal with both invertible and non-invertible functions on one operator (each keeps "
          "its own partial in the reference) is not supported on the MI355X path";
    return SCOTTY_ERR_UNSUPPORTED;
  }
  c.vt = vt;
  c.need = 0;
  c.n_aggs = (int32_t)aggs.size();
  for (size_t i = 0; i < aggs.size(); i++) {
    c.agg_kind[i] = aggs[i];
    c.need |= agg_need(aggs[i]);
  }
  // capacities
  if (sc == 0) {
    if (!keyed) {
      sc = sc_override > 0 ? sc_override : (1 << 20);
    } else if (sc_override > 0) {
      int64_t p = 1;  // keyed stores index slice positions with shifts (XKView): a power of two
      while (p < sc_override) p <<= 1;
      sc = (int32_t)p;
    } else {
      int64_t min_step = INT64_MAX;
      for (const XWinDef& w : wins) {
        if (w.kind == SCOTTY_WIN_TUMBLING) min_step = std::min(min_step, w.a);
        if (w.kind == SCOTTY_WIN_SLIDING) min_step = std::min(min_step, w.b);
      }
      int64_t est = 128;
      if (min_step != INT64_MAX && min_step > 0 && !has_ctx && !c.has_count)
        est = (max_fixed + std::max<int64_t>(max_lateness, 0)) / min_step + 24;
      int64_t p = 32;
      while (p < est && p < 1024) p <<= 1;  // grown on demand (replay capacity pre-check)
      sc = (int32_t)p;
    }
  }
  if (sesscap == 0) sesscap = sess_override > 0 ? sess_override : (keyed ? 64 : 4096);
  if (records && rcap_ == 0) rcap_ = keyed ? 256 : (1 << 20);
  c.sc = sc;
  sl.sc_sh = 0;
  while (((int64_t)1 << sl.sc_sh) < sc) sl.sc_sh++;
  c.sesscap = sesscap;
  c.ctx_alloc = ctx_alloc;
  c.rcap = rcap_;
  // context-free window table
  dfree(d_cf_kind); dfree(d_cf_meas); dfree(d_cf_a); dfree(d_cf_b);
  d_cf_kind = nullptr; d_cf_meas = nullptr; d_cf_a = nullptr; d_cf_b = nullptr;
  XCHK(dalloc(&d_cf_kind, kind.size()));
  XCHK(dalloc(&d_cf_meas, kind.size()));
  XCHK(dalloc(&d_cf_a, kind.size()));
  XCHK(dalloc(&d_cf_b, kind.size()));
  if (!kind.empty()) {
    XCHK(hipMemcpyAsync(d_cf_kind, kind.data(), kind.size() * 4, hipMemcpyHostToDevice, stream));
    XCHK(hipMemcpyAsync(d_cf_meas, meas.data(), meas.size() * 4, hipMemcpyHostToDevice, stream));
    XCHK(hipMemcpyAsync(d_cf_a, a.data(), a.size() * 8, hipMemcpyHostToDevice, stream));
    XCHK(hipMemcpyAsync(d_cf_b, b.data(), b.size() * 8, hipMemcpyHostToDevice, stream));
  }
  c.cf_kind = d_cf_kind;
  c.cf_measure = d_cf_meas;
  c.cf_a = d_cf_a;
  c.cf_b = d_cf_b;
  cfg = c;
  xq_need_grid = true;  // the union edge grid follows the registered windows
  XCHK(hipMemcpyAsync(d_cfg, &cfg, sizeof(XCfg), hipMemcpyHostToDevice, stream));
  if (nctx > ctx_alloc) {  // session windows registered (possibly mid-stream): widen the per-op session table
    int rc = grow_caps(sc, sesscap, nctx);
    if (rc) return rc;
  }
  if (records && !sl.rts && ops_cap > 0) {  // records switched on mid-stream: every existing set is empty
    int rc = alloc_records();
    if (rc) return rc;
  }
  XCHK(hipStreamSynchronize(stream));
  if (!keyed && n_ops == 0) {
    int rc = grow_ops(1);
    if (rc) return rc;
    XCHK(launch_xstate_init(d_st, 0, 1, nullptr, stream));
    n_ops = 1;
  }
  return SCOTTY_OK;
}

int XEngine::grow_ops(int64_t need) {
  if (need <= ops_cap) return SCOTTY_OK;
  int64_t cap = std::max<int64_t>(ops_cap * 2, keyed ? 1024 : 1);
  while (cap < need) cap *= 2;
  XCHK(hipStreamSynchronize(stream));
  auto grow = [&](auto** p, int64_t per_op) -> hipError_t {
    using T = std::remove_pointer_t<std::remove_reference_t<decltype(*p)>>;
    T* np = nullptr;
    hipError_t e = dalloc(&np, (size_t)(cap * per_op));
    if (e != hipSuccess) return e;
    if (*p && n_ops > 0) {
      e = hipMemcpyAsync(np, *p, (size_t)(n_ops * per_op) * sizeof(T), hipMemcpyDeviceToDevice, stream);
      if (e != hipSuccess) return e;
    }
    if (*p) {
      (void)hipStreamSynchronize(stream);
      dfree(*p);
    }
    *p = np;
    return hipSuccess;
  };
  if (ops_cap == 0) {  // the store's layout is fixed with the first allocation
    aos = keyed && (lane_mode() || lane_session_mode()) && vt != VT_F64;
    // MIN / MAX block summaries only if used (the functions are fixed before the first push: scotty_add_aggregation
    // refuses a function added after elements were processed)
    sl.kw_nf = (cfg.need & (NEED_MIN | NEED_MAX)) ? XK_NF : XK_NF_SUM;
  }
  XCHK(grow(&d_st, 1));
  if (aos) {  // key-interleaved store: rows (position, field) of cap words, re-strided from the old key capacity
    unsigned long long* nw = nullptr;
    const int64_t rows = (int64_t)sc * sl.kw_nf;
    XCHK(dalloc(&nw, (size_t)(rows * cap)));
    XCHK(hipMemsetAsync(nw, 0, (size_t)(rows * cap) * 8, stream));
    if (sl.kw && n_ops > 0)
      XCHK(hipMemcpy2DAsync(nw, cap * 8, sl.kw, ops_cap * 8, n_ops * 8, rows, hipMemcpyDeviceToDevice, stream));
    XCHK(hipStreamSynchronize(stream));
    dfree(sl.kw);
    sl.kw = nw;
    int sh = 0;
    while (((int64_t)1 << sh) < cap) sh++;
    sl.kc_sh = sh;
  } else {
    XCHK(grow(&sl.ts, sc)); XCHK(grow(&sl.te, sc)); XCHK(grow(&sl.tl, sc)); XCHK(grow(&sl.tf, sc));
    XCHK(grow(&sl.cs, sc)); XCHK(grow(&sl.cl, sc)); XCHK(grow(&sl.ty, sc)); XCHK(grow(&sl.cnt, sc));
    for (int k = 0; k < NPART; k++) XCHK(grow(&sl.p[k], sc));
    XCHK(grow(&sl.pc, sc)); XCHK(grow(&sl.ps, sc));
  }
  if (ctx_alloc > 0) {
    XCHK(grow(&ss.start, (int64_t)ctx_alloc * sesscap));
    XCHK(grow(&ss.end, (int64_t)ctx_alloc * sesscap));
  }
  if (keyed) XCHK(grow(&d_slot_key, 1));
  if (records) {
    XCHK(grow(&sl.rlo, sc)); XCHK(grow(&sl.rhi, sc)); XCHK(grow(&sl.nn, sc));
    XCHK(grow(&sl.rts, rcap_)); XCHK(grow(&sl.rv, rcap_));
  }
  XCHK(hipStreamSynchronize(stream));
  ops_cap = cap;
  return SCOTTY_OK;
}

// Record arrays for every allocated op (records enabled after slices existed: every record range is [0, 0)).
int XEngine::alloc_records() {
  XCHK(hipStreamSynchronize(stream));
  const int64_t rows = std::max<int64_t>(ops_cap, 1);
  XCHK(dalloc(&sl.rlo, rows * sc)); XCHK(dalloc(&sl.rhi, rows * sc)); XCHK(dalloc(&sl.nn, rows * sc));
  XCHK(dalloc(&sl.rts, rows * rcap_)); XCHK(dalloc(&sl.rv, rows * rcap_));
  XCHK(hipMemsetAsync(sl.rlo, 0, rows * sc * 8, stream));
  XCHK(hipMemsetAsync(sl.rhi, 0, rows * sc * 8, stream));
  // existing slices got nn from their counts: conservatively non-null iff they hold tuples (set by the kernels
  // on the next add); a zero fill is exact for slices created from now on
  XCHK(hipMemsetAsync(sl.nn, 0, rows * sc * 4, stream));
  XCHK(hipStreamSynchronize(stream));
  return SCOTTY_OK;
}

// Re-lay out the per-op slice / session tables with larger capacities (row = one op, 2-D copies).
int XEngine::grow_caps(int64_t need_sc, int64_t need_sess, int32_t need_ctx, int64_t need_rec) {
  int64_t nsc = sc, nss = sesscap, nrc = rcap_;
  while (nsc < need_sc) nsc *= 2;
  while (nss < need_sess) nss *= 2;
  while (records && nrc < need_rec) nrc *= 2;
  if (nrc > ((int64_t)1 << 34)) {
    err = "per-operator LazySlice record capacity would exceed the supported maximum";
    failed = true;
    return SCOTTY_ERR_NOMEM;
  }
  const int32_t nctx = std::max(ctx_alloc, need_ctx);
  if (nsc > (1 << 26) || nss > (1 << 24)) {
    err = "per-operator slice / session capacity would exceed the supported maximum";
    failed = true;
    return SCOTTY_ERR_NOMEM;
  }
  XCHK(hipStreamSynchronize(stream));
  const int64_t rows = std::max<int64_t>(ops_cap, 1);
  auto relayout = [&](auto** p, int64_t old_w, int64_t new_w, int64_t nrows, int64_t copy_rows) -> hipError_t {
    using T = std::remove_pointer_t<std::remove_reference_t<decltype(*p)>>;
    T* np = nullptr;
    hipError_t e = dalloc(&np, (size_t)(nrows * new_w));
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(np, 0, (size_t)(nrows * new_w) * sizeof(T), stream);
    if (e != hipSuccess) return e;
    if (*p && copy_rows > 0 && old_w > 0) {
      e = hipMemcpy2DAsync(np, new_w * sizeof(T), *p, old_w * sizeof(T), old_w * sizeof(T), copy_rows,
                           hipMemcpyDeviceToDevice, stream);
      if (e != hipSuccess) return e;
      (void)hipStreamSynchronize(stream);
    }
    dfree(*p);
    *p = np;
    return hipSuccess;
  };
  if (nsc != sc && sl.kw) {  // key-interleaved: positions are the outer index, the old store is a prefix
    unsigned long long* nw = nullptr;
    XCHK(dalloc(&nw, (size_t)(nsc * sl.kw_nf * rows)));
    XCHK(hipMemsetAsync(nw, 0, (size_t)(nsc * sl.kw_nf * rows) * 8, stream));
    XCHK(hipMemcpyAsync(nw, sl.kw, (size_t)(sc * sl.kw_nf * rows) * 8, hipMemcpyDeviceToDevice, stream));
    XCHK(hipStreamSynchronize(stream));
    dfree(sl.kw);
    sl.kw = nw;
  }
  if (nsc != sc && sl.ts) {
    XCHK(relayout(&sl.ts, sc, nsc, rows, n_ops)); XCHK(relayout(&sl.te, sc, nsc, rows, n_ops));
    XCHK(relayout(&sl.tl, sc, nsc, rows, n_ops)); XCHK(relayout(&sl.tf, sc, nsc, rows, n_ops));
    XCHK(relayout(&sl.cs, sc, nsc, rows, n_ops)); XCHK(relayout(&sl.cl, sc, nsc, rows, n_ops));
    XCHK(relayout(&sl.ty, sc, nsc, rows, n_ops)); XCHK(relayout(&sl.cnt, sc, nsc, rows, n_ops));
    for (int k = 0; k < NPART; k++) XCHK(relayout(&sl.p[k], sc, nsc, rows, n_ops));
    XCHK(relayout(&sl.pc, sc, nsc, rows, n_ops)); XCHK(relayout(&sl.ps, sc, nsc, rows, n_ops));
    if (records && sl.rlo) {
      XCHK(relayout(&sl.rlo, sc, nsc, rows, n_ops)); XCHK(relayout(&sl.rhi, sc, nsc, rows, n_ops));
      XCHK(relayout(&sl.nn, sc, nsc, rows, n_ops));
    }
  }
  if (records && nrc != rcap_ && sl.rts) {
    XCHK(relayout(&sl.rts, rcap_, nrc, rows, n_ops)); XCHK(relayout(&sl.rv, rcap_, nrc, rows, n_ops));
  }
  if (nss != sesscap || nctx != ctx_alloc) {
    // row = one op: ctx_alloc contexts x sesscap sessions; re-pitch contexts first, then widen each context
    int64_t* ns_start = nullptr;
    int64_t* ns_end = nullptr;
    XCHK(dalloc(&ns_start, (size_t)(rows * nctx * nss)));
    XCHK(dalloc(&ns_end, (size_t)(rows * nctx * nss)));
    XCHK(hipMemsetAsync(ns_start, 0, (size_t)(rows * nctx * nss) * 8, stream));
    XCHK(hipMemsetAsync(ns_end, 0, (size_t)(rows * nctx * nss) * 8, stream));
    if (ss.start && ctx_alloc > 0 && n_ops > 0) {
      for (int c = 0; c < ctx_alloc; c++) {
        XCHK(hipMemcpy2DAsync(ns_start + (int64_t)c * nss, (size_t)nctx * nss * 8, ss.start + (int64_t)c * sesscap,
                              (size_t)ctx_alloc * sesscap * 8, (size_t)sesscap * 8, n_ops, hipMemcpyDeviceToDevice,
                              stream));
        XCHK(hipMemcpy2DAsync(ns_end + (int64_t)c * nss, (size_t)nctx * nss * 8, ss.end + (int64_t)c * sesscap,
                              (size_t)ctx_alloc * sesscap * 8, (size_t)sesscap * 8, n_ops, hipMemcpyDeviceToDevice,
                              stream));
      }
      XCHK(hipStreamSynchronize(stream));
    }
    dfree(ss.start);
    dfree(ss.end);
    ss.start = ns_start;
    ss.end = ns_end;
  }
  sc = (int32_t)nsc;
  sl.sc_sh = 0;
  while (((int64_t)1 << sl.sc_sh) < sc) sl.sc_sh++;
  sesscap = (int32_t)nss;
  ctx_alloc = nctx;
  rcap_ = nrc;
  cfg.sc = sc;
  cfg.sesscap = sesscap;
  cfg.ctx_alloc = ctx_alloc;
  cfg.rcap = rcap_;
  XCHK(hipMemcpyAsync(d_cfg, &cfg, sizeof(XCfg), hipMemcpyHostToDevice, stream));
  XCHK(hipStreamSynchronize(stream));
  return SCOTTY_OK;
}

int XEngine::ensure_batch(int64_t n) {
  if (n <= bcap) return SCOTTY_OK;
  XCHK(hipStreamSynchronize(stream));
  int64_t cap = std::max<int64_t>(n, 1 << 16);
  dfree(d_slot); dfree(d_recA); dfree(d_recB); dfree(d_hist); dfree(d_scan32); dfree(d_rpart);
  dfree(d_ukey); dfree(d_ubeg); dfree(d_segcnt); dfree(d_segoff); dfree(d_segscan); dfree(d_tmaxt);
  const int rec = vt == VT_I32 ? 16 : 24;
  XCHK(dalloc(&d_slot, cap));
  XCHK(dalloc(&d_ukey, cap));
  XCHK(dalloc(&d_ubeg, cap));
  {
    const int64_t ns = seg_tiles(cap) + 1;
    XCHK(dalloc(&d_segcnt, ns));
    XCHK(dalloc(&d_segoff, ns));
    XCHK(dalloc(&d_segscan, ns / 512 + 64));
    XCHK(dalloc(&d_tmaxt, ns));
  }
  XCHK(dalloc((unsigned char**)&d_recA, cap * rec));
  XCHK(dalloc((unsigned char**)&d_recB, cap * rec));
  const int64_t nb = (cap + sort_tile() - 1) / sort_tile();
  XCHK(dalloc(&d_hist, (256 + 1024) * nb));  // 8-bit digit histograms, then the 10-bit ones (launch_sort_by_slot)
  XCHK(dalloc(&d_rpart, 3 * nb));
  XCHK(dalloc(&d_scan32, 1024 * nb / 512 + 64));
  XCHK(dalloc(&d_newpos, cap));
  bcap = cap;
  return SCOTTY_OK;
}

int XEngine::ensure_table(int64_t keys_needed, bool drop_new) {
  uint64_t want = 1024;
  while ((int64_t)want < 2 * keys_needed) want <<= 1;
  if (want <= tcap) return SCOTTY_OK;
  unsigned long long* nt = nullptr;
  XCHK(dalloc(&nt, want));
  XCHK(hipMemsetAsync(nt, 0, want * 8, stream));
  if (d_table) {
    XCHK(launch_rehash(d_table, tcap, nt, want - 1, drop_new ? 1 : 0, stream));
    XCHK(hipStreamSynchronize(stream));
    dfree(d_table);
  }
  d_table = nt;
  tcap = want;
  return SCOTTY_OK;
}

int XEngine::check_ready() {
  if (failed) return SCOTTY_ERR_STATE;
  return SCOTTY_OK;
}

XBatchArgs XEngine::batch_args() const {
  XBatchArgs a{};
  a.cfg = d_cfg;
  a.st = d_st;
  a.sl = sl;
  a.ss = ss;
  a.n_ops = (int32_t)n_ops;
  return a;
}

int XEngine::push(const int64_t* d_ts, const void* d_val, int64_t n) {
  if (n <= 0) return SCOTTY_OK;
  XBatchArgs a = batch_args();
  a.ts = d_ts;
  a.val = d_val;
  a.n = n;
  a.rec_stride = 0;
  if (!records) {
    XCHK(launch_replay(a, vt, stream));
    return SCOTTY_OK;
  }
  // records mode: capacity pre-check (slices, sessions, records); a deferred op is grown and relaunched
  a.need = d_need;
  for (int attempt = 0; attempt < 8; attempt++) {
    XCHK(hipMemsetAsync(d_need, 0, 32, stream));
    a.retry = attempt > 0;
    a.sl = sl;
    a.ss = ss;
    XCHK(launch_replay(a, vt, stream));
    XCHK(hipMemcpyAsync(h_misc, d_need, 24, hipMemcpyDeviceToHost, stream));
    XCHK(hipStreamSynchronize(stream));
    if (h_misc[0] == 0 && h_misc[1] == 0 && h_misc[2] == 0) return SCOTTY_OK;
    int rc = grow_caps(std::max<int64_t>(h_misc[0], sc), std::max<int64_t>(h_misc[1], sesscap), ctx_alloc,
                       std::max<int64_t>(h_misc[2], rcap_));
    if (rc) return rc;
  }
  err = "capacity growth did not converge";
  failed = true;
  return SCOTTY_ERR_NOMEM;
}

// Non-keyed micro-batch: classify (all CUs) -> compacted events (one wave, exact) -> apply (all CUs).  A
// round ends at the first out-of-order event that may modify sessions / older slices; the rest of the batch
// is then classified again against the updated operator (rounds are rare: record-breaking session growth).
int XEngine::push_batch(const int64_t* d_ts, const void* d_val, int64_t n) {
  const size_t vb = vt == VT_I32 ? 4 : 8;
  last_events = 0;
  last_segments = 0;
  last_quiet = 0;
  // The batch is processed in consecutive pieces, which the sequential reference cannot tell from one batch: the
  // quiet path takes the rest of the batch in one pass when it can; when it cannot, the event-exact path takes a
  // prefix and the quiet path is tried again on what follows.  A batch whose session structure changes only near its
  // start (the stream resuming after a silence: a new session whose start moves down with the first out-of-order
  // tuples) costs one short event-exact prefix, not rounds over the whole batch.  The prefix grows 4x with every
  // further refusal, so a batch that is not quiet anywhere reaches the event-exact path for all of it quickly.
  int64_t pos0 = 0;
  xq_trace.clear();
  int64_t chunk = xq_prefix > 0 ? xq_prefix : std::max<int64_t>(n / 32, (int64_t)1 << 20);
  chunk = (chunk + 4095) & ~(int64_t)4095;  // pieces start 16-byte aligned (the ingest's vector loads)
  // event-exact piece behind a located jump: the stream resuming after a silence opens a session whose start settles
  // within the first tuples (out-of-order tuples reach at most maxDelay below it), then the batch is quiet again
  int64_t chunk_jump = (int64_t)1 << 18;
  bool try_quiet = quiet_eligible();
  int jump_pieces = 0;
  if (try_quiet && xq_skip > 0) {  // backed off after consecutive refusals the batch itself caused (see below)
    xq_skip--;
    quiet_skipped++;
    try_quiet = false;
  }
  while (pos0 < n) {
    const int64_t rest = n - pos0;
    const unsigned char* val0 = (const unsigned char*)d_val + pos0 * vb;
    if (try_quiet) {
      int32_t res = XQ_NONE;
      int rc = push_quiet(d_ts + pos0, val0, rest, &res);
      if (rc) return rc;
      xq_trace.push_back((int64_t)res | (last_quiet_why & 0xFFFF) << 8 | pos0 << 24);
      if (pos0 == 0) last_quiet = res;  // the batch's own verdict (a committed remainder is counted below)
      else if (res == XQ_COMMITTED) quiet_tail_commits++;
      if (res == XQ_COMMITTED) {
        quiet_commits++;
        xq_refused_run = 0;
        return SCOTTY_OK;
      }
      quiet_fallbacks++;
      if (res == XQ_NOT_QUIET && (last_quiet_why & 3) != 0) {
        // tuples below the cell view or the last session's start (why 1 / 2).  Within a batch such a refusal is often
        // transient -- a resumed stream's new session settles within its first tuples (C3's pause step), and until
        // it has, the view of an unsorted slice list starts above the tuples still to come -- so the event-exact
        // prefix keeps growing 4x and the quiet path is tried on what follows (at most ~log4(n / prefix) attempts;
        // stopping at the first why-1 refusal sent 2^26 - 4096 tuples of C3's pause step through event-exact rounds,
        // profiles/r04/r04b_c3_quiet_attempts.txt).  Batches whose own verdict fails that way back the quiet path off
        // across batches (after two in a row: the next 1, 2, 4 .. 16 batches go straight to the event-exact path).
        if (pos0 == 0) {
          xq_refused_run++;
          if (xq_refused_run >= 2) xq_skip = std::min(1 << std::min(xq_refused_run - 2, 4), 16);
        }
      } else if (pos0 == 0) {
        xq_refused_run = 0;
      }
      // a session-gap jump among the piece's first 64 tuples (the prep's refusal located it), with the start band: the
      // event-exact path takes the tuples up to and including the jump (an even count, so the next piece starts
      // 16-byte aligned) and the quiet path is tried on the rest -- the resumed stream's new session then settles
      // inside the band in one pass (C3's pause step; exact_quiet.h).  At most two such pieces per batch: a stream
      // that jumps every few tuples goes on with the growing event-exact prefix below
      if (res == XQ_NOT_QUIET && last_quiet_why == 4 && last_quiet_jump_pos >= 0 && band_usable() && jump_pieces < 2) {
        const int64_t w = std::min(rest, (last_quiet_jump_pos + 2) & ~(int64_t)1);
        rc = push_exact(d_ts + pos0, val0, w);
        if (rc) return rc;
        quiet_jump_pieces++;
        jump_pieces++;
        pos0 += w;
        continue;
      }
      // the verdict failed only on session-gap jumps and located the first one: everything before its arrival tile
      // is quiet (the verdict's other conditions held for the whole rest) -- commit that prefix in one pass, then the
      // event-exact path from the jump on
      const int64_t J = res == XQ_NOT_QUIET && (last_quiet_why & ~(int64_t)12) == 0 ? last_quiet_jump : 0;
      if (J > 0 && J < rest) {
        res = XQ_NONE;
        rc = push_quiet(d_ts + pos0, val0, J, &res);
        if (rc) return rc;
        if (res == XQ_COMMITTED) {
          quiet_commits++;
          quiet_split_commits++;
          pos0 += J;
          const int64_t w = std::min(chunk_jump, n - pos0);
          rc = push_exact(d_ts + pos0, (const unsigned char*)d_val + pos0 * vb, w);
          if (rc) return rc;
          pos0 += w;
          chunk_jump *= 4;
          continue;
        }
        quiet_fallbacks++;
      }
    }
    const int64_t w = try_quiet && chunk < rest ? chunk : rest;
    int rc = push_exact(d_ts + pos0, val0, w);
    if (rc) return rc;
    pos0 += w;
    chunk *= 4;
  }
  return SCOTTY_OK;
}

// Event-exact batch path over [0, n): classify (all CUs) -> compacted events (one wave, exact) -> apply (all CUs).  A
// round ends at the first out-of-order event that may modify sessions / older slices; the rest is then classified
// again against the updated operator (rounds are rare: record-breaking session growth).
int XEngine::push_exact(const int64_t* d_ts, const void* d_val, int64_t n) {
  const size_t vb = vt == VT_I32 ? 4 : 8;
  int64_t pos0 = 0;
  TEv tx;
  int rct = tbegin(tx, SCOTTY_TIME_PUSH_OTHER);
  if (rct) return rct;
  struct TEnd {  // the event-exact path's device time (class PUSH_OTHER), also on early returns
    XEngine* e;
    TEv* t;
    int64_t n;
    ~TEnd() { (void)e->tend(*t, n); }
  } tend_guard{this, &tx, n};
  for (int64_t round = 0; pos0 < n; round++) {
    int64_t stop = -1;
    int rc = push_round(d_ts + pos0, (const unsigned char*)d_val + pos0 * vb, n - pos0, round > 0, &stop);
    if (rc) return rc;
    last_segments++;
    if (stop < 0) break;
    pos0 += stop;
    if (round > 4 * n + 16) {
      err = "event pass made no progress";
      failed = true;
      return SCOTTY_ERR_STATE;
    }
  }
  return SCOTTY_OK;
}


// ---------------------------------------------------------------- one-pass quiet path (exact_quiet.hip)
// Eligible configurations: non-keyed, time measure, Eager slices (no count windows, maxLateness > 0), and partials the
// grid ingest computes bit-identically (an int32 stream's sums wrap mod 2^32 there: SUM_I32 only).
bool XEngine::quiet_eligible() const {
  if (keyed || quiet_off || use_serial() || cfg.lazy || cfg.has_count || !cfg.has_time) return false;
  for (int i = 0; i < cfg.n_aggs; i++) {
    const int k = cfg.agg_kind[i] & 0xFFFF;
    if (vt == VT_I32 && (k == SCOTTY_AGG_SUM_I64 || k == SCOTTY_AGG_SUM_F64)) return false;
  }
  return true;
}

int XEngine::tbegin(TEv& e, int cls) {
  e.cls = cls;
  e.a = e.b = nullptr;
  if (!timing) return SCOTTY_OK;
  if (!ev_pool.empty()) {
    e.a = ev_pool.back().a;
    e.b = ev_pool.back().b;
    ev_pool.pop_back();
  } else {
    XCHK(hipEventCreate(&e.a));
    XCHK(hipEventCreate(&e.b));
  }
  XCHK(hipEventRecord(e.a, stream));
  return SCOTTY_OK;
}
int XEngine::tend(TEv& e, int64_t n) {
  if (!timing || !e.a) return SCOTTY_OK;
  XCHK(hipEventRecord(e.b, stream));
  e.n = n;
  ev_pending.push_back(e);
  e.a = nullptr;
  return SCOTTY_OK;
}
// after a synchronisation: completed intervals into their classes
int XEngine::collect_timing() {
  std::vector<TEv> keep;
  for (auto& e : ev_pending) {
    if (hipEventQuery(e.b) == hipErrorNotReady) {
      keep.push_back(e);
      continue;
    }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess && e.cls >= 0 && e.cls < 4) {
      t_ms[e.cls] += ms;
      t_cnt[e.cls]++;
      if (e.cls == SCOTTY_TIME_INGEST) t_tuples += e.n;
    }
    ev_pool.push_back(e);
  }
  ev_pending.swap(keep);
  return SCOTTY_OK;
}

// Union edge grid of the context-free time windows from the pending edge N (first entry) up to a horizon: the
// points nextGrid visits (S/StreamSlicer.java:103-116; TumblingWindow.java:29-31, SlidingWindow.java:41-43,
// FixedBandWindow.java:37-48), a k-way merge of arithmetic progressions.  Built on the host at synchronisation
// points only (the first push, a stale grid, a horizon running short).
int XEngine::xq_rebuild_grid() {
  XState s{};
  XCHK(hipMemcpyAsync(&s, d_st, sizeof(XState), hipMemcpyDeviceToHost, stream));
  XCHK(hipStreamSynchronize(stream));
  xq_hgrid.clear();
  if (!cfg.has_fixed) {
    xq_need_grid = false;
    return SCOTTY_OK;
  }
  const int64_t N = s.nextEdgeTs;
  if (N < 0 || !s.started) return SCOTTY_OK;  // not yet: the event-exact path runs, the grid is built later
  if (xq_gcap == 0) xq_gcap = 1 << 20;
  auto next_start = [](const XWinDef& w, int64_t t) -> int64_t {
    auto jadd_ = [](int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); };
    if (w.kind == SCOTTY_WIN_TUMBLING) return jadd_(t, w.a) - (w.a == -1 ? 0 : t % w.a);
    if (w.kind == SCOTTY_WIN_SLIDING) return jadd_(t, w.b) - (w.b == -1 ? 0 : t % w.b);
    if (t == INT64_MAX || t < w.a) return w.a;
    if (t >= w.a && t < jadd_(w.a, w.b)) return jadd_(w.a, w.b);
    return INT64_MAX;
  };
  const int64_t span = std::max<int64_t>(xq_span, 1);
  const int64_t front = std::max<int64_t>(s.maxEventTime, 0);
  const int64_t horizon = front > INT64_MAX / 2 ? INT64_MAX : front + std::max<int64_t>(64 * span, 600000);
  xq_hgrid.push_back(N);
  using Item = std::pair<int64_t, int>;
  std::priority_queue<Item, std::vector<Item>, std::greater<Item>> pq;
  bool infinite = false;
  for (int i = 0; i < (int)h_wins.size(); i++) {
    const XWinDef& w = h_wins[i];
    if (w.kind == SCOTTY_WIN_SESSION || w.measure != SCOTTY_MEASURE_TIME) continue;
    if (w.kind == SCOTTY_WIN_FIXED_BAND) {
      if (w.a > N) pq.push({w.a, -1});
      const int64_t e = (int64_t)((uint64_t)w.a + (uint64_t)w.b);
      if (e > N) pq.push({e, -1});
    } else {
      infinite = true;
      pq.push({next_start(w, N), i});
    }
  }
  while (!pq.empty() && (int64_t)xq_hgrid.size() < xq_gcap - 1) {
    const Item it = pq.top();
    pq.pop();
    if (it.first > xq_hgrid.back()) {
      if (it.first > horizon && infinite) break;
      xq_hgrid.push_back(it.first);
    }
    if (it.second >= 0) {
      const int64_t nx = next_start(h_wins[it.second], it.first);
      if (nx > it.first) pq.push({nx, it.second});
    }
  }
  if (!infinite && pq.empty()) xq_hgrid.push_back(INT64_MAX);
  if (!d_xq_grid) XCHK(dalloc(&d_xq_grid, xq_gcap));
  XCHK(hipMemcpyAsync(d_xq_grid, xq_hgrid.data(), xq_hgrid.size() * 8, hipMemcpyHostToDevice, stream));
  XCHK(hipStreamSynchronize(stream));
  xq_need_grid = false;
  return SCOTTY_OK;
}

int XEngine::xq_ensure(int64_t n) {
  if (xq_gcap == 0) xq_gcap = 1 << 20;
  if (!d_xq_meta) {
    XCHK(dalloc((unsigned char**)&d_xq_meta, sizeof(DevMeta)));
    XCHK(dalloc((unsigned char**)&d_xq_ctl, sizeof(XQCtl)));
    XCHK(dalloc(&d_xq_cix, CIX_CAP));
    XCHK(dalloc(&d_xq_cixmeta, 8));
    XCHK(dalloc(&d_xq_rank, xq_gcap));
    XCHK(dalloc(&d_xq_flag, xq_gcap));
    XCHK(dalloc(&d_xq_eg, xq_gcap));
    XCHK(dalloc(&d_xq_epos, 2 * xq_gcap));
    XCHK(dalloc(&d_xq_pmax, NT_MAX));
    if (!d_xq_grid) XCHK(dalloc(&d_xq_grid, xq_gcap));
  }
  if (xq_ccap < (int64_t)sc + xq_gcap) {  // cells: retained slices ++ grid cells, identity between batches
    XCHK(hipStreamSynchronize(stream));
    dfree(d_xq_ccnt); dfree(d_xq_ctmax);
    for (int k = 0; k < NPART; k++) dfree(d_xq_cpart[k]);
    xq_ccap = (int64_t)sc + xq_gcap;
    XCHK(dalloc(&d_xq_ccnt, xq_ccap));
    XCHK(dalloc(&d_xq_ctmax, xq_ccap));
    for (int k = 0; k < NPART; k++) XCHK(dalloc(&d_xq_cpart[k], xq_ccap));
    XCHK(launch_fill_u64(d_xq_ccnt, xq_ccap, 0, stream));
    XCHK(launch_fill_u64((unsigned long long*)d_xq_ctmax, xq_ccap, (unsigned long long)INT64_MIN, stream));
    XCHK(launch_fill_u64(d_xq_cpart[0], xq_ccap, 0, stream));
    XCHK(launch_fill_u64(d_xq_cpart[1], xq_ccap, (unsigned long long)INT64_MAX, stream));
    XCHK(launch_fill_u64(d_xq_cpart[2], xq_ccap, (unsigned long long)INT64_MIN, stream));
  }
  const int64_t nt = (n + TILE_MIN - 1) / TILE_MIN + 1;
  if (nt > xq_tcap) {
    XCHK(hipStreamSynchronize(stream));
    dfree(d_xq_tilemax);
    dfree(d_xq_tilemin);
    xq_tcap = std::max<int64_t>(nt, 1024);
    XCHK(dalloc(&d_xq_tilemax, xq_tcap));
    XCHK(dalloc(&d_xq_tilemin, xq_tcap));
  }
  return SCOTTY_OK;
}

// One HBM pass over the batch (grid ingest into cells), then the quiet verdict and commit on the device; one host
// synchronisation reads the verdict.  Nothing of the operator changes unless *result == XQ_COMMITTED.
int XEngine::push_quiet(const int64_t* d_ts, const void* d_val, int64_t n, int32_t* result) {
  *result = XQ_NONE;
  last_quiet_why = 0;
  last_quiet_jump = 0;
  last_quiet_jump_pos = -1;
  if (xq_need_grid) {
    int rc = xq_rebuild_grid();
    if (rc) return rc;
    if (xq_need_grid) {  // the stream has not reached a pending edge yet
      *result = XQ_GRID;
      return SCOTTY_OK;
    }
  }
  int rc = xq_ensure(n);
  if (rc) return rc;
  int64_t tile = TILE_MIN;
  while ((n + tile - 1) / tile > NT_MAX) tile <<= 1;
  const int64_t target_blocks = xq_ingest_blocks > 0 ? xq_ingest_blocks
                                                     : 256 * ingest_wgs_per_cu(vt, cfg.need);  // one round of resident workgroups
  int64_t per_wave = (n + target_blocks * 4 - 1) / (target_blocks * 4);
  per_wave = std::max(((per_wave + tile - 1) / tile) * tile, tile);
  const int64_t nblocks = (n + per_wave * 4 - 1) / (per_wave * 4);
  IngestArgs ia{};
  ia.ts = d_ts;
  ia.val = d_val;
  ia.n = n;
  ia.s_tstart = sl.ts;  // op 0
  ia.grid = d_xq_grid;
  ia.c_cnt = d_xq_ccnt;
  ia.c_tmax = d_xq_ctmax;
  for (int k = 0; k < NPART; k++) ia.c_part[k] = d_xq_cpart[k];
  ia.tilemax = d_xq_tilemax;
  const bool band = band_usable();
  ia.tilemin = band ? d_xq_tilemin : nullptr;  // the ingest's per-tile minima (the band's new session start)
  ia.meta = d_xq_meta;
  ia.per_wave = per_wave;
  ia.tile = tile;
  ia.cix = d_xq_cix;
  ia.cix_meta = d_xq_cixmeta;
  ia.cix_margin = std::max<int64_t>(4 * xq_span, 4000);
  XQArgs q{};
  q.ts = d_ts;
  q.n = n;
  q.tile = tile;
  q.cfg = d_cfg;
  q.st = d_st;
  q.sl = sl;
  q.ss = ss;
  q.grid = d_xq_grid;
  q.gcount = (int64_t)xq_hgrid.size();
  q.meta = d_xq_meta;
  q.c_cnt = d_xq_ccnt;
  q.c_tmax = d_xq_ctmax;
  for (int k = 0; k < NPART; k++) q.c_part[k] = d_xq_cpart[k];
  q.tilemax = d_xq_tilemax;
  q.tilemin = d_xq_tilemin;
  q.band = band ? 1 : 0;
  q.pmax = d_xq_pmax;
  q.rank = d_xq_rank;
  q.flag = d_xq_flag;
  q.eg = d_xq_eg;
  q.epos = d_xq_epos;
  q.ctl = (XQCtl*)d_xq_ctl;
  q.margin = std::max<int64_t>(16 * xq_span, 60000);
  const bool prof = getenv("SCOTTY_XQ_PROF") != nullptr;
  if (prof && !d_dbg) XCHK(dalloc(&d_dbg, 256));
  q.dbg = prof ? d_dbg : nullptr;
  TEv t0, t1, t2;
  if ((rc = tbegin(t0, SCOTTY_TIME_PUSH_OTHER))) return rc;
  XCHK(launch_xq_prep(q, stream));
  XCHK(launch_cix_build(ia, stream));
  if ((rc = tend(t0, 0))) return rc;
  if ((rc = tbegin(t1, SCOTTY_TIME_INGEST))) return rc;
  XCHK(launch_ingest(ia, vt, cfg.need, nblocks, stream, xq_ingest_mode));
  if ((rc = tend(t1, n))) return rc;
  if ((rc = tbegin(t2, SCOTTY_TIME_PUSH_OTHER))) return rc;
  XCHK(launch_xq_commit(q, stream));
  static_assert(sizeof(XQCtl) <= 16 * sizeof(int64_t), "XQCtl fits the mapped control block");
  XCHK(launch_copy_to_host(d_xq_ctl, h_misc_dev, sizeof(XQCtl), stream));
  if ((rc = tend(t2, 0))) return rc;
  XCHK(hipStreamSynchronize(stream));
  if (prof) {  // debugging aid: s_memtime deltas between the commit's phases
    long long h[16];
    XCHK(hipMemcpy(h, d_dbg, sizeof(h), hipMemcpyDeviceToHost));
    fprintf(stderr, "xq commit phase ticks:");
    for (int i = 1; i <= 3; i++) fprintf(stderr, " %lld", h[i] - h[i - 1]);
    fprintf(stderr, "\n");
  }
  XQCtl c;
  std::memcpy(&c, h_misc, sizeof(XQCtl));
  if (getenv("SCOTTY_XQ_DEBUG")) {  // debugging aid: the verdict's inputs
    DevMeta m;
    XCHK(hipMemcpy(&m, d_xq_meta, sizeof(DevMeta), hipMemcpyDeviceToHost));
    fprintf(stderr, "xq n=%lld res=%d why=%lld lo=%lld band_si=%lld band_s=%lld bmin=%lld bmax=%lld head=%lld tail=%lld "
            "cmin=%lld late=%llu ovf=%llu ncand=%lld\n", (long long)n, c.result, (long long)c.why, (long long)c.lo_bound,
            (long long)c.band_si, (long long)c.band_s, (long long)c.batch_min, (long long)c.batch_max,
            (long long)m.head, (long long)m.tail, (long long)m.cmin, (unsigned long long)m.late_push,
            (unsigned long long)m.overflow_push, (long long)c.ncand);
  }
  *result = c.result;
  last_quiet_why = c.why;
  last_quiet_jump = c.result == XQ_NOT_QUIET && c.jump_tile > 0 && c.jump_tile < (n + tile - 1) / tile ? c.jump_tile * tile : 0;
  last_quiet_jump_pos = c.result == XQ_NOT_QUIET ? c.jump_pos : -1;
  if (c.result == XQ_COMMITTED && c.band_si != -1 && c.batch_min < c.band_s) {
    quiet_band_moves++;
    if (c.band_si == -2) quiet_band_noedge++;
  }
  if (c.result == XQ_COMMITTED && c.batch_max > c.p_start) xq_span = std::max<int64_t>(c.batch_max - c.p_start, 1);
  if (c.result == XQ_GRID || (c.result == XQ_COMMITTED && c.rebuild)) xq_need_grid = true;
  if (timing) collect_timing();
  return SCOTTY_OK;
}

int XEngine::push_round(const int64_t* d_ts, const void* d_val, int64_t n, bool resume, int64_t* stop_at) {
  *stop_at = -1;
  if (n <= 0) return SCOTTY_OK;
  const int64_t T = xb_tile();
  const int64_t nt = (n + T - 1) / T;
  if (!xb_snap) {
    XCHK(dalloc((unsigned char**)&xb_snap, xb_snap_bytes()));
    XCHK(dalloc((unsigned char**)&xb_ctl, xb_ctl_bytes()));
    XCHK(dalloc(&xb_nstot, XMAXCTX));
  }
  if (nt > xb_tcap) {
    XCHK(hipStreamSynchronize(stream));
    dfree(xb_tmax); dfree(xb_pcarry); dfree(xb_segtail); dfree(xb_mcarry); dfree(xb_nscnt); dfree(xb_evcnt);
    dfree(xb_seghas); dfree(xb_tjump); dfree(xb_tmin);
    const int64_t c = std::max<int64_t>(nt, 64);
    XCHK(dalloc(&xb_tmax, c)); XCHK(dalloc(&xb_pcarry, c)); XCHK(dalloc(&xb_segtail, c));
    XCHK(dalloc(&xb_mcarry, c)); XCHK(dalloc(&xb_nscnt, (size_t)c * XMAXCTX)); XCHK(dalloc(&xb_evcnt, c));
    XCHK(dalloc(&xb_seghas, c));
    XCHK(dalloc(&xb_tjump, c));
    XCHK(dalloc(&xb_tmin, c));
    xb_tcap = c;
  }
  if (n > xb_ncap) {
    XCHK(hipStreamSynchronize(stream));
    dfree(xb_bits);
    XCHK(dalloc(&xb_bits, (size_t)(n / 32 + 2)));
    xb_ncap = n;
  }
  if (sc > xb_sufcap) {
    XCHK(hipStreamSynchronize(stream));
    dfree(xb_sufmin);
    xb_sufcap = sc;
    XCHK(dalloc(&xb_sufmin, xb_sufcap));
  }
  if ((int64_t)XMAXCTX * sesscap > xb_reachcap) {
    XCHK(hipStreamSynchronize(stream));
    dfree(xb_reach);
    xb_reachcap = (int64_t)XMAXCTX * std::max<int32_t>(sesscap, 1);
    XCHK(dalloc(&xb_reach, xb_reachcap));
  }
  XBArgs a{};
  a.ts = d_ts;
  a.val = d_val;
  a.n = n;
  a.ntiles = nt;
  a.cfg = d_cfg;
  a.st = d_st;
  a.sl = sl;
  a.ss = ss;
  a.snap = (XSnap*)xb_snap;
  a.reach = xb_reach;
  a.tmax = xb_tmax;
  a.pcarry = xb_pcarry;
  a.ns_cnt = xb_nscnt;
  a.ns_tot = xb_nstot;
  a.ev_cnt = xb_evcnt;
  a.seg_tail = xb_segtail;
  a.seg_has = xb_seghas;
  a.m_carry = xb_mcarry;
  a.evbits = xb_bits;
  a.ctl = (XBCtl*)xb_ctl;
  a.vt = vt;
  a.cfg_nctx_host = cfg.n_ctx;
  a.sufmin = xb_sufmin;
  a.tjump = xb_tjump;
  a.tmin = xb_tmin;
  // One host synchronisation per round: the event and new-session buffers keep their size from earlier rounds; a
  // round that outgrows them applies nothing (XBCtl.retry) and runs again with grown buffers.
  for (int attempt = 0;; attempt++) {
    a.ns_start = xb_nsstart;
    a.ns_pb = xb_nspb;
    a.ns_cap = xb_nscap;
    a.ev_pos = xb_evpos;
    a.ev_t = xb_evt;
    a.ev_v = xb_evv;
    a.ev_m = xb_evm;
    a.ev_cap = xb_evcap;
    a.ep_pos = xb_eppos;
    a.ep_tail = xb_eptail;
    a.ep_cap = xb_evcap + 4;
    XCHK(hipMemsetAsync(xb_ctl, 0, xb_ctl_bytes(), stream));
    // XBCtl.resume: a device-side fill (a pageable 4-byte host copy went through a staging buffer every round)
    if (resume) XCHK(hipMemsetD32Async((hipDeviceptr_t)((unsigned char*)xb_ctl + 48), 1, 1, stream));
    XCHK(xb_classify_phase(a, 0, stream));
    XCHK(xb_classify_phase(a, 1, stream));
    XCHK(xb_classify_phase(a, 2, stream));
    const bool prof = getenv("SCOTTY_XB_PROF") != nullptr;
    if (prof && !d_dbg) XCHK(dalloc(&d_dbg, 256));
    a.dbg = prof ? d_dbg : nullptr;
    XCHK(xb_events(a, stream));
    if (prof) {  // debugging aid: clock stamps of the event pass (100 MHz-ish s_memtime ticks, see MI355X guide)
      long long h[256];
      XCHK(hipMemcpyAsync(h, d_dbg, sizeof(h), hipMemcpyDeviceToHost, stream));
      XCHK(hipStreamSynchronize(stream));
      fprintf(stderr, "xb events pass stamps (%lld):", h[0]);
      for (int i = 2; i <= h[0] && i < 256; i++) fprintf(stderr, " %lld", h[i] - h[i - 1]);
      fprintf(stderr, "\n");
    }
    XCHK(xb_apply(a, stream));
    static_assert(sizeof(int64_t) * 9 >= 68, "XBCtl layout");
    XCHK(launch_copy2_to_host(xb_ctl, h_misc_dev, 72, xb_nstot, h_misc_dev + 9, cfg.n_ctx > 0 ? 8 * cfg.n_ctx : 0,
                              stream));
    XCHK(hipStreamSynchronize(stream));
    const int64_t nev = h_misc[0];
    const int32_t retry = ((const int32_t*)(h_misc + 8))[0];
    if (!retry) {
      last_events += nev;
      const int32_t stopped = ((const int32_t*)(h_misc + 5))[0];
      if (stopped) *stop_at = h_misc[3];  // XBCtl.seg_end
      const int32_t lost = ((const int32_t*)(h_misc + 6))[1];  // XBCtl.pad: simple tuples without a slice
      if (lost) {
        err = "internal: simple tuple without a slice (" + std::to_string(lost) + ")";
        failed = true;
        return SCOTTY_ERR_STATE;
      }
      return SCOTTY_OK;
    }
    if (attempt >= 2) {
      err = "internal: exact batch buffers did not converge";
      failed = true;
      return SCOTTY_ERR_STATE;
    }
    int64_t mx = 1;
    for (int k = 0; k < cfg.n_ctx; k++) mx = std::max<int64_t>(mx, h_misc[9 + k]);
    if (mx > xb_nscap) {
      dfree(xb_nsstart); dfree(xb_nspb);
      xb_nscap = std::max<int64_t>({mx, 2 * xb_nscap, (int64_t)1024});
      XCHK(dalloc(&xb_nsstart, (size_t)xb_nscap * XMAXCTX));
      XCHK(dalloc(&xb_nspb, (size_t)xb_nscap * XMAXCTX));
    }
    if (nev + 4 > xb_evcap) {
      dfree(xb_evpos); dfree(xb_evt); dfree(xb_evv); dfree(xb_evm); dfree(xb_eppos); dfree(xb_eptail);
      xb_evcap = std::max<int64_t>({nev + 4, 2 * xb_evcap, (int64_t)4096});
      XCHK(dalloc(&xb_evpos, xb_evcap)); XCHK(dalloc(&xb_evt, xb_evcap)); XCHK(dalloc(&xb_evv, xb_evcap));
      XCHK(dalloc(&xb_evm, xb_evcap)); XCHK(dalloc(&xb_eppos, xb_evcap + 4)); XCHK(dalloc(&xb_eptail, xb_evcap + 4));
    }
  }
  return SCOTTY_OK;
}

// Sort-free path (keyed_grid.hip) for one batch.  *deferred: -1 the batch did not qualify (nothing changed),
// else the number of tuples left marked for the replay path (keys new or not eligible in this batch).
int XEngine::push_kg(const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n, int64_t* deferred,
                     int32_t* flag_out) {
  *deferred = -1;
  *flag_out = -1;
  // compact key table over the known keys (<= 50 % load), rebuilt when keys were added
  uint64_t want = 2048;
  while ((int64_t)want < 2 * n_ops) want <<= 1;
  if ((want >> KG_RB) > (uint64_t)KG_NB_MAX) return SCOTTY_OK;  // > 2^21 keys: replay path
  if (want != kgcap) {
    XCHK(hipStreamSynchronize(stream));
    dfree(d_kgtab);
    XCHK(dalloc(&d_kgtab, want));
    kgcap = want;
    kg_built = -1;
  }
  if (kg_built != n_ops) {
    XCHK(hipMemsetAsync(d_kgtab, 0, kgcap * 8, stream));
    XCHK(launch_kg_build(d_slot_key, n_ops, d_kgtab, kgcap - 1, stream));
    kg_built = n_ops;
  }
  const int vb = vt == VT_I32 ? 4 : 8;
  const int rec = vt == VT_I32 ? 12 : 16;  // KRec<4> / KRec<8> (keyed_grid.hip)
  const int64_t nbk = (int64_t)(kgcap >> KG_RB);
  const int tile = kg_tile(vt, nbk, kg_variant);
  const int64_t ntiles = (n + tile - 1) / tile;
  const bool mm = (cfg.need & (NEED_MIN | NEED_MAX)) != 0;
  const int cm = kg_cells(mm);
  if (n_ops * cm > kg_pcap) {  // per-(key, cell) partials and deferral flags, zero between batches
    XCHK(hipStreamSynchronize(stream));
    dfree(d_kgpart); dfree(d_kgdflag);
    kg_pcap = std::max<int64_t>(ops_cap * cm, 4096);
    XCHK(dalloc(&d_kgpart, kg_pcap));
    XCHK(dalloc(&d_kgdflag, kg_pcap));
    XCHK(hipMemsetAsync(d_kgpart, 0, kg_pcap * sizeof(KPart), stream));
    XCHK(hipMemsetAsync(d_kgdflag, 0, kg_pcap, stream));
  }
  if (n > kg_ncap) {
    XCHK(hipStreamSynchronize(stream));
    dfree(d_kgrec); dfree(d_kgmark); dfree(d_kgblk);
    kg_ncap = std::max<int64_t>(n, 1 << 16);
    XCHK(dalloc((unsigned char**)&d_kgrec, (size_t)kg_ncap * rec));
    XCHK(dalloc(&d_kgmark, kg_ncap));
    XCHK(hipMemsetAsync(d_kgmark, 0, kg_ncap, stream));  // marks are reset by the gather that consumes them
    XCHK(dalloc(&d_kgblk, kg_ncap / 1024 + 64));
  }
  if (nbk * ntiles > kg_hcap) {
    XCHK(hipStreamSynchronize(stream));
    dfree(d_kghist); dfree(d_kgscan);
    kg_hcap = std::max<int64_t>(nbk * ntiles, 1 << 16);
    XCHK(dalloc(&d_kghist, kg_hcap));
    XCHK(dalloc(&d_kgscan, kg_hcap / 512 + 64));
  }
  if (!d_kgctl) {
    XCHK(dalloc((unsigned char**)&d_kgctl, sizeof(KgCtl)));
    XCHK(mapped_host_alloc(&h_kgctl, &h_kgctl_dev, sizeof(KgCtl)));
  }
  KgArgs a{};
  a.key = d_key;
  a.ts = d_ts;
  a.val = d_val;
  a.n = n;
  a.ktab = d_kgtab;
  a.kmask = kgcap - 1;
  a.nbk = (int32_t)nbk;
  a.ntiles = (int32_t)ntiles;
  a.cmax = cm;
  a.tile = tile;
  a.variant = kg_variant;
  // 8-byte records with the default kernels only (scotty_tune "keyed_grid_variant" 0: the 12-byte records, A/B)
  a.allow_compact = vt == VT_I32 && kg_variant >= 1 && tile == 8192 ? 1 : 0;
  a.part = d_kgpart;
  a.dflag = d_kgdflag;
  a.hist = d_kghist;
  a.rec = d_kgrec;
  a.mark = d_kgmark;
  a.ctl = (KgCtl*)d_kgctl;
  a.cfg = d_cfg;
  a.st = d_st;
  a.sl = sl;
  // device time: the data pass over the tuples (class INGEST: histogram, scan, partition, per-(key, cell) fold),
  // then the per-key commit (PUSH_OTHER)
  TEv t0, t1;
  int rc = tbegin(t0, SCOTTY_TIME_INGEST);
  if (rc) return rc;
  XCHK(launch_kg_partition(a, vt, stream));
  XCHK(launch_scan_i32(d_kghist, d_kghist, nbk * ntiles, d_kgscan, stream));
  XCHK(launch_kg_scatter(a, vt, stream));
  XCHK(launch_kg_bucket(a, vt, mm, n_ops, stream, 1));
  if ((rc = tend(t0, n))) return rc;
  if ((rc = tbegin(t1, SCOTTY_TIME_PUSH_OTHER))) return rc;
  XCHK(launch_kg_bucket(a, vt, mm, n_ops, stream, 2));
  KgCtl* hc = (KgCtl*)h_kgctl;
  static_assert(sizeof(KgCtl) % 4 == 0, "KgCtl copied in words");
  XCHK(launch_copy_to_host(d_kgctl, h_kgctl_dev, sizeof(KgCtl), stream));
  if ((rc = tend(t1, 0))) return rc;
  XCHK(hipStreamSynchronize(stream));
  if (timing) collect_timing();
  (void)vb;
  *flag_out = hc->flag;
  if (hc->flag) return SCOTTY_OK;
  *deferred = (int64_t)hc->deferred;
  for (int i = 0; i < KG_SHARDS; i++) last_kg_keys += (int64_t)hc->keys_shard[i];
  if (hc->deferred > 0) {  // tuples of keys the bucket kernel missed or the commit deferred: mark, clear the flags
    XCHK(launch_kg_mark_deferred(a, stream));
    if (hc->defer_keys > 0) XCHK(hipMemsetAsync(d_kgdflag, 0, n_ops, stream));
  }
  return SCOTTY_OK;
}

int XEngine::push_keyed(const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n) {
  if (n <= 0) return SCOTTY_OK;
  last_kg = 0;
  last_kg_deferred = 0;
  last_kg_keys = 0;
  kg_used = kg_replayed = 0;
  int rc;
  if (lane_mode() && !kg_off && n < ((int64_t)1 << 31)) rc = push_keyed_kg(d_key, d_ts, d_val, n, true);
  else rc = push_keyed_replay(d_key, d_ts, d_val, n);
  last_kg = kg_used ? (kg_replayed ? 2 : 1) : 0;
  return rc;
}

// One in-order range through the sort-free path: deferred keys' tuples replayed after it; a range over more grid
// cells than a bucket pass keeps cut into chunks of consecutive cells (split), each run the same way in order
// (a chunk's replay precedes the next chunk, so a key deferred in one chunk is current in the next); a range the
// path cannot take replayed whole.  Every tuple is processed once, in an order that keeps each key's arrival order.
int XEngine::push_keyed_kg(const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n, bool split) {
  if (n <= 0) return SCOTTY_OK;
  if (n_ops == 0) {  // no key known yet: every key is new
    kg_replayed = 1;
    return push_keyed_replay(d_key, d_ts, d_val, n);
  }
  int64_t deferred = -1;
  int32_t flag = 0;
  int rc = push_kg(d_key, d_ts, d_val, n, &deferred, &flag);
  if (rc) return rc;
  if (flag == 0) {
    kg_used = 1;
    if (deferred == 0) return SCOTTY_OK;
    // gather the deferred keys' tuples in arrival order, replay them
    kg_replayed = 1;
    last_kg_deferred += deferred;
    const int64_t nblk = (n + 1023) / 1024;
    XCHK(launch_kg_dcount(d_kgmark, n, d_kgblk, stream));
    XCHK(launch_scan_i32(d_kgblk, d_kgblk, nblk, d_kgscan, stream));
    if (deferred > kg_gcap) {
      XCHK(hipStreamSynchronize(stream));
      dfree(d_kgkey); dfree(d_kgts); dfree(d_kgval);
      kg_gcap = std::max<int64_t>(deferred, 1 << 16);
      XCHK(dalloc(&d_kgkey, kg_gcap));
      XCHK(dalloc(&d_kgts, kg_gcap));
      XCHK(dalloc((unsigned char**)&d_kgval, (size_t)kg_gcap * (vt == VT_I32 ? 4 : 8)));
    }
    XCHK(launch_kg_dgather(d_key, d_ts, d_val, d_kgmark, n, d_kgblk, d_kgkey, d_kgts, d_kgval, vt, stream));
    return push_keyed_replay(d_kgkey, d_kgts, d_kgval, deferred);
  }
  const int cm = kg_cells((cfg.need & (NEED_MIN | NEED_MAX)) != 0);
  if (split && flag == KG_CELLS) {
    constexpr int KMAX = 4096;
    if (!d_kggpts) {
      XCHK(dalloc(&d_kggpts, KMAX));
      XCHK(dalloc(&d_kgpos, KMAX + 1));
    }
    XCHK(launch_kg_bounds(d_ts, n, d_cfg, KMAX, d_kggpts, d_kgpos, stream));
    h_kgpos.resize(KMAX + 1);
    XCHK(hipMemcpyAsync(h_kgpos.data(), d_kgpos, 8, hipMemcpyDeviceToHost, stream));
    XCHK(hipStreamSynchronize(stream));
    const int64_t k = h_kgpos[0];
    const bool more = k == KMAX;  // the walk stopped at KMAX grid points: whole chunks now, the rest after
    const int64_t chunks = k < 0 ? 0 : (more ? k / cm : k / cm + 1);
    if (k > 0 && n / chunks >= kg_min_chunk) {
      XCHK(hipMemcpy(h_kgpos.data() + 1, d_kgpos + 1, k * 8, hipMemcpyDeviceToHost));
      bool mono = true;
      for (int64_t j = 1; j < k; j++) mono = mono && h_kgpos[1 + j] >= h_kgpos[j];
      if (mono) {
        // chunk c: cells [c*cm, (c+1)*cm), i.e. tuples from the first >= g_{c*cm} (cell 0: from 0)
        const int vb = vt == VT_I32 ? 4 : 8;
        int64_t p0 = 0;
        for (int64_t c = 0; c < chunks; c++) {
          const int64_t j = (c + 1) * cm;  // grid point g_j starts the next chunk (1-based)
          const int64_t p1 = j <= k ? h_kgpos[j] : n;
          if (p1 > p0) {
            rc = push_keyed_kg(d_key + p0, d_ts + p0, (const unsigned char*)d_val + p0 * vb, p1 - p0, false);
            if (rc) return rc;
          }
          p0 = p1;
        }
        if (p0 < n) {  // the rest of a walk cut at KMAX grid points, in order
          rc = push_keyed_kg(d_key + p0, d_ts + p0, (const unsigned char*)d_val + p0 * vb, n - p0, true);
          if (rc) return rc;
        }
        return SCOTTY_OK;
      }
    }
  }
  kg_replayed = 1;
  return push_keyed_replay(d_key, d_ts, d_val, n);
}

int XEngine::push_keyed_replay(const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n) {
  if (n <= 0) return SCOTTY_OK;
  int rc = ensure_batch(n);
  if (rc) return rc;
  if (!d_kmax) XCHK(dalloc(&d_kmax, 4));
  // 1. stable sort of the batch by KEY (arrival order kept within each key, which the reference's out-of-order
  //    handling depends on), over the bits the batch's largest key needs
  // device time: the sort, segment and key-table passes are PUSH_OTHER, the per-key replay kernel (the path's
  // largest single kernel) is INGEST, timed per launch
  TEv tk, ts0, tr;
  if ((rc = tbegin(tk, SCOTTY_TIME_PUSH_OTHER))) return rc;
  //    The lane-session replay of an int32 batch whose key bits and event-time span fit one 32-bit word sorts
  //    packed 8-byte records (keyed_kernels.hip, Rec<8>): the key range pass then also takes the timestamp range
  const bool pack_try = vt == VT_I32 && lane_session_mode() && !pack_off;
  // (one read of the keys, and of the timestamps when packing: also the sort's first digit histogram)
  const int64_t hist_nb = (bcap + sort_tile() - 1) / sort_tile();
  // (the 10-bit first digit's histogram only for the 10-bit sort A/B: scotty_tune "keyed_sort_digit10" 1)
  int32_t* d_hist10 = sort_digit10 == 1 ? d_hist + 256 * hist_nb : nullptr;
  XCHK(launch_range_hist(d_key, pack_try ? d_ts : nullptr, n, d_hist, d_hist10, d_rpart, d_kmax, stream));
  if ((rc = tend(tk, 0))) return rc;
  XCHK(hipMemcpyAsync(h_misc, d_kmax, 24, hipMemcpyDeviceToHost, stream));
  XCHK(hipStreamSynchronize(stream));
  const uint64_t kmax = (uint64_t)(uint32_t)h_misc[0];
  const int kb = bits_for((int64_t)kmax + 1);
  int rec = vt == VT_I32 ? 16 : 24;
  int64_t tbase = 0;
  int tb = 0;
  if (pack_try) {
    const int64_t tlo = (int64_t)(~(uint64_t)h_misc[1] ^ 0x8000000000000000ull);
    const int64_t thi = (int64_t)((uint64_t)h_misc[2] ^ 0x8000000000000000ull);
    const uint64_t span = (uint64_t)thi - (uint64_t)tlo;  // thi >= tlo (n > 0)
    if (span < ((uint64_t)1 << 31)) {
      tb = bits_for((int64_t)span + 1);
      if (tb + kb <= 32) {
        rec = 8;
        tbase = tlo;
      }
    }
  }
  last_rec_bytes = rec;
  void* sorted = nullptr;
  if ((rc = tbegin(ts0, SCOTTY_TIME_PUSH_OTHER))) return rc;
  XCHK(launch_sort_by_slot(rec, d_ts, d_val, d_key, n, kb, d_recA, d_recB, d_hist, d_hist10, d_scan32, &sorted, stream,
                           tbase, tb, true, sort_digit10));
  // 2. the batch's distinct keys in key order (segment u = [ubeg[u], ubeg[u + 1])) and its largest timestamp
  const int64_t nbs = seg_tiles(n);
  XCHK(launch_seg_count(rec, sorted, n, d_segcnt, (long long*)d_tmaxt, d_need + 3, stream, tbase, tb));
  XCHK(launch_scan_i32(d_segcnt, d_segoff, nbs, d_segscan, stream));
  XCHK(launch_seg_write(rec, sorted, n, d_segoff, d_ukey, d_ubeg, stream, tbase, tb));
  if ((rc = tend(ts0, 0))) return rc;
  XCHK(hipMemcpyAsync(h_misc, d_segoff + nbs - 1, 4, hipMemcpyDeviceToHost, stream));
  XCHK(hipMemcpyAsync((unsigned char*)h_misc + 4, d_segcnt + nbs - 1, 4, hipMemcpyDeviceToHost, stream));
  XCHK(hipStreamSynchronize(stream));
  const int64_t u_n = (int64_t)((const int32_t*)h_misc)[0] + (int64_t)((const int32_t*)h_misc)[1];
  // 3. distinct keys -> slots (KeyedScottyWindowOperator.processElement: HashMap.put(key, initWindowOperator()) for
  //    a key's first tuple): one probe per key of the batch.  A table that fills up mid-pass is grown (the pass's
  //    unassigned insertions dropped) and the pass re-run.
  rc = ensure_table(n_ops + u_n);
  if (rc) return rc;
  for (int attempt = 0;; attempt++) {
    XCHK(hipMemsetAsync(d_newcnt, 0, 8, stream));
    XCHK(hipMemsetAsync(d_full, 0, 4, stream));
    XCHK(launch_key_insert(d_ukey, u_n, d_table, tcap - 1, d_newpos, d_newcnt, d_full, d_slot, stream));
    XCHK(hipMemcpyAsync(h_misc, d_newcnt, 8, hipMemcpyDeviceToHost, stream));
    XCHK(hipMemcpyAsync(h_misc + 1, d_full, 4, hipMemcpyDeviceToHost, stream));
    XCHK(hipStreamSynchronize(stream));
    if ((int32_t)h_misc[1] == 0) break;
    if (attempt >= 8 || (int64_t)tcap >= ((int64_t)1 << 33)) {
      err = "key hash table full";
      failed = true;
      return SCOTTY_ERR_NOMEM;
    }
    rc = ensure_table((int64_t)tcap, true);  // 2x the slots
    if (rc) return rc;
  }
  const int64_t n_new = h_misc[0];
  if (n_new > 0) {
    rc = grow_ops(n_ops + n_new);
    if (rc) return rc;
    XCHK(launch_key_assign(d_table, d_newpos, n_new, n_ops, d_slot_key, stream));
    XCHK(launch_xstate_init(d_st, n_ops, n_ops + n_new, d_slot_key, stream));
    h_slot_key.resize(n_ops + n_new);
    XCHK(hipMemcpyAsync(h_slot_key.data() + n_ops, d_slot_key + n_ops, n_new * 4, hipMemcpyDeviceToHost, stream));
    n_ops += n_new;
    if ((int64_t)2 * n_ops > (int64_t)tcap) {
      rc = ensure_table(n_ops);
      if (rc) return rc;
    }
    XCHK(launch_slot(d_ukey, u_n, d_table, tcap - 1, d_slot, true, stream));  // the new keys' slots
  }
  // 4. every operator's segment of the sorted batch (empty for keys without tuples in it)
  if (seg_cap < n_ops) {
    XCHK(hipStreamSynchronize(stream));
    dfree(d_seg_b);
    dfree(d_seg_e);
    seg_cap = std::max<int64_t>(ops_cap, 1024);
    XCHK(dalloc(&d_seg_b, seg_cap));
    XCHK(dalloc(&d_seg_e, seg_cap));
  }
  XCHK(hipMemsetAsync(d_seg_b, 0, n_ops * 8, stream));
  XCHK(hipMemsetAsync(d_seg_e, 0, n_ops * 8, stream));
  XCHK(launch_seg_fill(d_ubeg, d_slot, u_n, n, d_seg_b, d_seg_e, stream));
  // 5. per-key replay; ops whose capacities might overflow are deferred, the tables grown, and relaunched
  XBatchArgs a = batch_args();
  a.ts = (const int64_t*)sorted;
  a.val = nullptr;
  a.n = n;
  a.seg_begin = d_seg_b;
  a.seg_end = d_seg_e;
  a.rec_stride = rec;
  a.pk_base = tbase;
  a.pk_bits = tb;
  a.need = d_need;
  a.ts_max_b = d_need + 3;
  if (lsdbg_on) {
    if (!d_lsdbg) {
      XCHK(dalloc(&d_lsdbg, 16));
      XCHK(hipMemsetAsync(d_lsdbg, 0, 16 * 8, stream));
    }
    a.dbg = d_lsdbg;
  }
  for (int attempt = 0; attempt < 6; attempt++) {
    XCHK(hipMemsetAsync(d_need, 0, 24, stream));
    a.retry = attempt > 0;
    a.sl = sl;
    a.ss = ss;
    // the wavefront replay does not track the lane paths' slice prefixes (XState.pvalid)
    if (!lane_mode() && !lane_session_mode()) prefix_stale = true;
    if ((rc = tbegin(tr, SCOTTY_TIME_INGEST))) return rc;
    XCHK(lane_mode()           ? launch_lane_replay(a, cfg, stream)
         : lane_session_mode() ? launch_lane_session(a, vt, lane_session_occ, stream)
         : lane_count_mode()   ? launch_lane_count(a, vt, stream)
                               : launch_replay(a, vt, stream));
    if ((rc = tend(tr, n))) return rc;
    XCHK(hipMemcpyAsync(h_misc, d_need, 24, hipMemcpyDeviceToHost, stream));
    XCHK(hipStreamSynchronize(stream));
    if (h_misc[0] == 0 && h_misc[1] == 0 && h_misc[2] == 0) return SCOTTY_OK;
    rc = grow_caps(std::max<int64_t>(h_misc[0], sc), std::max<int64_t>(h_misc[1], sesscap), ctx_alloc,
                   std::max<int64_t>(h_misc[2], rcap_));
    if (rc) return rc;
  }
  err = "capacity growth did not converge";
  failed = true;
  return SCOTTY_ERR_NOMEM;
}

int XEngine::ensure_rows(int64_t rows) {
  if (rows <= rcap) return SCOTTY_OK;
  XCHK(hipStreamSynchronize(stream));
  dfree(d_w_start); dfree(d_w_end); dfree(d_w_meas); dfree(d_w_op); dfree(d_w_key); dfree(d_has);
  for (int k = 0; k < SCOTTY_MAX_AGGS; k++) {
    dfree(d_vals[k]);
    d_vals[k] = nullptr;
  }
  const int64_t cap = std::max<int64_t>(rows + rows / 2, 1024);
  XCHK(dalloc(&d_w_start, cap));
  XCHK(dalloc(&d_w_end, cap));
  XCHK(dalloc(&d_w_meas, cap));
  XCHK(dalloc(&d_w_op, cap));
  XCHK(dalloc(&d_w_key, cap));
  XCHK(dalloc(&d_has, cap));
  for (int k = 0; k < cfg.n_aggs; k++) XCHK(dalloc(&d_vals[k], cap));
  rcap = cap;
  return SCOTTY_OK;
}

int XEngine::watermark(int64_t wm, XResult& r, bool to_host) {
  r.n = 0;
  r.dropped = 0;
  r.clear_cols(cfg.n_aggs);
  if (n_ops == 0) return SCOTTY_OK;
  if (wcap < n_ops) {
    XCHK(hipStreamSynchronize(stream));
    dfree(d_wcount); dfree(d_woff); dfree(d_scan64);
    wcap = std::max<int64_t>(ops_cap, 1024);
    XCHK(dalloc(&d_wcount, wcap));
    XCHK(dalloc(&d_woff, wcap));
    XCHK(dalloc(&d_scan64, wcap / 512 + 64));
  }
  XWmArgs a{};
  a.cfg = d_cfg;
  a.st = d_st;
  a.sl = sl;
  a.ss = ss;
  a.n_ops = (int32_t)n_ops;
  a.wm = wm;
  a.wcount = d_wcount;
  a.woff = d_woff;
  a.err_flag = (int32_t*)(d_misc + 0);
  a.dropped_total = (unsigned long long*)(d_misc + 1);
  a.op_err = (int32_t*)(d_misc + 2);
  a.slot_key = keyed ? d_slot_key : nullptr;
  // lane path: COUNT / integer SUM windows straight from the slice prefixes in the emit kernel, integer MIN / MAX from
  // the key-interleaved store's block summaries (XK_QN ...); f64 (and MIN / MAX outside that store) scan the slices
  // (wm_agg).  (MIN / MAX by a lane-per-key scan of each window's contained run in the key-major store measured
  // 2.46 ms per C4 watermark against 1.18 ms with wm_agg: the lanes walk 64 different lines per load.)
  const bool prefix_agg = lane_wm_mode() && !((cfg.need & NEED_SUM) && vt == VT_F64) &&
                          (!(cfg.need & (NEED_MIN | NEED_MAX)) || sl.kw != nullptr);
  a.prefix_reset = prefix_stale ? 1 : 0;
  // one-kernel watermark (rows from a host bound) for context-free windows only; sessions take the count pass
  const int64_t bound = prefix_agg && lane_mode() ? lane_row_bound(wm) : -1;
  if (bound >= 0) {  // one kernel: count, reserve, emit, aggregate, GC -- rows sized from the bound
    int rc = ensure_rows(std::max<int64_t>(bound, 1));
    if (rc) return rc;
    XCHK(hipMemsetAsync(d_misc, 0, 4 * 8, stream));
    a.row_count = (unsigned long long*)(d_misc + 3);
    a.n_rows = rcap;
    a.w_start = d_w_start;
    a.w_end = d_w_end;
    a.w_meas = d_w_meas;
    a.w_op = d_w_op;
    a.has_value = d_has;
    for (int k = 0; k < cfg.n_aggs; k++) a.values[k] = d_vals[k];
    a.w_key = d_w_key;
    TEv tw;
    int rct = tbegin(tw, SCOTTY_TIME_WATERMARK);
    if (rct) return rct;
    XCHK(launch_lane_wm_emit(a, true, stream));
    XCHK(launch_copy_to_host(d_misc, h_misc_dev, 4 * 8, stream));
    if ((rct = tend(tw, 0))) return rct;
    XCHK(hipStreamSynchronize(stream));
    if (timing) collect_timing();
    prefix_stale = false;
    have_wm = true;
    last_wm = wm;
    r.dropped = (uint64_t)h_misc[1];
    rc = op_error((int32_t)h_misc[2]);
    if (rc) return rc;
    if ((int32_t)h_misc[0] & 4) {
      err = "internal: watermark rows exceeded the host bound";
      failed = true;
      return SCOTTY_ERR_STATE;
    }
    return finish_rows((int64_t)h_misc[3], r, to_host, false);
  }
  const int64_t sbound = !keyed && n_ops == 1 && !lane_mode() ? single_row_bound(wm) : -1;
  if (sbound >= 0) {  // one operator: no count pass -- the emit kernel checks, emits and counts (rows from a bound)
    int rc = ensure_rows(std::max<int64_t>(sbound, 1));
    if (rc) return rc;
    if (!cfg.records) {  // 64-slice block summaries of the scan range for the window assembly (wm_blocks_kernel)
      const int64_t need_b = (int64_t)sc / XB_BLK + 2;
      if (xblk_cap < need_b) {
        XCHK(hipStreamSynchronize(stream));
        dfree(xblk.cnt); dfree(xblk.sum); dfree(xblk.mn); dfree(xblk.mx); dfree(xblk.ts_min); dfree(xblk.tl_max);
        XCHK(dalloc(&xblk.cnt, need_b)); XCHK(dalloc(&xblk.sum, need_b)); XCHK(dalloc(&xblk.mn, need_b));
        XCHK(dalloc(&xblk.mx, need_b)); XCHK(dalloc(&xblk.ts_min, need_b)); XCHK(dalloc(&xblk.tl_max, need_b));
        xblk_cap = need_b;
      }
      a.blk = xblk;
      a.blk.nbcap = xblk_cap;
    }
    a.single = 1;
    a.row_count = (unsigned long long*)(d_misc + 3);
    a.n_rows = sbound;
    a.w_start = d_w_start;
    a.w_end = d_w_end;
    a.w_meas = d_w_meas;
    a.w_op = d_w_op;
    a.has_value = d_has;
    for (int k = 0; k < cfg.n_aggs; k++) a.values[k] = d_vals[k];
    a.w_key = d_w_key;
    TEv tw;
    int rct = tbegin(tw, SCOTTY_TIME_WATERMARK);
    if (rct) return rct;
    a.zero4 = (unsigned long long*)d_misc;  // zeroed by the emit kernel (n_ops == 1: one wave) instead of a memset
    XCHK(launch_wm_emit(a, stream));
    if (a.blk.cnt) XCHK(launch_wm_blocks(a, stream));
    XCHK(launch_wm_agg(a, stream, 64));
    XCHK(launch_copy_to_host(d_misc, h_misc_dev, 4 * 8, stream));
    if ((rct = tend(tw, 0))) return rct;
    XCHK(hipStreamSynchronize(stream));
    r.dropped = (uint64_t)h_misc[1];
    rc = op_error((int32_t)h_misc[2]);
    if (rc) return rc;
    const int32_t ef = (int32_t)h_misc[0];
    if (ef & 1) {
      err = "processWatermark threw IndexOutOfBoundsException (empty session context / count trigger before the "
            "oldest slice, S/WindowManager.java:98-118)";
      return SCOTTY_ERR_INDEX;
    }
    if (ef & 4) {
      err = "internal: watermark rows exceeded the host bound";
      failed = true;
      return SCOTTY_ERR_STATE;
    }
    have_wm = true;
    last_wm = wm;
    rc = finish_rows((int64_t)h_misc[3], r, to_host, false);
    if (rc) return rc;
    if (ef & 2) {
      err = "processWatermark threw IndexOutOfBoundsException in LazyAggregateStore.aggregate (getSlice(-1))";
      return SCOTTY_ERR_INDEX;
    }
    if (timing) collect_timing();
    return SCOTTY_OK;
  }
  TEv tw1;
  int rct = tbegin(tw1, SCOTTY_TIME_WATERMARK);
  if (rct) return rct;
  XCHK(hipMemsetAsync(d_misc, 0, 3 * 8, stream));
  XCHK(lane_wm_mode() ? launch_lane_wm_count(a, stream) : launch_wm_count(a, stream));
  XCHK(launch_scan_i64(d_wcount, d_woff, n_ops, d_scan64, stream));
  XCHK(launch_copy_to_host(d_misc, h_misc_dev, 3 * 8, stream));
  XCHK(launch_copy_to_host(d_woff + n_ops - 1, h_misc_dev + 3, 8, stream));
  XCHK(launch_copy_to_host(d_wcount + n_ops - 1, h_misc_dev + 4, 8, stream));
  if ((rct = tend(tw1, 0))) return rct;
  XCHK(hipStreamSynchronize(stream));
  r.dropped = (uint64_t)h_misc[1];
  int rc = op_error((int32_t)h_misc[2]);
  if (rc) return rc;
  if ((int32_t)h_misc[0] & 1) {
    err = "processWatermark threw IndexOutOfBoundsException (empty session context / count trigger before the "
          "oldest slice, S/WindowManager.java:98-118)";
    return SCOTTY_ERR_INDEX;
  }
  const int64_t rows = h_misc[3] + h_misc[4];
  rc = ensure_rows(rows);
  if (rc) return rc;
  a.w_start = d_w_start;
  a.w_end = d_w_end;
  a.w_meas = d_w_meas;
  a.w_op = d_w_op;
  a.has_value = d_has;
  for (int k = 0; k < cfg.n_aggs; k++) a.values[k] = d_vals[k];
  a.w_key = d_w_key;
  a.n_rows = rows;
  TEv tw2;
  if ((rct = tbegin(tw2, SCOTTY_TIME_WATERMARK))) return rct;
  if (lane_wm_mode()) {
    XCHK(launch_lane_wm_emit(a, prefix_agg, stream));
    if (prefix_agg) prefix_stale = false;
  } else {
    XCHK(launch_wm_emit(a, stream));
  }
  if (!prefix_agg) XCHK(launch_wm_agg(a, stream, keyed ? 16 : 64));
  if ((rct = tend(tw2, 0))) return rct;
  have_wm = true;
  last_wm = wm;
  rc = finish_rows(rows, r, to_host, true);
  if (timing) collect_timing();
  return rc;
}

// Fatal per-operator errors recorded by the kernels (OR of 1 << XState.err over the ops).
int XEngine::op_error(int32_t op_err) {
  if (op_err & ~((1 << XERR_INDEX) | (1 << XERR_NPE) | (1 << XERR_NOELEM))) {
    failed = true;
    if (op_err & (1 << XERR_UNSUPPORTED))
      err = "an EagerSlice would have to move LazySlice records (slices created before the operator's slices "
            "became Lazy): not supported on the MI355X path";
    else if (op_err & (1 << XERR_REC_CAP))
      err = "internal: LazySlice record capacity exceeded after the pre-check";
    else if (op_err & (1 << XERR_SLICE_CAP))
      err = "per-operator slice capacity exceeded (scotty_tune \"slice_capacity\")";
    else if (op_err & (1 << XERR_SESS_CAP))
      err = "per-context session capacity exceeded (scotty_tune \"session_capacity\")";
    else if (op_err & (1 << XERR_HANG))
      err = "the reference StreamSlicer loops forever on this configuration (calculateNextFixedEdge returns "
            "Long.MIN_VALUE for a power-of-two time window size/slide, S/StreamSlicer.java:103-116)";
    else
      err = "operator failed";
    return (op_err & (1 << XERR_HANG)) || (op_err & (1 << XERR_UNSUPPORTED)) ? SCOTTY_ERR_UNSUPPORTED
                                                                               : SCOTTY_ERR_NOMEM;
  }
  return SCOTTY_OK;
}

// Upper bound of the rows one lane-path watermark can emit (LaneWindows: every key's last watermark is the
// engine's previous one, or -- keys created since -- max(0, wm - maxLateness), WindowManager.java:43-44; a
// window is emitted once its end passes it).  -1: no useful bound, use the count pass.
int64_t XEngine::lane_row_bound(int64_t wm) const {
  const double lo = std::max(0.0, (double)wm - (double)cfg.max_lateness);
  const double l0 = have_wm ? std::min(lo, (double)last_wm) : lo;
  const double span = std::max(0.0, (double)wm + 1.0 - l0);
  double per = 0;
  for (const XWinDef& w : h_wins) {
    if (w.kind == SCOTTY_WIN_TUMBLING && w.a > 0) per += std::floor(span / (double)w.a) + 2;
    else if (w.kind == SCOTTY_WIN_SLIDING && w.b > 0) per += std::floor(span / (double)w.b) + 2;
    else if (w.kind == SCOTTY_WIN_FIXED_BAND) per += 1;
    else return -1;
  }
  const double rows = per * (double)n_ops;
  return rows > 2e9 ? -1 : (int64_t)rows;
}

// Upper bound of the rows one watermark of the single (non-keyed) operator emits: context-free time windows by the
// lane bound's arithmetic (the operator's lastWatermark is at least the bound's l0), every session of every context
// (at most the session capacity); -1 (count windows): use the count pass.
int64_t XEngine::single_row_bound(int64_t wm) const {
  if (cfg.has_count) return -1;
  const double lo = std::max(0.0, (double)wm - (double)cfg.max_lateness);
  const double l0 = have_wm ? std::min(lo, (double)last_wm) : lo;
  const double span = std::max(0.0, (double)wm + 1.0 - l0);
  double rows = 0;
  for (const XWinDef& w : h_wins) {
    if (w.kind == SCOTTY_WIN_SESSION) rows += (double)sesscap;
    else if (w.kind == SCOTTY_WIN_TUMBLING && w.a > 0) rows += std::floor(span / (double)w.a) + 2;
    else if (w.kind == SCOTTY_WIN_SLIDING && w.b > 0) rows += std::floor(span / (double)w.b) + 2;
    else if (w.kind == SCOTTY_WIN_FIXED_BAND) rows += 1;
    else return -1;
  }
  return rows > 1e6 ? -1 : (int64_t)rows;
}

// check: a kernel may have flagged LazyAggregateStore.aggregate's getSlice(-1) (err_flag bit 1)
int XEngine::finish_rows(int64_t rows, XResult& r, bool to_host, bool check) {
  r.n = rows;
  r.d_start = d_w_start;
  r.d_end = d_w_end;
  r.d_meas = d_w_meas;
  r.d_key = d_w_key;
  r.d_has = d_has;
  for (int k = 0; k < cfg.n_aggs; k++) r.d_vals[k] = d_vals[k];
  TEv tc;
  int rct = tbegin(tc, SCOTTY_TIME_RESULT_COPY);
  if (rct) return rct;
  if (to_host && rows > 0) {
    r.start.resize(rows); r.end.resize(rows); r.meas.resize(rows); r.has.resize(rows); r.key.resize(rows);
    if ((int)r.vals.size() < cfg.n_aggs) r.vals.resize(cfg.n_aggs);
    for (int k = 0; k < cfg.n_aggs; k++) r.vals[k].resize(rows);
    XCHK(hipMemcpyAsync(r.start.data(), d_w_start, rows * 8, hipMemcpyDeviceToHost, stream));
    XCHK(hipMemcpyAsync(r.end.data(), d_w_end, rows * 8, hipMemcpyDeviceToHost, stream));
    XCHK(hipMemcpyAsync(r.meas.data(), d_w_meas, rows * 4, hipMemcpyDeviceToHost, stream));
    XCHK(hipMemcpyAsync(r.has.data(), d_has, rows, hipMemcpyDeviceToHost, stream));
    XCHK(hipMemcpyAsync(r.key.data(), d_w_key, rows * 4, hipMemcpyDeviceToHost, stream));
    for (int k = 0; k < cfg.n_aggs; k++)
      XCHK(hipMemcpyAsync(r.vals[k].data(), d_vals[k], rows * 8, hipMemcpyDeviceToHost, stream));
  }
  if ((rct = tend(tc, 0))) return rct;
  if (!check) {
    if (to_host && rows > 0) XCHK(hipStreamSynchronize(stream));
    return SCOTTY_OK;
  }
  XCHK(hipMemcpyAsync(h_misc, d_misc, 8, hipMemcpyDeviceToHost, stream));
  XCHK(hipStreamSynchronize(stream));
  if ((int32_t)h_misc[0] & 2) {
    err = "processWatermark threw IndexOutOfBoundsException in LazyAggregateStore.aggregate (getSlice(-1))";
    return SCOTTY_ERR_INDEX;
  }
  return SCOTTY_OK;
}

int XEngine::set_last_watermark(int64_t lw) {
  if (n_ops < 1) return SCOTTY_OK;
  last_wm = lw;  // the row bounds start from it
  have_wm = true;
  XCHK(hipMemcpyAsync((unsigned char*)d_st + offsetof(XState, lastWatermark), &lw, 8, hipMemcpyHostToDevice, stream));
  XCHK(hipStreamSynchronize(stream));
  return SCOTTY_OK;
}

int XEngine::slice_count(int64_t op, int64_t* out) {
  if (op < 0 || op >= n_ops) {
    *out = 0;
    return SCOTTY_OK;
  }
  XState s;
  XCHK(hipMemcpy(&s, d_st + op, sizeof(XState), hipMemcpyDeviceToHost));
  *out = s.tail - s.head;
  return SCOTTY_OK;
}

int XEngine::debug_dump(int64_t op, std::vector<int64_t>& out) {
  out.clear();
  if (op < 0 || op >= n_ops) return SCOTTY_ERR_ARG;
  XState s;
  XCHK(hipMemcpy(&s, d_st + op, sizeof(XState), hipMemcpyDeviceToHost));
  const int64_t S = s.tail - s.head, b = op * (int64_t)sc + s.head;
  out.push_back(S);
  std::vector<int64_t> tmp(std::max<int64_t>(S, 1));
  std::vector<int32_t> ty(std::max<int64_t>(S, 1));
  auto col = [&](const void* p) -> int {
    XCHK(hipMemcpy(tmp.data(), (const int64_t*)p + b, S * 8, hipMemcpyDeviceToHost));
    out.insert(out.end(), tmp.begin(), tmp.begin() + S);
    return SCOTTY_OK;
  };
  if (S > 0 && sl.kw) {  // key-interleaved store: the same columns, gathered (one word per position and field)
    const int64_t kc = (int64_t)1 << sl.kc_sh;
    auto kcol = [&](int f, bool ty32) -> int {
      XCHK(hipMemcpy2D(tmp.data(), 8, sl.kw + ((s.head * (int64_t)sl.kw_nf + f) << sl.kc_sh) + op, sl.kw_nf * kc * 8, 8, S,
                       hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < S; i++) out.push_back(ty32 ? (int64_t)(int32_t)tmp[i] : tmp[i]);
      return SCOTTY_OK;
    };
    for (int f : {XK_TS, XK_TE, XK_TL, XK_CNT, XK_CS, XK_CL})
      if (kcol(f, false)) return SCOTTY_ERR_HIP;
    if (kcol(XK_TY, true)) return SCOTTY_ERR_HIP;
  } else if (S > 0) {
    if (col(sl.ts) || col(sl.te) || col(sl.tl) || col(sl.cnt) || col(sl.cs) || col(sl.cl)) return SCOTTY_ERR_HIP;
    XCHK(hipMemcpy(ty.data(), sl.ty + b, S * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < S; i++) out.push_back(ty[i]);
  }
  out.push_back(cfg.n_ctx);
  for (int c = 0; c < cfg.n_ctx; c++) {
    const int ns = s.nsess[c];
    out.push_back(ns);
    const int64_t sb = (op * ctx_alloc + c) * (int64_t)sesscap;
    std::vector<int64_t> a(std::max(ns, 1)), e(std::max(ns, 1));
    if (ns) {
      XCHK(hipMemcpy(a.data(), ss.start + sb, ns * 8, hipMemcpyDeviceToHost));
      XCHK(hipMemcpy(e.data(), ss.end + sb, ns * 8, hipMemcpyDeviceToHost));
    }
    for (int i = 0; i < ns; i++) { out.push_back(a[i]); out.push_back(e[i]); }
  }
  out.push_back(s.maxEventTime); out.push_back(s.nextEdgeTs); out.push_back(s.currentCount);
  out.push_back(s.unsorted); out.push_back(s.head); out.push_back(s.tail);
  out.push_back(s.wlo); out.push_back(s.whi); out.push_back(s.lastWatermark); out.push_back(s.lastCount);
  if (records && S > 0) {  // record ranges, non-null flags, then the records themselves (ts, value)
    if (col(sl.rlo) || col(sl.rhi)) return SCOTTY_ERR_HIP;
    XCHK(hipMemcpy(ty.data(), sl.nn + b, S * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < S; i++) out.push_back(ty[i]);
    out.push_back(s.rend);
    std::vector<int64_t> rt(std::max<int64_t>(s.rend, 1)), rvv(std::max<int64_t>(s.rend, 1));
    if (s.rend > 0) {
      XCHK(hipMemcpy(rt.data(), sl.rts + op * rcap_, s.rend * 8, hipMemcpyDeviceToHost));
      XCHK(hipMemcpy(rvv.data(), sl.rv + op * rcap_, s.rend * 8, hipMemcpyDeviceToHost));
    }
    for (int64_t i = 0; i < s.rend; i++) { out.push_back(rt[i]); out.push_back(rvv[i]); }
  }
  return SCOTTY_OK;
}

int XEngine::read_states(std::vector<XState>& out) {
  out.resize(n_ops);
  if (n_ops) XCHK(hipMemcpy(out.data(), d_st, n_ops * sizeof(XState), hipMemcpyDeviceToHost));
  return SCOTTY_OK;
}

}  // namespace scotty
