// exact_engine.h -- host interface of the exact ("replay") engine (see exact_common.h).
#pragma once
#include <hip/hip_runtime.h>

#include <new>
#include <string>
#include <utility>
#include <vector>

#include "../../include/scotty_mi355x.h"
#include "exact_common.h"
#include "keyed_grid.h"

namespace scotty {

struct XWinDef {  // one Window of WindowOperator.addWindowAssigner, in registration order
  int kind, measure;
  int64_t a, b;
};

// Host result columns in pinned memory (the D2H copies run at DMA speed instead of being staged through pageable
// bounce buffers) that keep their capacity across watermarks and grow without zero-filling: a keyed watermark returns
// up to millions of rows (C4: 2^20 windows, ~33 MB per watermark).
template <class T>
struct PinnedAlloc {
  using value_type = T;
  PinnedAlloc() = default;
  template <class U>
  PinnedAlloc(const PinnedAlloc<U>&) {}
  T* allocate(size_t n) {
    void* p = nullptr;
    if (hipHostMalloc(&p, n * sizeof(T), hipHostMallocDefault) != hipSuccess) throw std::bad_alloc();
    return (T*)p;
  }
  void deallocate(T* p, size_t) { (void)hipHostFree(p); }
  template <class U>
  void construct(U* p) noexcept { ::new ((void*)p) U; }  // resize() leaves new elements uninitialised
  template <class U, class... A>
  void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
  template <class U>
  bool operator==(const PinnedAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const PinnedAlloc<U>&) const { return false; }
};
template <class T>
using pinned_vec = std::vector<T, PinnedAlloc<T>>;

struct XResult {
  int64_t n = 0;
  uint64_t dropped = 0;   // cumulative tuples dropped (reference: exception per tuple)
  // device columns (valid until the next watermark)
  const int64_t *d_start = nullptr, *d_end = nullptr;
  const int32_t* d_meas = nullptr;
  const uint32_t* d_key = nullptr;
  const uint8_t* d_has = nullptr;
  const int64_t* d_vals[SCOTTY_MAX_AGGS] = {};
  // host copies (when requested)
  pinned_vec<int64_t> start, end;
  pinned_vec<int32_t> meas;
  pinned_vec<uint32_t> key;
  pinned_vec<uint8_t> has;
  std::vector<pinned_vec<int64_t>> vals;
  // empty columns that keep their capacity (clear() frees nothing)
  void clear_cols(size_t n_aggs) {
    start.clear(); end.clear(); meas.clear(); has.clear(); key.clear();
    if (vals.size() < n_aggs) vals.resize(n_aggs);
    for (auto& v : vals) v.clear();
  }
};

class XEngine {
 public:
  ~XEngine();
  int init(int device, hipStream_t stream, int vt, bool keyed, std::string& err);
  // agg_inv[i]: function i is an InvertibleAggregateFunction (C/windowFunction/InvertibleAggregateFunction.java)
  int configure(const std::vector<XWinDef>& wins, const std::vector<int>& aggs, int64_t max_lateness,
                const std::vector<int>& agg_inv = {});
  int push(const int64_t* d_ts, const void* d_val, int64_t n);
  int push_keyed(const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n);
  int push_batch(const int64_t* d_ts, const void* d_val, int64_t n);  // non-keyed, batch-parallel
  int push_exact(const int64_t* d_ts, const void* d_val, int64_t n);  // event-exact rounds over [0, n)
  // non-keyed one-pass path (exact_quiet.hip): *result = XQ_COMMITTED, or why the batch needs the event-exact path
  int push_quiet(const int64_t* d_ts, const void* d_val, int64_t n, int32_t* result);
  bool quiet_eligible() const;
  bool quiet_off = false;      // A/B: every non-keyed batch through the event-exact path
  int64_t quiet_commits = 0, quiet_fallbacks = 0, quiet_tail_commits = 0;
  int32_t last_quiet = 0;      // XQ_* verdict of the last non-keyed push (0: not attempted)
  int64_t last_quiet_why = 0;  // XQCtl.why of the last verdict
  int64_t last_quiet_jump = 0;   // first tuple of the arrival tile holding the verdict's first session-gap jump (0: none)
  int64_t quiet_split_commits = 0;  // quiet prefixes committed up to a located jump
  // start band (exact_quiet.h): quiet batches may move the last session's start down (scotty_tune "quiet_band", on by
  // default; 0 sends such batches through the event-exact path)
  bool band_on = true;
  int64_t last_quiet_jump_pos = -1;  // the prep's refusal: arrival index of the first session-gap jump (< 64), else -1
  int64_t quiet_band_moves = 0;      // committed quiet batches that moved a session start (XQCtl.batch_min < band_s)
  int64_t quiet_band_noedge = 0;     // of those: no slice ended at the session start (band_si -2, only the start moved)
  int64_t quiet_jump_pieces = 0;     // event-exact pieces cut right behind a located jump (then the quiet path again)
  bool band_usable() const { return band_on && cfg.n_ctx == 1 && !cfg.lazy; }
  // first event-exact piece of a refused quiet batch, in tuples (scotty_tune "exact_prefix"; 0: max(n / 32, 2^20))
  int64_t xq_prefix = 0;
  // the quiet pass's ingest launch (A/B, scotty_tune "quiet_ingest_mode" / "quiet_ingest_blocks"): mode 7 = the loop
  // without the DQ2 deferred queue, -1 the default; blocks 0 = one round of resident workgroups
  int32_t xq_ingest_mode = -1;
  int64_t xq_ingest_blocks = 0;
  // batches whose own quiet verdict fails on their tuples (below the cell view / too late / past the grid horizon:
  // XQCtl.why bit 1; below the last session's start: bit 2) back the quiet path off: after two such batches in a row,
  // the next 1, 2, 4 .. 16 batches go straight to the event-exact path
  int32_t xq_refused_run = 0, xq_skip = 0;
  int64_t quiet_skipped = 0;        // batches that went to the event-exact path under that back-off
  // verdicts of the last batch's quiet attempts, in order: XQ_* | why << 8 | (attempt's first tuple) << 24 (debugging)
  std::vector<int64_t> xq_trace;
  // device time of the last pushes by class (HIP events; scotty_device_timing): 0 quiet ingest, 1 other push work
  bool timing = false;
  struct TEv {
    hipEvent_t a = nullptr, b = nullptr;
    int cls = 0;
    int64_t n = 0;
  };
  std::vector<TEv> ev_pending, ev_pool;
  double t_ms[4] = {0, 0, 0, 0};
  int64_t t_cnt[4] = {0, 0, 0, 0};
  int64_t t_tuples = 0;
  int collect_timing();
  int push_round(const int64_t* d_ts, const void* d_val, int64_t n, bool resume, int64_t* stop_at);
  int64_t last_events = 0, last_segments = 0;                          // statistics of the last push
  int watermark(int64_t wm, XResult& r, bool to_host);
  int slice_count(int64_t op, int64_t* out);
  int read_states(std::vector<XState>& out);
  int debug_dump(int64_t op, std::vector<int64_t>& out);  // slices + sessions of one op (tests / debugging)
  int64_t key_count() const { return keyed ? n_ops : 0; }
  int set_last_watermark(int64_t lw);  // non-keyed: watermarks seen before the first tuple

  std::string err;
  bool failed = false;
  int32_t sc_override = 0, sess_override = 0;
  bool serial = false;  // non-keyed: single-wavefront replay instead of the batch-parallel path (A/B)
  bool lane_off = false;  // keyed: force the wavefront-per-key replay even where the lane path applies (A/B)
  bool kg_off = false;    // keyed: no sort-free path (keyed_grid.hip), every batch sorted + replayed (A/B)
  // a batch over more grid cells than one bucket pass keeps is cut into chunks of consecutive cells when they
  // average at least this many tuples (below, the sort + replay path is cheaper than a pass per chunk)
  int64_t kg_min_chunk = 1 << 19;
  int32_t kg_variant = 1;   // sort-free path kernel variant (A/B)
  // last keyed push: 0 replay path only, 1 sort-free path only, 2 both (deferred keys / chunks replayed)
  int32_t last_kg = 0;
  int64_t last_kg_deferred = 0, last_kg_keys = 0;
  bool lane_mode() const {  // keyed_lane.hip: context-free time windows on Eager slices only
    return keyed && !lane_off && cfg.n_ctx == 0 && !cfg.has_count && !cfg.lazy && !records && cfg.n_cf > 0;
  }
  unsigned long long* d_lsdbg = nullptr;  // lane-session path counters (scotty_tune "lane_session_counters" 1)
  bool lsdbg_on = false;
  bool pack_off = false;          // keyed replay: 16-byte records even when a batch fits 8 ("keyed_pack_records" 0)
  int sort_digit10 = -1;          // keyed replay sort digits: 8-bit (-1 default, 0), 10-bit for 17-20-bit keys (1, A/B)
  int64_t last_rec_bytes = 0;     // the last keyed replay's record size (debug stat 107)
  int lane_session_occ = 2;       // lane-session kernel build: 2 (default) or 3 waves per SIMD ("keyed_lane_session" 1 / 2)
  bool lane_session_off = false;  // keyed: sessions through the wavefront replay instead (A/B, "keyed_lane_session" 0)
  bool lane_count_off = false;    // keyed: LazySlice record sets through the wavefront replay instead (A/B, "keyed_lane_count" 0)
  // keyed_lane_count.hip: LazySlice record sets (count windows), no session windows -- one lane per key
  bool lane_count_mode() const { return keyed && !lane_count_off && records && cfg.n_ctx == 0; }
  // keyed_lane_session.hip: time-measured session windows (beside context-free time windows) on Eager slices
  bool lane_session_mode() const {
    if (!keyed || lane_session_off || cfg.n_ctx == 0 || cfg.has_count || cfg.lazy || records || !cfg.has_time)
      return false;
    for (int k = 0; k < cfg.n_ctx; k++)
      if (cfg.ctx_measure[k] != 0) return false;
    return true;
  }
  // keyed_lane.hip's lane-per-key watermark (count / emit / scan range / GC): context-free windows, and sessions on
  // the lane-session path
  bool lane_wm_mode() const { return lane_mode() || lane_session_mode(); }
  // non-keyed: the single-wavefront replay (LazySlice record sets live only there)
  bool use_serial() const { return serial || records; }
  bool records = false;   // LazySlice record sets kept (XCfg.records)
  // lane path with integer values: the slice store is kept key-interleaved (XSlices.kw, XKView),
  // fixed with the first allocation -- the lane path cannot be switched off afterwards
  bool aos = false;
  bool layout_fixed() const { return aos; }

 private:
  void release();
  int grow_ops(int64_t need);
  int grow_caps(int64_t need_sc, int64_t need_sess, int32_t need_ctx, int64_t need_rec = 0);
  int alloc_records();
  int ensure_batch(int64_t n);
  int ensure_table(int64_t keys, bool drop_new = false);
  int ensure_rows(int64_t rows);
  int op_error(int32_t op_err);
  int64_t lane_row_bound(int64_t wm) const;
  int64_t single_row_bound(int64_t wm) const;
  int finish_rows(int64_t rows, XResult& r, bool to_host, bool check);
  int push_keyed_replay(const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n);
  int push_kg(const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n, int64_t* deferred,
              int32_t* flag);
  int push_keyed_kg(const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n, bool split);
  int kg_used = 0, kg_replayed = 0;
  bool prefix_stale = false;
  std::vector<XWinDef> h_wins;
  bool have_wm = false;   // a watermark was processed (last_wm: its value)
  int64_t last_wm = 0;  // ops were replayed without prefix tracking: the next lane watermark rebuilds them
  int check_ready();
  XBatchArgs batch_args() const;

  int device = 0;
  hipStream_t stream = nullptr;
  int vt = VT_I32;
  bool keyed = false;
  XCfg cfg{};
  XCfg* d_cfg = nullptr;
  int32_t *d_cf_kind = nullptr, *d_cf_meas = nullptr;
  int64_t *d_cf_a = nullptr, *d_cf_b = nullptr;
  int32_t sc = 0, sesscap = 0, ctx_alloc = 0;
  int64_t rcap_ = 0;  // records per op (records mode)
  unsigned long long* d_need = nullptr;
  int64_t n_ops = 0, ops_cap = 0;
  XState* d_st = nullptr;
  XSlices sl{};
  XSess ss{};
  // keyed
  unsigned long long* d_table = nullptr;
  uint64_t tcap = 0;
  uint32_t* d_newpos = nullptr;
  unsigned long long* d_newcnt = nullptr;
  int32_t* d_full = nullptr;
  uint32_t* d_slot_key = nullptr;
  std::vector<uint32_t> h_slot_key;
  // sort-free keyed path (keyed_grid.hip): compact key table, partition scratch, deferred-tuple gather
  unsigned long long* d_kgtab = nullptr;
  uint64_t kgcap = 0;
  int64_t kg_built = -1;
  int64_t kg_ncap = 0, kg_hcap = 0, kg_gcap = 0;
  int32_t *d_kghist = nullptr, *d_kgscan = nullptr, *d_kgblk = nullptr;
  void* d_kgrec = nullptr;
  uint8_t* d_kgmark = nullptr;
  void* d_kgctl = nullptr;
  void* h_kgctl = nullptr;   // pinned, host-mapped copy of the control block
  void* h_kgctl_dev = nullptr;
  uint32_t* d_kgkey = nullptr;
  int64_t* d_kgts = nullptr;
  void* d_kgval = nullptr;
  int64_t *d_kggpts = nullptr, *d_kgpos = nullptr;
  KPart* d_kgpart = nullptr;
  uint8_t* d_kgdflag = nullptr;
  int64_t kg_pcap = 0;
  std::vector<int64_t> h_kgpos;
  // batch scratch
  int64_t bcap = 0;
  uint32_t* d_slot = nullptr;         // replay path: the batch's distinct keys' slots
  uint32_t* d_ukey = nullptr;         // replay path: the batch's distinct keys (sorted), segment starts, per-tile counts
  int64_t* d_ubeg = nullptr;
  int32_t *d_segcnt = nullptr, *d_segoff = nullptr, *d_segscan = nullptr;
  int64_t* d_tmaxt = nullptr;
  unsigned long long* d_rpart = nullptr;  // range_hist_kernel's per-tile key / timestamp ranges (3 per sort tile)
  unsigned long long* d_kmax = nullptr;
  void *d_recA = nullptr, *d_recB = nullptr;
  int32_t *d_hist = nullptr, *d_scan32 = nullptr;
  int64_t seg_cap = 0;
  int64_t *d_seg_b = nullptr, *d_seg_e = nullptr;
  // watermark scratch + rows
  int64_t wcap = 0, rcap = 0;
  int64_t *d_wcount = nullptr, *d_woff = nullptr, *d_scan64 = nullptr;
  int64_t* d_misc = nullptr;
  int64_t* h_misc = nullptr;     // pinned, host-mapped
  int64_t* h_misc_dev = nullptr;
  int64_t *d_w_start = nullptr, *d_w_end = nullptr;
  int32_t *d_w_meas = nullptr, *d_w_op = nullptr;
  uint32_t* d_w_key = nullptr;
  uint8_t* d_has = nullptr;
  int64_t* d_vals[SCOTTY_MAX_AGGS] = {};
  // batch-parallel non-keyed path (exact_batch.hip)
  int64_t xb_tcap = 0, xb_ncap = 0, xb_nscap = 0, xb_evcap = 0, xb_reachcap = 0;
  void* xb_snap = nullptr;
  void* xb_ctl = nullptr;
  int64_t* xb_reach = nullptr;
  long long *xb_tmax = nullptr, *xb_pcarry = nullptr, *xb_segtail = nullptr, *xb_mcarry = nullptr;
  int64_t *xb_nscnt = nullptr, *xb_nstot = nullptr, *xb_nsstart = nullptr, *xb_nspb = nullptr;
  int64_t* xb_evcnt = nullptr;
  int32_t* xb_seghas = nullptr;
  int32_t* xb_tjump = nullptr;
  long long* xb_tmin = nullptr;  // per-tile minimum ts (quiet-tile test)  // per-tile session-jump flags (exact_batch.hip, xb_tilemax_kernel)
  uint32_t* xb_bits = nullptr;
  int64_t *xb_evpos = nullptr, *xb_evt = nullptr, *xb_evv = nullptr, *xb_eppos = nullptr;
  long long* xb_evm = nullptr;
  int32_t* xb_eptail = nullptr;
  int64_t* xb_sufmin = nullptr;
  int64_t xb_sufcap = 0;
  // one-pass quiet path (exact_quiet.hip): union edge grid, per-batch cells, ingest view of the store
  int xq_rebuild_grid();
  int xq_ensure(int64_t n);
  int tbegin(TEv& e, int cls);
  int tend(TEv& e, int64_t n);
  std::vector<int64_t> xq_hgrid;
  int64_t xq_gcap = 0, xq_ccap = 0, xq_tcap = 0;
  int64_t* d_xq_grid = nullptr;
  unsigned long long* d_xq_ccnt = nullptr;
  long long* d_xq_ctmax = nullptr;
  unsigned long long* d_xq_cpart[NPART] = {};
  long long* d_xq_tilemax = nullptr;
  long long* d_xq_tilemin = nullptr;
  long long* d_xq_pmax = nullptr;     // prefix maxima of the tile maxima (quiet scan -> edge kernel)
  int32_t *d_xq_rank = nullptr, *d_xq_flag = nullptr;
  int64_t *d_xq_eg = nullptr, *d_xq_epos = nullptr;
  DevMeta* d_xq_meta = nullptr;
  uint32_t* d_xq_cix = nullptr;
  int64_t* d_xq_cixmeta = nullptr;
  void* d_xq_ctl = nullptr;
  long long* d_dbg = nullptr;
  XBlocks xblk{};               // single operator: 64-slice block summaries of the watermark (wm_blocks_kernel)
  int64_t xblk_cap = 0;   // debugging aid (SCOTTY_XQ_PROF / SCOTTY_XB_PROF): clock stamps, this engine's device
  int64_t xq_span = 1000;       // event-time span of the last committed batch (grid horizon and cell-index sizing)
  bool xq_need_grid = true;     // (re)build the grid from the pending edge at the next push
};

}  // namespace scotty
