// count_engine.h -- host side of the count-window path (count_common.h, count_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/scotty_mi355x.h"
#include "count_common.h"
#include "exact_engine.h"

namespace scotty {

class CEngine {
 public:
  ~CEngine();
  int init(int device, hipStream_t stream, int vt, std::string& err);
  // WindowManager.addWindowAssigner / addAggregation / setMaxLateness (S/WindowManager.java:121-202)
  int configure(const std::vector<XWinDef>& wins, const std::vector<int>& aggs, int64_t max_lateness);
  int push(const int64_t* d_ts, const void* d_val, int64_t n, hipEvent_t ev0, hipEvent_t ev1);
  // sharding of one stream over G ranks (count_common.h CSHARD_HDR): every rank pushes its arrival chunk
  // (n_before tuples of lower ranks precede it in a micro-batch of n_total), the caller all-gathers the
  // records of shard_words() int64 each, every rank commits them
  int64_t shard_words() const { return cshard_words(shard_cap); }
  int shard_push(const int64_t* d_ts, const void* d_val, int64_t n, int64_t ts0, int64_t n_before, int64_t n_total,
                 int64_t ts_before, int64_t ts_last, int64_t* d_rec);
  int shard_commit(const int64_t* d_gathered, int world);
  int64_t shard_cap = 1 << 16;  // cells per rank record (scotty_tune "shard_count_cells")
  bool shard_async = false;     // scotty_tune "shard_async": shard_push returns without a host sync
  bool prefix_one = true;       // scotty_tune "count_prefix_one" 0: the watermark's prefix sums always by three kernels
  int watermark(int64_t wm, XResult& r, bool to_host);
  int set_last_watermark(int64_t lw) {
    last_wm = lw;
    return SCOTTY_OK;
  }
  int64_t slice_count();
  uint64_t dropped() const { return dropped_; }

  std::string err;
  bool failed = false;

  bool has_time_windows() const { return !twins.empty(); }
  int64_t last_nte = 0;
  double last_te_us = 0;  // host time of the last push's time-edge step (debug stat)  // time edges of the last push (debug stat)

 private:
  int grow_slices(int64_t need);
  int fail(int rc, const std::string& m) {
    err = m;
    failed = true;
    return rc;
  }
  int64_t next_point(int64_t x) const;  // smallest union count-grid point >= x (x >= 1)
  int prepare(int64_t C, int64_t n, int64_t range_lo, int64_t range_hi, CPushArgs& a, int64_t& ebound, int64_t& maxp,
              int64_t n_te = 0);
  int64_t batch_edges_bound(int64_t lo_count, int64_t hi_count) const;
  struct ShardTime {  // a rank's chunk within a global micro-batch (shard_push)
    int64_t ts0, n_before, n_total, ts_before, ts_last;
  };
  int time_edges(const int64_t* d_ts, int64_t n, CPushArgs& a, const ShardTime* sh);
  int64_t shard_te_bound = 0;  // time-edge candidates of the current sharded batch (all ranks)
  int64_t next_time_point(int64_t x) const;  // nextGrid over the time windows (calculateNextFixedEdge's min)
  int64_t shard_ts0 = INT64_MIN, shard_total = 0;
  long long* d_plan = nullptr;
  int plan_cap = 0;
  void trigger(int64_t last_c, int64_t cur_c, int64_t last_t, int64_t cur_t);

  int device = 0;
  hipStream_t stream = nullptr;
  int vt = VT_I32;
  std::vector<CWin> wins;   // count windows (the device edge marking)
  std::vector<CWin> twins;  // time windows: edges from the in-order stream's timestamps (time_edges)
  std::vector<CWin> reg;    // every window in registration order (triggers)
  std::vector<int> aggs;
  int need = 0;
  int64_t max_lateness = 1000, max_fixed = 0;
  bool prefix = false;  // every aggregation an invertible integer kind
  // StreamSlicer / WindowManager scalars the host tracks exactly (edges depend on counts only)
  int64_t count = 0;           // WindowManager.currentCount
  int64_t pending = INT64_MIN;  // StreamSlicer.min_next_edge_count
  int64_t last_wm = -1, last_count = 0;
  int64_t t_pending = INT64_MIN;
  int64_t tstep = 0;
  CSlices spare{};                 // second slice buffer set (grow_slices moves the retained range into it)
  int64_t spare_cap = 0;               // common period of the time windows (device-generated candidates), or 0  // StreamSlicer.min_next_edge_ts (time windows)
  int64_t h_prev_max = INT64_MIN; // StreamSlicer.maxEventTime after the last push (the stream is in order)
  bool started = false;
  // time edges of the current push
  int64_t tcap = 0, tecap = 0;
  int64_t *d_cand = nullptr, *d_cpos = nullptr, *d_te_pos = nullptr, *d_te_g = nullptr;
  int64_t *d_cflag = nullptr, *d_coff = nullptr, *d_cscan = nullptr;
  unsigned long long* d_nte = nullptr;
  int64_t* h_tmp = nullptr;  // pinned scratch (batch ends, edge count)
  uint64_t dropped_ = 0;
  int64_t tail_ub = 0, head_lb = 0;  // slice range bounds between synchronisations
  // slices [ts_sorted_from, tail) have nondecreasing tStart and tLast: only the stream's first tuple puts slices out of
  // order (its own slice, then the time edges its walk crosses below its timestamp, all at position 0)
  int64_t ts_sorted_from = 0;
  // device
  CMeta* d_meta = nullptr;
  CMeta* h_meta = nullptr;  // pinned, host-mapped
  CMeta* h_meta_dev = nullptr;
  CWin* d_wins = nullptr;
  int64_t scap = 0;
  CSlices sl{};
  int64_t ccap = 0;
  CCells cells{};
  int64_t bcap = 0, stcap = 0;
  uint32_t* d_bits = nullptr;
  int64_t *d_stepc = nullptr, *d_stepbase = nullptr, *d_scan = nullptr, *d_stepte = nullptr;
  uint32_t* d_steptp = nullptr;
  long long *d_stepmax = nullptr, *d_steppre = nullptr, *d_premax = nullptr;
  // watermark
  struct Row {
    int64_t start, end;
    int32_t meas;
  };
  std::vector<int32_t> h_meas;
  std::vector<Row> rows;
  bool trigger_segs(int64_t last_c, int64_t cur_c, int64_t last_t, int64_t cur_t);  // false: use trigger()
  CRowSeg* h_segs = nullptr;  // pinned: the runs, then nseg + 1 offsets
  int64_t segcap = 0;         // runs h_segs / d_segbuf hold
  int nseg = 0;
  void* d_segbuf = nullptr;
  int64_t wcap = 0, pcap = 0;
  int64_t *d_wstart = nullptr, *d_wend = nullptr;
  int32_t* d_meas = nullptr;
  uint8_t* d_has = nullptr;
  int64_t* d_vals[SCOTTY_MAX_AGGS] = {};
  unsigned long long *d_pre_cnt = nullptr, *d_pre_sum = nullptr, *d_bsum = nullptr;
  std::vector<int64_t> h_start, h_end;
  // host sources of asynchronous copies that outlive the call that queued them (the first walk's edges, an empty
  // shard chunk's record header): rewritten only after the stream's next synchronisation
  std::vector<int64_t> h_first_pos, h_first_g, h_shard_hdr;
};

}  // namespace scotty
