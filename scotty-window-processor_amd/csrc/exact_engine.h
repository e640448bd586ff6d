// exact_engine.h -- host interface of the exact ("replay") engine (see exact_common.h).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/scotty_mi355x.h"
#include "exact_common.h"

namespace scotty {

struct XWinDef {  // one Window of WindowOperator.addWindowAssigner, in registration order
  int kind, measure;
  int64_t a, b;
};

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
  std::vector<int64_t> start, end;
  std::vector<int32_t> meas;
  std::vector<uint32_t> key;
  std::vector<uint8_t> has;
  std::vector<std::vector<int64_t>> vals;
};

class XEngine {
 public:
  ~XEngine();
  int init(int device, hipStream_t stream, int vt, bool keyed, std::string& err);
  int configure(const std::vector<XWinDef>& wins, const std::vector<int>& aggs, int64_t max_lateness);
  int push(const int64_t* d_ts, const void* d_val, int64_t n);
  int push_keyed(const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n);
  int watermark(int64_t wm, XResult& r, bool to_host);
  int slice_count(int64_t op, int64_t* out);
  int read_states(std::vector<XState>& out);
  int64_t key_count() const { return keyed ? n_ops : 0; }
  int set_last_watermark(int64_t lw);  // non-keyed: watermarks seen before the first tuple

  std::string err;
  bool failed = false;
  int32_t sc_override = 0, sess_override = 0;

 private:
  void release();
  int grow_ops(int64_t need);
  int grow_caps(int64_t need_sc, int64_t need_sess, int32_t need_ctx);
  int ensure_batch(int64_t n);
  int ensure_table(int64_t keys);
  int ensure_rows(int64_t rows);
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
  // batch scratch
  int64_t bcap = 0;
  uint32_t* d_slot = nullptr;
  void *d_recA = nullptr, *d_recB = nullptr;
  int32_t *d_hist = nullptr, *d_scan32 = nullptr;
  int64_t seg_cap = 0;
  int64_t *d_seg_b = nullptr, *d_seg_e = nullptr;
  // watermark scratch + rows
  int64_t wcap = 0, rcap = 0;
  int64_t *d_wcount = nullptr, *d_woff = nullptr, *d_scan64 = nullptr;
  int64_t* d_misc = nullptr;
  int64_t* h_misc = nullptr;
  int64_t *d_w_start = nullptr, *d_w_end = nullptr;
  int32_t *d_w_meas = nullptr, *d_w_op = nullptr;
  uint32_t* d_w_key = nullptr;
  uint8_t* d_has = nullptr;
  int64_t* d_vals[SCOTTY_MAX_AGGS] = {};
};

}  // namespace scotty
