// scotty_engine.cpp -- host side of the MI355X operator: control state, edge grid, window triggering,
// and the C-ABI of include/scotty_mi355x.h.
//
// Per-tuple work never runs here: every tuple is read, assigned and aggregated by the gfx950 kernels
// (slicing_kernels.hip).  The host keeps what the reference keeps in scalars of the WindowManager /
// StreamSlicer (S/WindowManager.java:18-33, S/StreamSlicer.java:10-14), generates the triggered window
// list (pure arithmetic of C/windowType/*Window.triggerWindows) and the union edge grid of the
// context-free windows (their assignNextWindowStart), and sequences launches on one HIP stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <queue>
#include <string>
#include <vector>

#include "../../include/scotty_mi355x.h"
#include "dev_alloc.h"
#include "device_common.h"
#include "count_engine.h"
#include "exact_engine.h"
#include "host_ingest.h"

namespace scotty {
hipError_t launch_ingest(const IngestArgs& a, int vt, int need, int64_t nblocks, hipStream_t st, int mode);
void set_ingest_timing_events(hipEvent_t start, hipEvent_t stop);
int ingest_wgs_per_cu(int vt, int need);
hipError_t launch_cix_build(const IngestArgs& a, hipStream_t st);
hipError_t launch_first(const IngestArgs& a, hipStream_t st);
hipError_t launch_commit(const CommitArgs& a, hipStream_t st);
hipError_t launch_wm(const WmArgs& a, hipStream_t st);
hipError_t launch_cix_build(const IngestArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1);
hipError_t launch_commit(const CommitArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1);
hipError_t launch_wm(const WmArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1);
hipError_t launch_wm_publish(const void* d_src, void* h_dst_dev, int64_t bytes, hipStream_t st);
hipError_t launch_fill_u64(unsigned long long* p, int64_t n, unsigned long long v, hipStream_t st);
hipError_t launch_first_ge(const int64_t* ts, int64_t n, int64_t x, unsigned long long* out_idx, hipStream_t st);
hipError_t launch_shard_export(const ShardArgs& a, hipStream_t st);
hipError_t launch_shard_commit(const ShardArgs& a, hipStream_t st);
}  // namespace scotty

// Allocation poison (dev_alloc.h): -1 off, else the byte every new engine allocation is filled with.
namespace scotty {
static std::atomic<int> g_alloc_poison{[] {
  const char* e = getenv("SCOTTY_ALLOC_POISON");
  return (e && *e) ? (int)(strtol(e, nullptr, 0) & 0xFF) : -1;
}()};
int alloc_poison() { return g_alloc_poison.load(std::memory_order_relaxed); }

static thread_local char g_kernel_name[KN_N][96];
void note_kernel(int which, const char* fmt, int a, int b, int c, int d) {
  if (which >= 0 && which < KN_N) snprintf(g_kernel_name[which], sizeof(g_kernel_name[which]), fmt, a, b, c, d);
}
}  // namespace scotty

using namespace scotty;

namespace {

constexpr int64_t JMAX = INT64_MAX, JMIN = INT64_MIN;
inline int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
inline int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
inline int64_t jmod(int64_t a, int64_t b) { return b == -1 ? 0 : a % b; }

struct CFWin {  // context-free window (C/windowType/ContextFreeWindow.java)
  int kind;
  int64_t a, b;
  // assignNextWindowStart: TumblingWindow.java:29-31, SlidingWindow.java:41-43, FixedBandWindow.java:37-48
  int64_t next_start(int64_t t) const {
    if (kind == SCOTTY_WIN_TUMBLING) return jsub(jadd(t, a), jmod(t, a));
    if (kind == SCOTTY_WIN_SLIDING) return jsub(jadd(t, b), jmod(t, b));
    if (t == JMAX || t < a) return a;
    if (t >= a && t < jadd(a, b)) return jadd(a, b);
    return JMAX;
  }
  int64_t clear_delay() const { return kind == SCOTTY_WIN_FIXED_BAND ? b : a; }
};

// Device-time classes of scotty_device_timing (include/scotty_mi355x.h)
constexpr int NTCLS = 4;

}  // namespace

struct scotty_op {
  int device = 0;
  int vt = VT_I32;
  hipStream_t stream = nullptr;
  hipEvent_t order_ev = nullptr;  // scotty_stream_order
  hipEvent_t wm_ev = nullptr;     // grid watermark: the packed result has landed (the host waits on this, not the stream)
  bool cix_ready = false;         // the cell index on the device matches the current slice store (built at the end
                                  // of the last watermark, overlapping the host's result handling)
  bool shard_async = false;       // scotty_tune("shard_async", 1): shard pushes return without a host sync
  bool c_prefix_one = true;       // scotty_tune("count_prefix_one", 0): count-path prefix sums by three kernels (tests)
  std::string err;
  bool failed = false;

  // ---- WindowManager / StreamSlicer scalars
  std::vector<CFWin> windows;
  std::vector<int> aggs;      // SCOTTY_AGG_* kinds (without SCOTTY_AGG_INVERTIBLE)
  std::vector<int> agg_inv;   // 1: the function is an InvertibleAggregateFunction
  int need = 0;
  int64_t max_lateness = 1000;
  int64_t max_fixed_window_size = 0;
  bool has_fixed = false;
  bool started = false;            // store non-empty (at least one tuple processed)
  bool walk_pending = false;       // first context-free window added after tuples were processed
  int64_t last_watermark = -1;
  int64_t h_oldest = 0;            // t_start of the oldest retained slice (mirror)
  int64_t h_prev_max = JMIN;       // mirror of DevMeta.prev_max after the last sync
  int64_t last_span = 1000;        // event-time span of the last watermark interval (grid horizon sizing)

  // ---- union edge grid (host copy of d_grid)
  std::vector<int64_t> grid;
  bool grid_complete = false;

  // ---- device buffers
  int64_t scap = 0, gcap = 0, ccap = 0, tcap = 0;
  DevMeta* d_meta = nullptr;
  DevMeta* h_snap = nullptr;  // pinned
  int64_t* d_tstart = nullptr;
  int64_t* d_tlast = nullptr;
  unsigned long long* d_scnt = nullptr;
  unsigned long long* d_spart[NPART] = {};
  int64_t* d_grid = nullptr;
  unsigned long long* d_ccnt = nullptr;
  long long* d_ctmax = nullptr;
  unsigned long long* d_cpart[NPART] = {};
  long long* d_tilemax = nullptr;
  uint32_t* d_cix = nullptr;      // cell index (slicing_kernels.hip cix_build_kernel)
  int64_t* d_cixmeta = nullptr;
  long long* d_stamps = nullptr;  // ingest phase stamps (scotty_tune "ingest_stamps", a debugging aid)
  bool stamps_on = false;
  long long* d_pmax = nullptr;
  int32_t* d_rank = nullptr;
  int32_t* d_flag = nullptr;
  unsigned long long* d_scratch = nullptr;
  // watermark (window_kernels.hip): slice-block summaries, prefix sums, sparse tables, window definitions, and the
  // packed result buffer (device + pinned host copy, one transfer per watermark)
  int64_t nbcap = 0;
  unsigned long long* d_bcnt = nullptr;
  unsigned long long* d_bpart[NPART] = {};
  unsigned long long* d_pcnt = nullptr;
  unsigned long long* d_psum = nullptr;
  long long* d_stmin = nullptr;
  long long* d_stmax = nullptr;
  int64_t* d_wdef = nullptr;
  int64_t wdef_cap = 0;
  bool wdef_dirty = true;
  unsigned char* d_out = nullptr;
  unsigned char* h_out = nullptr;  // pinned, host-mapped
  void* h_out_dev = nullptr;       // device address of h_out (null: plain DMA transfer)
  int64_t out_cap = 0;

  // ---- pushes of the current watermark interval (replayed after a horizon overflow)
  struct Push {
    const int64_t* ts;
    const void* val;
    int64_t n;
    int64_t seq;
    int64_t base = 0;  // arrival index of ts[0] (SCOTTY_AGG_FIRST)
  };
  std::vector<Push> pending;
  std::vector<void*> owned;  // (unused since the host ingest arena; kept empty)
  HostIngest* ingest = nullptr;  // host columns -> HBM (pinned slots, copy stream, arena reset per watermark)
  int64_t push_seq = 0;
  uint64_t dropped = 0, processed = 0;
  // SCOTTY_AGG_FIRST (grid path): per-slice / per-cell arrival index of the first tuple (identity FIRST_NONE)
  bool first = false;
  int64_t arrivals = 0;  // tuples pushed so far (WindowManager.currentCount order, dropped ones included)
  long long* d_sfirst = nullptr;
  long long* d_cfirst = nullptr;

  int ingest_mode = -1;  // tuning knob (scotty_tune), -1 = default variant
  int64_t ingest_blocks = 0;  // tuning knob: target workgroups of the ingest launch (0: one round of resident ones)
  int64_t last_ingest_blocks = 0, last_ingest_streaming = 0;  // the last ingest launch (statistics)

  // ---- engine selection: the grid path (context-free time windows, non-keyed) or the exact engine
  //      (keyed ops, session windows, count windows); decided at the first push
  bool keyed = false;
  int mode = 0;                       // 0 undecided, 1 grid, 2 exact
  std::vector<XWinDef> xwins;         // every window, registration order
  XEngine* x = nullptr;
  CEngine* c = nullptr;  // mode 3: count-window path (count_engine.h)
  int32_t x_sc = 0, x_sess = 0;       // capacity knobs
  bool x_serial = false;
  bool x_quiet_off = false;  // exact engine: no one-pass quiet path (A/B)
  bool x_band_on = true;     // exact engine: quiet batches may move the last session's start (start band; scotty_tune)
  bool x_lane_off = false;
  bool x_kg_off = false;
  int64_t x_kg_chunk = -1;
  int64_t x_prefix = 0;      // exact engine: first event-exact prefix of a refused quiet batch (0: default)
  int32_t x_qmode = -1;      // exact engine: quiet-pass ingest loop (A/B: -1 default, 7 without the DQ2 queue)
  bool x_ls_off = false;     // exact engine: keyed sessions through the wavefront replay (A/B)
  bool x_lc_off = false;     // exact engine: keyed LazySlice record sets through the wavefront replay (A/B)
  int32_t x_ls_occ = 2;      // lane-session kernel's waves per SIMD (2 default, no VGPR spill; 3: A/B, profiles/r06/ab1/)
  bool x_pack_off = false;   // exact engine: keyed replay records always 16 bytes (A/B for the packed 8-byte ones)
  int x_digit10 = -1;        // exact engine: keyed replay sort digits ("keyed_sort_digit10": -1 default = 0 8-bit, 1 10-bit)
  bool x_lsdbg = false;      // lane-session path counters (debugging aid)
  int64_t x_qblocks = 0;     // exact engine: quiet-pass ingest workgroups (A/B: 0 default)
  int32_t x_kg_variant = -1;
  int64_t shard_count_total = 0;
  int64_t count_shard_cap = 1 << 16;
  bool x_count_on = false;   // "count_path" 1: the stream is in timestamp order -> count-only operators keep no
                             // LazySlice records and run on the count path (count_engine.cpp)
  uint64_t x_pushed = 0;
  std::vector<uint32_t> r_key;
  // sharded grid path (scotty_shard_*)
  int64_t shard_kc = 2048, shard_kg = 1024;
  int32_t* d_shrank = nullptr;
  int32_t* d_shflag = nullptr;
  int64_t shard_tile = TILE_MIN, shard_n = 0;
  XResult xr;

  // ---- timing: HIP events around every launch group on the op's stream, per device-time class
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending, ev_pool;  // ingest launches (class 0)
  struct TEv {
    int cls;
    hipEvent_t a, b;
  };
  std::vector<TEv> tev_pending;
  double t_ms = 0.0;
  uint64_t t_launches = 0, t_tuples = 0;
  double t_cls_ms[NTCLS] = {};
  uint64_t t_cls_n[NTCLS] = {};

  // ---- results
  std::vector<int32_t> r_measure;  // grid path: every window is a time window (SCOTTY_MEASURE_TIME == 0)
};

namespace {

int fail(scotty_op* op, int code, const std::string& m) {
  op->err = m;
  return code;
}

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      op->failed = true;                                                              \
      return fail(op, SCOTTY_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
    }                                                                                 \
  } while (0)

// Timed section of one device-time class: events recorded on the op's stream around a launch group.
int tbegin(scotty_op* op, scotty_op::TEv& e, int cls) {
  e.cls = cls;
  e.a = e.b = nullptr;
  if (!op->timing) return SCOTTY_OK;
  if (!op->ev_pool.empty()) {
    e.a = op->ev_pool.back().first;
    e.b = op->ev_pool.back().second;
    op->ev_pool.pop_back();
  } else {
    HIPCHK(hipEventCreate(&e.a));
    HIPCHK(hipEventCreate(&e.b));
  }
  HIPCHK(hipEventRecord(e.a, op->stream));
  return SCOTTY_OK;
}
// A timed launch group whose launch wrappers take the events and have the dispatches stamp them (hipExtLaunchKernel):
// no marker packets between dependent kernels.  tlaunch acquires the pair (null when timing is off), tlaunched files
// it for tresolve.
int tlaunch(scotty_op* op, scotty_op::TEv& e, int cls) {
  e.cls = cls;
  e.a = e.b = nullptr;
  if (!op->timing) return SCOTTY_OK;
  if (!op->ev_pool.empty()) {
    e.a = op->ev_pool.back().first;
    e.b = op->ev_pool.back().second;
    op->ev_pool.pop_back();
  } else {
    HIPCHK(hipEventCreate(&e.a));
    HIPCHK(hipEventCreate(&e.b));
  }
  return SCOTTY_OK;
}
void tlaunched(scotty_op* op, scotty_op::TEv& e) {
  if (op->timing && e.a) op->tev_pending.push_back(e);
}
int tend(scotty_op* op, scotty_op::TEv& e) {
  if (!op->timing || !e.a) return SCOTTY_OK;
  HIPCHK(hipEventRecord(e.b, op->stream));
  op->tev_pending.push_back(e);
  return SCOTTY_OK;
}
// after a synchronisation: fold every completed interval into its class; intervals still running (the cell index
// built behind a watermark's result transfer) stay pending until the next resolve
void tresolve(scotty_op* op) {
  std::vector<scotty_op::TEv> keep;
  for (auto& e : op->tev_pending) {
    if (hipEventQuery(e.b) == hipErrorNotReady) {
      keep.push_back(e);
      continue;
    }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
      op->t_cls_ms[e.cls] += ms;
      op->t_cls_n[e.cls]++;
    }
    op->ev_pool.push_back({e.a, e.b});
  }
  op->tev_pending.swap(keep);
}

int agg_value_type(int kind) {
  switch (kind) {
    case SCOTTY_AGG_SUM_I32: case SCOTTY_AGG_MIN_I32: case SCOTTY_AGG_MAX_I32: return VT_I32;
    case SCOTTY_AGG_SUM_I64: case SCOTTY_AGG_MIN_I64: case SCOTTY_AGG_MAX_I64: return VT_I64;
    case SCOTTY_AGG_SUM_F64: case SCOTTY_AGG_MIN_F64: case SCOTTY_AGG_MAX_F64: return VT_F64;
    case SCOTTY_AGG_COUNT: case SCOTTY_AGG_FIRST: return -1;
    default: return -2;
  }
}
int agg_need(int kind) {
  switch (kind) {
    case SCOTTY_AGG_SUM_I32: case SCOTTY_AGG_SUM_I64: case SCOTTY_AGG_SUM_F64: return NEED_SUM;
    case SCOTTY_AGG_MIN_I32: case SCOTTY_AGG_MIN_I64: case SCOTTY_AGG_MIN_F64: return NEED_MIN;
    case SCOTTY_AGG_MAX_I32: case SCOTTY_AGG_MAX_I64: case SCOTTY_AGG_MAX_F64: return NEED_MAX;
    default: return 0;
  }
}

// min over context-free time windows of assignNextWindowStart (StreamSlicer.calculateNextFixedEdge's loop,
// S/StreamSlicer.java:108-114)
int64_t next_edge(const scotty_op* op, int64_t t) {
  int64_t e = JMAX;
  for (const CFWin& w : op->windows) e = std::min(e, w.next_start(t));
  return e;
}

// Union edge grid: first entry is the pending edge N, then every point of the union of the windows'
// grids above N up to the horizon.  A finite grid (fixed-band windows only) ends with a JMAX sentinel.
void build_grid(scotty_op* op, int64_t n_pending, int64_t horizon_end) {
  op->grid.clear();
  op->grid_complete = false;
  if (n_pending == JMAX) {
    op->grid.push_back(JMAX);
    op->grid_complete = true;
    return;
  }
  op->grid.push_back(n_pending);
  // k-way merge of arithmetic progressions / fixed points
  using Item = std::pair<int64_t, size_t>;
  std::priority_queue<Item, std::vector<Item>, std::greater<Item>> pq;
  std::vector<int64_t> fixed_pts;
  bool infinite = false;
  for (size_t i = 0; i < op->windows.size(); i++) {
    const CFWin& w = op->windows[i];
    if (w.kind == SCOTTY_WIN_FIXED_BAND) {
      fixed_pts.push_back(w.a);
      fixed_pts.push_back(jadd(w.a, w.b));
    } else {
      infinite = true;
      pq.push({w.next_start(n_pending), i});
    }
  }
  for (int64_t p : fixed_pts)
    if (p > n_pending) pq.push({p, (size_t)-1});
  const int64_t cap = op->gcap - 1;
  while (!pq.empty() && (int64_t)op->grid.size() < cap) {
    Item it = pq.top();
    pq.pop();
    if (it.first <= op->grid.back()) {
      if (it.second != (size_t)-1) {
        const int64_t nx = op->windows[it.second].next_start(it.first);
        if (nx > it.first) pq.push({nx, it.second});  // a progression that wraps past Long.MAX_VALUE ends
      }
      continue;
    }
    if (it.first > horizon_end && infinite) break;
    op->grid.push_back(it.first);
    if (it.second != (size_t)-1) pq.push({op->windows[it.second].next_start(it.first), it.second});
  }
  if (!infinite && pq.empty()) {
    op->grid.push_back(JMAX);
    op->grid_complete = true;
  }
}

int upload_grid(scotty_op* op) {
  op->cix_ready = false;  // the cell index covers grid cells
  HIPCHK(hipMemcpyAsync(op->d_grid, op->grid.data(), op->grid.size() * 8, hipMemcpyHostToDevice, op->stream));
  // DevMeta.j0 = 0, gcount = grid.size()  (offsets of DevMeta fields)
  int64_t v[2] = {0, (int64_t)op->grid.size()};
  HIPCHK(hipMemcpyAsync(&op->d_meta->j0, v, 16, hipMemcpyHostToDevice, op->stream));
  HIPCHK(hipStreamSynchronize(op->stream));
  return SCOTTY_OK;
}

int alloc_all(scotty_op* op) {
  op->scap = 1 << 20;
  op->gcap = 1 << 20;
  op->ccap = op->scap + op->gcap;
  op->tcap = 0;
  HIPCHK(hipSetDevice(op->device));
  HIPCHK(hipStreamCreateWithFlags(&op->stream, hipStreamNonBlocking));
  op->ingest = new HostIngest();
  if (op->ingest->init(op->device, op->stream)) return fail(op, SCOTTY_ERR_HIP, "host ingest: stream / event creation");
  HIPCHK(dev_malloc(&op->d_meta, sizeof(DevMeta)));
  HIPCHK(hipHostMalloc(&op->h_snap, sizeof(DevMeta), hipHostMallocDefault));
  HIPCHK(hipMemset(op->d_meta, 0, sizeof(DevMeta)));
  HIPCHK(dev_malloc(&op->d_tstart, op->scap * 8));
  HIPCHK(dev_malloc(&op->d_tlast, op->scap * 8));
  HIPCHK(dev_malloc(&op->d_scnt, op->scap * 8));
  for (int k = 0; k < NPART; k++) HIPCHK(dev_malloc(&op->d_spart[k], op->scap * 8));
  HIPCHK(dev_malloc(&op->d_grid, op->gcap * 8));
  HIPCHK(dev_malloc(&op->d_ccnt, op->ccap * 8));
  HIPCHK(dev_malloc(&op->d_ctmax, op->ccap * 8));
  for (int k = 0; k < NPART; k++) HIPCHK(dev_malloc(&op->d_cpart[k], op->ccap * 8));
  HIPCHK(dev_malloc(&op->d_rank, op->gcap * 4));
  HIPCHK(dev_malloc(&op->d_flag, op->gcap * 4));
  HIPCHK(dev_malloc(&op->d_scratch, 64));
  HIPCHK(launch_fill_u64(op->d_ccnt, op->ccap, 0, op->stream));
  HIPCHK(launch_fill_u64((unsigned long long*)op->d_ctmax, op->ccap, (unsigned long long)INT64_MIN, op->stream));
  HIPCHK(launch_fill_u64(op->d_cpart[0], op->ccap, 0, op->stream));
  HIPCHK(launch_fill_u64(op->d_cpart[1], op->ccap, (unsigned long long)INT64_MAX, op->stream));
  HIPCHK(launch_fill_u64(op->d_cpart[2], op->ccap, (unsigned long long)INT64_MIN, op->stream));
  HIPCHK(hipStreamSynchronize(op->stream));
  return SCOTTY_OK;
}

int ensure_tiles(scotty_op* op, int64_t n) {
  int64_t nt = (n + TILE_MIN - 1) / TILE_MIN + 1;
  if (nt <= op->tcap) return SCOTTY_OK;
  HIPCHK(hipStreamSynchronize(op->stream));
  if (op->d_tilemax) HIPCHK(hipFree(op->d_tilemax));
  if (op->d_pmax) HIPCHK(hipFree(op->d_pmax));
  op->tcap = std::max(nt, (int64_t)1024);
  HIPCHK(dev_malloc(&op->d_tilemax, op->tcap * 8));
  HIPCHK(dev_malloc(&op->d_pmax, op->tcap * 8));
  return SCOTTY_OK;
}

// Slice-block summaries of the watermark path (window_kernels.hip), sized for the slice capacity.
int alloc_blocks(scotty_op* op) {
  if (op->d_bcnt) return SCOTTY_OK;
  op->nbcap = op->scap / SBLK + 1;
  HIPCHK(dev_malloc(&op->d_bcnt, op->nbcap * 8));
  for (int k = 0; k < NPART; k++) HIPCHK(dev_malloc(&op->d_bpart[k], op->nbcap * 8));
  HIPCHK(dev_malloc(&op->d_pcnt, op->nbcap * 8));
  HIPCHK(dev_malloc(&op->d_psum, op->nbcap * 8));
  HIPCHK(dev_malloc(&op->d_stmin, (size_t)ST_LEVELS * op->nbcap * 8));
  HIPCHK(dev_malloc(&op->d_stmax, (size_t)ST_LEVELS * op->nbcap * 8));
  return SCOTTY_OK;
}

// Packed watermark output (device + pinned host) of at least `bytes`.
int ensure_wm_out(scotty_op* op, int64_t bytes) {
  if (bytes <= op->out_cap) return SCOTTY_OK;
  HIPCHK(hipStreamSynchronize(op->stream));
  if (op->d_out) HIPCHK(hipFree(op->d_out));
  if (op->h_out) HIPCHK(hipHostFree(op->h_out));
  op->d_out = nullptr;
  op->h_out = nullptr;
  op->out_cap = std::max<int64_t>(bytes + bytes / 2, 1 << 16);
  op->out_cap = (op->out_cap + 15) & ~(int64_t)15;
  HIPCHK(dev_malloc(&op->d_out, op->out_cap));
  HIPCHK(hipHostMalloc(&op->h_out, op->out_cap, hipHostMallocMapped));
  op->h_out_dev = nullptr;
  if (hipHostGetDevicePointer(&op->h_out_dev, op->h_out, 0) != hipSuccess) op->h_out_dev = nullptr;
  return SCOTTY_OK;
}

// Window definitions (registration order) for the device triggers: kind, a, b.
int upload_wdefs(scotty_op* op) {
  if (!op->wdef_dirty) return SCOTTY_OK;
  const int64_t n = (int64_t)op->windows.size();
  if (n > op->wdef_cap) {
    HIPCHK(hipStreamSynchronize(op->stream));
    if (op->d_wdef) HIPCHK(hipFree(op->d_wdef));
    op->wdef_cap = std::max<int64_t>(n, 64);
    HIPCHK(dev_malloc(&op->d_wdef, op->wdef_cap * 3 * 8));
  }
  std::vector<int64_t> v;
  for (const CFWin& w : op->windows) {
    v.push_back(w.kind);
    v.push_back(w.a);
    v.push_back(w.b);
  }
  if (n > 0) {
    HIPCHK(hipMemcpyAsync(op->d_wdef, v.data(), v.size() * 8, hipMemcpyHostToDevice, op->stream));
    HIPCHK(hipStreamSynchronize(op->stream));  // v is pageable and local
  }
  op->wdef_dirty = false;
  return SCOTTY_OK;
}

// The first in-order tuple after the first context-free window exists runs StreamSlicer.determineSlices
// with min_next_edge_ts == Long.MIN_VALUE (S/StreamSlicer.java:52-84): calculateNextFixedEdge starts from
// Long.MAX_VALUE, whose assignNextWindowStart wraps negative, and the loop then walks up from te-maxLateness.
// Returns the edges appended (in order) and the resulting pending edge.
// Returns false when the reference would never leave this loop (see oracle: ORC_ERR_HANG).
bool first_walk(const scotty_op* op, int64_t te, std::vector<int64_t>& edges, int64_t& n_out) {
  auto calc = [&](int64_t cur_next, int64_t t) {  // calculateNextFixedEdge
    int64_t cur = cur_next == JMIN ? JMAX : cur_next;
    int64_t tc = std::max(jsub(t, op->max_lateness), cur);
    return next_edge(op, tc);
  };
  int64_t n = calc(JMIN, te);
  while (te > n) {
    if (n >= 0) edges.push_back(n);
    n = calc(n, te);
    if (n == JMIN) return false;
  }
  if (n == te) {
    edges.push_back(n);
    n = calc(n, te);
  }
  n_out = n;
  return true;
}

int compact_if_needed(scotty_op* op) {
  DevMeta& m = *op->h_snap;
  if (m.tail < op->scap / 2 || m.head == 0) return SCOTTY_OK;
  op->cix_ready = false;  // slices move
  const int64_t live = m.tail - m.head;
  int64_t* tmp = nullptr;
  HIPCHK(dev_malloc(&tmp, std::max<int64_t>(live, 1) * 8));
  int64_t* arrs[3 + NPART] = {op->d_tstart, op->d_tlast, (int64_t*)op->d_scnt, (int64_t*)op->d_spart[0],
                             (int64_t*)op->d_spart[1], (int64_t*)op->d_spart[2]};
  for (int64_t* a : arrs) {
    HIPCHK(hipMemcpyAsync(tmp, a + m.head, live * 8, hipMemcpyDeviceToDevice, op->stream));
    HIPCHK(hipMemcpyAsync(a, tmp, live * 8, hipMemcpyDeviceToDevice, op->stream));
  }
  if (op->d_sfirst) {
    HIPCHK(hipMemcpyAsync(tmp, op->d_sfirst + m.head, live * 8, hipMemcpyDeviceToDevice, op->stream));
    HIPCHK(hipMemcpyAsync(op->d_sfirst, tmp, live * 8, hipMemcpyDeviceToDevice, op->stream));
  }
  int64_t ht[2] = {0, live};
  HIPCHK(hipMemcpyAsync(&op->d_meta->head, ht, 16, hipMemcpyHostToDevice, op->stream));
  const int64_t zero = 0;  // block summaries follow slice indices: all of them are recomputed
  HIPCHK(hipMemcpyAsync(&op->d_meta->dirty_from, &zero, 8, hipMemcpyHostToDevice, op->stream));
  HIPCHK(hipStreamSynchronize(op->stream));
  HIPCHK(hipFree(tmp));
  m.head = 0;
  m.tail = live;
  m.dirty_from = 0;
  return SCOTTY_OK;
}

int sync_snapshot(scotty_op* op) {
  HIPCHK(hipMemcpyAsync(op->h_snap, op->d_meta, sizeof(DevMeta), hipMemcpyDeviceToHost, op->stream));
  HIPCHK(hipStreamSynchronize(op->stream));
  return SCOTTY_OK;
}

// Cell index build over the current slice store (cix_build_kernel, class PUSH_OTHER): it reads only operator state,
// so the grid watermark enqueues it behind the result transfer for the next micro-batch.
int enqueue_cix(scotty_op* op) {
  if (!op->d_cix) {
    HIPCHK(dev_malloc(&op->d_cix, CIX_CAP * 4));
    HIPCHK(dev_malloc(&op->d_cixmeta, 8 * 8));
  }
  IngestArgs ia{};
  ia.s_tstart = op->d_tstart;
  ia.grid = op->d_grid;
  ia.meta = op->d_meta;
  ia.cix = op->d_cix;
  ia.cix_meta = op->d_cixmeta;
  ia.cix_margin = std::max<int64_t>(4 * op->last_span, 4000);
  scotty_op::TEv tx;
  int rc = tlaunch(op, tx, SCOTTY_TIME_PUSH_OTHER);
  if (rc) return rc;
  HIPCHK(launch_cix_build(ia, op->stream, tx.a, tx.b));
  tlaunched(op, tx);
  return SCOTTY_OK;
}

// Ingest launch of one micro-batch (no host synchronisation); *tile_out = the arrival tile size used.
int enqueue_ingest(scotty_op* op, const int64_t* d_ts, const void* d_val, int64_t n, int64_t* tile_out) {
  int rc = ensure_tiles(op, n);
  if (rc) return rc;
  IngestArgs ia{};
  ia.ts = d_ts;
  ia.val = d_val;
  ia.n = n;
  ia.s_tstart = op->d_tstart;
  ia.grid = op->d_grid;
  ia.c_cnt = op->d_ccnt;
  ia.c_tmax = op->d_ctmax;
  for (int k = 0; k < NPART; k++) ia.c_part[k] = op->d_cpart[k];
  ia.tilemax = op->d_tilemax;
  ia.meta = op->d_meta;
  if (!op->d_cix) {
    HIPCHK(dev_malloc(&op->d_cix, CIX_CAP * 4));
    HIPCHK(dev_malloc(&op->d_cixmeta, 8 * 8));
  }
  ia.cix = op->d_cix;
  ia.cix_meta = op->d_cixmeta;
  ia.cix_margin = std::max<int64_t>(4 * op->last_span, 4000);
  if (!op->cix_ready) {
    rc = enqueue_cix(op);
    if (rc) return rc;
  }
  op->cix_ready = false;  // this micro-batch changes the slice store
  // tile: power of two >= TILE_MIN with at most NT_MAX tiles (the commit kernel keeps them in LDS)
  int64_t tile = TILE_MIN;
  while ((n + tile - 1) / tile > NT_MAX) tile <<= 1;
  // one round of resident workgroups, each wave streaming a tile-aligned contiguous range (a tune value overrides).
  // A stream whose last committed push was in order (< 1 % of its tuples outside their wave's current cell) takes the
  // streaming variant: the software-pipelined loop on fewer, longer waves (fewer concurrent DRAM streams: C2 ingest
  // 279 -> 264 us per 2^27 tuples, profiles/r04/r04f); out-of-order streams keep more waves to hide their slow paths
  // (C2s: 314 us with 1024 workgroups, 321 us with 512)
  const DevMeta& hs = *op->h_snap;
  const bool streaming = op->ingest_mode < 0 && op->ingest_blocks <= 0 && op->vt == VT_I32 &&
                         !(op->need & (NEED_MIN | NEED_MAX)) && hs.n_last > 0 && hs.slow_last * 100 < hs.n_last;
  const bool i32_sum = op->vt == VT_I32 && !(op->need & (NEED_MIN | NEED_MAX));
  const int64_t target_blocks = op->ingest_blocks > 0 ? op->ingest_blocks
                                : streaming          ? INGEST_STREAMING_WGS
                                : i32_sum            ? INGEST_OOO_I32_WGS
                                                     : 256 * ingest_wgs_per_cu(op->vt, op->need);
  int64_t per_wave = (n + target_blocks * 4 - 1) / (target_blocks * 4);
  per_wave = ((per_wave + tile - 1) / tile) * tile;
  if (per_wave < tile) per_wave = tile;
  ia.per_wave = per_wave;
  ia.tile = tile;
  const int64_t nblocks = (n + per_wave * 4 - 1) / (per_wave * 4);
  // the stamps buffer holds 8192 x 4 words, the commit's 16 at its end: a launch of more workgroups records none
  if (op->stamps_on && nblocks <= 8192 - 4) {
    if (!op->d_stamps) HIPCHK(dev_malloc(&op->d_stamps, 8192 * 4 * 8));
    ia.stamps = op->d_stamps;
  }
  std::pair<hipEvent_t, hipEvent_t> ev{};
  if (op->timing) {
    // timing mode only (scotty_enable_timing: the bench's instrumented steps, not its wall-clock ones): the work
    // queued before the ingest -- the cell index the last watermark enqueued behind itself -- finishes first, so the
    // start stamp of the ingest's dispatch cannot fall inside it (C1: 145 us by events against 134 us in the trace)
    HIPCHK(hipStreamSynchronize(op->stream));
    if (!op->ev_pool.empty()) {
      ev = op->ev_pool.back();
      op->ev_pool.pop_back();
    } else {
      HIPCHK(hipEventCreate(&ev.first));
      HIPCHK(hipEventCreate(&ev.second));
    }
    set_ingest_timing_events(ev.first, ev.second);
  }
  HIPCHK(launch_ingest(ia, op->vt, op->need, nblocks, op->stream, streaming ? INGEST_STREAMING : op->ingest_mode));
  op->last_ingest_blocks = nblocks;
  op->last_ingest_streaming = streaming ? 1 : 0;
  if (op->timing) {
    op->ev_pending.push_back(ev);
    op->t_tuples += n;
  }
  *tile_out = tile;
  return SCOTTY_OK;
}

// Runs the ingest + commit launches of one micro-batch (no host synchronisation).
int enqueue_push(scotty_op* op, const int64_t* d_ts, const void* d_val, int64_t n, int64_t seq, int64_t base) {
  int64_t tile = TILE_MIN;
  int rc = enqueue_ingest(op, d_ts, d_val, n, &tile);
  if (rc) return rc;
  if (op->first) {  // SCOTTY_AGG_FIRST: the cells' first arrival indices (first_kernel), before the commit folds them
    IngestArgs fa{};
    fa.ts = d_ts;
    fa.n = n;
    fa.s_tstart = op->d_tstart;
    fa.grid = op->d_grid;
    fa.meta = op->d_meta;
    fa.cix = op->d_cix;
    fa.cix_meta = op->d_cixmeta;
    fa.c_first = op->d_cfirst;
    fa.seq_base = base;
    scotty_op::TEv tf;
    rc = tbegin(op, tf, SCOTTY_TIME_PUSH_OTHER);
    if (rc) return rc;
    HIPCHK(launch_first(fa, op->stream));
    rc = tend(op, tf);
    if (rc) return rc;
  }
  CommitArgs ca{};
  ca.ts = d_ts;
  ca.n = n;
  ca.tile = tile;
  ca.max_lateness = op->max_lateness;
  ca.scap = op->scap;
  ca.grid = op->d_grid;
  ca.tilemax = op->d_tilemax;
  ca.pmax = op->d_pmax;
  ca.rank = op->d_rank;
  ca.flag = op->d_flag;
  ca.s_tstart = op->d_tstart;
  ca.s_tlast = op->d_tlast;
  ca.s_cnt = op->d_scnt;
  for (int k = 0; k < NPART; k++) ca.s_part[k] = op->d_spart[k];
  ca.c_cnt = op->d_ccnt;
  ca.c_tmax = op->d_ctmax;
  for (int k = 0; k < NPART; k++) ca.c_part[k] = op->d_cpart[k];
  ca.meta = op->d_meta;
  ca.need = op->need;
  ca.vt = op->vt;
  ca.push_seq = seq;
  ca.s_first = op->d_sfirst;
  ca.c_first = op->d_cfirst;
  scotty_op::TEv tc;
  rc = tlaunch(op, tc, SCOTTY_TIME_PUSH_OTHER);
  if (rc) return rc;
  if (op->stamps_on && op->d_stamps) ca.stamps = op->d_stamps + 8192 * 4 - 16;  // the commit's phase stamps
  HIPCHK(launch_commit(ca, op->stream, tc.a, tc.b));
  tlaunched(op, tc);
  return SCOTTY_OK;
}

// First tuple of the operator's life: StreamSlicer + SliceManager for tuple 0 (the store is empty).
int start_stream(scotty_op* op, int64_t ts0) {
  if (op->first && !op->d_sfirst) {  // SCOTTY_AGG_FIRST arrays (aggregations are fixed by the first push)
    HIPCHK(dev_malloc(&op->d_sfirst, op->scap * 8));
    HIPCHK(dev_malloc(&op->d_cfirst, op->ccap * 8));
    HIPCHK(launch_fill_u64((unsigned long long*)op->d_cfirst, op->ccap, (unsigned long long)FIRST_NONE, op->stream));
  }
  std::vector<int64_t> edges;
  int64_t n_pending = JMIN;
  if (op->has_fixed && !first_walk(op, ts0, edges, n_pending))
    return fail(op, SCOTTY_ERR_UNSUPPORTED,
                "the reference StreamSlicer loops forever on this configuration (calculateNextFixedEdge returns "
                "Long.MIN_VALUE for a power-of-two time window size/slide, S/StreamSlicer.java:103-116)");
  // SliceManager.processElement: an empty store first gets the slice [0, MAX) (S/SliceManager.java:49-51)
  if (edges.empty()) edges.push_back(0);
  const int64_t s0 = (int64_t)edges.size();
  std::vector<int64_t> zeros(s0, 0), idmin(s0, INT64_MAX), idmax(s0, INT64_MIN);
  HIPCHK(hipMemcpyAsync(op->d_tstart, edges.data(), s0 * 8, hipMemcpyHostToDevice, op->stream));
  HIPCHK(hipMemcpyAsync(op->d_tlast, edges.data(), s0 * 8, hipMemcpyHostToDevice, op->stream));
  HIPCHK(hipMemcpyAsync(op->d_scnt, zeros.data(), s0 * 8, hipMemcpyHostToDevice, op->stream));
  HIPCHK(hipMemcpyAsync(op->d_spart[0], zeros.data(), s0 * 8, hipMemcpyHostToDevice, op->stream));
  HIPCHK(hipMemcpyAsync(op->d_spart[1], idmin.data(), s0 * 8, hipMemcpyHostToDevice, op->stream));
  HIPCHK(hipMemcpyAsync(op->d_spart[2], idmax.data(), s0 * 8, hipMemcpyHostToDevice, op->stream));
  if (op->d_sfirst) HIPCHK(hipMemcpyAsync(op->d_sfirst, idmin.data(), s0 * 8, hipMemcpyHostToDevice, op->stream));
  DevMeta m{};
  m.head = 0;
  m.tail = s0;
  m.prev_max = ts0;  // maxEventTime after the first tuple
  m.oldest_start = edges[0];
  if (op->has_fixed) {
    build_grid(op, n_pending, std::max(ts0, (int64_t)0) + std::max<int64_t>(64 * op->last_span, 600000));
  } else {
    op->grid.clear();
  }
  m.j0 = 0;
  m.gcount = (int64_t)op->grid.size();
  if (!op->grid.empty())
    HIPCHK(hipMemcpyAsync(op->d_grid, op->grid.data(), op->grid.size() * 8, hipMemcpyHostToDevice, op->stream));
  HIPCHK(hipMemcpyAsync(op->d_meta, &m, sizeof(DevMeta), hipMemcpyHostToDevice, op->stream));
  HIPCHK(hipStreamSynchronize(op->stream));
  *op->h_snap = m;
  op->h_oldest = edges[0];
  op->h_prev_max = ts0;
  op->started = true;
  return SCOTTY_OK;
}

// Re-extend the grid horizon from the current pending edge (only at synchronisation points).
int maybe_extend_grid(scotty_op* op, bool force) {
  if (!op->has_fixed || op->grid_complete) return SCOTTY_OK;
  const DevMeta& m = *op->h_snap;
  const int64_t j0 = m.j0;
  const int64_t remaining = (int64_t)op->grid.size() - j0;
  const int64_t last = op->grid.back();
  const int64_t margin = std::max<int64_t>(16 * op->last_span, 60000);
  if (!force && remaining > 1024 && jsub(last, m.prev_max) > margin) return SCOTTY_OK;
  const int64_t n_pending = op->grid[j0];
  const int64_t need_to = std::max(m.batch_max, m.prev_max);
  build_grid(op, n_pending, jadd(need_to, std::max<int64_t>(64 * op->last_span, 600000)));
  if ((int64_t)op->grid.size() >= op->gcap - 1 && op->grid.back() <= need_to)
    return fail(op, SCOTTY_ERR_UNSUPPORTED, "micro-batch spans more edge-grid points than the grid capacity");
  return upload_grid(op);
}

int replay_after_overflow(scotty_op* op) {
  op->cix_ready = false;
  for (int attempt = 0; attempt < 4; attempt++) {
    DevMeta& m = *op->h_snap;
    if (!m.overflow) return SCOTTY_OK;
    if (m.overflow == 2) return fail(op, SCOTTY_ERR_NOMEM, "slice capacity exceeded");
    if (m.overflow == 3)
      return fail(op, SCOTTY_ERR_UNSUPPORTED, "sharded batch exceeded the exchange capacity or the edge-grid horizon "
                                              "(scotty_tune \"shard_cells\" / \"shard_cands\")");
    const int64_t failed = m.failed_push;
    static const int64_t zero = 0;  // (static: the copy may read it after this scope ends)
    HIPCHK(hipMemcpyAsync(&op->d_meta->overflow, &zero, 8, hipMemcpyHostToDevice, op->stream));
    m.overflow = 0;
    int rc = maybe_extend_grid(op, true);
    if (rc) return rc;
    for (auto& p : op->pending)
      if (p.seq >= failed) {
        rc = enqueue_push(op, p.ts, p.val, p.n, p.seq, p.base);
        if (rc) return rc;
      }
    rc = sync_snapshot(op);
    if (rc) return rc;
  }
  return fail(op, SCOTTY_ERR_UNSUPPORTED, "edge-grid horizon overflow could not be resolved");
}

// Number of windows WindowManager.assignContextFreeWindows triggers (S/WindowManager.java:104-118): the same loops as
// TumblingWindow / SlidingWindow / FixedBandWindow.triggerWindows, which the device runs again to emit them (the
// count only sizes the packed result transfer).  -1: more windows than any result buffer could hold.
// Upper bound of count_triggers in O(#definitions): triggered tumbling windows start in (last_wm - size, wm - size],
// sliding windows end in (last_wm, wm + 1] (one per slide), a fixed band emits at most once.  -1 when the values
// are too large for the bound to be exact arithmetic (the exact loops run instead).
int64_t bound_triggers(const scotty_op* op, int64_t last_wm, int64_t wm) {
  const int64_t LIM = (int64_t)1 << 61;
  if (wm > LIM || wm < -LIM || last_wm > LIM || last_wm < -LIM) return -1;
  const int64_t span = std::max<int64_t>(0, wm - last_wm + 1);
  int64_t n = 0;
  for (const CFWin& w : op->windows) {
    if (w.kind == SCOTTY_WIN_TUMBLING) {
      if (w.a > LIM) return -1;
      n += span / w.a + 2;
    } else if (w.kind == SCOTTY_WIN_SLIDING) {
      if (w.a > LIM || w.b > LIM) return -1;
      n += span / w.b + 2;
    } else {
      n += 1;
    }
    if (n > ((int64_t)1 << 31)) return -1;
  }
  return n;
}

int64_t count_triggers(const scotty_op* op, int64_t last_wm, int64_t wm) {
  int64_t n = 0;
  const int64_t limit = (int64_t)1 << 31;
  for (const CFWin& w : op->windows) {
    if (w.kind == SCOTTY_WIN_TUMBLING) {  // TumblingWindow.triggerWindows :34-39
      const int64_t size = w.a;
      const int64_t last_start = jsub(last_wm, jmod(jadd(last_wm, size), size));
      for (int64_t ws = last_start; jadd(ws, size) <= wm; ws = jadd(ws, size))
        if (++n > limit) return -1;
    } else if (w.kind == SCOTTY_WIN_SLIDING) {  // SlidingWindow.triggerWindows :50-57
      const int64_t size = w.a, slide = w.b;
      const int64_t last_start = jsub(wm, jmod(jadd(wm, slide), slide));
      int64_t it = 0;
      for (int64_t ws = last_start; jadd(ws, size) > last_wm; ws = jsub(ws, slide)) {
        if (ws >= 0 && jadd(ws, size) <= jadd(wm, 1)) n++;
        if (++it > limit || n > limit) return -1;
      }
    } else {  // FixedBandWindow.triggerWindows :51-57
      const int64_t e = jadd(w.a, w.b);
      if (last_wm <= e && e <= wm) n++;
    }
  }
  return n;
}

}  // namespace

// ====================================================================== C-ABI
extern "C" {

int scotty_create(scotty_op** out, int device, int value_type, uint32_t flags) {
  if (!out) return SCOTTY_ERR_ARG;
  *out = nullptr;
  if (value_type < VT_I32 || value_type > VT_F64) return SCOTTY_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SCOTTY_ERR_HIP;
  if (device < 0 || device >= ndev) return SCOTTY_ERR_ARG;
  scotty_op* op = new scotty_op();
  op->device = device;
  op->vt = value_type;
  op->keyed = (flags & SCOTTY_FLAG_KEYED) != 0;
  int rc = alloc_all(op);
  if (rc) {
    scotty_destroy(op);
    return rc;
  }
  *out = op;
  return SCOTTY_OK;
}

void scotty_destroy(scotty_op* op) {
  if (!op) return;
  (void)hipSetDevice(op->device);
  if (op->stream) (void)hipStreamSynchronize(op->stream);
  auto F = [](void* p) { if (p) (void)hipFree(p); };
  F(op->d_meta); F(op->d_tstart); F(op->d_tlast); F(op->d_scnt); F(op->d_grid); F(op->d_sfirst); F(op->d_cfirst);
  F(op->d_ccnt); F(op->d_ctmax); F(op->d_tilemax); F(op->d_pmax); F(op->d_rank); F(op->d_flag);
  F(op->d_scratch); F(op->d_bcnt); F(op->d_pcnt); F(op->d_psum); F(op->d_stmin); F(op->d_stmax); F(op->d_wdef);
  F(op->d_out);
  for (int k = 0; k < NPART; k++) { F(op->d_spart[k]); F(op->d_cpart[k]); F(op->d_bpart[k]); }
  for (void* p : op->owned) F(p);
  delete op->ingest;
  if (op->h_snap) (void)hipHostFree(op->h_snap);
  if (op->h_out) (void)hipHostFree(op->h_out);
  for (auto& e : op->tev_pending) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
  for (auto& e : op->ev_pending) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
  if (op->order_ev) (void)hipEventDestroy(op->order_ev);
  if (op->wm_ev) (void)hipEventDestroy(op->wm_ev);
  for (auto& e : op->ev_pool) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
  delete op->x;
  delete op->c;
  F(op->d_shrank); F(op->d_shflag); F(op->d_cix); F(op->d_cixmeta); F(op->d_stamps);
  if (op->stream) (void)hipStreamDestroy(op->stream);
  delete op;
}

const char* scotty_last_error(scotty_op* op) { return op ? op->err.c_str() : "null op"; }

int scotty_add_window(scotty_op* op, int kind, int measure, int64_t a, int64_t b) {
  if (!op) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (kind < SCOTTY_WIN_TUMBLING || kind > SCOTTY_WIN_FIXED_BAND || (measure != SCOTTY_MEASURE_TIME &&
                                                                     measure != SCOTTY_MEASURE_COUNT))
    return fail(op, SCOTTY_ERR_ARG, "unknown window kind / measure");
  if ((kind == SCOTTY_WIN_TUMBLING && a <= 0) || (kind == SCOTTY_WIN_SLIDING && (a <= 0 || b <= 0)))
    return fail(op, SCOTTY_ERR_ARG, "window size / slide must be positive");
  if (kind == SCOTTY_WIN_SESSION && a < 0) return fail(op, SCOTTY_ERR_ARG, "session gap must be >= 0");
  const bool exact_only = kind == SCOTTY_WIN_SESSION || measure == SCOTTY_MEASURE_COUNT;
  if (op->mode == 3) {  // count path: more count windows mid-stream (the pending count edge keeps its value)
    if (kind == SCOTTY_WIN_SESSION || measure != SCOTTY_MEASURE_COUNT)
      return fail(op, SCOTTY_ERR_UNSUPPORTED, "time / session window added to a count-path operator after elements "
                                              "were processed");
    op->xwins.push_back({kind, measure, a, b});
    int rc = op->c->configure(op->xwins, op->aggs, op->max_lateness);
    if (rc) {
      op->xwins.pop_back();
      return fail(op, rc, op->c->err);
    }
    return SCOTTY_OK;
  }
  if (op->mode == 2) {  // exact engine: reconfigure (windows may be added mid-stream, S/WindowManager.java:121-147)
    op->xwins.push_back({kind, measure, a, b});
    int rc = op->x->configure(op->xwins, op->aggs, op->max_lateness, op->agg_inv);
    if (rc) {
      op->xwins.pop_back();
      return fail(op, rc, op->x->err);
    }
    return SCOTTY_OK;
  }
  if (exact_only && op->mode == 1)
    return fail(op, SCOTTY_ERR_UNSUPPORTED,
                "session / count window added after elements were processed by the context-free grid path");
  op->xwins.push_back({kind, measure, a, b});
  if (exact_only) return SCOTTY_OK;
  CFWin w{kind, a, b};
  const bool had_fixed = op->has_fixed;
  if (op->started && !had_fixed)
    return fail(op, SCOTTY_ERR_UNSUPPORTED,
                "first context-free window added after elements were processed (edge walk would append "
                "slices out of order)");
  op->windows.push_back(w);
  op->wdef_dirty = true;
  op->max_fixed_window_size = std::max(op->max_fixed_window_size, w.clear_delay());  // S/WindowManager.java:124
  op->has_fixed = true;
  if (op->started) {
    // mid-stream addition: the pending edge N keeps its value (computed with the old grid); later edges
    // follow the new union grid (StreamSlicer.calculateNextFixedEdge only runs at the next crossing).
    int rc = sync_snapshot(op);
    if (rc) return rc;
    const int64_t n_pending = op->h_snap->gcount > 0 ? op->grid[op->h_snap->j0] : JMAX;
    build_grid(op, n_pending, jadd(op->h_snap->prev_max, std::max<int64_t>(64 * op->last_span, 600000)));
    rc = upload_grid(op);
    if (rc) return rc;
    rc = sync_snapshot(op);
    if (rc) return rc;
  }
  return SCOTTY_OK;
}

int scotty_add_aggregation(scotty_op* op, int kind_flags) {
  if (!op) return SCOTTY_ERR_ARG;
  const int kind = kind_flags & 0xFFFF;
  const bool inv = (kind_flags & SCOTTY_AGG_INVERTIBLE) != 0;
  if ((kind_flags & ~(0xFFFF | SCOTTY_AGG_INVERTIBLE)) != 0) return fail(op, SCOTTY_ERR_ARG, "unknown aggregation flags");
  if (inv && agg_need(kind) != NEED_SUM && kind != SCOTTY_AGG_COUNT)
    return fail(op, SCOTTY_ERR_ARG, "only sums and counts have an inverse (InvertibleAggregateFunction)");
  const int vt = agg_value_type(kind);
  if (vt == -2) return fail(op, SCOTTY_ERR_ARG, "unknown aggregation kind");
  if (vt >= 0 && vt != op->vt) return fail(op, SCOTTY_ERR_ARG, "aggregation kind does not match the value type");
  if ((int)op->aggs.size() >= SCOTTY_MAX_AGGS) return fail(op, SCOTTY_ERR_ARG, "too many aggregations");
  if (op->mode != 0)  // existing slices would lack the new function's state (S/state/AggregateState.java:44-50)
    return fail(op, SCOTTY_ERR_UNSUPPORTED, "aggregation added after elements were processed");
  op->aggs.push_back(kind);
  op->agg_inv.push_back(inv ? 1 : 0);
  op->need |= agg_need(kind);
  if (kind == SCOTTY_AGG_FIRST) op->first = true;
  return (int)op->aggs.size() - 1;
}

int scotty_set_max_lateness(scotty_op* op, int64_t l) {
  if (!op) return SCOTTY_ERR_ARG;
  op->max_lateness = l;
  if (op->mode == 3) {
    int rc = op->c->configure(op->xwins, op->aggs, op->max_lateness);
    if (rc) return fail(op, rc, op->c->err);
  }
  if (op->mode == 2) {
    int rc = op->x->configure(op->xwins, op->aggs, op->max_lateness, op->agg_inv);
    if (rc) return fail(op, rc, op->x->err);
  }
  return SCOTTY_OK;
}

// First push: the grid path serves non-keyed ops whose windows are all context-free time windows; every
// other configuration runs on the exact engine.
static int decide_mode(scotty_op* op) {
  if (op->mode != 0) return SCOTTY_OK;
  bool exact = op->keyed;
  for (const XWinDef& w : op->xwins)
    if (w.kind == SCOTTY_WIN_SESSION || w.measure == SCOTTY_MEASURE_COUNT) exact = true;
  if (!exact) {
    op->mode = 1;
    return SCOTTY_OK;
  }
  if (op->first) {
    op->failed = true;
    return fail(op, SCOTTY_ERR_UNSUPPORTED, "SCOTTY_AGG_FIRST runs on the grid path only (non-keyed operators with "
                                            "context-free time windows)");
  }
  // count path: context-free windows only, at least one of them on the count measure (time windows' edges come
  // from the in-order stream's timestamps, CEngine::time_edges)
  bool count_only = !op->keyed && !op->xwins.empty() && op->x_count_on;
  for (const XWinDef& w : op->xwins)
    if (w.kind == SCOTTY_WIN_SESSION) count_only = false;
  if (count_only) {  // count_common.h: edges are a function of counts, one micro-batch = segmented reduction
    op->c = new CEngine();
    std::string e;
    int rc = op->c->init(op->device, op->stream, op->vt, e);
    if (!rc) rc = op->c->configure(op->xwins, op->aggs, op->max_lateness);
    if (!rc && op->last_watermark != -1) rc = op->c->set_last_watermark(op->last_watermark);
    op->c->shard_cap = op->count_shard_cap;
    op->c->shard_async = op->shard_async;
    op->c->prefix_one = op->c_prefix_one;
    if (rc) {
      op->failed = true;
      return fail(op, rc, e.empty() ? op->c->err : e);
    }
    op->mode = 3;
    return SCOTTY_OK;
  }
  op->x = new XEngine();
  op->x->sc_override = op->x_sc;
  op->x->sess_override = op->x_sess;
  op->x->serial = op->x_serial;
  op->x->quiet_off = op->x_quiet_off;
  op->x->band_on = op->x_band_on;
  op->x->lane_off = op->x_lane_off;
  op->x->kg_off = op->x_kg_off;
  if (op->x_kg_chunk >= 0) op->x->kg_min_chunk = op->x_kg_chunk;
  if (op->x_kg_variant >= 0) op->x->kg_variant = op->x_kg_variant;
  op->x->xq_prefix = op->x_prefix;
  op->x->xq_ingest_mode = op->x_qmode;
  op->x->xq_ingest_blocks = op->x_qblocks;
  op->x->lane_session_off = op->x_ls_off;
  op->x->lane_session_occ = op->x_ls_occ;
  op->x->lane_count_off = op->x_lc_off;
  op->x->pack_off = op->x_pack_off;
  op->x->sort_digit10 = op->x_digit10;
  op->x->lsdbg_on = op->x_lsdbg;
  op->x->timing = op->timing;  // scotty_enable_timing before the first push (the natural order) reaches the engine
  std::string e;
  int rc = op->x->init(op->device, op->stream, op->vt, op->keyed, e);
  if (!rc) rc = op->x->configure(op->xwins, op->aggs, op->max_lateness, op->agg_inv);
  if (!rc && !op->keyed && op->last_watermark != -1) rc = op->x->set_last_watermark(op->last_watermark);
  if (rc) {
    op->failed = true;
    return fail(op, rc, op->x->err);
  }
  op->mode = 2;
  return SCOTTY_OK;
}

static int push_impl(scotty_op* op, const int64_t* d_ts, const void* d_val, int64_t n, const int64_t* h_ts0) {
  if (n <= 0) return SCOTTY_OK;
  int rc = decide_mode(op);
  if (rc) return rc;
  if (op->mode == 3) {
    op->pending.push_back({d_ts, d_val, n, op->push_seq++});
    op->x_pushed += (uint64_t)n;
    std::pair<hipEvent_t, hipEvent_t> ev{};
    if (op->timing) {
      if (!op->ev_pool.empty()) {
        ev = op->ev_pool.back();
        op->ev_pool.pop_back();
      } else {
        HIPCHK(hipEventCreate(&ev.first));
        HIPCHK(hipEventCreate(&ev.second));
      }
    }
    // device-time classes of the count path: the whole push on the op's stream (marker events: the interval holds
    // any bubble a host read inside the push leaves, so push_other is an upper bound), less the ingest launch, whose
    // dispatch stamps its own pair (ev) -> ingest
    scotty_op::TEv tp;
    rc = tbegin(op, tp, SCOTTY_TIME_PUSH_OTHER);
    if (rc) return rc;
    rc = op->c->push(d_ts, d_val, n, ev.first, ev.second);
    if (rc) return fail(op, rc, op->c->err);
    rc = tend(op, tp);
    if (rc) return rc;
    if (op->timing) {
      op->ev_pending.push_back(ev);
      op->t_tuples += n;
    }
    return SCOTTY_OK;
  }
  if (op->mode == 2) {
    op->pending.push_back({d_ts, d_val, n, op->push_seq++});
    op->x_pushed += (uint64_t)n;
    rc = op->x->use_serial() ? op->x->push(d_ts, d_val, n) : op->x->push_batch(d_ts, d_val, n);
    if (rc) return fail(op, rc, op->x->err);
    return SCOTTY_OK;
  }
  if (!op->started) {
    int64_t ts0;
    if (h_ts0) ts0 = *h_ts0;
    else HIPCHK(hipMemcpy(&ts0, d_ts, 8, hipMemcpyDeviceToHost));
    rc = start_stream(op, ts0);
    if (rc) return rc;
  }
  const int64_t seq = op->push_seq++;
  const int64_t base = op->arrivals;
  op->arrivals += n;
  op->pending.push_back({d_ts, d_val, n, seq, base});
  return enqueue_push(op, d_ts, d_val, n, seq, base);
}

static size_t value_bytes(const scotty_op* op) { return op->vt == VT_I32 ? 4 : 8; }

int scotty_process_elements(scotty_op* op, const int64_t* ts, const void* val, size_t n) {
  if (!op || (n && (!ts || !val))) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (op->keyed) return fail(op, SCOTTY_ERR_ARG, "keyed operator: use scotty_process_keyed_elements");
  if (n == 0) return SCOTTY_OK;
  // host columns -> HBM (host_ingest.h): pinned slots DMA'd in place, pageable input chunked through pinned
  // staging; the copies stay in the ingest arena until the watermark (the grid path may replay a push)
  int64_t* d_ts = nullptr;
  void* d_val = nullptr;
  HIPCHK(op->ingest->stage(ts, val, nullptr, n, value_bytes(op), true, &d_ts, &d_val, nullptr));
  return push_impl(op, d_ts, d_val, (int64_t)n, ts);
}

int scotty_host_buffers(scotty_op* op, size_t n, int64_t** ts, void** val, uint32_t** key) {
  if (!op || !ts || !val || (op->keyed && !key)) return SCOTTY_ERR_ARG;
  HIPCHK(op->ingest->host_buffers(n, value_bytes(op), op->keyed, ts, val, key));
  return SCOTTY_OK;
}

int scotty_process_elements_device(scotty_op* op, const int64_t* d_ts, const void* d_val, size_t n) {
  if (!op || (n && (!d_ts || !d_val))) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (op->keyed) return fail(op, SCOTTY_ERR_ARG, "keyed operator: use scotty_process_keyed_elements_device");
  if (((uintptr_t)d_ts & 15) || ((uintptr_t)d_val & 15))
    return fail(op, SCOTTY_ERR_ARG, "device buffers must be 16-byte aligned");
  return push_impl(op, d_ts, d_val, (int64_t)n, nullptr);
}

static int keyed_push(scotty_op* op, const uint32_t* d_key, const int64_t* d_ts, const void* d_val, int64_t n) {
  int rc = decide_mode(op);
  if (rc) return rc;
  op->x_pushed += (uint64_t)n;
  rc = op->x->push_keyed(d_key, d_ts, d_val, n);
  if (rc) return fail(op, rc, op->x->err);
  return SCOTTY_OK;
}

int scotty_process_keyed_elements(scotty_op* op, const uint32_t* key, const int64_t* ts, const void* val, size_t n) {
  if (!op || (n && (!ts || !val || !key))) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (!op->keyed) return fail(op, SCOTTY_ERR_ARG, "not a keyed operator (create with SCOTTY_FLAG_KEYED)");
  if (n == 0) return SCOTTY_OK;
  // keyed pushes complete inside the call: the device copy goes to reusable scratch, not the arena
  int64_t* d_ts = nullptr;
  void* d_val = nullptr;
  uint32_t* d_key = nullptr;
  HIPCHK(op->ingest->stage(ts, val, key, n, value_bytes(op), false, &d_ts, &d_val, &d_key));
  return keyed_push(op, d_key, d_ts, d_val, (int64_t)n);
}

int scotty_process_keyed_elements_device(scotty_op* op, const uint32_t* d_key, const int64_t* d_ts,
                                         const void* d_val, size_t n) {
  if (!op || (n && (!d_ts || !d_val || !d_key))) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (!op->keyed) return fail(op, SCOTTY_ERR_ARG, "not a keyed operator (create with SCOTTY_FLAG_KEYED)");
  if (n == 0) return SCOTTY_OK;
  return keyed_push(op, d_key, d_ts, d_val, (int64_t)n);
}

// watermark of the exact engine
static int exact_watermark(scotty_op* op, int64_t wm, scotty_windows* out, bool to_host) {
  XResult& r = op->xr;
  const uint64_t dropped_before = op->dropped;
  scotty_op::TEv tw;
  if (op->mode == 3) {
    int rt = tbegin(op, tw, SCOTTY_TIME_WATERMARK);
    if (rt) return rt;
  }
  int rc = op->mode == 3 ? op->c->watermark(wm, r, to_host) : op->x->watermark(wm, r, to_host);
  if (rc) return fail(op, rc, op->mode == 3 ? op->c->err : op->x->err);
  if (op->mode == 3) {  // device-time classes of the interval (scotty_enable_timing): ingest launches, the rest
    rc = tend(op, tw);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(op->stream));
    for (auto& e : op->ev_pending) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) {
        op->t_ms += ms;
        op->t_cls_ms[SCOTTY_TIME_INGEST] += ms;
        op->t_cls_ms[SCOTTY_TIME_PUSH_OTHER] -= ms;  // inside a push interval
      }
      op->t_launches++;
      op->t_cls_n[SCOTTY_TIME_INGEST]++;
      op->ev_pool.push_back(e);
    }
    op->ev_pending.clear();
    tresolve(op);
  }
  op->dropped = r.dropped;
  op->processed = op->x_pushed - r.dropped;
  for (void* p : op->owned) (void)hipFree(p);
  op->owned.clear();
  op->ingest->reset();
  op->pending.clear();
  if (out) {
    std::memset(out, 0, sizeof(*out));
    out->n_windows = (size_t)r.n;
    out->n_aggs = (int32_t)op->aggs.size();
    if (to_host) {
      out->start = r.start.data();
      out->end = r.end.data();
      out->measure = r.meas.data();
      out->has_value = r.has.data();
      for (size_t k = 0; k < op->aggs.size() && k < r.vals.size(); k++) out->values[k] = r.vals[k].data();
      out->key = op->keyed ? r.key.data() : nullptr;
    } else {
      out->start = r.d_start;
      out->end = r.d_end;
      out->measure = r.d_meas;
      out->has_value = r.d_has;
      for (size_t k = 0; k < op->aggs.size(); k++) out->values[k] = r.d_vals[k];
      out->key = op->keyed ? r.d_key : nullptr;
    }
  }
  if (op->dropped > dropped_before) {
    op->err = "tuples older than the oldest retained slice were dropped (reference: IndexOutOfBoundsException)";
    return SCOTTY_WARN_LATE_DROPPED;
  }
  return SCOTTY_OK;
}

int scotty_process_watermark_device(scotty_op* op, int64_t wm, scotty_windows* out) {
  if (!op) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (op->mode != 2 && op->mode != 3) {
    if (op->mode == 0 && op->keyed) {  // keyed op without any tuple yet: no operators, no windows
      if (out) std::memset(out, 0, sizeof(*out));
      return SCOTTY_OK;
    }
    return fail(op, SCOTTY_ERR_UNSUPPORTED, "device results are provided by the exact engine and count path only");
  }
  return exact_watermark(op, wm, out, false);
}

static int64_t shard_words(const scotty_op* op) { return SHARD_HDR + 6 * op->shard_kc + 2 * op->shard_kg; }

size_t scotty_shard_xbytes(scotty_op* op) {
  if (!op) return 0;
  if (op->mode == 0 && !op->keyed && !op->xwins.empty()) (void)decide_mode(op);
  if (op->mode == 3) return (size_t)op->c->shard_words() * 8;
  return (size_t)shard_words(op) * 8;
}

static ShardArgs shard_args(scotty_op* op) {
  ShardArgs a{};
  a.tile = op->shard_tile;
  a.max_lateness = op->max_lateness;
  a.scap = op->scap;
  a.grid = op->d_grid;
  a.tilemax = op->d_tilemax;
  a.s_tstart = op->d_tstart;
  a.s_tlast = op->d_tlast;
  a.s_cnt = op->d_scnt;
  for (int k = 0; k < NPART; k++) a.s_part[k] = op->d_spart[k];
  a.c_cnt = op->d_ccnt;
  a.c_tmax = op->d_ctmax;
  for (int k = 0; k < NPART; k++) a.c_part[k] = op->d_cpart[k];
  a.meta = op->d_meta;
  a.rank_buf = op->d_shrank;
  a.flag_buf = op->d_shflag;
  a.kc_cap = op->shard_kc;
  a.kg_cap = op->shard_kg;
  a.need = op->need;
  a.vt = op->vt;
  return a;
}

int scotty_shard_push(scotty_op* op, const int64_t* d_ts, const void* d_val, size_t n, int64_t ts0, void* d_xbuf) {
  if (!op || !d_xbuf || (n && (!d_ts || !d_val))) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (op->keyed) return fail(op, SCOTTY_ERR_UNSUPPORTED, "keyed operators shard by key: no exchange needed");
  if (((uintptr_t)d_ts & 15) || ((uintptr_t)d_val & 15))  // the ingest kernels load 16 B per lane
    return fail(op, SCOTTY_ERR_ARG, "device buffers must be 16-byte aligned");
  int rc = decide_mode(op);
  if (rc) return rc;
  if (op->mode == 3)
    return fail(op, SCOTTY_ERR_ARG, "count windows: use scotty_shard_push_counted (the chunk's count offset)");
  if (op->mode != 1)
    return fail(op, SCOTTY_ERR_UNSUPPORTED, "sharding needs context-free time windows or count windows only");
  if (op->first) return fail(op, SCOTTY_ERR_UNSUPPORTED, "SCOTTY_AGG_FIRST operators are not sharded");
  if (!op->has_fixed) return fail(op, SCOTTY_ERR_UNSUPPORTED, "sharding needs at least one context-free window");
  if (!op->d_shrank) {
    HIPCHK(dev_malloc(&op->d_shrank, op->shard_kg * 4));
    HIPCHK(dev_malloc(&op->d_shflag, op->shard_kg * 4));
  }
  if (!op->started) {
    rc = start_stream(op, ts0);
    if (rc) return rc;
  }
  int64_t tile = TILE_MIN;
  if (n > 0) {
    rc = enqueue_ingest(op, d_ts, d_val, (int64_t)n, &tile);
    if (rc) return rc;
  } else {
    HIPCHK(hipMemsetAsync(op->d_tilemax, 0xFF, 8, op->stream));
  }
  op->shard_tile = tile;
  op->shard_n = (int64_t)n;
  ShardArgs a = shard_args(op);
  a.ts = d_ts;
  a.n = (int64_t)n;
  a.xbuf = (int64_t*)d_xbuf;
  HIPCHK(launch_shard_export(a, op->stream));
  // the record is complete when the caller starts the all-gather -- unless the caller orders its collective's stream
  // after the op's stream itself (shard_async + scotty_stream_order)
  if (!op->shard_async) HIPCHK(hipStreamSynchronize(op->stream));
  return SCOTTY_OK;
}

static int shard_push_counted(scotty_op* op, const int64_t* d_ts, const void* d_val, size_t n, int64_t ts0,
                              int64_t n_before, int64_t n_total, bool timed, int64_t ts_before, int64_t ts_last,
                              void* d_xbuf) {
  if (!op || !d_xbuf || (n && (!d_ts || !d_val))) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (op->keyed) return fail(op, SCOTTY_ERR_UNSUPPORTED, "keyed operators shard by key: no exchange needed");
  if (((uintptr_t)d_ts & 15) || ((uintptr_t)d_val & 15))
    return fail(op, SCOTTY_ERR_ARG, "device buffers must be 16-byte aligned");
  int rc = decide_mode(op);
  if (rc) return rc;
  if (op->mode != 3) return scotty_shard_push(op, d_ts, d_val, n, ts0, d_xbuf);
  if (!timed && op->c->has_time_windows())
    return fail(op, SCOTTY_ERR_ARG, "count + time windows: use scotty_shard_push_timed (the batch's timestamp "
                                    "bounds decide the time edges)");
  rc = op->c->shard_push(d_ts, d_val, (int64_t)n, ts0, n_before, n_total, ts_before, ts_last, (int64_t*)d_xbuf);
  if (rc) return fail(op, rc, op->c->err);
  op->shard_count_total = n_total;
  return SCOTTY_OK;
}

int scotty_shard_bounds(scotty_op* op, const int64_t* d_ts, size_t n, int64_t* first_last) {
  if (!op || !first_last || (n && !d_ts)) return SCOTTY_ERR_ARG;
  first_last[0] = first_last[1] = INT64_MIN;
  if (n == 0) return SCOTTY_OK;
  HIPCHK(hipMemcpyAsync(first_last, d_ts, 8, hipMemcpyDeviceToHost, op->stream));
  HIPCHK(hipMemcpyAsync(first_last + 1, d_ts + n - 1, 8, hipMemcpyDeviceToHost, op->stream));
  HIPCHK(hipStreamSynchronize(op->stream));
  return SCOTTY_OK;
}

int scotty_shard_push_counted(scotty_op* op, const int64_t* d_ts, const void* d_val, size_t n, int64_t ts0,
                              int64_t n_before, int64_t n_total, void* d_xbuf) {
  return shard_push_counted(op, d_ts, d_val, n, ts0, n_before, n_total, false, INT64_MIN, INT64_MIN, d_xbuf);
}

int scotty_shard_push_timed(scotty_op* op, const int64_t* d_ts, const void* d_val, size_t n, int64_t ts0,
                            int64_t n_before, int64_t n_total, int64_t ts_before, int64_t ts_last, void* d_xbuf) {
  return shard_push_counted(op, d_ts, d_val, n, ts0, n_before, n_total, true, ts_before, ts_last, d_xbuf);
}

int scotty_shard_commit(scotty_op* op, const void* d_gathered, int world) {
  if (!op || !d_gathered || world < 1 || world > 64) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (op->mode == 3) {
    int rc = op->c->shard_commit((const int64_t*)d_gathered, world);
    if (rc) return fail(op, rc, op->c->err);
    op->x_pushed += (uint64_t)op->shard_count_total;  // replicated state: every rank counts the whole batch
    return SCOTTY_OK;
  }
  if (op->mode != 1 || !op->d_shrank) return fail(op, SCOTTY_ERR_STATE, "scotty_shard_push must come first");
  ShardArgs a = shard_args(op);
  a.gathered = (const int64_t*)d_gathered;
  a.world = world;
  HIPCHK(launch_shard_commit(a, op->stream));
  return SCOTTY_OK;
}

int64_t scotty_key_count(scotty_op* op) { return (op && op->x) ? op->x->key_count() : 0; }

int scotty_process_watermark(scotty_op* op, int64_t wm, scotty_windows* out) {
  if (!op) return SCOTTY_ERR_ARG;
  if (op->failed) return fail(op, SCOTTY_ERR_STATE, "operator failed earlier: " + op->err);
  if (op->mode == 2 || op->mode == 3) return exact_watermark(op, wm, out, true);
  if (op->keyed) {  // keyed op without any tuple yet: no per-key operators exist
    if (out) std::memset(out, 0, sizeof(*out));
    return SCOTTY_OK;
  }
  int rc;
  const uint64_t dropped_before = op->dropped;
  // WindowManager.processWatermark (S/WindowManager.java:41-80)
  if (op->last_watermark == -1) op->last_watermark = std::max((int64_t)0, jsub(wm, op->max_lateness));
  int64_t nw = 0, res_cap = 0;
  const unsigned char* res = nullptr;
  if (!op->started) {
    op->last_watermark = wm;
  } else {
    // lastWatermark is raised to the oldest slice's start (S/WindowManager.java:51-55)
    int64_t last_wm = op->last_watermark;
    if (last_wm < op->h_oldest) last_wm = op->h_oldest;
    int64_t cap = bound_triggers(op, last_wm, wm);  // row capacity; the device writes the true count
    if (cap < 0) cap = count_triggers(op, last_wm, wm);
    if (cap < 0) return fail(op, SCOTTY_ERR_NOMEM, "watermark triggers more than 2^31 windows");
    const WmLayout L(cap, (int)op->aggs.size());
    rc = alloc_blocks(op);
    if (!rc) rc = ensure_wm_out(op, L.total);
    if (!rc) rc = upload_wdefs(op);
    if (rc) return rc;
    const int64_t remove_from = jsub(jsub(wm, op->max_lateness), op->max_fixed_window_size);
    WmArgs wa{};
    wa.meta = op->d_meta;
    wa.s_tstart = op->d_tstart;
    wa.s_tlast = op->d_tlast;
    wa.s_cnt = op->d_scnt;
    for (int k = 0; k < NPART; k++) wa.s_part[k] = op->d_spart[k];
    wa.b_cnt = op->d_bcnt;
    for (int k = 0; k < NPART; k++) wa.b_part[k] = op->d_bpart[k];
    wa.p_cnt = op->d_pcnt;
    wa.p_sum = op->d_psum;
    wa.st_min = op->d_stmin;
    wa.st_max = op->d_stmax;
    wa.nbcap = op->nbcap;
    wa.wdef = op->d_wdef;
    wa.n_defs = (int32_t)op->windows.size();
    wa.last_wm = last_wm;
    wa.wm = wm;
    wa.remove_from = remove_from;
    wa.n_windows = cap;
    wa.out = op->d_out;
    wa.hout = (unsigned char*)op->h_out_dev;  // rows written straight into host-mapped memory: no publish copy
    wa.n_aggs = (int32_t)op->aggs.size();
    for (size_t k = 0; k < op->aggs.size(); k++) wa.agg_kind[k] = op->aggs[k];
    wa.need = op->need;
    wa.s_first = op->d_sfirst;
    wa.vt = op->vt;
    for (int attempt = 0; attempt < 2; attempt++) {
      // triggers + window assembly + GC (window_kernels.hip), then ONE transfer of the packed result
      scotty_op::TEv tw, tc;
      rc = tlaunch(op, tw, SCOTTY_TIME_WATERMARK);
      if (rc) return rc;
      HIPCHK(launch_wm(wa, op->stream, tw.a, tw.b));
      tlaunched(op, tw);
      if (!op->h_out_dev) {  // no host-mapped result buffer: one DMA transfer (class RESULT_COPY)
        rc = tbegin(op, tc, SCOTTY_TIME_RESULT_COPY);
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(op->h_out, op->d_out, L.total, hipMemcpyDeviceToHost, op->stream));
        rc = tend(op, tc);
        if (rc) return rc;
      }
      // the next micro-batch's cell index is built while the host handles this result
      if (!op->wm_ev) HIPCHK(hipEventCreateWithFlags(&op->wm_ev, hipEventDisableTiming));
      HIPCHK(hipEventRecord(op->wm_ev, op->stream));
      rc = enqueue_cix(op);
      if (rc) return rc;
      op->cix_ready = true;
      HIPCHK(hipEventSynchronize(op->wm_ev));
      std::memcpy(op->h_snap, op->h_out, sizeof(DevMeta));
      if (!op->h_snap->overflow) break;
      rc = replay_after_overflow(op);
      if (rc) {
        op->failed = true;
        return rc;
      }
    }
    if (op->h_snap->overflow) {
      op->failed = true;
      return fail(op, SCOTTY_ERR_UNSUPPORTED, "edge-grid horizon overflow");
    }
    std::memcpy(&nw, op->h_out + WM_HDR_N, 8);
    if (nw < 0 || nw > cap) {
      op->failed = true;
      return fail(op, SCOTTY_ERR_STATE, "internal: device triggered " + std::to_string(nw) + " windows, capacity " +
                                            std::to_string(cap));
    }
    res_cap = cap;
    res = op->h_out;
    op->last_watermark = wm;
    // bookkeeping at the synchronisation point
    const DevMeta& m = *op->h_snap;
    op->last_span = std::max<int64_t>(1, jsub(m.prev_max, op->h_prev_max));
    op->h_prev_max = m.prev_max;
    op->h_oldest = m.oldest_start;
    op->dropped = m.late_total;
    op->processed = m.processed_total;
    rc = maybe_extend_grid(op, false);
    if (rc) return rc;
    rc = compact_if_needed(op);
    if (rc) return rc;
  }
  // timing of the launches of this interval
  for (auto& e : op->ev_pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e.first, e.second) == hipSuccess) {
      op->t_ms += ms;
      op->t_cls_ms[SCOTTY_TIME_INGEST] += ms;
    }
    op->t_launches++;
    op->t_cls_n[SCOTTY_TIME_INGEST]++;
    op->ev_pool.push_back(e);
  }
  op->ev_pending.clear();
  tresolve(op);
  for (void* p : op->owned) (void)hipFree(p);
  op->owned.clear();
  op->ingest->reset();
  op->pending.clear();
  if (out) {
    // results: AggregateWindowState.getAggValues / hasValue (S/state/AggregateWindowState.java:41-49), lowered on
    // the device; the columns point into the pinned result buffer (valid until the next call on the op)
    std::memset(out, 0, sizeof(*out));
    out->n_windows = (size_t)nw;
    out->n_aggs = (int32_t)op->aggs.size();
    if (nw > 0) {
      const WmLayout L(res_cap, (int)op->aggs.size());  // columns are res_cap rows apart
      if ((int64_t)op->r_measure.size() < nw) op->r_measure.assign(nw, SCOTTY_MEASURE_TIME);
      out->start = (const int64_t*)(res + L.start);
      out->end = (const int64_t*)(res + L.end);
      out->measure = op->r_measure.data();
      out->has_value = (const uint8_t*)(res + L.has);
      for (size_t k = 0; k < op->aggs.size(); k++) out->values[k] = (const int64_t*)(res + L.vals + 8 * res_cap * k);
    }
  }
  if (op->dropped > dropped_before) {
    op->err = "tuples older than the oldest retained slice were dropped (reference: IndexOutOfBoundsException)";
    return SCOTTY_WARN_LATE_DROPPED;
  }
  return SCOTTY_OK;
}

uint64_t scotty_dropped_count(scotty_op* op) { return op ? op->dropped : 0; }
uint64_t scotty_processed_count(scotty_op* op) { return op ? op->processed : 0; }
int64_t scotty_slice_count(scotty_op* op) {
  if (!op) return 0;
  if (op->mode == 3) return op->c->slice_count();
  if (op->mode == 2) {
    if (op->keyed) return -1;
    int64_t c = 0;
    if (op->x->slice_count(0, &c)) return -1;
    return c;
  }
  if (!op->started) return 0;
  if (sync_snapshot(op)) return -1;
  return op->h_snap->tail - op->h_snap->head;
}

int64_t scotty_first_indices(scotty_op* op, int64_t* out, size_t cap) {
  if (!op || (cap && !out)) return SCOTTY_ERR_ARG;
  if (!op->first) return fail(op, SCOTTY_ERR_ARG, "no SCOTTY_AGG_FIRST aggregation registered");
  if (!op->started) return 0;
  if (sync_snapshot(op)) return SCOTTY_ERR_HIP;
  const DevMeta& m = *op->h_snap;
  const int64_t live = m.tail - m.head;
  if (live <= 0) return 0;
  std::vector<int64_t> v((size_t)live);
  HIPCHK(hipMemcpy(v.data(), op->d_sfirst + m.head, (size_t)live * 8, hipMemcpyDeviceToHost));
  std::vector<int64_t> f;
  for (int64_t x : v)
    if (x != FIRST_NONE) f.push_back(x);
  std::sort(f.begin(), f.end());
  f.erase(std::unique(f.begin(), f.end()), f.end());
  for (size_t i = 0; i < f.size() && i < cap; i++) out[i] = f[i];
  return (int64_t)f.size();
}

int scotty_enable_timing(scotty_op* op, int on) {
  if (!op) return SCOTTY_ERR_ARG;
  op->timing = on != 0;
  if (op->x) {  // exact engine: its own HIP-event classes (quiet ingest, other push work, watermark, result copy)
    op->x->timing = on != 0;
    for (int k = 0; k < 4; k++) {
      op->x->t_ms[k] = 0.0;
      op->x->t_cnt[k] = 0;
    }
    op->x->t_tuples = 0;
  }
  op->t_ms = 0.0;
  op->t_launches = 0;
  op->t_tuples = 0;
  for (int k = 0; k < NTCLS; k++) {
    op->t_cls_ms[k] = 0.0;
    op->t_cls_n[k] = 0;
  }
  return SCOTTY_OK;
}

int scotty_device_timing(scotty_op* op, int cls, double* total_ms, uint64_t* intervals) {
  if (!op || cls < 0 || cls >= NTCLS) return SCOTTY_ERR_ARG;
  if (op->mode == 2 && op->x) {
    (void)op->x->collect_timing();
    if (total_ms) *total_ms = op->x->t_ms[cls];
    if (intervals) *intervals = op->x->t_cnt[cls];
    return SCOTTY_OK;
  }
  if (total_ms) *total_ms = op->t_cls_ms[cls];
  if (intervals) *intervals = op->t_cls_n[cls];
  return SCOTTY_OK;
}

int scotty_ingest_timing(scotty_op* op, double* total_ms, uint64_t* launches, uint64_t* tuples) {
  if (!op) return SCOTTY_ERR_ARG;
  if (total_ms) *total_ms = op->t_ms;
  if (launches) *launches = op->t_launches;
  if (tuples) *tuples = op->t_tuples;
  return SCOTTY_OK;
}

// Tuning knobs (include/scotty_mi355x.h): capacities of the exact engine, grid ingest variant.
int scotty_tune(scotty_op* op, const char* key, int64_t value) {
  if (!op || !key) return SCOTTY_ERR_ARG;
  if (std::strcmp(key, "ingest_blocks") == 0) {
    if (value < 1 || value > (1 << 20)) return SCOTTY_ERR_ARG;
    op->ingest_blocks = value;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "ingest_stamps") == 0) {  // per-workgroup phase clock stamps of the ingest (debugging aid)
    op->stamps_on = value != 0;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "ingest_mode") == 0) {  // ingest loop (A/B only, launch_ingest): 7 pipelined without the DQ2
                                                // queue; int32 COUNT / SUM also 6 plain, 22 plain + DQ2, 23 the default
    if (value != -1 && value != 6 && value != 7 && value != 22 && value != 23) return SCOTTY_ERR_ARG;
    op->ingest_mode = (int)value;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "shard_cells") == 0 || std::strcmp(key, "shard_cands") == 0) {
    if (op->d_shrank || value < 16 || value > (1 << 22)) return SCOTTY_ERR_ARG;
    (key[6] == 'c' && key[7] == 'e' ? op->shard_kc : op->shard_kg) = value;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "exact_serial") == 0) {
    if (op->mode != 0) return SCOTTY_ERR_ARG;
    op->x_serial = value != 0;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "exact_quiet") == 0) {  // 0: non-keyed exact batches skip the one-pass quiet path (A/B)
    op->x_quiet_off = value == 0;
    if (op->x) op->x->quiet_off = op->x_quiet_off;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "quiet_band") == 0) {  // 1: quiet batches may move the session start (exact_quiet.h)
    op->x_band_on = value != 0;
    if (op->x) op->x->band_on = op->x_band_on;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "exact_prefix") == 0) {  // first event-exact piece of a refused quiet batch (tuples, >= 4096)
    if (value != 0 && (value < 4096 || value > ((int64_t)1 << 40))) return SCOTTY_ERR_ARG;
    op->x_prefix = value;
    if (op->x) op->x->xq_prefix = value;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "keyed_lane_count") == 0) {  // 0: keyed LazySlice record sets (count windows) through the
    if (op->mode != 0 || value < 0 || value > 1) return SCOTTY_ERR_ARG;  // wavefront replay (A/B); 1 lane per key (default)
    op->x_lc_off = value == 0;
    if (op->x) op->x->lane_count_off = op->x_lc_off;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "keyed_lane_session") == 0) {  // 0: keyed sessions through the wavefront replay (A/B),
    if (op->mode != 0 || value < 0 || value > 2) return SCOTTY_ERR_ARG;  // 1 lane kernel 2-waves build (default), 2 3-waves
    // (the store layout follows the kernel at the first push: the lane kernel's key-interleaved store cannot be
    // handed to the wavefront replay later)
    if (op->x && op->x->key_count() > 0 && (value == 0) != op->x_ls_off) return SCOTTY_ERR_STATE;
    op->x_ls_off = value == 0;
    op->x_ls_occ = value == 2 ? 3 : 2;
    if (op->x) {
      op->x->lane_session_off = op->x_ls_off;
      op->x->lane_session_occ = op->x_ls_occ;
    }
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "keyed_sort_digit10") == 0) {  // keyed replay sort: 10-bit digits for 17-20-bit keys (A/B)
    if (value < -1 || value > 2) return fail(op, SCOTTY_ERR_ARG, "keyed_sort_digit10 is -1, 0, 1 or 2");
    op->x_digit10 = (int)value;
    if (op->x) op->x->sort_digit10 = op->x_digit10;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "keyed_pack_records") == 0) {  // 1 (default): the lane-session replay sorts packed 8-byte
    if (op->mode != 0 || value < 0 || value > 1) return SCOTTY_ERR_ARG;  // records when a batch fits; 0: 16-byte (A/B)
    op->x_pack_off = value == 0;
    if (op->x) op->x->pack_off = op->x_pack_off;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "lane_session_counters") == 0) {  // debugging aid: count the lane-session kernel's paths
    if (op->mode != 0 || value < 0 || value > 1) return SCOTTY_ERR_ARG;  // (debug stats 103-106)
    op->x_lsdbg = value != 0;
    if (op->x) op->x->lsdbg_on = op->x_lsdbg;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "quiet_ingest_mode") == 0) {  // exact engine's quiet pass: -1 default loop, 7 without DQ2 (A/B)
    if (value != -1 && value != 7) return SCOTTY_ERR_ARG;
    op->x_qmode = (int32_t)value;
    if (op->x) op->x->xq_ingest_mode = op->x_qmode;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "quiet_ingest_blocks") == 0) {  // exact engine's quiet pass: ingest workgroups (A/B, 0 default)
    if (value < 0 || value > 65536) return SCOTTY_ERR_ARG;
    op->x_qblocks = value;
    if (op->x) op->x->xq_ingest_blocks = value;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "shard_count_cells") == 0) {  // cells per rank record of the count path's exchange
    if (op->mode != 0 || value < 16 || value > (1 << 24)) return SCOTTY_ERR_ARG;
    op->count_shard_cap = value;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "count_path") == 0) {  // 1: in-order stream promised -> count path (no LazySlice records)
    if (op->mode != 0) return SCOTTY_ERR_ARG;
    op->x_count_on = value != 0;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "keyed_grid") == 0) {  // 0: keyed batches always sorted + replayed (no sort-free path)
    if (op->mode != 0) return SCOTTY_ERR_ARG;
    op->x_kg_off = value == 0;
    if (op->x) op->x->kg_off = op->x_kg_off;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "count_prefix_one") == 0) {  // 0: the count watermark's prefix sums by three kernels (tests)
    if (value < 0 || value > 1) return SCOTTY_ERR_ARG;
    op->c_prefix_one = value != 0;
    if (op->c) op->c->prefix_one = op->c_prefix_one;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "shard_async") == 0) {  // shard pushes without a host sync (the caller orders its streams)
    if (value < 0 || value > 1) return SCOTTY_ERR_ARG;
    op->shard_async = value != 0;
    if (op->c) op->c->shard_async = op->shard_async;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "keyed_grid_variant") == 0) {  // sort-free path kernel variant (A/B only: 0 baseline, 1 default)
    if (op->mode != 0 || value < 0 || value > 1) return SCOTTY_ERR_ARG;
    op->x_kg_variant = (int32_t)value;
    if (op->x) op->x->kg_variant = op->x_kg_variant;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "keyed_grid_chunk") == 0) {  // min average tuples per chunk of a many-cell batch
    if (op->mode != 0 || value < 0) return SCOTTY_ERR_ARG;
    op->x_kg_chunk = value;
    if (op->x) op->x->kg_min_chunk = value;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "keyed_lane") == 0) {  // 0: wavefront-per-key replay even where the lane path applies
    if (op->mode != 0) return SCOTTY_ERR_ARG;
    if (op->x && op->x->layout_fixed() && value == 0) return SCOTTY_ERR_ARG;  // the record store needs the lane path
    op->x_lane_off = value == 0;
    if (op->x) op->x->lane_off = op->x_lane_off;
    return SCOTTY_OK;
  }
  if (std::strcmp(key, "slice_capacity") == 0 || std::strcmp(key, "session_capacity") == 0) {
    if (op->mode != 0 || value <= 0 || value > (1 << 26)) return SCOTTY_ERR_ARG;
    (key[1] == 'l' ? op->x_sc : op->x_sess) = (int32_t)value;
    return SCOTTY_OK;
  }
  return SCOTTY_ERR_ARG;
}

// Internal (not in the header): allocations made from now on are filled with `byte` (0..255), or left as allocated
// (exact engine: zero-filled) for byte < 0.  Returns the previous setting.  Tests of never-written reads only.
int scotty_debug_alloc_poison(int byte) {
  return scotty::g_alloc_poison.exchange(byte < 0 ? -1 : (byte & 0xFF));
}

// Internal (not in the header): grid-path statistics (0: tuples added with global atomics since creation).
int64_t scotty_debug_grid_stat(scotty_op* op, int which) {
  if (!op || op->mode != 1 || !op->d_meta) return -1;
  DevMeta m;
  if (hipMemcpy(&m, op->d_meta, sizeof(DevMeta), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (which == 0) return (int64_t)m.glb_slow;
  if (which >= 1 && which <= 5 && op->d_cixmeta) {  // cell index: base, shift, buckets, full, span end
    int64_t cm[8];
    if (hipMemcpy(cm, op->d_cixmeta, sizeof(cm), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return cm[which - 1];
  }
  if (which == 6) return m.tail - m.head;
  if (which == 7) return m.gcount - m.j0;
  if (which == 8) return m.prev_max;
  if (which == 9) return op->last_ingest_blocks;
  if (which == 10) return op->last_ingest_streaming;
  if (which == 11) return (int64_t)op->h_snap->slow_last;
  return -1;
}

// Internal (not in the header): the last grid ingest's phase stamps (s_memtime ticks), [workgroups][4]: start, LDS
// window ready, every wave's range done, window flushed to the cells.  Returns the workgroups copied.
// The last commit's phase stamps (8: start, prefix maxima, candidates, edge decision, ambiguous scans, ranks and
// appends, fold, before the meta write), in the same buffer's last 16 words.
int64_t scotty_debug_commit_stamps(scotty_op* op, long long* out) {
  if (!op || !op->d_stamps) return -1;
  if (hipMemcpy(out, op->d_stamps + 8192 * 4 - 16, 8 * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return 7;
}
int64_t scotty_debug_ingest_stamps(scotty_op* op, long long* out, int64_t max_blocks) {
  if (!op || !op->d_stamps) return -1;
  const int64_t nb = std::min<int64_t>(std::min<int64_t>(op->last_ingest_blocks, 8192), max_blocks);
  if (hipMemcpy(out, op->d_stamps, nb * 4 * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return nb;
}

// Internal (not in the header): statistics of the last push of the exact engine (0 events, 1 rounds; keyed:
// 2 path of the last push (0 replay, 1 sort-free, 2 sort-free + replay of deferred keys), 3 deferred tuples,
// 4 keys committed on the sort-free path).
// Internal (not in the header): the rocprofv3 name of the calling thread's last launch of kernel class `which`
// (KN_* in device_common.h), "" if none -- the bench ties PMC traffic files to the kernel they measured.
const char* scotty_debug_kernel_name(int which) {
  return (which >= 0 && which < KN_N) ? g_kernel_name[which] : "";
}

int64_t scotty_debug_stat(scotty_op* op, int which) {
  if (!op) return -1;
  if (which == 5) return op->mode;  // 1 grid path, 2 exact engine, 3 count path
  if (which == 6) return op->c ? op->c->last_nte : -1;
  if (which == 7) return op->c ? (int64_t)op->c->last_te_us : -1;
  if (!op->x) return -1;
  switch (which) {
    case 0: return op->x->last_events;
    case 1: return op->x->last_segments;
    case 2: return op->x->last_kg;
    case 3: return op->x->last_kg_deferred;
    case 4: return op->x->last_kg_keys;
    case 8: return op->x->last_quiet;       // XQ_* verdict of the last non-keyed push (exact_quiet.h)
    case 9: return op->x->quiet_commits;
    case 10: return op->x->quiet_fallbacks;
    case 11: return op->x->last_quiet_why;
    case 12: return op->x->quiet_tail_commits;  // batches whose remainder committed after an event-exact prefix
    case 13: return op->x->quiet_split_commits;  // quiet prefixes committed up to a located session-gap jump
    case 14: return op->x->quiet_skipped;        // batches sent to the event-exact path by the quiet back-off
    case 15: return (int64_t)op->x->xq_trace.size();  // quiet attempts of the last batch; 16 + k: attempt k's trace
    case 100: return op->x->quiet_band_moves;   // committed quiet batches that moved a session start (start band)
    case 101: return op->x->quiet_jump_pieces;  // event-exact pieces cut right behind a located session-gap jump
    case 102: return op->x->quiet_band_noedge;  // of the band moves: sessions opened without a slice edge (start only)
    case 103: case 104: case 105: case 106: {  // lane-session path counters (tune "lane_session_counters"): general,
      unsigned long long v = 0;                // fast in-order, fast late (registers), fast late (memory) tuples
      if (op->x->d_lsdbg && hipMemcpy(&v, op->x->d_lsdbg + (which - 103), 8, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
      return (int64_t)v;
    }
    case 107: return op->x->last_rec_bytes;
    case 110: case 111: case 112: case 113: case 114: case 115: case 116: case 117: case 118: case 119: {
      // lane-session general-path tuples by the reason they left the fast path (keyed_lane_session.hip `why`)
      unsigned long long v = 0;
      if (op->x->d_lsdbg && hipMemcpy(&v, op->x->d_lsdbg + 4 + (which - 110), 8, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
      return (int64_t)v;
    }  // the last keyed replay's record bytes (8 packed, 16, 24)
    default:
      if (which >= 16 && which - 16 < (int)op->x->xq_trace.size()) return op->x->xq_trace[which - 16];
      return -1;
  }
}

// Internal (not in the header): state of one operator of the exact engine, for tests and debugging.
int64_t scotty_debug_dump(scotty_op* op, int64_t key_slot, int64_t* out, int64_t cap) {
  if (!op || !op->x) return SCOTTY_ERR_STATE;
  std::vector<int64_t> v;
  int rc = op->x->debug_dump(key_slot, v);
  if (rc) return rc;
  for (int64_t i = 0; i < (int64_t)v.size() && i < cap; i++) out[i] = v[i];
  return (int64_t)v.size();
}

int scotty_sync(scotty_op* op) {
  if (!op) return SCOTTY_ERR_ARG;
  HIPCHK(hipStreamSynchronize(op->stream));
  return SCOTTY_OK;
}

int scotty_stream_order(scotty_op* op, void* stream, int op_waits) {
  if (!op) return SCOTTY_ERR_ARG;
  if (!op->order_ev) HIPCHK(hipEventCreateWithFlags(&op->order_ev, hipEventDisableTiming));
  hipStream_t ext = (hipStream_t)stream;
  if (op_waits) {
    HIPCHK(hipEventRecord(op->order_ev, ext));
    HIPCHK(hipStreamWaitEvent(op->stream, op->order_ev, 0));
  } else {
    HIPCHK(hipEventRecord(op->order_ev, op->stream));
    HIPCHK(hipStreamWaitEvent(ext, op->order_ev, 0));
  }
  return SCOTTY_OK;
}

void* scotty_op_stream(scotty_op* op) { return op ? (void*)op->stream : nullptr; }

}  // extern "C"
