// exact_common.h -- data layout of the exact ("replay") engine, shared by host and gfx950 kernels.
//
// The exact engine runs the reference operator's per-tuple state machine (S/StreamSlicer.java:36-141,
// S/SliceManager.java:27-192, C/windowType/SessionWindow.java:40-116) for MANY operators at once: one
// wavefront owns one operator (one key of a keyed stream, or the single operator of a non-keyed stream)
// and walks that operator's micro-batch in arrival order, 64 tuples at a time.  Tuples whose effect
// commutes (no slice edge, no session modification) are reduced cooperatively per slice; the rare tuples
// that change structure ("events") are executed exactly, wave-uniformly.  It serves every configuration
// the grid path (slicing_kernels.hip) does not: session windows, count windows and keyed operators.
//
// HBM layout (SoA, operator-major):
//   XState   [n_ops]            StreamSlicer / WindowManager scalars of each operator
//   slices   [n_ops * sc]       tStart tEnd tLast tFirst cStart cLast (i64), type (i32), cnt + 3 partials
//   sessions [n_ops * nctx * sesscap]  active sessions (start, end) of each SessionContext
//   cfg                         windows + functions shared by all operators (same for every key, as the
//                               Flink connector builds every per-key operator identically,
//                               flink-connector/.../KeyedScottyWindowOperator.java:41-49)
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "device_common.h"

namespace scotty {

// Key table entries (keyed_kernels.hip, keyed_grid.hip): key << 32 | 1 << 31 | slot; 0 = empty.  The occupied bit
// keeps every uint32 key representable (a (key + 1) << 32 tag wrapped key 0xFFFFFFFF to the empty tag); slot field
// 0x7FFFFFFF = inserted in this batch, slot not yet assigned (the entry's low word is then 0xFFFFFFFF).
constexpr uint32_t KTAB_PENDING = 0xFFFFFFFFu;  // low word of a pending entry / a tuple's unassigned slot
__host__ __device__ inline unsigned long long ktab_tag(uint32_t key) {
  return ((unsigned long long)key << 32) | 0x80000000ull;
}
__host__ __device__ inline bool ktab_is(unsigned long long e, uint32_t key) {
  return (e & 0xFFFFFFFF80000000ull) == ktab_tag(key);
}
__host__ __device__ inline uint32_t ktab_key(unsigned long long e) { return (uint32_t)(e >> 32); }
// slot of an entry (KTAB_PENDING for a pending one)
__host__ __device__ inline uint32_t ktab_slot(unsigned long long e) {
  const uint32_t w = (uint32_t)e;
  return w == KTAB_PENDING ? KTAB_PENDING : (w & 0x7FFFFFFFu);
}

constexpr int XMAXCTX = 4;        // session windows per operator
constexpr int XMAXMODS = 8;       // WindowModifications produced by one updateContext call (<= 4 in practice)
constexpr int SCOTTY_MAX_AGGS_ = 8;  // == SCOTTY_MAX_AGGS

// Slice.Type (S/slice/Slice.java:86-121): Fixed, or Flexible(counter).  Stored in an int32:
// XTYPE_FIXED, or the flexible counter; bit 30 marks a LazySlice (SliceFactory.createSlice, :17-22).
constexpr int32_t XTYPE_FIXED = (int32_t)0x80000000;
constexpr int32_t XTYPE_LAZY = 0x40000000;

// exception codes of the reference, recorded per operator
enum : int32_t {
  XERR_NONE = 0,
  XERR_INDEX = 1,        // IndexOutOfBoundsException (tuple dropped; counted)
  XERR_UNSUPPORTED = 2,  // LazySlice record movement (not on the MI355X path yet) -- fatal
  XERR_SLICE_CAP = 3,    // per-operator slice capacity exceeded -- fatal
  XERR_SESS_CAP = 4,     // per-context session capacity exceeded -- fatal
  XERR_HANG = 5,         // reference would loop forever in StreamSlicer (power-of-two size/slide) -- fatal
  XERR_WM_INDEX = 6,     // processWatermark threw (empty session context / count trigger) -- fatal for the call
  XERR_NPE = 7,          // NullPointerException: a LazySlice ran out of records while records move (tuple failed,
                         // counted; the state keeps the reference's partial changes)
  XERR_NOELEM = 8,       // NoSuchElementException (TreeSet.first() on an emptied record set; same handling)
  XERR_REC_CAP = 9,      // per-operator record capacity exceeded (internal; the pre-check prevents it) -- fatal
};
// a tuple whose processing threw one of these is counted as failed, like the reference's per-tuple exception
__host__ __device__ inline bool xerr_tuple_failed(int32_t e) { return e == XERR_INDEX || e == XERR_NPE || e == XERR_NOELEM; }

struct XCfg {
  int32_t n_cf;           // context-free windows (registration order)
  int32_t n_ctx;          // context-aware (session) windows (registration order)
  int32_t has_fixed, has_ctx, has_count, has_time, session_case, lazy;
  // LazySlice record sets (S/slice/LazySlice.java:14-54, ST/memory/MemorySetState.java): kept when slices are Lazy;
  // invertible: every function is an InvertibleAggregateFunction (removal = liftAndInvert), else recompute()
  int32_t records, invertible;
  int64_t rcap;           // records per operator (arena capacity)
  int32_t need, vt;
  int32_t sc;             // slice capacity per operator
  int32_t sesscap;        // session capacity per context per operator
  int32_t ctx_alloc;      // session contexts allocated per operator (>= n_ctx)
  int64_t max_lateness, max_fixed;
  int64_t gap[XMAXCTX];
  int32_t ctx_measure[XMAXCTX];
  int32_t n_aggs;
  int32_t agg_kind[SCOTTY_MAX_AGGS_];   // SCOTTY_AGG_* of include/scotty_mi355x.h, registration order
  // context-free windows, SoA [n_cf]
  const int32_t* cf_kind;
  const int32_t* cf_measure;
  const int64_t* cf_a;
  const int64_t* cf_b;
};

struct XState {          // 128 B
  int64_t maxEventTime, nextEdgeTs, nextEdgeCount, currentCount;   // S/StreamSlicer.java:10-14, WindowManager
  int64_t lastWatermark, lastCount;                                 // S/WindowManager.java:18-33
  int32_t head, tail;                                               // retained slices [head, tail) of the op
  int32_t started, unsorted;                                        // store non-empty; tStart order broken
  int32_t err, key;                                                 // fatal error; key of this op
  int32_t nsess[XMAXCTX];
  // context c's session count through constant indices only: a runtime index into nsess keeps the whole XState of
  // a kernel in scratch memory (every field access then a scratch round trip)
  __host__ __device__ int32_t ns(int c) const {
    return c == 0 ? nsess[0] : c == 1 ? nsess[1] : c == 2 ? nsess[2] : nsess[3];
  }
  __host__ __device__ void set_ns(int c, int32_t v) {
    if (c == 0) nsess[0] = v;
    else if (c == 1) nsess[1] = v;
    else if (c == 2) nsess[2] = v;
    else nsess[3] = v;
  }
  uint64_t dropped;                                                 // tuples whose processing threw
  int64_t wlo, whi;                                                 // watermark: slice scan range
  int32_t pending;                                                  // batch deferred: capacity too small
  int32_t pvalid;                                                   // lane path: slice prefixes valid below this
  int64_t rend;                                                     // records: end of the live arena range
};

struct XSlices {
  int64_t *ts, *te, *tl, *tf, *cs, *cl;
  int32_t* ty;
  unsigned long long* cnt;
  unsigned long long* p[NPART];
  // records mode (XCfg.records): slice s owns arena records [rlo[s], rhi[s]) of its op (rhi[s] == rlo[s+1]: the
  // slices' record sets lie in slice order, each sorted by ts, no duplicate ts -- the TreeSet<StreamRecord>
  // ordered by ts only, S/slice/StreamRecord.java:25-27); nn[s]: the partial is non-null (AggregateValueState
  // keeps a value after liftAndInvert even at count 0)
  int64_t *rlo, *rhi;
  int32_t* nn;
  int64_t *rts, *rv;      // arena [n_ops * rcap]: record ts, value bits
  // lane path (keyed_lane.hip, keyed_grid.hip): running prefixes of cnt and of the wrapping integer sum over the
  // op's slice positions 0..i (positions below head keep their values until a compaction), valid for positions
  // below XState.pvalid -- a window's COUNT / SUM is then two reads instead of a scan of its slices
  unsigned long long *pc, *ps;
  // lane path for COUNT / integer SUM functions: the store kept key-interleaved instead (XKView, the columns above
  // unused): word (op, slice position i, field f) at kw[((i * kw_nf + f) << kc_sh) + op], so the lanes of a
  // wavefront -- consecutive keys -- touching the same field of the same slice position read or write one
  // contiguous 512-B run instead of 64 scattered lines.  Keys advance in lockstep in a steady stream (one slice per
  // grid interval each, compacted at the same batch), so their positions coincide.  sc and the key capacity are
  // powers of two (sc_sh, kc_sh their logs).
  unsigned long long* kw;
  int32_t sc_sh, kc_sh;
  int32_t kw_nf;  // fields per position: XK_NF with MIN / MAX functions (their block summaries), else XK_NF_SUM
};

// Fields of the key-interleaved store (XSlices.kw), one 8-byte word each (ty in the low half of its word).
// MIN / MAX window assembly (keyed_lane.hip, lane_wm_emit_kernel) keeps block summaries of p[1] / p[2] over blocks of
// XK_MB consecutive slice positions: QN / QX the min / max from the block's first position up to this one (valid below
// XState.pvalid, like PC / PS), SN / SX from this position to the block's end (kept for complete blocks only: the
// emit kernel recomputes them for every complete block that holds a position at or above pvalid) -- a window of
// positions [lo, hi) then reads SN[lo], QN at the end of each whole block and QN[hi - 1], not each of its slices.
// Operators without MIN / MAX keep only the first XK_NF_SUM fields per position (the summaries are last).
enum : int {
  XK_TS, XK_TE, XK_TL, XK_TF, XK_CS, XK_CL, XK_CNT, XK_P0, XK_P1, XK_P2, XK_PC, XK_PS, XK_TY,
  XK_NF_SUM,
  XK_QN = XK_NF_SUM, XK_SN, XK_QX, XK_SX, XK_NF
};
constexpr int XK_MB = 16;  // slice positions per MIN / MAX summary block

// Column views of the key-interleaved store with the syntax of XSlices' columns (q.ts[j], q.p[k][j], q.ts + base
// with j = op * sc + i), so one kernel body serves both layouts (template parameter V = XSlices or XKView).
struct XKCol0 {
  unsigned long long* w;
  int64_t off;
  int32_t sc_sh, kc_sh;
  int32_t f, nf;
  __host__ __device__ unsigned long long* addr(int64_t j) const {
    j += off;
    const int64_t op = j >> sc_sh, i = j & ((((int64_t)1) << sc_sh) - 1);
    return w + (((i * nf + f) << kc_sh) + op);
  }
};
template <typename T>
struct XKCol : XKCol0 {
  __host__ __device__ T& operator[](int64_t j) const { return *(T*)addr(j); }
  __host__ __device__ XKCol operator+(int64_t j) const {
    XKCol c = *this;
    c.off += j;
    return c;
  }
};
struct XKParts {
  XKCol0 c;
  __host__ __device__ XKCol<unsigned long long> operator[](int k) const {
    XKCol<unsigned long long> r;
    static_cast<XKCol0&>(r) = c;
    r.f = XK_P0 + k;
    return r;
  }
};
struct XKView {
  XKCol<int64_t> ts, te, tl, tf, cs, cl;
  XKCol<unsigned long long> cnt;
  XKParts p;
  XKCol<unsigned long long> pc, ps;
  XKCol<int64_t> qn, sn, qx, sx;  // MIN / MAX block summaries (XK_QN ...)
  XKCol<int32_t> ty;
  __host__ __device__ XKView() {}
  __host__ __device__ explicit XKView(const XSlices& s) {
    XKCol0 b{s.kw, 0, s.sc_sh, s.kc_sh, 0, s.kw_nf};
    auto col = [&](auto& c, int f) {
      static_cast<XKCol0&>(c) = b;
      c.f = f;
    };
    col(ts, XK_TS); col(te, XK_TE); col(tl, XK_TL); col(tf, XK_TF); col(cs, XK_CS); col(cl, XK_CL);
    col(cnt, XK_CNT); col(pc, XK_PC); col(ps, XK_PS); col(ty, XK_TY);
    col(qn, XK_QN); col(sn, XK_SN); col(qx, XK_QX); col(sx, XK_SX);
    p.c = b;
  }
};
template <typename V>
__host__ __device__ inline V xview(const XSlices& s);
template <>
__host__ __device__ inline XSlices xview<XSlices>(const XSlices& s) { return s; }
template <>
__host__ __device__ inline XKView xview<XKView>(const XSlices& s) { return XKView(s); }

struct XSess {
  int64_t *start, *end;
};

// one micro-batch, arrival ordered; ops[] lists the operators that have tuples, seg[op] = [begin, end)
struct XBatchArgs {
  const int64_t* ts;
  const void* val;
  const int32_t* op_of;     // nullable: operator of each sorted tuple (keyed) -- unused by the replay itself
  const int64_t* seg_begin; // [n_ops] (null: the single operator owns [0, n))
  const int64_t* seg_end;
  int64_t n;
  int32_t n_ops;
  const XCfg* cfg;
  XState* st;
  XSlices sl;
  XSess ss;
  int32_t rec_stride;       // keyed: tuples are AoS records (ts at +0, value at +8, op at +rec_stride-4)
  int32_t retry;            // process only ops marked pending by an earlier launch
  unsigned long long* need; // [3] capacity pre-check: max slices / sessions / records an op may need (atomicMax)
  // nullable: the batch's largest timestamp, biased (ts ^ 1 << 63, an unsigned order) -- seg_kernel's by-product; the
  // lane-session kernel bounds a started key's capacity need with it before it reads the key's tuples
  const unsigned long long* ts_max_b;
  // rec_stride 8 (lane-session replay of an int32 batch only): packed records {key << pk_bits | ts - pk_base, value}
  int64_t pk_base;
  int32_t pk_bits;
  unsigned long long* dbg;  // nullable: lane-session path counters (general / fast in-order / fast late in registers /
                            // fast late in memory tuples), debugging aid
};

// Block summaries of one operator's slices for the watermark (exact_kernels.hip, wm_blocks_kernel): block b covers
// slice positions [XB_BLK * b, XB_BLK * (b + 1)); a block not wholly inside the scan range [wlo, whi) gets ts_min =
// INT64_MIN, so no window takes it whole
constexpr int XB_BLK = 64;
struct XBlocks {
  unsigned long long *cnt, *sum;   // COUNT; wrapping integer sum or f64 sum bits
  long long *mn, *mx;              // MIN / MAX partials (order-preserving keys for f64)
  long long *ts_min, *tl_max;      // smallest tStart / largest tLast of the block (whole-block containment test)
  int64_t nbcap;
};

struct XWmArgs {
  unsigned long long* zero4;  // single mode: the 4 control words the emit kernel zeroes first (no host memset launch)
  const XCfg* cfg;
  XState* st;
  XSlices sl;
  XSess ss;
  int32_t n_ops;
  int64_t wm;
  // pass 1 output: windows per op; pass 2 input: exclusive offsets
  int64_t* wcount;
  const int64_t* woff;
  // pass 2 outputs (rows)
  int64_t* w_start;
  int64_t* w_end;
  int32_t* w_meas;
  int32_t* w_op;
  int32_t* err_flag;
  unsigned long long* dropped_total;   // count pass: sum of XState.dropped
  int32_t* op_err;                     // count pass: OR of (1 << XState.err)
  // pass 3 outputs: lowered values (AggregateWindowState.getAggValues, S/state/AggregateWindowState.java:41-49)
  uint8_t* has_value;
  int64_t* values[SCOTTY_MAX_AGGS_];
  uint32_t* w_key;                      // key of the row's op (keyed)
  const uint32_t* slot_key;            // nullable
  int64_t n_rows;
  int32_t prefix_reset;                // lane path: recompute every op's slice prefixes from position 0
  unsigned long long* row_count;       // lane path / single mode: rows written by the emit kernel (n_rows = capacity)
  int32_t single;                      // one operator: wm_emit_kernel counts, checks and emits (no count pass)
  // one operator, Eager slices: 64-slice block summaries over the scan range [wlo, whi) (wm_blocks_kernel), read by
  // wm_agg_kernel for the blocks a window contains whole; null: every window scans its slices
  XBlocks blk;
};

}  // namespace scotty
