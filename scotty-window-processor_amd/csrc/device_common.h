// device_common.h -- data layout shared by the host engine and the gfx950 kernels.
//
// HBM layout of one operator (all SoA, 64-bit words):
//   slices   [SCAP]  t_start, t_last, cnt(u64), part[3] (sum | min | max)   -- LazyAggregateStore's SliceList
//   grid     [GCAP]  sorted union edge grid of the context-free time windows  -- StreamSlicer's edge function
//   cells    [CCAP]  per-micro-batch partials: old slices ++ grid cells        -- refined slices of one batch
//   tilemax  [TCAP]  max ts of each 4096-tuple arrival tile                    -- edge first-crossing lookups
//   meta             DevMeta (device-resident slicer / store scalars)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace scotty {

constexpr int TILE_MIN = 4096;    // tuples per arrival-order tile (tilemax granularity), power of two
constexpr int NT_MAX = 8192;      // tiles per micro-batch held in the commit kernel's LDS
constexpr int WCAP = 1024;        // cells in a workgroup's LDS window
constexpr int64_t CIX_CAP = 1 << 20;  // entries of the cell index (ts bucket -> first cell), see cix_build_kernel
constexpr int LCIX = 2048;        // cell-index entries staged in LDS for a workgroup's window
constexpr int NPART = 3;          // partial slots per slice/cell: 0 sum, 1 min, 2 max
constexpr int ING_SC = 24;        // block scalars of the ingest kernel (int64)
constexpr int DEFER_CAP = 320;    // per-wave deferred out-of-order queue of the ingest kernel (entries)

enum : int { VT_I32 = 0, VT_I64 = 1, VT_F64 = 2 };
// launch_ingest's mode for a stream whose last push was in order (DevMeta.slow_last): the software-pipelined loop on
// fewer, longer waves (r04f A/B on C2: 279 -> 264 us per 2^27 tuples; an out-of-order stream wants the default)
constexpr int INGEST_STREAMING = -2;
// workgroups of the streaming launch (C2, same-box sweeps: 416-480 -> 0.257-0.261 ms, 512 -> 0.267, 1024 -> 0.285;
// profiles/r05/ab_c2_blocks.json)
constexpr int INGEST_STREAMING_WGS = 448;
// workgroups of the int32 COUNT / SUM launch for out-of-order streams (C2s with the DQ2 queue: 704-896 -> 0.305-0.309
// ms, 1024 -> 0.342; profiles/r05/ab_c2s_dq2_blocks.json)
constexpr int INGEST_OOO_I32_WGS = 768;
enum : int { NEED_SUM = 1, NEED_MIN = 2, NEED_MAX = 4 };
constexpr int64_t FIRST_NONE = INT64_MAX;  // identity of a FIRST partial (no tuple yet)

// The rocprofv3 name of the last launch of a measured kernel class on this thread ("ingest_kernel<0, 1, 23>", as the
// profiler prints the template instance), so the bench can tie a PMC traffic file to the kernel it measured
// (scotty_debug_kernel_name).  Defined in scotty_engine.cpp.
enum : int {
  KN_INGEST = 0, KN_KG_HIST = 1, KN_KG_SCATTER = 2, KN_KG_BUCKET = 3, KN_COUNT_INGEST = 4, KN_LANE_SESSION = 5,
  KN_REPLAY = 6, KN_N = 7
};
void note_kernel(int which, const char* fmt, int a = 0, int b = 0, int c = 0, int d = 0);

// Device-resident scalars.  The StreamSlicer state (maxEventTime, min_next_edge_ts) lives here so
// consecutive micro-batches need no host round trip (S/StreamSlicer.java:10-14).
struct DevMeta {
  int64_t head, tail;        // retained slices are [head, tail) of the slice arrays
  int64_t prev_max;          // StreamSlicer.maxEventTime
  int64_t j0;                // grid index of min_next_edge_ts (the pending edge N)
  int64_t gcount;            // valid grid entries
  int64_t batch_max;         // scratch: max ts of the last push (valid also on overflow)
  int64_t n_emitted;         // edges appended by the last push
  int64_t overflow;          // != 0: a push exceeded the grid horizon / slice capacity; nothing committed
  int64_t failed_push;       // push sequence number that overflowed
  int64_t push_seq;          // pushes committed or attempted since creation
  int64_t oldest_start;      // t_start[head] after the last GC (host mirror)
  uint64_t late_push, overflow_push;   // per-push counters (reset by the commit kernel)
  uint64_t late_total, processed_total;
  uint64_t glb_slow;          // statistics: tuples the ingest kernel added with global atomics (outside the LDS window)
  int64_t cmin;               // lowest cell index the current push's ingest added to (commit folds from there)
  int64_t dirty_from;         // lowest slice index whose partials changed since the last watermark (block summaries)
  int64_t whead;              // head before the last watermark's GC (window assembly reads [whead, tail))
  uint64_t slow_push;         // tuples of the current push outside their wave's current cell (ingest slow path)
  uint64_t slow_last, n_last; // the last committed push's slow-path tuples and size (the host picks the next launch)
  int64_t view_s0_on;         // != 0: cell 0 of the ingest's view starts at view_s0 instead of t_start[head] (the exact
  int64_t view_s0;            //   engine's start band, exact_quiet.h; the slice store itself is not written before a verdict)
};

struct IngestArgs {
  const int64_t* ts;
  const void* val;
  int64_t n;
  // slices (read-only here)
  const int64_t* s_tstart;
  // grid
  const int64_t* grid;
  // cells (atomically accumulated)
  unsigned long long* c_cnt;
  long long* c_tmax;
  unsigned long long* c_part[NPART];
  // tile maxima; tile minima (nullable: only the exact engine's quiet path asks for them -- launch_ingest then runs
  // the MODE bit-3 instantiation)
  long long* tilemax;
  long long* tilemin;
  DevMeta* meta;
  int64_t per_wave;          // tuples per wave (multiple of tile)
  int64_t tile;              // tuples per tile (power of two >= TILE_MIN, nT <= NT_MAX)
  // cell index (built per push by cix_build_kernel): cix[k] = cell of ts cix_meta[0] + (k << cix_meta[1])
  uint32_t* cix;
  int64_t* cix_meta;         // [base, shift, n, cells indexed, ts end of the indexed range]
  int64_t cix_margin;        // ms past the stream front (prev_max) the index covers
  long long* stamps;         // nullable: per-workgroup clock stamps [blocks][4] (debugging aid, "ingest_stamps")
  long long* c_first;        // SCOTTY_AGG_FIRST (first_kernel): per cell, the arrival index of its first tuple
  int64_t seq_base;          //   arrival index of ts[0]
};

struct CommitArgs {
  const int64_t* ts;
  int64_t n;
  int64_t tile;
  int64_t max_lateness;
  int64_t scap;              // slice capacity
  const int64_t* grid;
  long long* tilemax;
  long long* pmax;           // scratch [TCAP]
  int32_t* rank;             // scratch [GCAP]
  int32_t* flag;             // scratch [GCAP]
  int64_t* s_tstart;
  int64_t* s_tlast;
  unsigned long long* s_cnt;
  unsigned long long* s_part[NPART];
  unsigned long long* c_cnt;
  long long* c_tmax;
  unsigned long long* c_part[NPART];
  DevMeta* meta;
  int need;
  int vt;
  int64_t push_seq;
  long long* stamps;         // nullable: phase clock stamps (scotty_tune "ingest_stamps"; a debugging aid)
  long long* s_first;        // nullable (no SCOTTY_AGG_FIRST): per slice, the arrival index of its first tuple
  long long* c_first;        //   per cell (first_kernel), folded by min and reset to FIRST_NONE
};

// ---- watermark of the grid path (window_kernels.hip): window assembly over slice-block summaries.
// Slices are grouped in blocks of SBLK consecutive slice-array entries.  Per block: count, sum, min, max; an
// inclusive prefix over the blocks of count and (integer) sum -- int wrap arithmetic is exactly invertible, so
// a run of whole blocks is P[last] - P[first-1]; a sparse table over block minima / maxima (level k covers 2^k
// blocks) answers min / max of a run of whole blocks with two lookups.  A window [sa, sb) of slices is the
// partial head block + the run of whole blocks + the partial tail block.
constexpr int SBLK = 64;
constexpr int ST_LEVELS = 15;      // 2^14 blocks * 64 = 2^20 slices (the slice capacity)
constexpr int WM_HDR = 512;        // packed watermark output: header bytes (DevMeta snapshot + counts)
constexpr int WM_HDR_N = 448;      // offset of the device's window count in the header

struct WmArgs {
  DevMeta* meta;
  const int64_t* s_tstart;
  const int64_t* s_tlast;
  const unsigned long long* s_cnt;
  const unsigned long long* s_part[NPART];
  // block summaries (index = slice index / SBLK)
  unsigned long long* b_cnt;
  unsigned long long* b_part[NPART];
  unsigned long long* p_cnt;       // inclusive prefix of b_cnt
  unsigned long long* p_sum;       // inclusive prefix of b_part[0] (integer value types)
  long long* st_min;               // [ST_LEVELS][nbcap], level 0 = b_part[1]
  long long* st_max;
  int64_t nbcap;
  // window definitions (registration order): kind, a, b per definition
  const int64_t* wdef;
  int32_t n_defs;
  int64_t last_wm, wm, remove_from;
  int64_t n_windows;               // row capacity of the packed output (an upper bound of the triggered windows,
                                   // computed on the host in O(#definitions)); the device writes the true count
  unsigned char* out;              // packed output (device): header, start[n], end[n], values[n_aggs][n], has[n]
  unsigned char* hout;             // nullable: the same layout in host-mapped memory, written directly (no publish copy)
  int32_t n_aggs;
  int32_t agg_kind[8];
  int need;
  int vt;
  const long long* s_first;        // nullable: SCOTTY_AGG_FIRST per-slice partials
};

// byte offsets of the packed watermark output's columns for n windows and n_aggs aggregations
struct WmLayout {
  int64_t start, end, vals, has, total;
  __host__ __device__ WmLayout(int64_t n, int n_aggs) {
    start = WM_HDR;
    end = start + 8 * n;
    vals = end + 8 * n;
    has = vals + 8 * n * n_aggs;
    total = has + ((n + 7) / 8) * 8;
  }
};

// Time/arrival-range sharding of one non-keyed micro-batch over G ranks: rank r ingests
// arrival chunk r into the replicated cell layout, exports its first-crossing records and touched cells
// (ShardArgs.xbuf, identical size on every rank), the caller all-gathers the records, and every rank commits
// the same slice edges and partials.  Exchange record of one rank, int64 words:
//   [0..15]   header: chunk max, late tuples, horizon-overflow tuples, touched cells, local candidates, n
//   cells     kc_cap x {cell index, cnt, tmax, sum, min, max}
//   cands     kg_cap x {a local tuple reaches g (0/1), local part of the edge rule (0/1)}
constexpr int SHARD_HDR = 16;
struct ShardArgs {
  const int64_t* ts;
  int64_t n;
  int64_t tile;
  int64_t max_lateness;
  int64_t scap;
  const int64_t* grid;
  long long* tilemax;
  int64_t* s_tstart;
  int64_t* s_tlast;
  unsigned long long* s_cnt;
  unsigned long long* s_part[NPART];
  unsigned long long* c_cnt;
  long long* c_tmax;
  unsigned long long* c_part[NPART];
  DevMeta* meta;
  int32_t* rank_buf;          // scratch [kg_cap]
  int32_t* flag_buf;          // scratch [kg_cap]
  int64_t kc_cap, kg_cap;
  int64_t* xbuf;              // export: this rank's record
  const int64_t* gathered;    // commit: world records
  int32_t world;
  int need, vt;
};

}  // namespace scotty
