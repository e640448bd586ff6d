// keyed_grid.h -- the keyed engine's sort-free path (keyed_grid.hip): layout shared by host and kernels.
#pragma once
#include <stdint.h>

#include "exact_common.h"

namespace scotty {

constexpr int KG_RB = 10;                // table positions per bucket region = 1 << KG_RB
constexpr int KG_R = 1 << KG_RB;
constexpr int KG_SPILL = 64;             // linear-probe spill past the region end kept in LDS
constexpr int KG_RP = KG_R + KG_SPILL;
constexpr int KG_NB_MAX = 4096;          // buckets (LDS counters of the partition kernels)
constexpr int KG_MAXCELL = 8;            // batch grid cells the control block can describe
constexpr int KG_EMAX = 8;               // slice edges one key may append in one batch on this path
constexpr int KG_SHARDS = 32;            // shards of the committed-keys counter

// batch-level reasons the whole batch goes to the replay path (KgCtl.flag)
enum : int32_t {
  KG_UNSORTED = 1,   // timestamps not non-decreasing in arrival order
  KG_SPAN = 2,       // ts_last - ts_first does not fit 32 bits (cell offsets are u32)
  KG_CELLS = 4,      // the batch covers more grid intervals than the bucket kernel keeps in LDS
  KG_GRID = 8,       // grid walk did not advance (reference's calculateNextFixedEdge hang / overflow)
};

struct KgCtl {
  int32_t flag, ncell;
  unsigned long long deferred;     // tuples left to the replay path (keys new / not eligible this batch)
  int32_t compact, pad0;           // the partition writes 8-byte records this batch (see KgArgs.allow_compact)
  unsigned long long defer_keys;   // known keys deferred
  int64_t ts_first, ts_last;
  int64_t bg[KG_MAXCELL];          // bg[c] (c >= 1): lower bound of batch cell c (a grid point); bg[0] = ts_first
  unsigned long long keys_shard[KG_SHARDS];  // keys committed on this path, per commit-workgroup shard
};

// per-(key, cell) partials of one batch, at slot * cells + cell (cnt 0: untouched; the commit resets it)
struct KPart {
  uint32_t cnt, tmin, tmax, pad;   // tuples, min / max ts - ts_first
  unsigned long long sum;          // wrapping integer sum of the lifted values, or f64 bits
  long long vmin, vmax;            // lifted MIN / MAX partials
};

struct KgArgs {
  const uint32_t* key;
  const int64_t* ts;
  const void* val;
  int64_t n;
  const unsigned long long* ktab;  // compact key table: ((key + 1) << 32) | slot, capacity kmask + 1
  uint64_t kmask;
  int32_t nbk;                     // buckets = (kmask + 1) >> KG_RB
  int32_t ntiles;                  // ceil(n / KG_TILE)
  int32_t cmax;                    // cells the bucket kernel variant keeps
  int32_t tile;                    // tuples per partition tile
  int32_t variant;                 // kernel variant (A/B, scotty_tune "keyed_grid_variant")
  int32_t allow_compact;           // int32 values, default kernels: 8-byte records when the batch's ts span fits the
                                   // bits the key leaves (key hash bits outside the bucket, ts offset, value)
  int32_t* hist;                   // [nbk][ntiles], scanned in place (exclusive)
  void* rec;                       // bucket-ordered records
  uint8_t* mark;                   // [n] tuple deferred to the replay path (reset by the gather)
  KPart* part;                     // [n_ops * cmax]
  uint8_t* dflag;                  // [n_ops] key deferred by the commit (reset by the host)
  KgCtl* ctl;
  const XCfg* cfg;
  XState* st;
  XSlices sl;
};

}  // namespace scotty
