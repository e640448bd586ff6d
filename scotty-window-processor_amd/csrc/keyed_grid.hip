// keyed_grid.hip -- sort-free path of the keyed engine for its common case: every window a context-free time
// window on Eager slices (the lane path's subset, keyed_lane.hip) and a batch whose timestamps are non-decreasing
// in arrival order (so every key's tuples are in order).  BASELINE configs[3] (C4) is this case.
//
// The reference keeps one SlicingWindowOperator per key (flink-connector/.../KeyedScottyWindowOperator.java:56-86)
// and runs StreamSlicer.determineSlices + SliceManager.processElement per tuple (S/StreamSlicer.java:36-116,
// S/SliceManager.java:47-87).  For in-order tuples of one key the outcome of a batch is a function of per-cell
// partials only, where the cells are the batch's grid intervals (the union grid of the windows' edges, shared by
// every key):
//   * a grid point g at or above the key's pending edge N becomes a slice edge iff g == N (crossed), or
//     g == nextGrid(m(g)), or e(g) - g < maxLateness -- e(g) the key's first tuple >= g (its minimum ts at or above
//     g, the tuples being in order), m(g) its running max before e(g) (the grid path's rule, slicing_kernels.hip
//     commit_kernel (c), applied per key);
//   * a tuple lands in the slice of the last edge <= its ts, so a cell's tuples all land in one slice.
// Hence no sort: tuples are partitioned by the hash bucket of their key (two passes over the batch, no probe),
// one workgroup per bucket probes its slice of the key table in LDS, folds its tuples into per-(key, cell)
// partials with LDS atomics, and then one lane per key decides the edges and writes the slices and StreamSlicer
// scalars in the lane path's layout (XState + slice SoA), so keys move freely between the paths.
//
// Keys this path cannot take in a batch (new keys, or state the rule does not cover: an empty store, an edge
// walk longer than KG_EMAX, a full slice store) are deferred whole: their tuples are marked, gathered in arrival
// order and replayed by the sort + lane path.  Batch-level conditions (unsorted, span, cells) send the whole batch
// there.  Both keep the result exact.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keyed_grid.h"

namespace scotty {
namespace kg {

constexpr int64_t JMAX = INT64_MAX, JMIN = INT64_MIN;
constexpr int64_t ID_MIN = INT64_MAX;  // identity of a min partial
constexpr int64_t ID_MAX = INT64_MIN;

__device__ __forceinline__ int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
__device__ __forceinline__ int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
__device__ __forceinline__ int64_t jmod(int64_t a, int64_t b) { return b == -1 ? 0 : a % b; }

__device__ __forceinline__ uint32_t khash(uint32_t x) {  // murmur3 finaliser (the key table's hash)
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t khash_inv(uint32_t x) {  // inverse of khash (the murmur3 finaliser is a bijection)
  x ^= x >> 16;
  x *= 0x7ed1b41du;
  x ^= x >> 13;
  x ^= x >> 26;
  x *= 0xa5cb9243u;
  x ^= x >> 16;
  return x;
}

// 8-byte records (KgCtl.compact): word 0 = the key's hash bits outside the bucket field | ts offset << (32 - bb),
// word 1 = the int32 value; bb = log2(buckets).  The bucket kernel knows the bucket of every record it reads, so the
// full hash -- and through khash_inv the key -- is recovered exactly.
__device__ __forceinline__ uint32_t compact_word(uint32_t key, uint32_t toff, int bb) {
  const uint32_t h = khash(key);
  const uint32_t lo = h & ((1u << KG_RB) - 1), hi = h >> (KG_RB + bb);
  return lo | (hi << KG_RB) | (toff << (32 - bb));
}
__device__ __forceinline__ void compact_decode(uint32_t w, uint32_t bk, int bb, uint32_t& key, uint32_t& toff) {
  toff = w >> (32 - bb);
  const uint32_t rest = w & ((1u << (32 - bb)) - 1);
  const uint32_t h = ((rest >> KG_RB) << (KG_RB + bb)) | (bk << KG_RB) | (rest & ((1u << KG_RB) - 1));
  key = khash_inv(h);
}

__device__ __forceinline__ int64_t f64_key(double d) {
  const int64_t b = __double_as_longlong(d);
  return b ^ ((b >> 63) & 0x7FFFFFFFFFFFFFFFLL);
}

// assignNextWindowStart (TumblingWindow.java:29-31, SlidingWindow.java:41-43, FixedBandWindow.java:37-48); the
// union grid's next point after x is the minimum over the windows (StreamSlicer.calculateNextFixedEdge, :103-116)
__device__ __forceinline__ int64_t next_grid(const XCfg* c, int64_t x) {
  int64_t e = JMAX;
  for (int w = 0; w < c->n_cf; w++) {
    const int k = c->cf_kind[w];
    const int64_t a = c->cf_a[w], b = c->cf_b[w];
    int64_t r;
    if (k == 0) r = jsub(jadd(x, a), jmod(x, a));
    else if (k == 1) r = jsub(jadd(x, b), jmod(x, b));
    else if (x == JMAX || x < a) r = a;
    else if (x >= a && x < jadd(a, b)) r = jadd(a, b);
    else r = JMAX;
    e = min(e, r);
  }
  return e;
}

__device__ __forceinline__ uint32_t bucket_of(uint32_t key, uint64_t kmask) {
  return (uint32_t)(((uint64_t)khash(key) & kmask) >> KG_RB);
}

// XCD-aware tile order: consecutive tiles on one XCD (workgroups are dealt to the 8 XCDs round robin), so the
// partial lines of adjacent bucket runs meet in one L2
__device__ __forceinline__ int64_t tile_of(int ntiles) {
  const int per = (ntiles + 7) >> 3;
  return (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
}

// ---------------------------------------------------------------- compact key table
__global__ void kg_build_kernel(const uint32_t* slot_key, int64_t n_ops, unsigned long long* tab, uint64_t mask) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_ops; s += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t key = slot_key[s];
    const unsigned long long e = ktab_tag(key) | (unsigned long long)(uint32_t)s;
    uint64_t h = (uint64_t)khash(key) & mask;
    while (atomicCAS(&tab[h], 0ull, e) != 0ull) h = (h + 1) & mask;
  }
}

// ---------------------------------------------------------------- batch grid (one lane)
__global__ void kg_prep_kernel(KgArgs a) {
  if (threadIdx.x != 0) return;
  KgCtl& c = *a.ctl;
  const int64_t f = a.ts[0], l = a.ts[a.n - 1];
  int32_t flag = 0;
  if (l < f) flag |= KG_UNSORTED;
  if ((uint64_t)l - (uint64_t)f >= 0xFFFFFFF0ull) flag |= KG_SPAN;
  int32_t nc = 1;
  c.bg[0] = f;
  int64_t x = f;
  while (!flag) {
    const int64_t g = next_grid(a.cfg, x);
    if (g <= x) {  // no progress: the reference's calculateNextFixedEdge hang, or overflow
      flag |= KG_GRID;
      break;
    }
    if (g > l) break;
    if (nc >= a.cmax) {
      flag |= KG_CELLS;
      break;
    }
    c.bg[nc++] = g;
    x = g;
  }
  c.flag = flag;
  c.ncell = nc;
  c.ts_first = f;
  c.ts_last = l;
  c.deferred = 0;
  {
    const int bb = 31 - __clz(a.nbk);
    c.compact = (a.allow_compact && !flag && (a.nbk & (a.nbk - 1)) == 0 && bb >= 1 && bb <= 16 &&
                 (uint64_t)l - (uint64_t)f < ((uint64_t)1 << bb)) ? 1 : 0;
  }
  c.defer_keys = 0;
  for (int i = 0; i < KG_SHARDS; i++) c.keys_shard[i] = 0;
}

// ---------------------------------------------------------------- partition: histogram
// HT consecutive tiles per workgroup, so each bucket row of the [bucket][tile] matrix is written HT counts at a time
// (one 16-byte run per bucket, not one scattered dword per bucket and tile)
constexpr int PT = 512;  // partition threads
constexpr int HT = 4;
__global__ __launch_bounds__(PT) void kg_hist_kernel(KgArgs a) {
  __shared__ int32_t cnt[HT][KG_NB_MAX];
  const int64_t t0 = (int64_t)blockIdx.x * HT;
  const int tid = threadIdx.x;
  for (int j = 0; j < HT; j++)
    for (int b = tid; b < a.nbk; b += PT) cnt[j][b] = 0;
  __syncthreads();
  for (int j = 0; j < HT && t0 + j < a.ntiles; j++) {
    const int64_t i0 = (t0 + j) * a.tile, i1 = min(a.n, i0 + a.tile);
    if (((uintptr_t)(a.key + i0) & 15) == 0) {  // 16-B loads: 4 keys per lane per load, 16 keys in flight
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4* kp = (const u32x4*)(a.key + i0);
      const int64_t nv = (i1 - i0) >> 2;
      constexpr int UV = 4;
      int64_t v = tid;
      for (; v + (UV - 1) * PT < nv; v += UV * PT) {
        u32x4 k[UV];
#pragma unroll
        for (int u = 0; u < UV; u++) k[u] = __builtin_nontemporal_load(kp + v + u * PT);
#pragma unroll
        for (int u = 0; u < UV; u++) {
          atomicAdd(&cnt[j][bucket_of(k[u].x, a.kmask)], 1);
          atomicAdd(&cnt[j][bucket_of(k[u].y, a.kmask)], 1);
          atomicAdd(&cnt[j][bucket_of(k[u].z, a.kmask)], 1);
          atomicAdd(&cnt[j][bucket_of(k[u].w, a.kmask)], 1);
        }
      }
      for (; v < nv; v += PT) {
        const u32x4 k = __builtin_nontemporal_load(kp + v);
        atomicAdd(&cnt[j][bucket_of(k.x, a.kmask)], 1);
        atomicAdd(&cnt[j][bucket_of(k.y, a.kmask)], 1);
        atomicAdd(&cnt[j][bucket_of(k.z, a.kmask)], 1);
        atomicAdd(&cnt[j][bucket_of(k.w, a.kmask)], 1);
      }
      for (int64_t i = i0 + nv * 4 + tid; i < i1; i += PT)
        atomicAdd(&cnt[j][bucket_of(__builtin_nontemporal_load(a.key + i), a.kmask)], 1);
      continue;
    }
    constexpr int U = 8;  // keys loaded per round before their atomics: 8 loads in flight per lane
    int64_t i = i0 + tid;
    for (; i + (U - 1) * PT < i1; i += U * PT) {
      uint32_t k[U];
#pragma unroll
      for (int u = 0; u < U; u++) k[u] = __builtin_nontemporal_load(a.key + i + u * PT);
#pragma unroll
      for (int u = 0; u < U; u++) atomicAdd(&cnt[j][bucket_of(k[u], a.kmask)], 1);
    }
    for (; i < i1; i += PT) atomicAdd(&cnt[j][bucket_of(__builtin_nontemporal_load(a.key + i), a.kmask)], 1);
  }
  __syncthreads();
  const int nt = (int)min((int64_t)HT, a.ntiles - t0);
  for (int b = tid; b < a.nbk; b += PT) {
    int32_t* row = a.hist + (int64_t)b * a.ntiles + t0;
    for (int j = 0; j < nt; j++) row[j] = cnt[j][b];
  }
}

// records: 4-byte values {key, ts - ts_first, value} (12 B); 8-byte values {key, ts - ts_first, value} (16 B).  A
// record carries no tuple index: a tuple the bucket kernel cannot fold (its key is not in the bucket's LDS table
// slice) is found again by kg_mark_deferred_kernel with the same probe rule.
template <int VB>
struct KRec;
template <>
struct KRec<4> {
  uint32_t x, y, z;
  __device__ uint32_t key() const { return x; }
  __device__ uint32_t toff() const { return y; }
  __device__ int64_t vbits() const { return (int64_t)(int32_t)z; }
  __device__ static KRec load(const void* p, int64_t i) {
    const uint32_t* q = (const uint32_t*)p + 3 * i;
    return KRec{q[0], q[1], q[2]};
  }
  __device__ void store(void* p, int64_t i) const {
    uint32_t* q = (uint32_t*)p + 3 * i;
    q[0] = x;
    q[1] = y;
    q[2] = z;
  }
  __device__ void store_lds(uint32_t* s, int i) const {
    s[3 * i] = x;
    s[3 * i + 1] = y;
    s[3 * i + 2] = z;
  }
  __device__ static KRec load_lds(const uint32_t* s, int i) { return KRec{s[3 * i], s[3 * i + 1], s[3 * i + 2]}; }
  __device__ void set(uint32_t k, uint32_t toff) {
    x = k;
    y = toff;
  }
  __device__ static KRec make(uint32_t k, uint32_t toff, const void* val, int64_t i) {
    return KRec{k, toff, (uint32_t)((const int32_t*)val)[i]};
  }
};
template <>
struct KRec<8> {
  uint4 w;
  __device__ uint32_t key() const { return w.x; }
  __device__ uint32_t toff() const { return w.y; }
  __device__ int64_t vbits() const { return (int64_t)(((uint64_t)w.w << 32) | w.z); }
  __device__ static KRec load(const void* p, int64_t i) { return KRec{((const uint4*)p)[i]}; }
  __device__ void store(void* p, int64_t i) const { ((uint4*)p)[i] = w; }
  __device__ void store_lds(uint32_t* s, int i) const { ((uint4*)s)[i] = w; }
  __device__ static KRec load_lds(const uint32_t* s, int i) { return KRec{((const uint4*)s)[i]}; }
  __device__ void set(uint32_t k, uint32_t toff) {
    w.x = k;
    w.y = toff;
  }
  __device__ static KRec make(uint32_t k, uint32_t toff, const void* val, int64_t i) {
    const uint64_t v = (uint64_t)((const int64_t*)val)[i];
    return KRec{make_uint4(k, toff, (uint32_t)v, (uint32_t)(v >> 32))};
  }
};

// A tile's records and buckets.  Every load is unconditional (the index clamped to the batch), so the tile's loads
// are all in flight before the first is used -- a load under `if (i < n)` whose value is used after the branch joins
// is waited for with vmcnt(0) there, which serialised the IT rounds.  Tuples past the batch count into the sentinel
// bucket NBS (never scanned, never stored).
template <int VB, int IT, int ST, int NBS>
__device__ __forceinline__ bool tile_records(const KgArgs& a, int64_t i0, int tid, int64_t f, int32_t* cnt,
                                             KRec<VB> (&rec)[IT], int32_t (&bk)[IT], int32_t (&rk)[IT]) {
  uint32_t kk[IT];
  int64_t tt[IT], tp[IT];
#pragma unroll
  for (int j = 0; j < IT; j++) {
    const int64_t i = i0 + j * ST + tid;
    const int64_t ic = i < a.n ? i : a.n - 1;
    kk[j] = __builtin_nontemporal_load(a.key + ic);
    tt[j] = a.ts[ic];
    tp[j] = a.ts[ic > 0 ? ic - 1 : 0];
    rec[j] = KRec<VB>::make(0, 0, a.val, ic);
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < IT; j++) {
    const int64_t i = i0 + j * ST + tid;
    const bool in = i < a.n;
    bad |= in && i > 0 && tp[j] > tt[j];  // not in order: the bucket and commit kernels see the flag and skip
    rec[j].set(kk[j], (uint32_t)(tt[j] - f));
    bk[j] = in ? (int32_t)bucket_of(kk[j], a.kmask) : NBS;
    rk[j] = atomicAdd(&cnt[bk[j]], 1);
  }
  return bad;
}

// Scatter into bucket runs, staged in LDS: a tile is counted per bucket, ranked, laid out bucket by bucket in LDS
// and written as contiguous per-bucket runs (a wave writes a few runs, not 64 scattered records).  Order inside a
// bucket is not kept: the per-cell partials commute (counts, wrapping integer sums, min/max; f64 sums
// reassociate, within SUM_F64's stated tolerance).
template <int VB, int T, int NBS, int ST>
__global__ __launch_bounds__(ST) void kg_scatter_kernel(KgArgs a) {
  constexpr int IT = T / ST;
  constexpr int PER = NBS / ST;
  __shared__ __attribute__((aligned(16))) uint32_t stage[T * (VB == 4 ? 3 : 4)];
  __shared__ int32_t cnt[NBS + 1], tst[NBS], base[NBS];
  __shared__ int32_t wsum[ST / 64];
  if (a.ctl->flag) return;
  const int64_t tile = tile_of(a.ntiles);
  if (tile >= a.ntiles) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t f = a.ctl->ts_first;
  const int64_t i0 = tile * T;
  KRec<VB> rec[IT];
  int32_t bk[IT], rk[IT];
  for (int b = tid; b < a.nbk; b += ST) {
    cnt[b] = 0;
    base[b] = a.hist[(int64_t)b * a.ntiles + tile];
  }
  __syncthreads();
  const bool bad = tile_records<VB, IT, ST, NBS>(a, i0, tid, f, cnt, rec, bk, rk);
  if (__ballot(bad) && (tid & 63) == 0) atomicOr(&a.ctl->flag, KG_UNSORTED);
  __syncthreads();
  // tile-local exclusive scan of the bucket counts
  int32_t loc[PER], s = 0;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int idx = tid * PER + q;
    loc[q] = s;
    s += idx < a.nbk ? cnt[idx] : 0;
  }
  int32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  int32_t ex = inc - s;
  for (int w = 0; w < wid; w++) ex += wsum[w];
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int idx = tid * PER + q;
    if (idx < a.nbk) tst[idx] = ex + loc[q];
  }
  __syncthreads();
  const int nt = (int)min((int64_t)T, a.n - i0);
  if (VB == 4 && a.ctl->compact) {  // 8-byte records: staged with their bucket, 8 bytes written
    const int bb = 31 - __clz(a.nbk);
#pragma unroll
    for (int j = 0; j < IT; j++)
      if (bk[j] < NBS) {
        const int q = tst[bk[j]] + rk[j];
        const KRec<4>& r4 = reinterpret_cast<const KRec<4>&>(rec[j]);
        stage[3 * q] = compact_word(r4.x, r4.y, bb);
        stage[3 * q + 1] = r4.z;
        stage[3 * q + 2] = (uint32_t)bk[j];
      }
    __syncthreads();
    for (int i = tid; i < nt; i += ST) {
      const uint32_t w0 = stage[3 * i], w1 = stage[3 * i + 1], b = stage[3 * i + 2];
      ((uint2*)a.rec)[(int64_t)base[b] + (i - tst[b])] = make_uint2(w0, w1);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < IT; j++)
    if (bk[j] < NBS) rec[j].store_lds(stage, tst[bk[j]] + rk[j]);
  __syncthreads();
  for (int i = tid; i < nt; i += ST) {
    const KRec<VB> r = KRec<VB>::load_lds(stage, i);
    const uint32_t b = bucket_of(r.key(), a.kmask);
    r.store(a.rec, (int64_t)base[b] + (i - tst[b]));
  }
}

// ---------------------------------------------------------------- bucket: per-(key, cell) partials in LDS
template <int CM, bool MM>
struct KgLds {
  unsigned long long tab[KG_RP];
  uint32_t cnt[KG_RP * CM], tmin[KG_RP * CM], tmax[KG_RP * CM];
  unsigned long long sum[KG_RP * CM];
  long long vmin[MM ? KG_RP * CM : 1], vmax[MM ? KG_RP * CM : 1];
};

__device__ __forceinline__ int lds_probe(const unsigned long long* tab, uint32_t key, uint64_t kmask,
                                         uint64_t region) {
  for (int p = (int)(((uint64_t)khash(key) & kmask) - region); p < KG_RP; p++) {
    const unsigned long long e = tab[p];
    if (ktab_is(e, key)) return p;
    if (e == 0) return -1;
  }
  return -1;
}

template <int VT, bool MM>
__device__ __forceinline__ void lift(int64_t vb, int64_t& mn, int64_t& mx) {
  if (VT == VT_F64) {
    const double d = __longlong_as_double(vb);
    mn = d != d ? INT64_MIN : f64_key(d);
    mx = d != d ? INT64_MAX : f64_key(d);
  } else {
    mn = vb;
    mx = vb;
  }
}

template <int VT>
__device__ __forceinline__ unsigned long long add_sum(unsigned long long acc, unsigned long long v) {
  if (VT == VT_F64)
    return (unsigned long long)__double_as_longlong(__longlong_as_double((long long)acc) +
                                                    __longlong_as_double((long long)v));
  return acc + v;
}

// One workgroup per bucket: probe the bucket's slice of the key table in LDS, fold the bucket's records into
// per-(key, cell) partials with LDS atomics, write the partials of every touched key to its slot (KPart).
// Records whose key is not in the table (new keys, or probed past the spill) are marked for the replay path.
template <int VT, bool MM, int U>
__device__ __forceinline__ void kg_bucket_body(const KgArgs& a);
// COUNT / SUM: 74 KB of LDS and <= 64 VGPRs, two workgroups per CU; MIN / MAX: one (87 KB)
template <int VT, bool MM, int U = 2>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void kg_bucket_kernel(KgArgs a) {
  kg_bucket_body<VT, MM, U>(a);
}
template <int VT, bool MM>
__global__ __launch_bounds__(1024) void kg_bucket_mm_kernel(KgArgs a) {
  kg_bucket_body<VT, MM, 2>(a);
}
// U: records loaded per round before they are folded (U loads in flight per lane)
template <int VT, bool MM, int U>
__device__ __forceinline__ void kg_bucket_body(const KgArgs& a) {
  constexpr int CM = MM ? 2 : 3;
  constexpr int VB = VT == VT_I32 ? 4 : 8;
  __shared__ KgLds<CM, MM> L;
  __shared__ unsigned long long s_miss;
  if (a.ctl->flag) return;
  const int tid = threadIdx.x, nt = blockDim.x;
  const uint32_t bk = blockIdx.x;
  const uint64_t region = (uint64_t)bk << KG_RB;
  const int nc = a.ctl->ncell;
  const int64_t f = a.ctl->ts_first;
  for (int p = tid; p < KG_RP; p += nt) L.tab[p] = a.ktab[(region + p) & a.kmask];
  for (int q = tid; q < KG_RP * CM; q += nt) {
    L.cnt[q] = 0;
    L.tmin[q] = 0xFFFFFFFFu;
    L.tmax[q] = 0;
    L.sum[q] = 0;
    if (MM) {
      L.vmin[q] = ID_MIN;
      L.vmax[q] = ID_MAX;
    }
  }
  if (tid == 0) s_miss = 0;
  __syncthreads();
  uint32_t bgo[CM];  // cell lower bounds as offsets from ts_first
#pragma unroll
  for (int c = 0; c < CM; c++) bgo[c] = c < nc ? (uint32_t)(a.ctl->bg[c] - f) : 0xFFFFFFFFu;
  const int64_t r0 = a.hist[(int64_t)bk * a.ntiles];
  const int64_t r1 = (int)bk + 1 < a.nbk ? a.hist[(int64_t)(bk + 1) * a.ntiles] : a.n;
  uint32_t miss = 0;
  auto fold = [&](const KRec<VB>& rec) {
    const int p = lds_probe(L.tab, rec.key(), a.kmask, region);
    if (p < 0) {  // found again and marked by kg_mark_deferred_kernel
      miss++;
      return;
    }
    const uint32_t to = rec.toff();
    int c = 0;
#pragma unroll
    for (int k = 1; k < CM; k++) c += to >= bgo[k] ? 1 : 0;
    const int q = p * CM + c;
    const int64_t vb = rec.vbits();
    atomicAdd(&L.cnt[q], 1u);
    atomicMin(&L.tmin[q], to);
    atomicMax(&L.tmax[q], to);
    if (VT == VT_F64) atomicAdd((double*)&L.sum[q], __longlong_as_double(vb));
    else atomicAdd(&L.sum[q], (unsigned long long)vb);
    if (MM) {
      int64_t mn, mx;
      lift<VT, MM>(vb, mn, mx);
      atomicMin(&L.vmin[q], (long long)mn);
      atomicMax(&L.vmax[q], (long long)mx);
    }
  };
  int64_t r = r0 + tid;
  if (VB == 4 && a.ctl->compact) {  // 8-byte records: key and ts offset decoded from the hash word and the bucket
    const int bb = 31 - __clz(a.nbk);
    const uint2* cr = (const uint2*)a.rec;
    auto fold_c = [&](uint2 w) {
      uint32_t key, toff;
      compact_decode(w.x, bk, bb, key, toff);
      KRec<VB> rec;
      reinterpret_cast<KRec<4>&>(rec) = KRec<4>{key, toff, w.y};
      fold(rec);
    };
    for (; r + (U - 1) * nt < r1; r += U * nt) {
      uint2 w[U];
#pragma unroll
      for (int u = 0; u < U; u++) w[u] = cr[r + u * nt];
#pragma unroll
      for (int u = 0; u < U; u++) fold_c(w[u]);
    }
    for (; r < r1; r += nt) fold_c(cr[r]);
  } else {
    for (; r + (U - 1) * nt < r1; r += U * nt) {
      KRec<VB> rc[U];
#pragma unroll
      for (int u = 0; u < U; u++) rc[u] = KRec<VB>::load(a.rec, r + u * nt);
#pragma unroll
      for (int u = 0; u < U; u++) fold(rc[u]);
    }
    for (; r < r1; r += nt) fold(KRec<VB>::load(a.rec, r));
  }
  if (miss) atomicAdd(&s_miss, (unsigned long long)miss);
  __syncthreads();
  for (int p = tid; p < KG_RP; p += nt) {
    const unsigned long long e = L.tab[p];
    if (e == 0) continue;
    if (bucket_of(ktab_key(e), a.kmask) != bk) continue;  // a neighbour bucket's key
    uint32_t tot = 0;
#pragma unroll
    for (int c = 0; c < CM; c++) tot += L.cnt[p * CM + c];
    if (tot == 0) continue;
    KPart* kp = a.part + (int64_t)ktab_slot(e) * CM;
    for (int c = 0; c < nc; c++) {
      const int q = p * CM + c;
      KPart w;
      w.cnt = L.cnt[q];
      w.tmin = L.tmin[q];
      w.tmax = L.tmax[q];
      w.pad = 0;
      w.sum = L.sum[q];
      w.vmin = MM ? L.vmin[q] : ID_MIN;
      w.vmax = MM ? L.vmax[q] : ID_MAX;
      kp[c] = w;
    }
  }
  if (tid == 0 && s_miss) atomicAdd(&a.ctl->deferred, s_miss);
}

// ---------------------------------------------------------------- commit: one lane per key
// One key: decide the batch's edges (StreamSlicer.determineSlices in-order branch, S/StreamSlicer.java:51-86),
// fold the cells into slices (SliceManager.appendSlice / processElement, S/SliceManager.java:27-38, :47-87).
// Returns false (nothing written) when the key must be replayed instead.
template <int VT, bool MM, int CM, class V>
__device__ bool kg_commit_key(const KgArgs& a, const KPart* kp, uint32_t slot, int nc, int64_t f,
                              const int64_t* bg) {
  const XCfg* cfg = a.cfg;
  XState* sp = a.st + slot;
  const int64_t M = sp->maxEventTime, N0 = sp->nextEdgeTs, cc = sp->currentCount;
  const int32_t head = sp->head, tail = sp->tail;
  if (sp->err || !sp->started || tail <= head || N0 == JMIN || sp->pending) return false;
  uint32_t cn[CM];
  int64_t tmn[CM], tmx[CM];
  int64_t ek = JMAX, xk = JMIN;
#pragma unroll
  for (int c = 0; c < CM; c++) {
    cn[c] = c < nc ? kp[c].cnt : 0;
    tmn[c] = cn[c] ? f + (int64_t)kp[c].tmin : JMAX;
    tmx[c] = cn[c] ? f + (int64_t)kp[c].tmax : JMIN;
    ek = min(ek, tmn[c]);
    xk = max(xk, tmx[c]);
  }
  if (ek < M) return false;  // first tuple would take the out-of-order branch (t < maxEventTime)
  const int64_t Lt = cfg->max_lateness;
  int64_t edges[KG_EMAX], ecs[KG_EMAX];
  int ne = 0;
  int64_t g = N0, prev = JMIN;
  bool first = true;
  for (int it = 0; g <= xk; it++) {
    if (it >= 64 || g < 0) return false;
    int64_t e, m, cb = 0;
    if (g <= f) {
      e = ek;
      m = M;
    } else {
      int i = 1;
      while (i < nc && bg[i] != g) i++;
      if (i >= nc) return false;  // not a batch grid point: cannot happen for a grid walk from N
      e = JMAX;
      m = M;
#pragma unroll
      for (int c = 0; c < CM; c++) {
        if (c < i) {
          m = max(m, tmx[c]);
          cb += cn[c];
        } else {
          e = min(e, tmn[c]);
        }
      }
    }
    const bool edge = first || prev <= m || jsub(e, g) < Lt;
    if (edge) {
      if (ne == KG_EMAX) return false;
      edges[ne] = g;
      ecs[ne] = jadd(cc, cb);
      ne++;
    }
    int64_t gn = next_grid(cfg, g);
    if (Lt >= 0) {  // grid points <= ek - maxLateness precede every tuple: none of them can become an edge
      const int64_t lb = jsub(ek, Lt);
      if (lb > g && lb <= ek) gn = next_grid(cfg, lb);
    }
    if (gn <= g) return false;  // hang / overflow: the replay path reports it
    prev = g;
    g = gn;
    first = false;
  }
  const int64_t sc = cfg->sc;
  int32_t h = head, t = tail;
  if (t + ne > sc) {
    if (h == 0 || (t - h) + ne > sc) return false;  // the replay path grows the store
  }
  const V q = xview<V>(a.sl);
  const int64_t b = (int64_t)slot * sc;
  if (t + ne > sc) {  // compact [head, tail) to the front (as the lane replay does)
    const int n = t - h;
    for (int i = 0; i < n; i++) {
      const int64_t s = b + h + i, d = b + i;
      q.ts[d] = q.ts[s]; q.te[d] = q.te[s]; q.tl[d] = q.tl[s]; q.tf[d] = q.tf[s];
      q.cs[d] = q.cs[s]; q.cl[d] = q.cl[s]; q.ty[d] = q.ty[s]; q.cnt[d] = q.cnt[s];
      for (int k = 0; k < NPART; k++) q.p[k][d] = q.p[k][s];
    }
    h = 0;
    t = n;
  }
  // per target slice k (0: the open slice, k >= 1: edge k-1's new slice): a cell lands in the slice of the last
  // edge at or below its lower bound
  uint64_t tot = 0;
  bool cn_open = false;
  for (int k = 0; k <= ne; k++) {
    uint64_t n_ = 0;
    unsigned long long s_ = 0;
    int64_t mn = JMAX, mx = JMIN, vmn = ID_MIN, vmx = ID_MAX;
    for (int c = 0; c < nc && c < CM; c++) {
      if (!cn[c]) continue;
      const int64_t lo = c == 0 ? f : bg[c];
      int kk = 0;
      while (kk < ne && edges[kk] <= lo) kk++;
      if (kk != k) continue;
      n_ += cn[c];
      s_ = add_sum<VT>(s_, kp[c].sum);
      mn = min(mn, tmn[c]);
      mx = max(mx, tmx[c]);
      if (MM) {
        vmn = min(vmn, (int64_t)kp[c].vmin);
        vmx = max(vmx, (int64_t)kp[c].vmax);
      }
    }
    tot += n_;
    if (k == 0) {
      cn_open = n_ != 0;
      const int64_t j = b + t - 1;
      if (n_) {
        q.tl[j] = max(q.tl[j], mx);
        q.tf[j] = min(q.tf[j], mn);
        q.cl[j] = jadd(q.cl[j], (int64_t)n_);
        q.cnt[j] = q.cnt[j] + n_;
        if (cfg->need & NEED_SUM) q.p[0][j] = add_sum<VT>(q.p[0][j], s_);
        if (MM) {
          q.p[1][j] = (unsigned long long)min((int64_t)q.p[1][j], vmn);
          q.p[2][j] = (unsigned long long)max((int64_t)q.p[2][j], vmx);
        }
      }
      if (ne) {
        q.te[j] = edges[0];
        q.ty[j] = XTYPE_FIXED;
      }
    } else {
      const int64_t j = b + t + k - 1, st = edges[k - 1];
      q.ts[j] = st;
      q.te[j] = k < ne ? edges[k] : JMAX;
      q.ty[j] = k < ne ? XTYPE_FIXED : 1;
      q.cs[j] = ecs[k - 1];
      q.tl[j] = n_ ? max(st, mx) : st;
      q.tf[j] = n_ ? mn : JMAX;
      q.cl[j] = jadd(ecs[k - 1], (int64_t)n_);
      q.cnt[j] = n_;
      q.p[0][j] = s_;
      if (MM) {
        q.p[1][j] = (unsigned long long)vmn;
        q.p[2][j] = (unsigned long long)vmx;
      }
    }
  }
  sp->pvalid = h != head ? 0 : min(sp->pvalid, cn_open ? t - 1 : t);  // slice prefixes from here on go stale
  sp->maxEventTime = max(M, xk);
  sp->nextEdgeTs = g;  // the first grid point above the key's last tuple
  sp->currentCount = jadd(cc, (int64_t)tot);
  sp->head = h;
  sp->tail = t + ne;
  return true;
}

template <int VT, bool MM, class V>
__global__ __launch_bounds__(256) void kg_commit_kernel(KgArgs a, int64_t n_ops) {
  constexpr int CM = MM ? 2 : 3;
  __shared__ unsigned long long s_def_t, s_def_k, s_keys;
  const int tid = threadIdx.x;
  if (tid == 0) s_def_t = s_def_k = s_keys = 0;
  __syncthreads();
  const int64_t slot = (int64_t)blockIdx.x * blockDim.x + tid;
  if (!a.ctl->flag && slot < n_ops) {
    const int nc = a.ctl->ncell;
    KPart* kp = a.part + slot * CM;
    uint32_t tot = 0;
    for (int c = 0; c < nc; c++) tot += kp[c].cnt;
    if (tot) {
      int64_t bg[CM];
      for (int c = 0; c < CM; c++) bg[c] = c < nc ? a.ctl->bg[c] : JMAX;
      if (kg_commit_key<VT, MM, CM, V>(a, kp, (uint32_t)slot, nc, a.ctl->ts_first, bg)) {
        atomicAdd(&s_keys, 1ull);
      } else {
        a.dflag[slot] = 1;
        atomicAdd(&s_def_t, (unsigned long long)tot);
        atomicAdd(&s_def_k, 1ull);
      }
      for (int c = 0; c < nc; c++) kp[c].cnt = 0;  // consumed
    }
  }
  __syncthreads();
  if (tid == 0) {
    if (s_def_t) atomicAdd(&a.ctl->deferred, s_def_t);
    if (s_def_k) atomicAdd(&a.ctl->defer_keys, s_def_k);
    // every workgroup commits keys: a sharded counter (one word serialises its atomics), summed by the host
    if (s_keys) atomicAdd(&a.ctl->keys_shard[blockIdx.x % KG_SHARDS], s_keys);
  }
}

// Tuples left to the replay path: keys the bucket kernel could not fold (not in the bucket's LDS slice of the key
// table -- new keys, or probed past the spill: the same rule as lds_probe) and known keys the commit deferred (rare:
// capacity, long edge walks, state the rule does not cover)
__global__ void kg_mark_deferred_kernel(KgArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t key = a.key[i];
    const uint64_t h = (uint64_t)khash(key) & a.kmask;
    const uint64_t region = (h >> KG_RB) << KG_RB;
    bool m = true;
    for (int p = (int)(h - region); p < KG_RP; p++) {
      const unsigned long long e = a.ktab[(region + p) & a.kmask];
      if (ktab_is(e, key)) {
        m = a.dflag[ktab_slot(e)] != 0;
        break;
      }
      if (e == 0) break;
    }
    if (m) a.mark[i] = 1;
  }
}

// ---------------------------------------------------------------- chunk plan of a batch over many grid cells
// The batch's grid points g_1 < g_2 < ... in (ts[0], ts[n-1]] (at most kmax) and, for every g_j, the first tuple
// with ts >= g_j (the batch being in order, chunks of consecutive cells are consecutive tuple ranges).  out[0]:
// count (-1: the grid walk did not advance); out[1 + j]: position of g_{j+1}.
__global__ __launch_bounds__(1024) void kg_bounds_kernel(const int64_t* ts, int64_t n, const XCfg* cfg, int kmax,
                                                         int64_t* gpts, int64_t* out) {
  __shared__ int s_cnt;
  if (threadIdx.x == 0) {
    const int64_t l = ts[n - 1];
    int64_t x = ts[0];
    int k = 0;
    while (k < kmax) {
      const int64_t g = next_grid(cfg, x);
      if (g <= x) {
        k = -1;
        break;
      }
      if (g > l) break;
      gpts[k++] = g;
      x = g;
    }
    s_cnt = k;
    out[0] = k;
  }
  __syncthreads();
  const int k = s_cnt;
  for (int j = threadIdx.x; j < k; j += blockDim.x) {
    const int64_t g = gpts[j];
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ts[mid] < g) lo = mid + 1; else hi = mid;
    }
    out[1 + j] = lo;
  }
}

// ---------------------------------------------------------------- gather of deferred tuples (arrival order)
constexpr int GT = 1024;
__global__ __launch_bounds__(GT) void kg_dcount_kernel(const uint8_t* mark, int64_t n, int32_t* blk) {
  const int64_t i = (int64_t)blockIdx.x * GT + threadIdx.x;
  const int c = __syncthreads_count(i < n && mark[i] != 0);
  if (threadIdx.x == 0) blk[blockIdx.x] = c;
}

template <int VB>
__global__ __launch_bounds__(GT) void kg_dgather_kernel(const uint32_t* key, const int64_t* ts, const void* val,
                                                        uint8_t* mark, int64_t n, const int32_t* blk_off,
                                                        uint32_t* okey, int64_t* ots, void* oval) {
  __shared__ int32_t ws[GT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t i = (int64_t)blockIdx.x * GT + tid;
  const bool m = i < n && mark[i] != 0;
  const unsigned long long bal = __ballot(m);
  if (lane == 0) ws[wid] = __popcll(bal);
  __syncthreads();
  int32_t before = 0;
  for (int w = 0; w < wid; w++) before += ws[w];
  if (m) {
    const int64_t o = (int64_t)blk_off[blockIdx.x] + before + __popcll(bal & ((1ull << lane) - 1));
    okey[o] = key[i];
    ots[o] = ts[i];
    if (VB == 4) ((int32_t*)oval)[o] = ((const int32_t*)val)[i];
    else ((int64_t*)oval)[o] = ((const int64_t*)val)[i];
    mark[i] = 0;
  }
}

}  // namespace kg

// ---------------------------------------------------------------- host wrappers
hipError_t launch_kg_build(const uint32_t* slot_key, int64_t n_ops, unsigned long long* tab, uint64_t mask,
                           hipStream_t st) {
  if (n_ops <= 0) return hipSuccess;
  const unsigned g = (unsigned)std::min<int64_t>((n_ops + 255) / 256, 8192);
  hipLaunchKernelGGL(kg::kg_build_kernel, dim3(g), dim3(256), 0, st, slot_key, n_ops, tab, mask);
  return hipGetLastError();
}

hipError_t launch_kg_partition(const KgArgs& a, int vt, hipStream_t st) {
  hipLaunchKernelGGL(kg::kg_prep_kernel, dim3(1), dim3(64), 0, st, a);
  note_kernel(KN_KG_HIST, "kg_hist_kernel");
  hipLaunchKernelGGL(kg::kg_hist_kernel, dim3((unsigned)((a.ntiles + kg::HT - 1) / kg::HT)), dim3(kg::PT), 0, st, a);
  return hipGetLastError();
}

// tuples per partition tile: the LDS stage holds one tile (int32 values with <= 2048 buckets: 8192 tuples; else 4096).
// Variant 0 (A/B baseline, scotty_tune "keyed_grid_variant"): 512-thread scatter workgroups and 12-byte records only.
// (Measured and removed: a persistent software-pipelined scatter and a 72-KB two-workgroups-per-CU scatter, both equal
// or slower, profiles/r03/r03k_c4_variant_ab.log; round 5: the tile's loads issued behind the bucket bases with the
// previous timestamp from the next lower lane, 0.96 vs 1.01 ms data pass, profiles/r05/ab_c4_variants.json.)
int kg_tile(int vt, int64_t nbk, int variant) {
  (void)variant;
  return vt == VT_I32 && nbk <= 2048 ? 8192 : 4096;
}

hipError_t launch_kg_scatter(const KgArgs& a, int vt, hipStream_t st) {
  const unsigned grid = (unsigned)(((a.ntiles + 7) / 8) * 8);
  if (vt == VT_I32) {
    if (a.tile == 8192 && a.variant == 1) {
      note_kernel(KN_KG_SCATTER, "kg_scatter_kernel<4, 8192, 2048, 1024>");
      hipLaunchKernelGGL((kg::kg_scatter_kernel<4, 8192, 2048, 1024>), dim3(grid), dim3(1024), 0, st, a);
    } else if (a.tile == 8192) {
      note_kernel(KN_KG_SCATTER, "kg_scatter_kernel<4, 8192, 2048, 512>");
      hipLaunchKernelGGL((kg::kg_scatter_kernel<4, 8192, 2048, 512>), dim3(grid), dim3(512), 0, st, a);
    } else {
      note_kernel(KN_KG_SCATTER, "kg_scatter_kernel<4, 4096, 4096, 512>");
      hipLaunchKernelGGL((kg::kg_scatter_kernel<4, 4096, 4096, 512>), dim3(grid), dim3(512), 0, st, a);
    }
  } else {
    note_kernel(KN_KG_SCATTER, "kg_scatter_kernel<8, 4096, 4096, 512>");
    hipLaunchKernelGGL((kg::kg_scatter_kernel<8, 4096, 4096, 512>), dim3(grid), dim3(512), 0, st, a);
  }
  return hipGetLastError();
}

// which: 1 the bucket kernel, 2 the commit kernel (3 both, in that order)
hipError_t launch_kg_bucket(const KgArgs& a, int vt, bool mm, int64_t n_ops, hipStream_t st, int which) {
  const dim3 grid((unsigned)a.nbk), block(1024);
  const dim3 cgrid((unsigned)((n_ops + 255) / 256)), cblock(256);
  const bool B = (which & 1) != 0, C = (which & 2) != 0;
  if (a.sl.kw && mm) {  // key-interleaved store with MIN / MAX (integer values)
    if (vt == VT_I32) {
      if (B) note_kernel(KN_KG_BUCKET, "kg_bucket_mm_kernel<0, true>");
      if (B) hipLaunchKernelGGL((kg::kg_bucket_mm_kernel<VT_I32, true>), grid, block, 0, st, a);
      if (C) hipLaunchKernelGGL((kg::kg_commit_kernel<VT_I32, true, XKView>), cgrid, cblock, 0, st, a, n_ops);
    } else {
      if (B) note_kernel(KN_KG_BUCKET, "kg_bucket_mm_kernel<1, true>");
      if (B) hipLaunchKernelGGL((kg::kg_bucket_mm_kernel<VT_I64, true>), grid, block, 0, st, a);
      if (C) hipLaunchKernelGGL((kg::kg_commit_kernel<VT_I64, true, XKView>), cgrid, cblock, 0, st, a, n_ops);
    }
    return hipGetLastError();
  }
  if (a.sl.kw) {  // key-interleaved store: COUNT / integer SUM
    if (vt == VT_I32) {
      // 8 records in flight per lane (A/B r03k: 2 -> 8 cut the data pass 1.14 -> 1.02 ms per 2^26 tuples)
      if (B) note_kernel(KN_KG_BUCKET, "kg_bucket_kernel<0, false, 8>");
      if (B) hipLaunchKernelGGL((kg::kg_bucket_kernel<VT_I32, false, 8>), grid, block, 0, st, a);
      if (C) hipLaunchKernelGGL((kg::kg_commit_kernel<VT_I32, false, XKView>), cgrid, cblock, 0, st, a, n_ops);
    } else {
      if (B) note_kernel(KN_KG_BUCKET, "kg_bucket_kernel<1, false, 8>");
      if (B) hipLaunchKernelGGL((kg::kg_bucket_kernel<VT_I64, false, 8>), grid, block, 0, st, a);
      if (C) hipLaunchKernelGGL((kg::kg_commit_kernel<VT_I64, false, XKView>), cgrid, cblock, 0, st, a, n_ops);
    }
    return hipGetLastError();
  }
#define SCOTTY_KG(V)                                                                                   \
  do {                                                                                                 \
    if (mm) {                                                                                          \
      if (B) note_kernel(KN_KG_BUCKET, "kg_bucket_mm_kernel<%d, true>", V);                           \
      if (B) hipLaunchKernelGGL((kg::kg_bucket_mm_kernel<V, true>), grid, block, 0, st, a);           \
      if (C) hipLaunchKernelGGL((kg::kg_commit_kernel<V, true, XSlices>), cgrid, cblock, 0, st, a, n_ops);  \
    } else {                                                                                           \
      if (B) note_kernel(KN_KG_BUCKET, "kg_bucket_kernel<%d, false, 2>", V);                          \
      if (B) hipLaunchKernelGGL((kg::kg_bucket_kernel<V, false>), grid, block, 0, st, a);             \
      if (C) hipLaunchKernelGGL((kg::kg_commit_kernel<V, false, XSlices>), cgrid, cblock, 0, st, a, n_ops); \
    }                                                                                                  \
  } while (0)
  if (vt == VT_I32) SCOTTY_KG(VT_I32);
  else if (vt == VT_I64) SCOTTY_KG(VT_I64);
  else SCOTTY_KG(VT_F64);
#undef SCOTTY_KG
  return hipGetLastError();
}

hipError_t launch_kg_mark_deferred(const KgArgs& a, hipStream_t st) {
  const unsigned g = (unsigned)std::min<int64_t>((a.n + 255) / 256, 16384);
  hipLaunchKernelGGL(kg::kg_mark_deferred_kernel, dim3(g), dim3(256), 0, st, a);
  return hipGetLastError();
}

int kg_cells(bool mm) { return mm ? 2 : 3; }

hipError_t launch_kg_bounds(const int64_t* ts, int64_t n, const XCfg* cfg, int kmax, int64_t* gpts, int64_t* out,
                            hipStream_t st) {
  hipLaunchKernelGGL(kg::kg_bounds_kernel, dim3(1), dim3(1024), 0, st, ts, n, cfg, kmax, gpts, out);
  return hipGetLastError();
}

hipError_t launch_kg_dcount(const uint8_t* mark, int64_t n, int32_t* blk, hipStream_t st) {
  hipLaunchKernelGGL(kg::kg_dcount_kernel, dim3((unsigned)((n + kg::GT - 1) / kg::GT)), dim3(kg::GT), 0, st, mark, n,
                     blk);
  return hipGetLastError();
}

hipError_t launch_kg_dgather(const uint32_t* key, const int64_t* ts, const void* val, uint8_t* mark, int64_t n,
                             const int32_t* blk_off, uint32_t* okey, int64_t* ots, void* oval, int vt,
                             hipStream_t st) {
  const dim3 grid((unsigned)((n + kg::GT - 1) / kg::GT)), block(kg::GT);
  if (vt == VT_I32)
    hipLaunchKernelGGL(kg::kg_dgather_kernel<4>, grid, block, 0, st, key, ts, val, mark, n, blk_off, okey, ots, oval);
  else
    hipLaunchKernelGGL(kg::kg_dgather_kernel<8>, grid, block, 0, st, key, ts, val, mark, n, blk_off, okey, ots, oval);
  return hipGetLastError();
}

}  // namespace scotty
