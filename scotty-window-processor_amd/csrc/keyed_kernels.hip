// keyed_kernels.hip -- gfx950 kernels that turn an arrival-ordered keyed micro-batch into per-operator
// segments for the exact engine (exact_kernels.hip).
//
// The reference keeps one SlicingWindowOperator per key in a HashMap and feeds each key's tuples in
// arrival order (flink-connector/.../KeyedScottyWindowOperator.java:56-66).  Here:
//   1. an LDS-staged, stable LSD radix sort of the (ts, value, key) records by key, 8 bits per pass over the
//      bits the batch's largest key needs: radix_hist (per-tile digit counts) -> scan -> radix_scatter (tile
//      ranked stably in LDS with wave ballots, written out as contiguous per-digit runs).  Stability keeps
//      every key's tuples in arrival order, which the reference's out-of-order handling depends on;
//   2. seg_count / seg_write: the batch's distinct keys and where each one's run starts;
//   3. key_insert / key_assign: a device open-addressing hash table maps each distinct key to a dense operator
//      slot (new keys get the next free slots: the HashMap.put of initWindowOperator, :57-60) -- one probe
//      per key of the batch, not per tuple;
//   4. seg_fill: [begin, end) of every operator's run.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exact_common.h"

namespace scotty {
namespace k {

constexpr int RB = 8;                 // radix bits per pass
constexpr int RADIX = 1 << RB;
constexpr int SORT_THREADS = 256;
constexpr int SORT_ITEMS = 8;
constexpr int SORT_TILE = SORT_THREADS * SORT_ITEMS;  // 2048 records per tile

__device__ __forceinline__ uint32_t hash32(uint32_t x) {  // murmur3 finaliser
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

// ---------------------------------------------------------------- hash table
constexpr uint64_t KEY_PROBE_MAX = 2048;
// entries: ktab_tag(key) | slot (exact_common.h); 0 = empty; low word KTAB_PENDING = inserted in this batch, slot not
// yet assigned
__global__ void key_insert_kernel(const uint32_t* keys, int64_t n, unsigned long long* table, uint64_t mask,
                                  uint32_t* new_pos, unsigned long long* new_count, int32_t* full, uint32_t* slot) {
  // also records each tuple's slot when its key already has one (0xFFFFFFFF: key new in this batch, fixed up by
  // slot_kernel<true> after key_assign) -- in the steady state of a keyed stream one probe pass does both
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t key = keys[i];
    uint64_t h = hash32(key) & mask;
    uint32_t sl = KTAB_PENDING;
    for (uint64_t probe = 0; probe <= mask; probe++) {
      unsigned long long e = table[h];
      if (ktab_is(e, key)) {
        sl = ktab_slot(e);
        break;
      }
      if (e == 0) {
        const unsigned long long prev = atomicCAS(&table[h], 0ull, ktab_tag(key) | KTAB_PENDING);
        if (prev == 0) {
          const unsigned long long p = atomicAdd(new_count, 1ull);
          new_pos[p] = (uint32_t)h;
          break;
        }
        if (ktab_is(prev, key)) break;
      }
      h = (h + 1) & mask;
      // a probe run this long means the table is (nearly) full for this batch's new keys: the host doubles it
      // and re-runs the pass (bounded, so a batch of many new keys cannot scan a full table per tuple)
      if (probe == mask || probe >= KEY_PROBE_MAX) {
        atomicOr(full, 1);
        break;
      }
    }
    slot[i] = sl;
  }
}

__global__ void key_assign_kernel(unsigned long long* table, const uint32_t* new_pos, int64_t n_new, int64_t base,
                                  uint32_t* slot_key) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_new; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t h = new_pos[i];
    const unsigned long long e = table[h];
    const uint32_t key = ktab_key(e);
    table[h] = ktab_tag(key) | (unsigned long long)(uint32_t)(base + i);
    slot_key[base + i] = key;
  }
}

// drop_new: leave out keys inserted by an unfinished key_insert pass (slot placeholder 0xFFFFFFFF), so that pass
// can be re-run from scratch on the grown table
__global__ void rehash_kernel(const unsigned long long* old_t, uint64_t old_n, unsigned long long* nt, uint64_t mask,
                              int drop_new) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)old_n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long e = old_t[i];
    if (e == 0) continue;
    if (drop_new && (uint32_t)e == KTAB_PENDING) continue;
    uint64_t h = hash32(ktab_key(e)) & mask;
    while (atomicCAS(&nt[h], 0ull, e) != 0ull) h = (h + 1) & mask;
  }
}

template <bool FIXUP>
__global__ void slot_kernel(const uint32_t* keys, int64_t n, const unsigned long long* table, uint64_t mask,
                            uint32_t* slot) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (FIXUP && slot[i] != KTAB_PENDING) continue;
    const uint32_t key = keys[i];
    uint64_t h = hash32(key) & mask;
    unsigned long long e = 0;
    for (uint64_t probe = 0; probe <= mask; probe++) {
      e = table[h];
      if (ktab_is(e, key)) break;
      h = (h + 1) & mask;
    }
    slot[i] = ktab_slot(e);
  }
}

// ---------------------------------------------------------------- records
// REC = 16: {ts i64, val i32, slot u32};  REC = 24: {ts i64, val 64-bit, slot u32, pad}.  `slot` is the sort key:
// the tuple's key on the replay path (push_keyed_replay).
// REC = 8, packed: {w u32 = key << tb | (ts - tbase), val i32} -- an int32 batch whose key bits plus the bits of its
// event-time span fit one word (C4s: 2^20 keys, ~1.5 s of milliseconds: 20 + 11 bits).  Half the bytes of every
// sort pass, segment scan and replay read; the sort digits start at bit tb, so key order is word order.
struct PackP {
  int64_t tbase;  // the batch's smallest timestamp
  int32_t tb;     // timestamp-offset bits (< 32); the key takes the bits above
};
template <int REC>
struct Rec;
template <>
struct __attribute__((packed, aligned(8))) Rec<8> {
  uint32_t slot;  // the packed word
  int32_t v;
};
template <>
struct __attribute__((packed, aligned(16))) Rec<16> {
  int64_t ts;
  int32_t v;
  uint32_t slot;
};
template <>
struct __attribute__((packed, aligned(8))) Rec<24> {
  int64_t ts;
  int64_t v;
  uint32_t slot;
  uint32_t pad;
};

// a sorted record's key and timestamp
template <int REC>
__device__ __forceinline__ uint32_t rec_key(const Rec<REC>& r, const PackP& pk) {
  if constexpr (REC == 8) return r.slot >> pk.tb;
  else return r.slot;
}
template <int REC>
__device__ __forceinline__ int64_t rec_ts(const Rec<REC>& r, const PackP& pk) {
  if constexpr (REC == 8) return pk.tbase + (int64_t)(r.slot & ((1u << pk.tb) - 1u));
  else return r.ts;
}

// Register image of a record as plain 32-bit words (a packed struct copy would be lowered through scratch)
template <int REC>
struct RV;
template <>
struct RV<8> {
  uint2 a;
  __device__ uint32_t slot() const { return a.x; }
  __device__ static RV load(const void* p, int64_t i) { return RV{((const uint2*)p)[i]}; }
  __device__ void store(void* p, int64_t i) const { ((uint2*)p)[i] = a; }
  __device__ static RV make(const int64_t* ts, const void* val, const uint32_t* slot, int64_t i, const PackP& pk) {
    return RV{make_uint2((slot[i] << pk.tb) | (uint32_t)(ts[i] - pk.tbase), (uint32_t)((const int32_t*)val)[i])};
  }
};
template <>
struct RV<16> {
  uint4 a;
  __device__ uint32_t slot() const { return a.w; }
  __device__ static RV load(const void* p, int64_t i) { return RV{((const uint4*)p)[i]}; }
  __device__ void store(void* p, int64_t i) const { ((uint4*)p)[i] = a; }
  __device__ static RV make(const int64_t* ts, const void* val, const uint32_t* slot, int64_t i, const PackP&) {
    const uint64_t t = (uint64_t)ts[i];
    return RV{make_uint4((uint32_t)t, (uint32_t)(t >> 32), (uint32_t)((const int32_t*)val)[i], slot[i])};
  }
};
template <>
struct RV<24> {
  uint2 a, b, c;
  __device__ uint32_t slot() const { return c.x; }
  __device__ static RV load(const void* p, int64_t i) {
    const uint2* q = (const uint2*)p + 3 * i;
    return RV{q[0], q[1], q[2]};
  }
  __device__ void store(void* p, int64_t i) const {
    uint2* q = (uint2*)p + 3 * i;
    q[0] = a;
    q[1] = b;
    q[2] = c;
  }
  __device__ static RV make(const int64_t* ts, const void* val, const uint32_t* slot, int64_t i, const PackP&) {
    const uint64_t t = (uint64_t)ts[i], v = (uint64_t)((const int64_t*)val)[i];
    return RV{make_uint2((uint32_t)t, (uint32_t)(t >> 32)), make_uint2((uint32_t)v, (uint32_t)(v >> 32)),
              make_uint2(slot[i], 0u)};
  }
};

// A histogram workgroup counts HIST_TILES consecutive sort tiles, so each digit row of the [digit][tile] matrix is
// written HIST_TILES counts at a time (a 32-byte run per digit, not one scattered dword per digit and tile: 256 partial
// lines per tile were most of the histogram passes' HBM writes)
constexpr int HIST_TILES = 8;
template <int R = RADIX>
__device__ __forceinline__ void hist_rows_out(const int32_t (&cnt)[HIST_TILES][R], int32_t* hist, int64_t nblocks,
                                              int64_t t0, int nt, int tid) {
  for (int d = tid; d < R; d += SORT_THREADS) {
    int32_t* row = hist + (int64_t)d * nblocks + t0;
    for (int j = 0; j < nt; j++) row[j] = cnt[j][d];
  }
}

// FIRST: input is SoA (ts, val, slot arrays); else AoS records.  B: digit bits (8, or 10 for a 2-pass sort of 17-20-bit
// keys -- one pass fewer than 8-bit digits)
template <int REC, bool FIRST, int SI, int B = RB>
__global__ __launch_bounds__(SORT_THREADS) void radix_hist_kernel(const Rec<REC>* in, const int64_t* ts,
                                                                   const void* val, const uint32_t* slot, int64_t n,
                                                                   int shift, int32_t* hist, int64_t nblocks,
                                                                   PackP pk) {
  constexpr int TILE = SORT_THREADS * SI;
  constexpr int RADIX = 1 << B;
  __shared__ int32_t cnt[HIST_TILES][RADIX];
  const int tid = threadIdx.x;
  for (int d = tid; d < HIST_TILES * RADIX; d += SORT_THREADS) (&cnt[0][0])[d] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * HIST_TILES;
  const int nt = (int)min((int64_t)HIST_TILES, nblocks - t0);
  for (int j = 0; j < nt; j++) {
    const int64_t base = (t0 + j) * TILE;
    uint32_t sv[SI];
#pragma unroll
    for (int r = 0; r < SI; r++) {  // every load issued before the first is used (indices clamped)
      const int64_t i = min(base + r * SORT_THREADS + tid, n - 1);
      sv[r] = FIRST ? (REC == 8 ? slot[i] << pk.tb : slot[i]) : in[i].slot;
    }
#pragma unroll
    for (int r = 0; r < SI; r++)
      if (base + r * SORT_THREADS + tid < n) atomicAdd(&cnt[j][(sv[r] >> shift) & (RADIX - 1)], 1);
  }
  __syncthreads();
  hist_rows_out<RADIX>(cnt, hist, nblocks, t0, nt, tid);
}

// Stable scatter of one tile.  Each wavefront ranks its own contiguous SI * 64-record sub-tile against
// wave-private digit counters in LDS (8 ballots per record, no block barrier between rounds); one barrier
// then turns the per-wave counts into tile positions.  Arrival order inside the tile = (wave, round, lane).
template <int REC, bool FIRST, int SI, int B = RB>
__global__ __launch_bounds__(SORT_THREADS) void radix_scatter_kernel(const Rec<REC>* in, const int64_t* ts,
                                                                      const void* val, const uint32_t* slot,
                                                                      int64_t n, int shift, const int32_t* offs,
                                                                      int64_t nblocks, Rec<REC>* out, PackP pk) {
  constexpr int TILE = SORT_THREADS * SI;
  constexpr int RADIX = 1 << B;
  // digits per thread in the tile scan (a 4-bit last pass: the first 16 threads hold one digit each)
  constexpr int PER = RADIX >= SORT_THREADS ? RADIX / SORT_THREADS : 1;
  static_assert(RADIX < SORT_THREADS || PER * SORT_THREADS == RADIX, "digit count must be a multiple of the workgroup");
  __shared__ __attribute__((aligned(16))) unsigned char smem[REC * TILE + 4 * 6 * RADIX];
  void* stage = smem;                                                      // [TILE] records
  int32_t* wc = (int32_t*)(smem + sizeof(Rec<REC>) * TILE);               // [4][RADIX] per-wave counters
  int32_t* tot = wc + 4 * RADIX;                                           // [4] wave partial sums (scan)
  int32_t* tstart = tot + RADIX;                                           // [RADIX] tile digit starts
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // XCD-aware tile order: workgroups are dealt to the 8 XCDs round robin, so XCD x takes the consecutive tiles
  // [x * per, (x + 1) * per) -- the runs adjacent tiles write for one digit are adjacent in memory and now meet in
  // one L2, which merges their partial lines before they go to HBM
  const int64_t per = (nblocks + 7) >> 3;
  const int64_t tile = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (tile >= nblocks) return;
  const int64_t base = tile * TILE;
  constexpr int WAVE_ITEMS = SI * 64;
  for (int d = tid; d < 4 * RADIX; d += SORT_THREADS) wc[d] = 0;
  __syncthreads();
  RV<REC> item[SI];
  int32_t dig[SI], rank[SI];
  int32_t* mine = wc + wid * RADIX;
  const unsigned long long lt = (1ull << lane) - 1;
#pragma unroll
  for (int r = 0; r < SI; r++) {
    const int64_t i = base + wid * WAVE_ITEMS + r * 64 + lane;
    int d = -1;
    if (i < n) {
      item[r] = FIRST ? RV<REC>::make(ts, val, slot, i, pk) : RV<REC>::load(in, i);
      d = (item[r].slot() >> shift) & (RADIX - 1);
    }
    dig[r] = d;
    unsigned long long peers = __ballot(d >= 0);
#pragma unroll
    for (int b = 0; b < B; b++) {
      const unsigned long long bb = __ballot(d >= 0 && ((d >> b) & 1));
      peers &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int before = d >= 0 ? mine[d] : 0;
    rank[r] = before + __popcll(peers & lt);
    __builtin_amdgcn_wave_barrier();
    if (d >= 0 && (peers & lt) == 0) mine[d] = before + __popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // digits tid * PER .. + PER: per-wave exclusive offsets and the tile's exclusive digit scan
  {
    int32_t c[PER][4], v[PER], ex[PER], s = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int d = tid * PER + q;
      const bool dv = d < RADIX;
      c[q][0] = dv ? wc[d] : 0;
      c[q][1] = dv ? wc[RADIX + d] : 0;
      c[q][2] = dv ? wc[2 * RADIX + d] : 0;
      c[q][3] = dv ? wc[3 * RADIX + d] : 0;
      v[q] = c[q][0] + c[q][1] + c[q][2] + c[q][3];
      ex[q] = s;
      s += v[q];
    }
    int32_t inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t u = __shfl_up(inc, o);
      if (lane >= o) inc += u;
    }
    if (lane == 63) tot[wid] = inc;
    __syncthreads();
    int32_t add = 0;
    for (int w = 0; w < wid; w++) add += tot[w];
    // (the reads above precede these writes of wc: the barrier in the wave-sum exchange separates them)
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int d = tid * PER + q;
      if (d >= RADIX) continue;
      const int32_t st0 = inc - s + add + ex[q];
      tstart[d] = st0;
      wc[d] = st0;
      wc[RADIX + d] = st0 + c[q][0];
      wc[2 * RADIX + d] = st0 + c[q][0] + c[q][1];
      wc[3 * RADIX + d] = st0 + c[q][0] + c[q][1] + c[q][2];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < SI; r++)
    if (dig[r] >= 0) item[r].store(stage, mine[dig[r]] + rank[r]);
  __syncthreads();
  // write out per-digit runs
  const int64_t cnt_tile = min((int64_t)TILE, n - base);
  for (int i = tid; i < cnt_tile; i += SORT_THREADS) {
    const RV<REC> rr = RV<REC>::load(stage, i);
    const int d = (rr.slot() >> shift) & (RADIX - 1);
    const int64_t g = (int64_t)offs[(int64_t)d * nblocks + tile] + (i - tstart[d]);
    rr.store(out, g);
  }
}

// ---------------------------------------------------------------- the batch's keys, after the sort by key
// The replay path sorts the batch by KEY (stable: arrival order kept within a key) and maps each distinct key to its
// operator slot once, instead of looking up every tuple's key before the sort (67 M random probes of the key table per
// 2^26-tuple batch).  range_hist_kernel: the largest key (the sort's bit count), the timestamp range (the packed
// records' fit test) and the first digit's histogram.  seg_count / seg_write: the positions
// where the key changes, compacted in position order (per-tile counts, exclusive scan, write), so segment u spans
// [ubeg[u], ubeg[u + 1]); seg_count also keeps each tile's largest timestamp (tmax_reduce: the batch's, biased).
constexpr int SEG_ITEMS = 16;
constexpr int SEG_THREADS = 256;
constexpr int SEG_TILE = SEG_ITEMS * SEG_THREADS;

// The key / timestamp range and the sort's first digit histogram in one read of the batch: block b = sort tiles
// [HIST_TILES b, HIST_TILES (b + 1)) (radix_hist_kernel<.., FIRST>'s tiling; the first digit is key & 0xFF for every record layout, so it does not wait
// for the layout choice the range decides).  part[3 b ..]: the block's largest key, ~ smallest and largest biased
// timestamp (range_reduce_kernel folds them: no same-address atomics from thousands of blocks)
// H10: the first 10-bit digit's histogram into hist10 as well (key & 0x3FF: the 2-pass sort, sort_passes<.., 10>)
template <int SI, bool H10>
__global__ __launch_bounds__(SORT_THREADS) void range_hist_kernel(const uint32_t* keys, const int64_t* ts, int64_t n,
                                                                  int32_t* hist, int32_t* hist10, int64_t nblocks,
                                                                  unsigned long long* part) {
  constexpr int TILE = SORT_THREADS * SI;
  __shared__ int32_t cnt[HIST_TILES][RADIX];
  __shared__ int32_t cnt10[H10 ? HIST_TILES : 1][H10 ? 1024 : 1];
  __shared__ unsigned long long s_r[3][SORT_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int d = tid; d < HIST_TILES * RADIX; d += SORT_THREADS) (&cnt[0][0])[d] = 0;
  if (H10)
    for (int d = tid; d < HIST_TILES * 1024; d += SORT_THREADS) (&cnt10[0][0])[d] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * HIST_TILES;
  const int nt = (int)min((int64_t)HIST_TILES, nblocks - t0);
  unsigned long long m = 0, nlo = 0, hi = 0;
  for (int j = 0; j < nt; j++) {
    const int64_t base = (t0 + j) * TILE;
    uint32_t k[SI];
    int64_t t[SI];
#pragma unroll
    for (int r = 0; r < SI; r++) {  // every load issued before the first is used (indices clamped)
      const int64_t i = min(base + r * SORT_THREADS + tid, n - 1);
      k[r] = keys[i];
      t[r] = ts ? ts[i] : 0;
    }
#pragma unroll
    for (int r = 0; r < SI; r++) {
      if (base + r * SORT_THREADS + tid < n) {
        atomicAdd(&cnt[j][k[r] & (RADIX - 1)], 1);
        if (H10) atomicAdd(&cnt10[j][k[r] & 1023], 1);
        m = max(m, (unsigned long long)k[r]);
        const unsigned long long b = (unsigned long long)t[r] ^ 0x8000000000000000ull;
        nlo = max(nlo, ~b);
        hi = max(hi, b);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m = max(m, (unsigned long long)__shfl_xor((long long)m, o));
    nlo = max(nlo, (unsigned long long)__shfl_xor((long long)nlo, o));
    hi = max(hi, (unsigned long long)__shfl_xor((long long)hi, o));
  }
  if (lane == 0) {
    s_r[0][wid] = m;
    s_r[1][wid] = nlo;
    s_r[2][wid] = hi;
  }
  __syncthreads();
  hist_rows_out(cnt, hist, nblocks, t0, nt, tid);
  if constexpr (H10) hist_rows_out<1024>(cnt10, hist10, nblocks, t0, nt, tid);
  if (tid < 3) {
    unsigned long long v = 0;
    for (int w = 0; w < SORT_THREADS / 64; w++) v = max(v, s_r[tid][w]);
    part[3 * blockIdx.x + tid] = v;
  }
}

__global__ __launch_bounds__(1024) void range_reduce_kernel(const unsigned long long* part, int64_t nb,
                                                             unsigned long long* range) {
  __shared__ unsigned long long s_r[3][16];
  unsigned long long v[3] = {0, 0, 0};
  for (int64_t b = threadIdx.x; b < nb; b += 1024)
    for (int j = 0; j < 3; j++) v[j] = max(v[j], part[3 * b + j]);
  for (int j = 0; j < 3; j++) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[j] = max(v[j], (unsigned long long)__shfl_xor((long long)v[j], o));
    if ((threadIdx.x & 63) == 0) s_r[j][threadIdx.x >> 6] = v[j];
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long r = 0;
    for (int w = 0; w < 16; w++) r = max(r, s_r[threadIdx.x][w]);
    range[threadIdx.x] = r;
  }
}

// wave w of tile b: records [b * SEG_TILE + w * 64 * SEG_ITEMS, + 64 * SEG_ITEMS), read 64 consecutive records per
// round (lane = record, coalesced); a segment starts where the key differs from the previous record's
template <int REC>
__device__ __forceinline__ void seg_wave_scan(const Rec<REC>* r, int64_t n, int64_t w0, int lane,
                                              uint64_t (&starts)[SEG_ITEMS], uint32_t (&keys)[SEG_ITEMS],
                                              long long& tmax, const PackP& pk) {
  // the record before the wave's range
  uint32_t prev_last = w0 > 0 && w0 - 1 < n ? rec_key<REC>(r[w0 - 1], pk) : 0;
  tmax = INT64_MIN;
#pragma unroll
  for (int k = 0; k < SEG_ITEMS; k++) {
    const int64_t i = w0 + (int64_t)k * 64 + lane;
    uint32_t key = 0;
    long long t = INT64_MIN;
    if (i < n) {
      const Rec<REC> ri = r[i];
      key = rec_key<REC>(ri, pk);
      t = rec_ts<REC>(ri, pk);
    }
    const uint32_t up = (uint32_t)__shfl_up((int)key, 1);
    const uint32_t prev = lane == 0 ? prev_last : up;
    starts[k] = __ballot(i < n && (i == 0 || key != prev));
    keys[k] = key;
    prev_last = (uint32_t)__shfl((int)key, 63);
    tmax = max(tmax, t);
  }
}

template <int REC>
__global__ __launch_bounds__(SEG_THREADS) void seg_count_kernel(const Rec<REC>* r, int64_t n, int32_t* cnt,
                                                                 long long* tmax_tile, PackP pk) {
  __shared__ int s_c[SEG_THREADS / 64];
  __shared__ long long s_t[SEG_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint64_t starts[SEG_ITEMS];
  uint32_t keys[SEG_ITEMS];
  long long tm;
  seg_wave_scan<REC>(r, n, (int64_t)blockIdx.x * SEG_TILE + (int64_t)wid * 64 * SEG_ITEMS, lane, starts, keys, tm,
                     pk);
  int c = 0;
#pragma unroll
  for (int k = 0; k < SEG_ITEMS; k++) c += __popcll(starts[k]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tm = max(tm, (long long)__shfl_xor(tm, o));
  if (lane == 0) {
    s_c[wid] = c;
    s_t[wid] = tm;
  }
  __syncthreads();
  if (tid == 0) {
    int t = 0;
    long long m = INT64_MIN;
    for (int w = 0; w < SEG_THREADS / 64; w++) {
      t += s_c[w];
      m = max(m, s_t[w]);
    }
    cnt[blockIdx.x] = t;
    tmax_tile[blockIdx.x] = m;
  }
}

template <int REC>
__global__ __launch_bounds__(SEG_THREADS) void seg_write_kernel(const Rec<REC>* r, int64_t n, const int32_t* off,
                                                                 uint32_t* ukey, int64_t* ubeg, PackP pk) {
  __shared__ int s_c[SEG_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * SEG_TILE + (int64_t)wid * 64 * SEG_ITEMS;
  uint64_t starts[SEG_ITEMS];
  uint32_t keys[SEG_ITEMS];
  long long tm;
  seg_wave_scan<REC>(r, n, w0, lane, starts, keys, tm, pk);
  int c = 0;
#pragma unroll
  for (int k = 0; k < SEG_ITEMS; k++) c += __popcll(starts[k]);
  if (lane == 0) s_c[wid] = c;
  __syncthreads();
  int base = off[blockIdx.x];
  for (int w = 0; w < wid; w++) base += s_c[w];
  const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
  for (int k = 0; k < SEG_ITEMS; k++) {
    if ((starts[k] >> lane) & 1) {
      const int q = base + __popcll(starts[k] & lt);
      ukey[q] = keys[k];
      ubeg[q] = w0 + (int64_t)k * 64 + lane;
    }
    base += __popcll(starts[k]);
  }
}

__global__ __launch_bounds__(1024) void tmax_reduce_kernel(const long long* tmax_tile, int64_t nb,
                                                            unsigned long long* tmax_b) {
  __shared__ long long s_t[16];
  long long m = INT64_MIN;
  for (int64_t b = threadIdx.x; b < nb; b += 1024) m = max(m, tmax_tile[b]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (long long)__shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) s_t[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; w++) m = max(m, s_t[w]);
    *tmax_b = (unsigned long long)m ^ 0x8000000000000000ull;
  }
}

// segment u of the sorted batch -> its operator's [begin, end)
__global__ void seg_fill_kernel(const int64_t* ubeg, const uint32_t* uslot, int64_t u_n, int64_t n, int64_t* seg_begin,
                                int64_t* seg_end) {
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < u_n; u += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t s = uslot[u];
    seg_begin[s] = ubeg[u];
    seg_end[s] = u + 1 < u_n ? ubeg[u + 1] : n;
  }
}

// ---------------------------------------------------------------- scans (int32 and int64, exclusive)
template <typename T>
__global__ __launch_bounds__(1024) void scan_block_kernel(const T* in, T* out, int64_t n, T* block_sums) {
  __shared__ T ws[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t i = (int64_t)blockIdx.x * 1024 + tid;
  const T v = i < n ? in[i] : (T)0;
  T inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  T add = 0;
  for (int w = 0; w < wid; w++) add += ws[w];
  if (i < n) out[i] = inc - v + add;
  if (tid == 1023) block_sums[blockIdx.x] = inc + add;
}
template <typename T>
__global__ void scan_add_kernel(T* out, int64_t n, const T* block_off) {
  const int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  if (i < n) out[i] += block_off[blockIdx.x];
}

// Large int32 scans: reduce-then-scan over 4096-element tiles (a wavefront owns 1024 contiguous elements as 4 rows
// of 64 lanes x int4, so every load and store instruction is a contiguous 1 KB).  Two passes over the data --
// read (tile sums), read + write (scan) -- instead of the one-element-per-thread block scan plus a separate add
// pass over the whole array.
constexpr int SC_T = 256, SC_TILE = 4096;
__device__ __forceinline__ int32_t wave_incl_scan(int32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}
__device__ __forceinline__ void tile_load(const int32_t* in, int64_t n, int64_t w0, int lane, bool full,
                                          int4 (&v)[4]) {
  if (full) {
    const int4* p = (const int4*)(in + w0);
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = p[q * 64 + lane];
  } else {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t e = w0 + (int64_t)(q * 64 + lane) * 4;
      v[q] = make_int4(e < n ? in[e] : 0, e + 1 < n ? in[e + 1] : 0, e + 2 < n ? in[e + 2] : 0,
                       e + 3 < n ? in[e + 3] : 0);
    }
  }
}
__global__ __launch_bounds__(SC_T) void scan_reduce_i32_kernel(const int32_t* in, int64_t n, int32_t* sums) {
  __shared__ int32_t ws[SC_T / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * SC_TILE;
  int4 v[4];
  tile_load(in, n, b0 + wid * 1024, lane, b0 + SC_TILE <= n, v);
  int32_t s = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) s += v[q].x + v[q].y + v[q].z + v[q].w;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) ws[wid] = s;
  __syncthreads();
  if (tid == 0) sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}
__global__ __launch_bounds__(SC_T) void scan_apply_i32_kernel(const int32_t* in, int32_t* out, int64_t n,
                                                              const int32_t* tile_off) {
  __shared__ int32_t ws[SC_T / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * SC_TILE, w0 = b0 + wid * 1024;
  const bool full = b0 + SC_TILE <= n;
  int4 v[4];
  tile_load(in, n, w0, lane, full, v);
  int32_t ex[4], carry = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int32_t c = v[q].x + v[q].y + v[q].z + v[q].w;
    const int32_t inc = wave_incl_scan(c, lane);
    ex[q] = carry + inc - c;
    carry += __shfl(inc, 63);
  }
  if (lane == 0) ws[wid] = carry;
  __syncthreads();
  int32_t base = tile_off[blockIdx.x];
  for (int w = 0; w < wid; w++) base += ws[w];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    int4 o;
    o.x = base + ex[q];
    o.y = o.x + v[q].x;
    o.z = o.y + v[q].y;
    o.w = o.z + v[q].z;
    const int64_t e = w0 + (int64_t)(q * 64 + lane) * 4;
    if (full) {
      ((int4*)out)[e >> 2] = o;
    } else {
      if (e < n) out[e] = o.x;
      if (e + 1 < n) out[e + 1] = o.y;
      if (e + 2 < n) out[e + 2] = o.z;
      if (e + 3 < n) out[e + 3] = o.w;
    }
  }
}

// The tile sums (<= 64 Ki of them): one workgroup, a contiguous run per thread -- one launch instead of the
// block scan's three.
constexpr int SS_T = 1024, SS_MAX = 65536;
__global__ __launch_bounds__(SS_T) void scan_small_i32_kernel(int32_t* a, int n) {
  __shared__ int32_t ws[SS_T / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int per = (n + SS_T - 1) / SS_T, i0 = tid * per, i1 = min(n, i0 + per);
  int32_t s = 0;
  for (int i = i0; i < i1; i++) s += a[i];
  const int32_t inc = wave_incl_scan(s, lane);
  if (lane == 63) ws[wid] = inc;
  __syncthreads();
  int32_t run = inc - s;
  for (int w = 0; w < wid; w++) run += ws[w];
  for (int i = i0; i < i1; i++) {
    const int32_t v = a[i];
    a[i] = run;
    run += v;
  }
}

}  // namespace k

// ---------------------------------------------------------------- host wrappers
// exclusive scan in place-capable (in may equal out); tmp needs >= 2 * ceil(n/1024) + ... elements (recursive)
template <typename T>
static hipError_t scan_rec(const T* in, T* out, int64_t n, T* tmp, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = (n + 1023) / 1024;
  T* sums = tmp;
  T* rest = tmp + nb;
  hipLaunchKernelGGL(k::scan_block_kernel<T>, dim3((unsigned)nb), dim3(1024), 0, st, in, out, n, sums);
  if (nb > 1) {
    hipError_t e = scan_rec<T>(sums, sums, nb, rest, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k::scan_add_kernel<T>, dim3((unsigned)nb), dim3(1024), 0, st, out, n, sums);
  }
  return hipGetLastError();
}
hipError_t launch_scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t st) {
  return scan_rec<int64_t>(in, out, n, tmp, st);
}
hipError_t launch_scan_i32(const int32_t* in, int32_t* out, int64_t n, int32_t* tmp, hipStream_t st) {
  if (n < ((int64_t)1 << 20) || (((uintptr_t)in | (uintptr_t)out) & 15)) return scan_rec<int32_t>(in, out, n, tmp, st);
  const int64_t nb = (n + k::SC_TILE - 1) / k::SC_TILE;  // tmp: nb tile sums + the recursion's (< 2 nb / 1024 more)
  hipLaunchKernelGGL(k::scan_reduce_i32_kernel, dim3((unsigned)nb), dim3(k::SC_T), 0, st, in, n, tmp);
  if (nb <= k::SS_MAX) {
    hipLaunchKernelGGL(k::scan_small_i32_kernel, dim3(1), dim3(k::SS_T), 0, st, tmp, (int)nb);
  } else {
    const hipError_t e = scan_rec<int32_t>(tmp, tmp, nb, tmp + nb, st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k::scan_apply_i32_kernel, dim3((unsigned)nb), dim3(k::SC_T), 0, st, in, out, n, tmp);
  return hipGetLastError();
}

static unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)); }

hipError_t launch_key_insert(const uint32_t* keys, int64_t n, unsigned long long* table, uint64_t mask,
                             uint32_t* new_pos, unsigned long long* new_count, int32_t* full, uint32_t* slot,
                             hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k::key_insert_kernel, dim3(grid_for(n)), dim3(256), 0, st, keys, n, table, mask, new_pos,
                     new_count, full, slot);
  return hipGetLastError();
}
hipError_t launch_key_assign(unsigned long long* table, const uint32_t* new_pos, int64_t n_new, int64_t base,
                             uint32_t* slot_key, hipStream_t st) {
  if (n_new <= 0) return hipSuccess;
  hipLaunchKernelGGL(k::key_assign_kernel, dim3(grid_for(n_new)), dim3(256), 0, st, table, new_pos, n_new, base,
                     slot_key);
  return hipGetLastError();
}
hipError_t launch_rehash(const unsigned long long* old_t, uint64_t old_n, unsigned long long* nt, uint64_t mask,
                         int drop_new, hipStream_t st) {
  hipLaunchKernelGGL(k::rehash_kernel, dim3(grid_for((int64_t)old_n)), dim3(256), 0, st, old_t, old_n, nt, mask,
                     drop_new);
  return hipGetLastError();
}
hipError_t launch_slot(const uint32_t* keys, int64_t n, const unsigned long long* table, uint64_t mask,
                       uint32_t* slot, bool fixup, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (fixup) hipLaunchKernelGGL(k::slot_kernel<true>, dim3(grid_for(n)), dim3(256), 0, st, keys, n, table, mask, slot);
  else hipLaunchKernelGGL(k::slot_kernel<false>, dim3(grid_for(n)), dim3(256), 0, st, keys, n, table, mask, slot);
  return hipGetLastError();
}

int64_t sort_tile() { return k::SORT_TILE; }  // the smallest tile (sizes the histogram buffers)

// one LSD pass: digit histogram per tile (or range_hist_kernel's, pass 0 with hist0), its scan, the stable scatter
template <int REC, int SI, int B>
static void sort_pass(int p, bool hist0, int shift, const void* src, void* dst, const int64_t* ts, const void* val,
                      const uint32_t* slot, int64_t n, int32_t* hist, int32_t* scan_tmp, hipStream_t st, k::PackP pk,
                      hipError_t& e) {
  using R = k::Rec<REC>;
  const int64_t nb = (n + k::SORT_THREADS * SI - 1) / (k::SORT_THREADS * SI);
  const unsigned hb = (unsigned)((nb + k::HIST_TILES - 1) / k::HIST_TILES);
  const unsigned sb = (unsigned)(8 * ((nb + 7) / 8));  // scatter: XCD-aware tile order (radix_scatter_kernel)
  if (p == 0 && hist0) {
    // the first digit's histogram is range_hist_kernel's
  } else if (p == 0)
    hipLaunchKernelGGL((k::radix_hist_kernel<REC, true, SI, B>), dim3(hb), dim3(k::SORT_THREADS), 0, st,
                       (const R*)nullptr, ts, val, slot, n, shift, hist, nb, pk);
  else
    hipLaunchKernelGGL((k::radix_hist_kernel<REC, false, SI, B>), dim3(hb), dim3(k::SORT_THREADS), 0, st,
                       (const R*)src, ts, val, slot, n, shift, hist, nb, pk);
  e = launch_scan_i32(hist, hist, ((int64_t)1 << B) * nb, scan_tmp, st);
  if (e != hipSuccess) return;
  if (p == 0)
    hipLaunchKernelGGL((k::radix_scatter_kernel<REC, true, SI, B>), dim3(sb), dim3(k::SORT_THREADS), 0, st,
                       (const R*)nullptr, ts, val, slot, n, shift, hist, nb, (R*)dst, pk);
  else
    hipLaunchKernelGGL((k::radix_scatter_kernel<REC, false, SI, B>), dim3(sb), dim3(k::SORT_THREADS), 0, st,
                       (const R*)src, ts, val, slot, n, shift, hist, nb, (R*)dst, pk);
}

// narrow_last: the last pass sorts the top bits_last <= 4 key bits with 4-bit digits (16 digit runs per tile instead
// of 256, half the ballots per record; keys of 17-20 bits: 8 + 8 + 4)
template <int REC, int SI, int B = k::RB>
static hipError_t sort_passes(const int64_t* ts, const void* val, const uint32_t* slot, int64_t n, int passes,
                              void* bufA, void* bufB, int32_t* hist, int32_t* scan_tmp, void** result, hipStream_t st,
                              k::PackP pk, bool hist0, bool narrow_last = false) {
  void* src = nullptr;
  void* dst = bufA;
  for (int p = 0; p < passes; p++) {
    const int shift = p * B + (REC == 8 ? pk.tb : 0);
    hipError_t e = hipSuccess;
    if (narrow_last && p == passes - 1 && p > 0)
      sort_pass<REC, SI, 4>(p, hist0, shift, src, dst, ts, val, slot, n, hist, scan_tmp, st, pk, e);
    else
      sort_pass<REC, SI, B>(p, hist0, shift, src, dst, ts, val, slot, n, hist, scan_tmp, st, pk, e);
    if (e != hipSuccess) return e;
    src = dst;
    dst = dst == bufA ? bufB : bufA;
  }
  *result = src;
  return hipGetLastError();
}

// Stable sort of the batch by slot into records (AoS, rec bytes 8 (packed: tbase / tb), 16 or 24).  bufA/bufB: n
// records each; hist: RADIX * ceil(n / sort_tile()) int32, hist10: 1024 * ceil(n / sort_tile()) int32 or null (range_hist
// writes the first-digit histograms); scan_tmp: int32 scratch.  Result lands in *result.  Digits: 8 bits; with hist10
// and digit10 != 0, 10 bits (two passes instead of three for 17-20-bit keys: one read + write of the batch and one
// histogram pass fewer, but ranking 1024 digits per tile in LDS makes each scatter twice as slow -- C4s, 2^26 tuples,
// 2^20 keys: 652 + 607 us scatters, 323 us range + first histograms, 205 us second histogram = 1.93 ms against
// 1.53 ms for three 8-bit passes, profiles/r06/prof; kept as the scotty_tune "keyed_sort_digit10" 1 A/B).
hipError_t launch_sort_by_slot(int rec, const int64_t* ts, const void* val, const uint32_t* slot, int64_t n,
                               int slot_bits, void* bufA, void* bufB, int32_t* hist, int32_t* hist10,
                               int32_t* scan_tmp, void** result, hipStream_t st, int64_t tbase, int tb, bool hist0,
                               int digit10) {
  const k::PackP pk{tbase, tb};
  const bool ten = hist10 && digit10 != 0 && slot_bits > 16 && slot_bits <= 20;
  if (ten) {
    int passes = (slot_bits + 9) / 10;
    if (passes < 1) passes = 1;
    if (rec == 8)
      return sort_passes<8, k::SORT_ITEMS, 10>(ts, val, slot, n, passes, bufA, bufB, hist10, scan_tmp, result, st, pk,
                                               hist0);
    if (rec == 16)
      return sort_passes<16, k::SORT_ITEMS, 10>(ts, val, slot, n, passes, bufA, bufB, hist10, scan_tmp, result, st,
                                                pk, hist0);
    return sort_passes<24, k::SORT_ITEMS, 10>(ts, val, slot, n, passes, bufA, bufB, hist10, scan_tmp, result, st, pk,
                                              hist0);
  }
  int passes = (slot_bits + k::RB - 1) / k::RB;
  if (passes < 1) passes = 1;
  // a last pass over at most 4 key bits takes 4-bit digits (digit10 == 2: 8-bit digits throughout, the A/B)
  const bool narrow = digit10 != 2 && passes > 1 && slot_bits - k::RB * (passes - 1) <= 4;
  // (4096-record tiles for 16-byte records, SI = 16: histogram 291 -> 240 us but scatter 593 -> 803 us per 2^26
  // records -- the 70-KB stage halves the resident workgroups; profiles/r05/c4s_sort_by_key/)
  // packed 8-byte records: 2048-record tiles like the others (4096, SI = 16: histogram 350 -> 285 us but scatter
  // 700 -> 893 us per two passes over 2^26 records, profiles/r05/c4s_packed/)
  if (rec == 8)
    return sort_passes<8, k::SORT_ITEMS>(ts, val, slot, n, passes, bufA, bufB, hist, scan_tmp, result, st, pk, hist0,
                                         narrow);
  if (rec == 16)
    return sort_passes<16, k::SORT_ITEMS>(ts, val, slot, n, passes, bufA, bufB, hist, scan_tmp, result, st, pk, hist0,
                                          narrow);
  return sort_passes<24, k::SORT_ITEMS>(ts, val, slot, n, passes, bufA, bufB, hist, scan_tmp, result, st, pk, hist0,
                                        narrow);
}

// range[0] the largest key, range[1] ~ the smallest and range[2] the largest timestamp biased (ts ^ 1 << 63; with ts
// only), and the first sort digit's histogram; part: 3 * sort tiles
hipError_t launch_range_hist(const uint32_t* keys, const int64_t* ts, int64_t n, int32_t* hist, int32_t* hist10,
                             unsigned long long* part, unsigned long long* range, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = (n + k::SORT_TILE - 1) / k::SORT_TILE, hb = (nb + k::HIST_TILES - 1) / k::HIST_TILES;
  if (hist10)
    hipLaunchKernelGGL((k::range_hist_kernel<k::SORT_ITEMS, true>), dim3((unsigned)hb), dim3(k::SORT_THREADS), 0, st,
                       keys, ts, n, hist, hist10, nb, part);
  else
    hipLaunchKernelGGL((k::range_hist_kernel<k::SORT_ITEMS, false>), dim3((unsigned)hb), dim3(k::SORT_THREADS), 0, st,
                       keys, ts, n, hist, hist10, nb, part);
  hipLaunchKernelGGL(k::range_reduce_kernel, dim3(1), dim3(1024), 0, st, part, hb, range);
  return hipGetLastError();
}
int64_t seg_tiles(int64_t n) { return (n + k::SEG_TILE - 1) / k::SEG_TILE; }
// segment starts of a batch sorted by key: cnt [seg_tiles(n)] (scanned in place), tmax_tile [seg_tiles(n)]
hipError_t launch_seg_count(int rec, const void* recs, int64_t n, int32_t* cnt, long long* tmax_tile,
                            unsigned long long* tmax_b, hipStream_t st, int64_t tbase, int tb) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = seg_tiles(n);
  const k::PackP pk{tbase, tb};
  if (rec == 8)
    hipLaunchKernelGGL(k::seg_count_kernel<8>, dim3((unsigned)nb), dim3(k::SEG_THREADS), 0, st,
                       (const k::Rec<8>*)recs, n, cnt, tmax_tile, pk);
  else if (rec == 16)
    hipLaunchKernelGGL(k::seg_count_kernel<16>, dim3((unsigned)nb), dim3(k::SEG_THREADS), 0, st,
                       (const k::Rec<16>*)recs, n, cnt, tmax_tile, pk);
  else
    hipLaunchKernelGGL(k::seg_count_kernel<24>, dim3((unsigned)nb), dim3(k::SEG_THREADS), 0, st,
                       (const k::Rec<24>*)recs, n, cnt, tmax_tile, pk);
  hipLaunchKernelGGL(k::tmax_reduce_kernel, dim3(1), dim3(1024), 0, st, tmax_tile, nb, tmax_b);
  return hipGetLastError();
}
hipError_t launch_seg_write(int rec, const void* recs, int64_t n, const int32_t* off, uint32_t* ukey, int64_t* ubeg,
                            hipStream_t st, int64_t tbase, int tb) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = seg_tiles(n);
  const k::PackP pk{tbase, tb};
  if (rec == 8)
    hipLaunchKernelGGL(k::seg_write_kernel<8>, dim3((unsigned)nb), dim3(k::SEG_THREADS), 0, st,
                       (const k::Rec<8>*)recs, n, off, ukey, ubeg, pk);
  else if (rec == 16)
    hipLaunchKernelGGL(k::seg_write_kernel<16>, dim3((unsigned)nb), dim3(k::SEG_THREADS), 0, st,
                       (const k::Rec<16>*)recs, n, off, ukey, ubeg, pk);
  else
    hipLaunchKernelGGL(k::seg_write_kernel<24>, dim3((unsigned)nb), dim3(k::SEG_THREADS), 0, st,
                       (const k::Rec<24>*)recs, n, off, ukey, ubeg, pk);
  return hipGetLastError();
}
hipError_t launch_seg_fill(const int64_t* ubeg, const uint32_t* uslot, int64_t u_n, int64_t n, int64_t* seg_begin,
                           int64_t* seg_end, hipStream_t st) {
  if (u_n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k::seg_fill_kernel, dim3(grid_for(u_n)), dim3(256), 0, st, ubeg, uslot, u_n, n, seg_begin,
                     seg_end);
  return hipGetLastError();
}

}  // namespace scotty
