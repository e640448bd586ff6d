// window_kernels.hip -- gfx950 watermark of the grid path: window triggers, window assembly, GC.
//
// Replaces, per processWatermark (S/WindowManager.java:41-80):
//   * the context-free triggers, WindowManager.assignContextFreeWindows (S/WindowManager.java:104-118) with
//     TumblingWindow.triggerWindows (C/windowType/TumblingWindow.java:34-39), SlidingWindow.triggerWindows
//     (C/windowType/SlidingWindow.java:50-57), FixedBandWindow.triggerWindows (C/windowType/FixedBandWindow.java:51-57),
//     generated on the device in registration order (one thread per window definition, a block scan of the counts);
//   * LazyAggregateStore.aggregate (S/aggregationstore/LazyAggregateStore.java:83-111) with
//     AggregateWindowState.containsSlice / addState (S/state/AggregateWindowState.java:25-53): the contained slices
//     of a window are a contiguous range [sa, sb) (first tStart >= start, first tLast >= end; tStart and tLast both
//     increase for context-free slices), found by a wavefront-cooperative search (64 probes per round: 3 rounds for
//     2^18 slices), and folded from slice-block summaries -- prefix sums for count / integer sums (Java int / long
//     wrap is exact modular arithmetic, so differences are bit-exact), a sparse table for min / max, block sums for
//     double sums (no prefix differences on floats) -- plus at most two partial blocks read directly;
//   * AggregateWindowState.getAggValues / hasValue (S/state/AggregateWindowState.java:41-49): values are lowered to
//     the function's result type on the device and written as SoA columns of one packed buffer, so the host copies
//     the whole result with ONE transfer;
//   * WindowManager.clearAfterWatermark -> LazyAggregateStore.removeSlices (S/WindowManager.java:82-95,
//     S/aggregationstore/LazyAggregateStore.java:138-146).
// Two launches per watermark: wm_prep_kernel (one workgroup: dirty block summaries, prefix, sparse table, triggers,
// GC, metadata snapshot) and wm_windows_kernel (one wavefront per triggered window).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/scotty_mi355x.h"
#include "device_common.h"

namespace scotty {
namespace wk {

__device__ __forceinline__ int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
__device__ __forceinline__ int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
__device__ __forceinline__ int64_t jmod(int64_t a, int64_t b) { return b == -1 ? 0 : a % b; }

__device__ __forceinline__ uint64_t wsum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, o);
  return v;
}
__device__ __forceinline__ double wsumf(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int64_t wmin64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (int64_t)__shfl_xor((long long)v, o));
  return v;
}
__device__ __forceinline__ int64_t wmax64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (int64_t)__shfl_xor((long long)v, o));
  return v;
}

constexpr int64_t ID_MIN = INT64_MAX;  // identity of the min partial (order-preserving keys)
constexpr int64_t ID_MAX = INT64_MIN;

// Inclusive block scan (1024 threads) of a u64 sum; `w` is LDS scratch of 16 entries.  Returns the inclusive
// prefix of this thread; *total gets the block total.
__device__ __forceinline__ uint64_t block_scan_u64(uint64_t v, unsigned long long* w, int lane, int wid,
                                                   uint64_t* total) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = (uint64_t)__shfl_up((unsigned long long)v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) w[wid] = v;
  __syncthreads();
  uint64_t before = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint64_t x = w[k];
    if (k < wid) before += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return v + before;
}

// ---- context-free window triggers of one definition (registration order inside the definition follows the
//      reference's loops exactly).  EMIT=false only counts.
template <bool EMIT>
__device__ int64_t trigger_def(int kind, int64_t a, int64_t b, int64_t last_wm, int64_t wm, int64_t* o_start,
                               int64_t* o_end) {
  int64_t n = 0;
  if (kind == SCOTTY_WIN_TUMBLING) {  // TumblingWindow.triggerWindows :34-39
    const int64_t size = a;
    const int64_t last_start = jsub(last_wm, jmod(jadd(last_wm, size), size));
    for (int64_t ws = last_start; jadd(ws, size) <= wm; ws = jadd(ws, size)) {
      if (EMIT) {
        o_start[n] = ws;
        o_end[n] = jadd(ws, size);
      }
      n++;
    }
  } else if (kind == SCOTTY_WIN_SLIDING) {  // SlidingWindow.triggerWindows :50-57
    const int64_t size = a, slide = b;
    const int64_t last_start = jsub(wm, jmod(jadd(wm, slide), slide));
    for (int64_t ws = last_start; jadd(ws, size) > last_wm; ws = jsub(ws, slide)) {
      if (ws >= 0 && jadd(ws, size) <= jadd(wm, 1)) {
        if (EMIT) {
          o_start[n] = ws;
          o_end[n] = jadd(ws, size);
        }
        n++;
      }
    }
  } else if (kind == SCOTTY_WIN_FIXED_BAND) {  // FixedBandWindow.triggerWindows :51-57
    const int64_t e = jadd(a, b);
    if (last_wm <= e && e <= wm) {
      if (EMIT) {
        o_start[0] = a;
        o_end[0] = e;
      }
      n = 1;
    }
  }
  return n;
}

// ---- wavefront-cooperative lower bound: first i in [lo, hi) with key[i] >= x (hi if none).  64 probes per
//      round narrow the range 64-fold (3 dependent rounds for 2^18 slices instead of 18 for a scalar bisection).
__device__ __forceinline__ int64_t wave_lower_bound(const int64_t* key, int64_t lo, int64_t hi, int64_t x, int lane) {
  while (hi - lo > 64) {
    const int64_t stride = (hi - lo + 63) >> 6;
    const int64_t p = lo + (int64_t)lane * stride;
    const bool pred = p < hi && key[p] >= x;
    const unsigned long long bal = __ballot(pred);
    if (bal == 0) {
      const int64_t last = lo + 63 * stride < hi ? lo + 63 * stride : lo + ((hi - 1 - lo) / stride) * stride;
      lo = last + 1;
    } else {
      const int f = __ffsll((long long)bal) - 1;
      if (f == 0) return lo;
      const int64_t pf = lo + (int64_t)f * stride;
      lo = pf - stride + 1;
      hi = pf;
    }
  }
  const int64_t p = lo + lane;
  const unsigned long long bal = __ballot(p < hi && key[p] >= x);
  return bal ? lo + __ffsll((long long)bal) - 1 : hi;
}

// ================================================================ wm_prep (one workgroup of 1024 threads)
__global__ __launch_bounds__(1024) void wm_prep_kernel(WmArgs a) {
  __shared__ unsigned long long s_w[16];
  __shared__ int64_t s_nh;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  DevMeta* meta = a.meta;
  // Every thread reads the operator's scalars itself (one line, uniform addresses) and issues its first trigger
  // definition's loads at once, and the last wave runs the GC search while the others summarise the dirty blocks:
  // this one-workgroup kernel is bound by its chain of dependent global accesses, not by its work
  const int64_t ovf = meta->overflow, head = meta->head, tail = meta->tail, dirty_from = meta->dirty_from;
  int kind0 = -1;
  int64_t wa0 = 0, wb0 = 0;
  if (tid < a.n_defs) {
    kind0 = (int)a.wdef[3 * tid];
    wa0 = a.wdef[3 * tid + 1];
    wb0 = a.wdef[3 * tid + 2];
  }
  const WmLayout L(a.n_windows, a.n_aggs);
  if (ovf != 0) {  // an earlier push of the interval overflowed: the host replays, nothing is assembled
    if (tid == 0) {
      *(DevMeta*)a.out = *meta;
      *(int64_t*)(a.out + WM_HDR_N) = -1;
      if (a.hout) {
        *(DevMeta*)a.hout = *meta;
        *(int64_t*)(a.hout + WM_HDR_N) = -1;
      }
    }
    return;
  }
  // ---- 5 (early). GC (WindowManager.clearAfterWatermark): drop [head, idx) with idx the last slice whose
  //      tStart <= remove_from; the window kernel still reads the pre-GC range [whead, tail)
  if (wid == 15) {
    int64_t nh = head;
    if (tail > head) {  // idx = (count of tStart <= remove_from) - 1
      const int64_t cnt_le = a.remove_from == INT64_MAX
                                 ? tail
                                 : wave_lower_bound(a.s_tstart, head, tail, a.remove_from + 1, lane);
      nh = max(nh, cnt_le - 1);
    }
    if (lane == 0) s_nh = nh;
  }
  const int64_t dirty = min(max(dirty_from, (int64_t)0), tail);
  const bool need_min = (a.need & NEED_MIN) != 0, need_max = (a.need & NEED_MAX) != 0;
  const bool need_sum = (a.need & NEED_SUM) != 0;
  const bool f64 = a.vt == VT_F64;

  // ---- 1. summaries of the blocks whose slices changed since the last watermark (wavefront per block)
  const int64_t hb = head / SBLK;
  const int64_t b0 = max(dirty / SBLK, hb);
  const int64_t b_end = (tail + SBLK - 1) / SBLK;
  for (int64_t b = b0 + wid; b < b_end; b += 16) {
    const int64_t s = b * SBLK + lane;
    uint64_t c = 0, sw = 0;
    double sf = 0.0;
    int64_t mn = ID_MIN, mx = ID_MAX;
    if (s < tail) {
      c = a.s_cnt[s];
      if (need_sum) {
        if (f64) sf = __longlong_as_double((long long)a.s_part[0][s]);
        else sw = a.s_part[0][s];
      }
      if (need_min) mn = (int64_t)a.s_part[1][s];
      if (need_max) mx = (int64_t)a.s_part[2][s];
    }
    c = wsum64(c);
    if (need_sum) {
      if (f64) sf = wsumf(sf);
      else sw = wsum64(sw);
    }
    if (need_min) mn = wmin64(mn);
    if (need_max) mx = wmax64(mx);
    if (lane == 0) {
      a.b_cnt[b] = c;
      if (need_sum) a.b_part[0][b] = f64 ? (unsigned long long)__double_as_longlong(sf) : sw;
      if (need_min) a.b_part[1][b] = (unsigned long long)mn;
      if (need_max) a.b_part[2][b] = (unsigned long long)mx;
    }
  }
  __threadfence_block();
  __syncthreads();

  // ---- 2. inclusive prefix over blocks [b0, b_end) of count and integer sum (carry = prefix of block b0-1;
  //      P[b] - P[b-1] == b_cnt[b] holds for every block ever summarised, so P[-1] = 0 and any stale base cancels)
  {
    uint64_t carry_c = b0 > 0 ? a.p_cnt[b0 - 1] : 0;
    uint64_t carry_s = (need_sum && !f64 && b0 > 0) ? a.p_sum[b0 - 1] : 0;
    for (int64_t base = b0; base < b_end; base += 1024) {
      const int64_t b = base + tid;
      uint64_t tot;
      const uint64_t ic = block_scan_u64(b < b_end ? a.b_cnt[b] : 0, s_w, lane, wid, &tot);
      if (b < b_end) a.p_cnt[b] = carry_c + ic;
      carry_c += tot;
      if (need_sum && !f64) {
        const uint64_t is = block_scan_u64(b < b_end ? a.b_part[0][b] : 0, s_w, lane, wid, &tot);
        if (b < b_end) a.p_sum[b] = carry_s + is;
        carry_s += tot;
      }
    }
  }
  // ---- 3. sparse table over block minima / maxima: level k, entry i = [i, i + 2^k) blocks; only entries that
  //      cover a dirty block are recomputed, and none below the head block
  if (need_min || need_max) {
    for (int k = 1; k < ST_LEVELS; k++) {
      const int64_t span = (int64_t)1 << k, half = span >> 1;
      if (span > b_end - hb) break;
      const int64_t lo = max(hb, b0 - span + 1), hi = b_end - span + 1;
      __threadfence_block();
      __syncthreads();
      const long long* pmn = k == 1 ? (const long long*)a.b_part[1] : a.st_min + (int64_t)(k - 1) * a.nbcap;
      const long long* pmx = k == 1 ? (const long long*)a.b_part[2] : a.st_max + (int64_t)(k - 1) * a.nbcap;
      long long* qmn = a.st_min + (int64_t)k * a.nbcap;
      long long* qmx = a.st_max + (int64_t)k * a.nbcap;
      for (int64_t i = lo + tid; i < hi; i += 1024) {
        if (need_min) qmn[i] = min(pmn[i], pmn[i + half]);
        if (need_max) qmx[i] = max(pmx[i], pmx[i + half]);
      }
    }
  }

  // ---- 4. triggers in registration order: count per definition, scan, emit
  int64_t* o_start = (int64_t*)(a.out + L.start);
  int64_t* o_end = (int64_t*)(a.out + L.end);
  uint64_t emitted = 0;
  for (int base = 0; base < a.n_defs; base += 1024) {
    const int d = base + tid;
    int kind = -1;
    int64_t wa = 0, wb = 0, cnt = 0;
    if (d < a.n_defs) {
      if (base == 0) {
        kind = kind0;
        wa = wa0;
        wb = wb0;
      } else {
        kind = (int)a.wdef[3 * d];
        wa = a.wdef[3 * d + 1];
        wb = a.wdef[3 * d + 2];
      }
      cnt = trigger_def<false>(kind, wa, wb, a.last_wm, a.wm, nullptr, nullptr);
    }
    uint64_t tot;
    const uint64_t incl = block_scan_u64((uint64_t)cnt, s_w, lane, wid, &tot);
    const int64_t off = (int64_t)(emitted + incl) - cnt;
    if (cnt > 0 && off + cnt <= a.n_windows)
      trigger_def<true>(kind, wa, wb, a.last_wm, a.wm, o_start + off, o_end + off);
    emitted += tot;
  }
  __threadfence_block();
  __syncthreads();

  // ---- 6. the new head (the GC search above) and the watermark's header
  if (tid == 0) {
    const int64_t nh = s_nh;
    meta->whead = head;
    meta->head = nh;
    if (tail > nh) meta->oldest_start = a.s_tstart[nh];
    meta->dirty_from = tail;
    *(DevMeta*)a.out = *meta;
    *(int64_t*)(a.out + WM_HDR_N) = (int64_t)emitted;
    if (a.hout) {
      *(DevMeta*)a.hout = *meta;
      *(int64_t*)(a.hout + WM_HDR_N) = (int64_t)emitted;
    }
  }
}

__device__ __forceinline__ double key_to_f64(int64_t k) {  // inverse of the order-preserving f64 key
  return __longlong_as_double((long long)(k ^ ((k >> 63) & 0x7FFFFFFFFFFFFFFFLL)));
}

// lowered value of one aggregation kind (AggregateValueState.getValue -> lower, S/state/AggregateValueState.java:75-79)
__device__ __forceinline__ int64_t lower_value(int kind, uint64_t cnt, uint64_t sw, int64_t mn, int64_t mx,
                                               int64_t first) {
  switch (kind) {
    case SCOTTY_AGG_FIRST: return first;
    case SCOTTY_AGG_SUM_I32: return (int64_t)(int32_t)(uint32_t)sw;
    case SCOTTY_AGG_COUNT: return (int64_t)(int32_t)(uint32_t)cnt;
    case SCOTTY_AGG_MIN_I32: case SCOTTY_AGG_MIN_I64: return mn;
    case SCOTTY_AGG_MAX_I32: case SCOTTY_AGG_MAX_I64: return mx;
    case SCOTTY_AGG_SUM_I64: case SCOTTY_AGG_SUM_F64: return (int64_t)sw;
    case SCOTTY_AGG_MIN_F64:
      return (int64_t)__double_as_longlong(mn == INT64_MIN ? __longlong_as_double(0x7FF8000000000000LL) : key_to_f64(mn));
    case SCOTTY_AGG_MAX_F64:
      return (int64_t)__double_as_longlong(mx == INT64_MAX ? __longlong_as_double(0x7FF8000000000000LL) : key_to_f64(mx));
  }
  return 0;
}

// ================================================================ wm_windows (one wavefront per window)
__global__ __launch_bounds__(256) void wm_windows_kernel(WmArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wi >= a.n_windows) return;
  const DevMeta* meta = a.meta;
  if (meta->overflow) return;
  if (wi >= *(const int64_t*)(a.out + WM_HDR_N)) return;  // rows the triggers actually produced
  const WmLayout L(a.n_windows, a.n_aggs);
  const int64_t head = meta->whead, tail = meta->tail;
  const int64_t ws = ((const int64_t*)(a.out + L.start))[wi];
  const int64_t we = ((const int64_t*)(a.out + L.end))[wi];
  if (a.hout && lane == 0) {  // the row straight into host-mapped memory
    ((int64_t*)(a.hout + L.start))[wi] = ws;
    ((int64_t*)(a.hout + L.end))[wi] = we;
  }
  const int64_t sa = wave_lower_bound(a.s_tstart, head, tail, ws, lane);
  const int64_t sb = wave_lower_bound(a.s_tlast, head, tail, we, lane);
  const bool need_min = (a.need & NEED_MIN) != 0, need_max = (a.need & NEED_MAX) != 0;
  const bool need_sum = (a.need & NEED_SUM) != 0;
  const bool f64 = a.vt == VT_F64;
  uint64_t cnt = 0, sw = 0;
  double sf = 0.0;
  int64_t mn = ID_MIN, mx = ID_MAX;
  auto add_slice = [&](int64_t s) {
    const uint64_t c = a.s_cnt[s];
    if (c == 0) return;
    cnt += c;
    if (need_sum) {
      if (f64) sf += __longlong_as_double((long long)a.s_part[0][s]);
      else sw += a.s_part[0][s];
    }
    if (need_min) mn = min(mn, (int64_t)a.s_part[1][s]);
    if (need_max) mx = max(mx, (int64_t)a.s_part[2][s]);
  };
  if (sb > sa) {
    const int64_t bf = (sa + SBLK - 1) / SBLK, bl = sb / SBLK;  // whole blocks [bf, bl)
    if (bf < bl) {
      if (sa + lane < bf * SBLK) add_slice(sa + lane);   // partial head block
      if (bl * SBLK + lane < sb) add_slice(bl * SBLK + lane);  // partial tail block
      if (f64 && need_sum) {  // double sums: block sums folded directly (no prefix differences on floats)
        for (int64_t b = bf + lane; b < bl; b += 64) sf += __longlong_as_double((long long)a.b_part[0][b]);
      }
      if (lane == 0) {
        cnt += a.p_cnt[bl - 1] - (bf > 0 ? a.p_cnt[bf - 1] : 0);
        if (need_sum && !f64) sw += a.p_sum[bl - 1] - (bf > 0 ? a.p_sum[bf - 1] : 0);
        if (need_min || need_max) {
          const int64_t len = bl - bf;
          const int k = 63 - __clzll((unsigned long long)len);
          const int64_t j = bl - ((int64_t)1 << k);
          if (need_min) {
            const long long* t = k == 0 ? (const long long*)a.b_part[1] : a.st_min + (int64_t)k * a.nbcap;
            mn = min(mn, (int64_t)min(t[bf], t[j]));
          }
          if (need_max) {
            const long long* t = k == 0 ? (const long long*)a.b_part[2] : a.st_max + (int64_t)k * a.nbcap;
            mx = max(mx, (int64_t)max(t[bf], t[j]));
          }
        }
      }
    } else {
      for (int64_t s = sa + lane; s < sb; s += 64) add_slice(s);
    }
  }
  cnt = wsum64(cnt);
  if (need_sum) {
    if (f64) sf = wsumf(sf);
    else sw = wsum64(sw);
  }
  if (need_min) mn = wmin64(mn);
  if (need_max) mx = wmax64(mx);
  if (f64 && need_sum) sw = (uint64_t)__double_as_longlong(sf);
  const bool has = cnt != 0;
  // SCOTTY_AGG_FIRST: AggregateValueState.merge clones the first non-empty partial and folds the rest into it with a
  // combine that keeps partialAggregate1 (S/state/AggregateValueState.java:55-69), so the window's value is the FIRST
  // partial of the first non-empty slice in [sa, sb), slice order: 64 slices per probe, whole empty blocks skipped
  // with their summaries (64 blocks per probe)
  int64_t first = 0;
  if (a.s_first && has) {
    int64_t s0 = sa, found = -1;
    while (s0 < sb && found < 0) {
      if (s0 % SBLK == 0 && s0 + SBLK <= sb) {
        const int64_t bl = sb / SBLK;  // blocks [s0 / SBLK, bl) lie wholly inside the range
        const int64_t b = s0 / SBLK + lane;
        const unsigned long long nb = __ballot(b < bl && a.b_cnt[b] != 0);
        if (nb == 0) {
          s0 = min(bl, s0 / SBLK + 64) * SBLK;
          continue;
        }
        s0 = (s0 / SBLK + __ffsll((long long)nb) - 1) * SBLK;
      }
      const int64_t s1 = min(sb, (s0 / SBLK + 1) * SBLK);  // to the next block boundary
      const unsigned long long ns = __ballot(s0 + lane < s1 && a.s_cnt[s0 + lane] != 0);
      if (ns) found = s0 + __ffsll((long long)ns) - 1;
      s0 = s1;
    }
    if (found >= 0) first = (int64_t)a.s_first[found];
  }
  unsigned char* const o = a.hout ? a.hout : a.out;  // values and flags are read by the host only
  if (lane < a.n_aggs) {
    const int64_t v = has ? lower_value(a.agg_kind[lane], cnt, sw, mn, mx, first) : 0;
    ((int64_t*)(o + L.vals))[(int64_t)lane * a.n_windows + wi] = v;
  }
  if (lane == 0) o[L.has + wi] = has ? 1 : 0;
}

// The packed result into host-mapped pinned memory: one small kernel (16-byte stores over PCIe) instead of a DMA
// transfer, whose setup latency dominated these few-KB copies of every watermark.
__global__ __launch_bounds__(256) void wm_publish_kernel(const uint4* src, uint4* dst, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

__global__ __launch_bounds__(64) void copy_words_kernel(const uint32_t* src, uint32_t* dst, int64_t n) {
  for (int64_t i = threadIdx.x; i < n; i += 64) dst[i] = src[i];
}

}  // namespace wk

namespace wk {
__global__ __launch_bounds__(64) void copy2_words_kernel(const uint32_t* s1, uint32_t* d1, int64_t n1, const uint32_t* s2,
                                                         uint32_t* d2, int64_t n2) {
  for (int64_t i = threadIdx.x; i < n1; i += 64) d1[i] = s1[i];
  for (int64_t i = threadIdx.x; i < n2; i += 64) d2[i] = s2[i];
}
}  // namespace wk

hipError_t launch_copy2_to_host(const void* d_src1, void* h_dst1_dev, size_t bytes1, const void* d_src2, void* h_dst2_dev,
                                size_t bytes2, hipStream_t st) {
  hipLaunchKernelGGL(wk::copy2_words_kernel, dim3(1), dim3(64), 0, st, (const uint32_t*)d_src1, (uint32_t*)h_dst1_dev,
                     (int64_t)(bytes1 / 4), (const uint32_t*)d_src2, (uint32_t*)h_dst2_dev, (int64_t)(bytes2 / 4));
  return hipGetLastError();
}

hipError_t launch_copy_to_host(const void* d_src, void* h_dst_dev, size_t bytes, hipStream_t st) {
  hipLaunchKernelGGL(wk::copy_words_kernel, dim3(1), dim3(64), 0, st, (const uint32_t*)d_src, (uint32_t*)h_dst_dev,
                     (int64_t)(bytes / 4));
  return hipGetLastError();
}

hipError_t launch_wm_publish(const void* d_src, void* h_dst_dev, int64_t bytes, hipStream_t st) {
  const int64_t n16 = (bytes + 15) / 16;
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(64, (n16 + 255) / 256));
  hipLaunchKernelGGL(wk::wm_publish_kernel, dim3(blocks), dim3(256), 0, st, (const uint4*)d_src, (uint4*)h_dst_dev, n16);
  return hipGetLastError();
}

// e0 / e1 (nullable): timing events stamped by the dispatches themselves (hipExtLaunchKernel): e0 with wm_prep's start,
// e1 with the last launch's end
hipError_t launch_wm(const WmArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const bool more = a.n_windows > 0;
  if (e0 || e1) hipExtLaunchKernelGGL(wk::wm_prep_kernel, dim3(1), dim3(1024), 0, st, e0, more ? nullptr : e1, 0, a);
  else hipLaunchKernelGGL(wk::wm_prep_kernel, dim3(1), dim3(1024), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !more) return e;
  const dim3 grid((unsigned)((a.n_windows + 3) / 4));
  if (e1) hipExtLaunchKernelGGL(wk::wm_windows_kernel, grid, dim3(256), 0, st, nullptr, e1, 0, a);
  else hipLaunchKernelGGL(wk::wm_windows_kernel, grid, dim3(256), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_wm(const WmArgs& a, hipStream_t st) { return launch_wm(a, st, nullptr, nullptr); }

}  // namespace scotty
