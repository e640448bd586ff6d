// key_router.cpp -- host-side key-hash router for the keyed operator over G GPUs.
//
// The keyed connector receives tuples that the SPE has already routed by key: Flink's keyBy assigns key k to
// operator index keyGroup(k) * parallelism / maxParallelism, keyGroup(k) = murmurHash(k.hashCode()) % maxParallelism
// (the reference relies on it, F/KeyedScottyWindowOperator.java:56-66: one operator instance sees only its key
// groups).  A producer that feeds G GPUs from one host buffer (the Java shim's off-heap segment) needs the same
// split on the host: scotty_route_keyed is a stable counting sort of a micro-batch by that shard, on T threads
// (per-thread shard histograms over contiguous blocks, exclusive scan, in-order scatter), so each shard's
// sub-batch keeps its arrival order -- every key's operator sees its tuples in the same order as unrouted.
// No collective and no device work: each rank then pushes its sub-batch through scotty_process_keyed_elements.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/scotty_mi355x.h"

namespace {

// MathUtils.murmurHash(int) / bitMix(int) of the SPE (Java int arithmetic: wrap, >>> is a logical shift).
inline int32_t murmur_int(uint32_t code) {
  uint32_t c = code;
  c *= 0xcc9e2d51u;
  c = (c << 15) | (c >> 17);
  c *= 0x1b873593u;
  c = (c << 13) | (c >> 19);
  c = c * 5u + 0xe6546b64u;
  c ^= 4u;
  c ^= c >> 16;
  c *= 0x85ebca6bu;
  c ^= c >> 13;
  c *= 0xc2b2ae35u;
  c ^= c >> 16;
  const int32_t s = (int32_t)c;
  if (s >= 0) return s;
  if (s != INT32_MIN) return -s;
  return 0;
}

inline int shard_of(uint32_t key, int world, int maxp) {
  const int group = murmur_int(key) % maxp;  // KeyGroupRangeAssignment.computeKeyGroupForKeyHash
  return (int)((int64_t)group * world / maxp);  // computeOperatorIndexForKeyGroup
}

}  // namespace

extern "C" int32_t scotty_key_shard(uint32_t key, int world, int max_parallelism) {
  if (world <= 0) return SCOTTY_ERR_ARG;
  if (max_parallelism <= 0) max_parallelism = 128;
  if (world > max_parallelism) return SCOTTY_ERR_ARG;
  return shard_of(key, world, max_parallelism);
}

extern "C" int scotty_route_keyed(const uint32_t* key, const int64_t* ts, const void* val, size_t val_bytes,
                                  size_t n, int world, int max_parallelism, int threads, uint32_t* out_key,
                                  int64_t* out_ts, void* out_val, uint64_t* offsets) {
  if (world <= 0 || !offsets || (val_bytes != 4 && val_bytes != 8)) return SCOTTY_ERR_ARG;
  if (max_parallelism <= 0) max_parallelism = 128;
  if (world > max_parallelism) return SCOTTY_ERR_ARG;
  if (n && (!key || !ts || !val || !out_key || !out_ts || !out_val)) return SCOTTY_ERR_ARG;
  const int W = world, P = max_parallelism;
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  const size_t min_block = (size_t)1 << 16;  // below this a thread costs more than it saves
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, (n + min_block - 1) / min_block));
  const size_t block = (n + T - 1) / std::max(T, 1);
  // shard ids of the batch, computed once (1 B or 2 B per tuple) and reused by the scatter
  const bool narrow = W <= 256;
  std::vector<uint8_t> sid8(narrow ? n : 0);
  std::vector<uint16_t> sid16(narrow ? 0 : n);
  std::vector<uint64_t> hist((size_t)T * W, 0);

  auto run = [&](auto&& fn) {
    if (T == 1) {
      fn(0);
      return;
    }
    std::vector<std::thread> th;
    th.reserve(T);
    for (int t = 0; t < T; t++) th.emplace_back(fn, t);
    for (auto& x : th) x.join();
  };
  run([&](int t) {
    const size_t lo = std::min(n, (size_t)t * block), hi = std::min(n, lo + block);
    uint64_t* h = &hist[(size_t)t * W];
    for (size_t i = lo; i < hi; i++) {
      const int s = shard_of(key[i], W, P);
      if (narrow)
        sid8[i] = (uint8_t)s;
      else
        sid16[i] = (uint16_t)s;
      h[s]++;
    }
  });
  // exclusive scan, shard-major then thread: thread t's tuples of shard s follow those of threads < t
  uint64_t run_off = 0;
  for (int s = 0; s < W; s++) {
    offsets[s] = run_off;
    for (int t = 0; t < T; t++) {
      const uint64_t c = hist[(size_t)t * W + s];
      hist[(size_t)t * W + s] = run_off;
      run_off += c;
    }
  }
  offsets[W] = run_off;
  run([&](int t) {
    const size_t lo = std::min(n, (size_t)t * block), hi = std::min(n, lo + block);
    uint64_t* pos = &hist[(size_t)t * W];
    const unsigned char* v = (const unsigned char*)val;
    unsigned char* ov = (unsigned char*)out_val;
    for (size_t i = lo; i < hi; i++) {
      const int s = narrow ? sid8[i] : sid16[i];
      const uint64_t o = pos[s]++;
      out_key[o] = key[i];
      out_ts[o] = ts[i];
      if (val_bytes == 4)
        std::memcpy(ov + o * 4, v + i * 4, 4);
      else
        std::memcpy(ov + o * 8, v + i * 8, 8);
    }
  });
  return SCOTTY_OK;
}
