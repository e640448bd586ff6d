// c4_fold_probe.hip -- VERDICT r05 item 2's proposal for the C4 data pass, measured: one read of the batch folding
// every tuple straight into a per-(key, cell) partial table with device-scope atomics (2^20 keys x 2 cells: the table
// is 32 MB of sums + 8 MB of counts -- resident in the 256 MB MALL), instead of the partition (kg_hist + kg_scatter +
// kg_bucket, 0.94 ms per 2^26-tuple batch).  Keys are dense (slot = key: no probing, the atomics' best
// case), uniform random as in the bench's C4 stream, timestamps in order over two cells.
//   stream : the same loads reduced to a checksum (the read alone)
//   fold2  : + atomicAdd of the value (u64) and of the count (u32) into the tuple's (key, cell)
//   fold4  : + atomicMin / atomicMax of the ts offset (u32): the partials the commit kernel needs (kg_bucket's four)
// The tables are zeroed between passes (not timed); the count total is checked against n.
// Build: hipcc -O3 --offload-arch=gfx950 -o c4_fold_probe tools/c4_fold_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                               \
    }                                                         \
  } while (0)

constexpr int KEY_BITS = 20;

__device__ __forceinline__ uint32_t mix(uint64_t i) {
  uint64_t x = i * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 32;
  return (uint32_t)x;
}

__global__ void gen_kernel(uint32_t* key, int64_t* ts, int32_t* val, int64_t n, int64_t rate) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    key[i] = mix(i) & ((1u << KEY_BITS) - 1);
    ts[i] = i / rate;
    val[i] = (int32_t)mix(i + 0x1234567ull);
  }
}

// MODE 0: stream; 2: fold2; 4: fold4
template <int MODE>
__global__ __launch_bounds__(256) void fold_kernel(const uint32_t* key, const int64_t* ts, const int32_t* val, int64_t n,
                                                   int64_t mid, unsigned long long* sum, uint32_t* cnt, uint32_t* tmin,
                                                   uint32_t* tmax, unsigned long long* chk) {
  unsigned long long acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = __builtin_nontemporal_load(key + i);
    const int64_t t = __builtin_nontemporal_load(ts + i);
    const int32_t v = __builtin_nontemporal_load(val + i);
    const uint32_t q = (k << 1) | (t >= mid ? 1u : 0u);
    if (MODE == 0) {
      acc += k ^ (uint64_t)t ^ (uint32_t)v;
    } else {
      atomicAdd(&sum[q], (unsigned long long)(int64_t)v);
      atomicAdd(&cnt[q], 1u);
      if (MODE == 4) {
        atomicMin(&tmin[q], (uint32_t)t);
        atomicMax(&tmax[q], (uint32_t)t);
      }
    }
  }
  if (MODE == 0) {
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(chk, acc);
  }
}

int main() {
  const int64_t n = (int64_t)1 << 26, rate = n / 1000, mid = 500;
  const int64_t slots = (int64_t)2 << KEY_BITS;
  uint32_t *key, *cnt, *tmin, *tmax;
  int64_t* ts;
  int32_t* val;
  unsigned long long *sum, *chk;
  CK(hipMalloc(&key, n * 4));
  CK(hipMalloc(&ts, n * 8));
  CK(hipMalloc(&val, n * 4));
  CK(hipMalloc(&sum, slots * 8));
  CK(hipMalloc(&cnt, slots * 4));
  CK(hipMalloc(&tmin, slots * 4));
  CK(hipMalloc(&tmax, slots * 4));
  CK(hipMalloc(&chk, 8));
  hipLaunchKernelGGL(gen_kernel, dim3(4096), dim3(256), 0, 0, key, ts, val, n, rate);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes = (double)n * 16;
  for (int mode : {0, 2, 4}) {
    for (int grid : {1024, 4096, 16384}) {
      std::vector<float> ms;
      for (int r = 0; r < 6; r++) {
        CK(hipMemsetAsync(sum, 0, slots * 8, 0));
        CK(hipMemsetAsync(cnt, 0, slots * 4, 0));
        CK(hipMemsetAsync(tmin, 0xFF, slots * 4, 0));
        CK(hipMemsetAsync(tmax, 0, slots * 4, 0));
        CK(hipMemsetAsync(chk, 0, 8, 0));
        CK(hipEventRecord(a, 0));
        if (mode == 0)
          hipLaunchKernelGGL(fold_kernel<0>, dim3(grid), dim3(256), 0, 0, key, ts, val, n, mid, sum, cnt, tmin, tmax, chk);
        else if (mode == 2)
          hipLaunchKernelGGL(fold_kernel<2>, dim3(grid), dim3(256), 0, 0, key, ts, val, n, mid, sum, cnt, tmin, tmax, chk);
        else
          hipLaunchKernelGGL(fold_kernel<4>, dim3(grid), dim3(256), 0, 0, key, ts, val, n, mid, sum, cnt, tmin, tmax, chk);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t = 0;
        CK(hipEventElapsedTime(&t, a, b));
        if (r >= 1) ms.push_back(t);
      }
      float sumt = 0;
      for (float t : ms) sumt += t;
      const float avg = sumt / ms.size();
      unsigned long long total = 0;
      if (mode != 0) {
        std::vector<uint32_t> h(slots);
        CK(hipMemcpy(h.data(), cnt, slots * 4, hipMemcpyDeviceToHost));
        for (uint32_t c : h) total += c;
      }
      printf("%s grid %5d: %.3f ms per 2^26 tuples (%.0f GB/s of input)%s\n",
             mode == 0 ? "stream" : mode == 2 ? "fold2 " : "fold4 ", grid, avg, bytes / (avg * 1e-3) / 1e9,
             mode == 0 ? "" : (total == (unsigned long long)n ? ", counts sum to n" : ", COUNT MISMATCH"));
    }
  }
  return 0;
}
