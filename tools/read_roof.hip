// read_roof.hip -- the achievable HBM read rate of the grid ingest's access pattern on this MI355X, for the roofline
// discussion: 2^27 int64 timestamps + 2^27 int32 values (1.61 GB, C2's micro-batch) read once with
// 16-byte non-temporal loads, each wave streaming a contiguous range (the ingest's decomposition), reduced to one
// word per wave so nothing is dead code.  Prints GB/s per grid size.  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef long long ll2 __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));

// each wave: per_wave tuples [w0, w0 + per_wave): ts as 2 x int64 per lane per load, values as 4 x int32
template <int UNROLL>
__global__ __launch_bounds__(256) void read_kernel(const int64_t* ts, const int32_t* val, int64_t n, int64_t per_wave,
                                                  unsigned long long* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t w0 = wave * per_wave, w1 = min(n, w0 + per_wave);
  unsigned long long acc = 0;
  // 256 tuples per step: ts 2 KB (2 loads of 16 B per lane), values 1 KB (1 load per lane)
  for (int64_t b = w0; b + 256 * UNROLL <= w1; b += 256 * UNROLL) {
    ll2 t[2 * UNROLL];
    i4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      const ll2* tp = (const ll2*)(ts + b + u * 256);
      t[2 * u] = __builtin_nontemporal_load(tp + lane);
      t[2 * u + 1] = __builtin_nontemporal_load(tp + 64 + lane);
      v[u] = __builtin_nontemporal_load((const i4*)(val + b + u * 256) + lane);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      acc += (unsigned long long)(t[2 * u].x ^ t[2 * u + 1].y) + (unsigned)(v[u].x + v[u].w);
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) out[wave] = acc;
}

int main() {
  const int64_t n = (int64_t)1 << 27;
  int64_t* ts;
  int32_t* val;
  unsigned long long* out;
  CK(hipMalloc(&ts, n * 8));
  CK(hipMalloc(&val, n * 4));
  CK(hipMalloc(&out, (1 << 20) * 8));
  CK(hipMemset(ts, 1, n * 8));
  CK(hipMemset(val, 2, n * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes = (double)n * 12;
  const int grids[] = {256, 512, 768, 1024, 1536, 2048, 4096, 8192};
  for (int unroll : {1, 2, 4}) {
    for (int g : grids) {
      const int64_t waves = (int64_t)g * 4;
      int64_t per_wave = (n + waves - 1) / waves;
      per_wave = (per_wave + 256 * unroll - 1) / (256 * unroll) * (256 * unroll);
      std::vector<float> ms;
      for (int r = 0; r < 12; r++) {
        CK(hipEventRecord(a, 0));
        if (unroll == 1) hipLaunchKernelGGL(read_kernel<1>, dim3(g), dim3(256), 0, 0, ts, val, n, per_wave, out);
        else if (unroll == 2) hipLaunchKernelGGL(read_kernel<2>, dim3(g), dim3(256), 0, 0, ts, val, n, per_wave, out);
        else hipLaunchKernelGGL(read_kernel<4>, dim3(g), dim3(256), 0, 0, ts, val, n, per_wave, out);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t = 0;
        CK(hipEventElapsedTime(&t, a, b));
        if (r >= 2) ms.push_back(t);
      }
      float best = 1e30f, sum = 0;
      for (float t : ms) {
        best = t < best ? t : best;
        sum += t;
      }
      const float avg = sum / ms.size();
      printf("unroll %d grid %5d: avg %.1f us = %.0f GB/s (best %.1f us = %.0f GB/s)\n", unroll, g, avg * 1e3,
             bytes / (avg * 1e-3) / 1e9, best * 1e3, bytes / (best * 1e-3) / 1e9);
    }
  }
  return 0;
}
