// pmc_calib.hip -- known-byte kernels for calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 per access pattern
// (MI355X_MICROARCH.md, HBM: FETCH_SIZE reports 1/2 of a wide coalesced streaming read; "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").  Each calib_* kernel reads or writes
// exactly the bytes its name says, in the load / store shape of one of the product's measured kernels:
//   calib_read16      16-B-per-lane coalesced loads            (ingest_kernel, kg_hist_kernel, count_ingest_kernel)
//   calib_read_mix    per lane: u32 key + i64 ts + i32 value   (kg_scatter_kernel's tile loads)
//   calib_read8       8-B-per-lane coalesced loads             (kg_bucket_kernel's 8-byte records)
//   calib_read4       4-B-per-lane coalesced loads
//   calib_write8_runs 8-B stores, 4 lanes per 32-B run, runs at scattered positions (kg_scatter_kernel's bucket runs)
//   calib_write16     16-B-per-lane coalesced stores
// Every measured kernel is preceded by calib_flush (a 1 GiB streaming read of another buffer) so its bytes come from
// HBM, not the 256 MiB Infinity Cache.  tools/traffic.py divides the known bytes by the counters -> per-pattern factors.
// Build: hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib
// Run:   rocprofv3 --pmc FETCH_SIZE -d <dir> -o run -- tools/pmc_calib   (and a separate pass with WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void calib_flush(const u32x4* p, int64_t n4, unsigned* out) {
  unsigned acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    acc += v.x ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads; practically never stores
}

__global__ __launch_bounds__(256) void calib_read16(const u32x4* p, int64_t n4, unsigned* out) {
  unsigned acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ __launch_bounds__(256) void calib_read_mix(const uint32_t* key, const int64_t* ts, const int32_t* val,
                                                      int64_t n, unsigned* out) {
  unsigned acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint32_t k = __builtin_nontemporal_load(key + i);
    const int64_t t = ts[i];
    const int32_t v = val[i];
    acc += k ^ (unsigned)t ^ (unsigned)v;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ __launch_bounds__(256) void calib_read8(const uint2* p, int64_t n, unsigned* out) {
  unsigned acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint2 v = p[i];
    acc += v.x ^ v.y;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ __launch_bounds__(256) void calib_read4(const uint32_t* p, int64_t n, unsigned* out) {
  unsigned acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += __builtin_nontemporal_load(p + i);
  if (acc == 0x9e3779b9u) out[0] = acc;
}

// n records of 8 B, in runs of 4 (32 B); run r goes to slot perm(r) (an odd multiplier mod the run count, a power of
// two: a bijection), so every byte of the output is written exactly once
__global__ __launch_bounds__(256) void calib_write8_runs(uint2* p, int64_t n) {
  const int64_t runs = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i >> 2;
    const int64_t slot = (int64_t)(((uint64_t)r * 0x9E3779B1ull) & (uint64_t)(runs - 1));
    p[slot * 4 + (i & 3)] = make_uint2((uint32_t)i, (uint32_t)r);
  }
}

__global__ __launch_bounds__(256) void calib_write16(u32x4* p, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
    p[i] = v;
  }
}

int main() {
  const int64_t N = (int64_t)1 << 26;  // records / tuples per kernel (the keyed leg's batch)
  const int64_t FL = (int64_t)1 << 30; // flush buffer bytes
  void *flush, *a, *b, *c, *w;
  unsigned* out;
  CK(hipMalloc(&flush, FL));
  CK(hipMalloc(&a, N * 16));  // read16 / read8 / read4 source, write16 target
  CK(hipMalloc(&b, N * 8));   // ts (read_mix)
  CK(hipMalloc(&c, N * 4));   // values (read_mix)
  CK(hipMalloc(&w, N * 8));   // write8_runs target; keys (read_mix) in its first N * 4 bytes
  CK(hipMalloc(&out, 64));
  CK(hipMemset(flush, 3, FL));
  CK(hipMemset(a, 1, N * 16));
  CK(hipMemset(b, 2, N * 8));
  CK(hipMemset(c, 5, N * 4));
  CK(hipMemset(w, 7, N * 8));
  const dim3 G(2048), B(256);
  auto fl = [&]() { hipLaunchKernelGGL(calib_flush, G, B, 0, 0, (const u32x4*)flush, FL / 16, out); };
  for (int rep = 0; rep < 3; rep++) {
    fl();
    hipLaunchKernelGGL(calib_read16, G, B, 0, 0, (const u32x4*)a, N, out);          // 16 B x N
    fl();
    hipLaunchKernelGGL(calib_read_mix, G, B, 0, 0, (const uint32_t*)w, (const int64_t*)b, (const int32_t*)c, N,
                       out);                                                          // 16 B x N
    fl();
    hipLaunchKernelGGL(calib_read8, G, B, 0, 0, (const uint2*)a, N, out);            // 8 B x N
    fl();
    hipLaunchKernelGGL(calib_read4, G, B, 0, 0, (const uint32_t*)a, N, out);         // 4 B x N
    fl();
    hipLaunchKernelGGL(calib_write8_runs, G, B, 0, 0, (uint2*)w, N);                 // 8 B x N written
    fl();
    hipLaunchKernelGGL(calib_write16, G, B, 0, 0, (u32x4*)a, N);                     // 16 B x N written
  }
  CK(hipDeviceSynchronize());
  printf("{\"N\": %lld, \"read_bytes\": {\"calib_read16\": %lld, \"calib_read_mix\": %lld, \"calib_read8\": %lld, "
         "\"calib_read4\": %lld}, \"write_bytes\": {\"calib_write8_runs\": %lld, \"calib_write16\": %lld}}\n",
         (long long)N, (long long)(N * 16), (long long)(N * 16), (long long)(N * 8), (long long)(N * 4),
         (long long)(N * 8), (long long)(N * 16));
  return 0;
}
