// Standalone check of launch_scan_i32 (both the block-scan and the reduce-then-scan paths) against a host
// exclusive scan, in place and out of place, over ragged sizes.  Build: see tools/gpu_scan.sh.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../scotty-window-processor_amd/csrc/keyed_kernels.hip"

int main() {
  const int64_t sizes[] = {1, 1000, 4096, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, 4096 * 300 + 17, 16777216, 16777216 + 4095, 268435456 + 4097};
  int bad = 0;
  for (int64_t n : sizes) {
    std::vector<int32_t> h(n), ref(n), got(n);
    srand((unsigned)n);
    for (int64_t i = 0; i < n; i++) h[i] = rand() % 9;
    int64_t acc = 0;
    for (int64_t i = 0; i < n; i++) { ref[i] = (int32_t)acc; acc += h[i]; }
    int32_t *din, *dout, *tmp;
    if (hipMalloc(&din, n * 4) || hipMalloc(&dout, n * 4) || hipMalloc(&tmp, (n / 1024 + 64) * 8)) return 3;
    for (int inplace = 0; inplace < 2; inplace++) {
      hipMemcpy(din, h.data(), n * 4, hipMemcpyHostToDevice);
      int32_t* o = inplace ? din : dout;
      if (scotty::launch_scan_i32(din, o, n, tmp, 0) != hipSuccess) { printf("launch failed n=%lld\n", (long long)n); return 2; }
      hipMemcpy(got.data(), o, n * 4, hipMemcpyDeviceToHost);
      int64_t first = -1;
      for (int64_t i = 0; i < n && first < 0; i++) if (got[i] != ref[i]) first = i;
      printf("n=%lld inplace=%d %s\n", (long long)n, inplace, first < 0 ? "ok" : "MISMATCH");
      if (first >= 0) { printf("  at %lld: got %d want %d\n", (long long)first, got[first], ref[first]); bad++; }
    }
    hipFree(din); hipFree(dout); hipFree(tmp);
  }
  printf(bad ? "scan_check FAILED\n" : "scan_check all ok\n");
  return bad ? 1 : 0;
}
