// dev_alloc.h -- device / host-mapped allocations of the engines, with a poison knob.
//
// No kernel may read device memory its engine has not written: reused memory holds a previous owner's bytes.  To
// check that, SCOTTY_ALLOC_POISON=<byte> (e.g. 0xA5; a debugging knob) fills every new
// engine allocation with that byte, so a read of never-written state yields wild indices / values at its first use
// instead of the zeros a fresh mapping happens to hold.  Without the knob the exact engine still zero-fills its
// allocations (defence in depth; exact_engine.cpp), the grid and count engines leave them as allocated.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <string.h>

namespace scotty {

// the poison byte, or -1 when the knob is off (scotty_engine.cpp; the environment sets it at load, the internal
// scotty_debug_alloc_poison sets it at run time for the tests)
int alloc_poison();

// fill [p, p + bytes) with `byte` on the null stream and wait (the engines' streams are non-blocking: the fill must
// be complete before any of them can touch the buffer)
inline hipError_t dev_fill_sync(void* p, int byte, size_t bytes) {
  hipError_t e = hipMemsetAsync(p, byte, bytes, nullptr);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(nullptr);
}

// hipMalloc; poisoned when the knob is on
inline hipError_t dev_malloc(void** p, size_t bytes) {
  *p = nullptr;
  hipError_t e = hipMalloc(p, bytes ? bytes : 1);
  if (e != hipSuccess) return e;
  const int pb = alloc_poison();
  return pb >= 0 ? dev_fill_sync(*p, pb, bytes ? bytes : 1) : hipSuccess;
}
template <typename T>
inline hipError_t dev_malloc(T** p, size_t bytes) {
  return dev_malloc((void**)p, bytes);
}

// pinned host-mapped memory (host address *h, device address *d); poisoned when the knob is on
inline hipError_t mapped_host_alloc(void** h, void** d, size_t bytes) {
  hipError_t e = hipHostMalloc(h, bytes, hipHostMallocMapped);
  if (e != hipSuccess) return e;
  const int pb = alloc_poison();
  if (pb >= 0) memset(*h, pb, bytes);
  return hipHostGetDevicePointer(d, *h, 0);
}

}  // namespace scotty
