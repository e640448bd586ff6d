// host_copy.h -- small device-to-host reads through host-mapped pinned memory.
//
// The engines read a few bytes of control state back after their launches (event counts, batch flags, watermark
// scalars).  A DMA transfer of such a block costs ~10-20 us of setup; a one-wave kernel writing it into
// host-mapped pinned memory costs a kernel launch, and the host reads the bytes once the stream (or an event)
// has completed.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "dev_alloc.h"  // mapped_host_alloc

namespace scotty {

// copy `bytes` (a multiple of 4) from device memory to the device address of a host-mapped buffer
hipError_t launch_copy_to_host(const void* d_src, void* h_dst_dev, size_t bytes, hipStream_t st);
// two ranges in one launch (bytes2 may be 0)
hipError_t launch_copy2_to_host(const void* d_src1, void* h_dst1_dev, size_t bytes1, const void* d_src2, void* h_dst2_dev,
                                size_t bytes2, hipStream_t st);

}  // namespace scotty
