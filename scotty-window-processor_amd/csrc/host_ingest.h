// host_ingest.h -- host-to-HBM ingest of micro-batches handed over in host memory.
//
// The reference's callers hand tuples over one processElement at a time on the JVM heap; the C-ABI takes a
// micro-batch of host columns.  Moving them to HBM is PCIe-bound (~55 GB/s), so the path keeps the link busy:
//   * two pinned staging slots per operator, persistent (no per-push allocation); a caller that fills a slot
//     obtained from scotty_host_buffers hands over pinned memory, which is DMA'd in place with no CPU copy;
//   * pageable input is copied into the slots chunk by chunk, the CPU copy of chunk k+1 overlapping the DMA of
//     chunk k on a copy stream (events guard slot reuse);
//   * the device copies live in a bump arena reset at each watermark (pushes of the grid path stay resident until
//     then: a capacity overflow replays them), grown by whole chunks, so the steady state allocates nothing;
//   * the operator's compute stream waits on the copy stream's event: kernels of the push start as soon as the
//     last chunk lands, and the call returns without a device synchronisation.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace scotty {

class HostIngest {
 public:
  ~HostIngest();
  int init(int device, hipStream_t compute);
  // Pinned slot for up to n tuples (ts int64, value vb bytes, key uint32 if keyed); waits until the slot's last
  // DMA has finished.  Slots alternate between calls.
  hipError_t host_buffers(size_t n, size_t vb, bool keyed, int64_t** ts, void** val, uint32_t** key);
  // Device copies of host columns (pinned slot or pageable), enqueued ahead of the compute stream's next work.
  // persist: kept until reset() (else the copy may be overwritten by the next stage call).
  hipError_t stage(const int64_t* ts, const void* val, const uint32_t* key, size_t n, size_t vb, bool persist,
                   int64_t** d_ts, void** d_val, uint32_t** d_key);
  void reset();  // watermark: the arena's copies are no longer referenced
  uint64_t bytes_h2d = 0;

 private:
  struct Slot {
    unsigned char* h = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;
    bool pending = false;
  };
  hipError_t ensure_slot(Slot& s, size_t bytes);
  hipError_t wait_slot(Slot& s);
  hipError_t device_space(size_t bytes, bool persist, unsigned char** out);
  int slot_of(const void* p) const;
  hipError_t copy_columns(unsigned char* dst, const unsigned char* const* src, const size_t* width, int ncol,
                          size_t n, bool pinned_src);

  int device_ = 0;
  hipStream_t compute_ = nullptr, copy_ = nullptr;
  hipEvent_t landed_ = nullptr;
  Slot user_[2];   // handed out by host_buffers
  Slot chunk_[2];  // pageable input, chunk by chunk
  int next_user_ = 0, next_chunk_ = 0;
  // bump arena: chunks of device memory; the last one is filled, reset() keeps one chunk of the largest use seen
  std::vector<std::pair<unsigned char*, size_t>> chunks_;
  size_t used_ = 0, high_ = 0;
  unsigned char* scratch_ = nullptr;  // non-persistent copies (keyed pushes complete before the call returns)
  size_t scratch_bytes_ = 0;
};

}  // namespace scotty
