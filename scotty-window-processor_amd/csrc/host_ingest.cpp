// host_ingest.cpp -- see host_ingest.h.
#include "host_ingest.h"

#include <algorithm>
#include <cstring>

namespace scotty {

namespace {
constexpr size_t kChunkTuples = (size_t)1 << 22;  // pageable input: tuples per CPU copy / DMA chunk
size_t round16(size_t b) { return (b + 15) & ~(size_t)15; }
}  // namespace

#define HI_CHK(expr)                 \
  do {                               \
    hipError_t _e = (expr);          \
    if (_e != hipSuccess) return _e; \
  } while (0)

HostIngest::~HostIngest() {
  for (Slot* s0 : {&user_[0], &user_[1], &chunk_[0], &chunk_[1]}) {
    Slot& s = *s0;
    if (s.done) (void)hipEventSynchronize(s.done);
    if (s.h) (void)hipHostFree(s.h);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  if (copy_) (void)hipStreamSynchronize(copy_);
  for (auto& c : chunks_) (void)hipFree(c.first);
  if (scratch_) (void)hipFree(scratch_);
  if (landed_) (void)hipEventDestroy(landed_);
  if (copy_) (void)hipStreamDestroy(copy_);
}

int HostIngest::init(int device, hipStream_t compute) {
  device_ = device;
  compute_ = compute;
  if (hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking) != hipSuccess) return -1;
  if (hipEventCreateWithFlags(&landed_, hipEventDisableTiming) != hipSuccess) return -1;
  for (Slot* s : {&user_[0], &user_[1], &chunk_[0], &chunk_[1]})
    if (hipEventCreateWithFlags(&s->done, hipEventDisableTiming) != hipSuccess) return -1;
  return 0;
}

hipError_t HostIngest::wait_slot(Slot& s) {
  if (s.pending) {
    HI_CHK(hipEventSynchronize(s.done));
    s.pending = false;
  }
  return hipSuccess;
}

hipError_t HostIngest::ensure_slot(Slot& s, size_t bytes) {
  if (s.bytes >= bytes) return hipSuccess;
  HI_CHK(wait_slot(s));
  if (s.h) HI_CHK(hipHostFree(s.h));
  s.h = nullptr;
  s.bytes = 0;
  HI_CHK(hipHostMalloc((void**)&s.h, bytes, hipHostMallocDefault));
  s.bytes = bytes;
  return hipSuccess;
}

int HostIngest::slot_of(const void* p) const {
  const unsigned char* q = (const unsigned char*)p;
  for (int k = 0; k < 2; k++)
    if (user_[k].h && q >= user_[k].h && q < user_[k].h + user_[k].bytes) return k;
  return -1;
}

hipError_t HostIngest::host_buffers(size_t n, size_t vb, bool keyed, int64_t** ts, void** val, uint32_t** key) {
  Slot& s = user_[next_user_];
  next_user_ ^= 1;
  const size_t o_val = round16(n * 8), o_key = o_val + round16(n * vb);
  HI_CHK(ensure_slot(s, std::max<size_t>(o_key + (keyed ? round16(n * 4) : 0), 64)));
  HI_CHK(wait_slot(s));
  *ts = (int64_t*)s.h;
  *val = s.h + o_val;
  if (key) *key = keyed ? (uint32_t*)(s.h + o_key) : nullptr;
  return hipSuccess;
}

hipError_t HostIngest::device_space(size_t bytes, bool persist, unsigned char** out) {
  if (!persist) {
    if (scratch_bytes_ < bytes) {
      HI_CHK(hipStreamSynchronize(compute_));
      if (scratch_) HI_CHK(hipFree(scratch_));
      scratch_ = nullptr;
      HI_CHK(hipMalloc(&scratch_, bytes));
      scratch_bytes_ = bytes;
    }
    *out = scratch_;
    return hipSuccess;
  }
  if (chunks_.empty() || used_ + bytes > chunks_.back().second) {  // a new chunk; the older ones stay referenced
    unsigned char* p = nullptr;
    const size_t sz = std::max(bytes, std::max(high_, (size_t)1 << 26));
    HI_CHK(hipMalloc(&p, sz));
    chunks_.push_back({p, sz});
    used_ = 0;
  }
  *out = chunks_.back().first + used_;
  used_ += round16(bytes);
  return hipSuccess;
}

void HostIngest::reset() {
  size_t total = 0;
  for (size_t k = 0; k + 1 < chunks_.size(); k++) total += chunks_[k].second;
  total += used_;
  high_ = std::max(high_, total);
  if (chunks_.size() > 1) {  // merge: next interval's pushes fit one chunk
    for (auto& c : chunks_) (void)hipFree(c.first);
    chunks_.clear();
  }
  used_ = 0;
}

// Columns src[c] (width[c] bytes per tuple) -> dst packed as consecutive 16-byte-aligned columns.  Pinned source:
// one DMA per column.  Pageable: chunks through the two slots, CPU copy of the next chunk overlapping the DMA of
// the previous one.
hipError_t HostIngest::copy_columns(unsigned char* dst, const unsigned char* const* src, const size_t* width,
                                    int ncol, size_t n, bool pinned_src) {
  size_t off[3], o = 0;
  for (int c = 0; c < ncol; c++) {
    off[c] = o;
    o += round16(n * width[c]);
  }
  if (pinned_src) {
    for (int c = 0; c < ncol; c++)
      HI_CHK(hipMemcpyAsync(dst + off[c], src[c], n * width[c], hipMemcpyHostToDevice, copy_));
    bytes_h2d += o;
    return hipSuccess;
  }
  size_t per = 0;
  for (int c = 0; c < ncol; c++) per += width[c];
  const size_t chunk = std::min(n, kChunkTuples);
  for (size_t b = 0; b < n; b += chunk) {
    const size_t m = std::min(chunk, n - b);
    Slot& s = chunk_[next_chunk_];
    next_chunk_ ^= 1;
    HI_CHK(ensure_slot(s, chunk * per + 64 * ncol));
    HI_CHK(wait_slot(s));  // its previous DMA has read it
    size_t so = 0;
    for (int c = 0; c < ncol; c++) {
      std::memcpy(s.h + so, src[c] + b * width[c], m * width[c]);
      HI_CHK(hipMemcpyAsync(dst + off[c] + b * width[c], s.h + so, m * width[c], hipMemcpyHostToDevice, copy_));
      so += round16(m * width[c]);
    }
    HI_CHK(hipEventRecord(s.done, copy_));
    s.pending = true;
  }
  bytes_h2d += n * per;
  return hipSuccess;
}

hipError_t HostIngest::stage(const int64_t* ts, const void* val, const uint32_t* key, size_t n, size_t vb,
                             bool persist, int64_t** d_ts, void** d_val, uint32_t** d_key) {
  const size_t o_val = round16(n * 8), o_key = o_val + round16(n * vb);
  const size_t bytes = o_key + (key ? round16(n * 4) : 0);
  unsigned char* d = nullptr;
  HI_CHK(device_space(bytes, persist, &d));
  if (!persist) HI_CHK(hipStreamSynchronize(compute_));  // the scratch copy's previous reader is done
  // the copy stream starts after everything already queued on the compute stream that reads these bytes
  HI_CHK(hipEventRecord(landed_, compute_));
  HI_CHK(hipStreamWaitEvent(copy_, landed_, 0));
  const unsigned char* src[3] = {(const unsigned char*)ts, (const unsigned char*)val, (const unsigned char*)key};
  const size_t width[3] = {8, vb, 4};
  const int ncol = key ? 3 : 2;
  const int k = slot_of(ts);
  const bool pinned = k >= 0 && slot_of(val) == k && (!key || slot_of(key) == k);
  HI_CHK(copy_columns(d, src, width, ncol, n, pinned));
  if (pinned) {  // the caller's slot is free again once this DMA is done
    HI_CHK(hipEventRecord(user_[k].done, copy_));
    user_[k].pending = true;
  }
  HI_CHK(hipEventRecord(landed_, copy_));
  HI_CHK(hipStreamWaitEvent(compute_, landed_, 0));
  *d_ts = (int64_t*)d;
  *d_val = d + o_val;
  if (d_key) *d_key = key ? (uint32_t*)(d + o_key) : nullptr;
  return hipSuccess;
}

}  // namespace scotty
