// HBM GPU object store implementation. See gpu_store.h.
#include "gpu_store.h"

#include <stdlib.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace rmm {
namespace hip {

namespace {
constexpr uint64_t kAlignG = 256;
constexpr uint64_t kSpillChunk = 64ull << 20;  // input bytes per compression chunk
constexpr uint64_t kSpillMagic = 0x4c4c495053555047ull;   // "GPUSPILL": chunks packed back to back
constexpr uint64_t kSpillMagic2 = 0x324c495053555047ull;  // "GPUSPIL2": device-placed, each chunk 64-byte aligned
constexpr uint64_t kSpillMaxDeviceChunks = 4096;          // device-placed spills up to 256 GiB
constexpr uint32_t kTagGpuSpill = 0x47505553u;           // "GPUS"
inline uint64_t AlignG(uint64_t v) { return (v + kAlignG - 1) & ~(kAlignG - 1); }

ObjectId ToOid(const std::string& s) {
  ObjectId o;
  memset(o.b, 0, kIdSize);
  memcpy(o.b, s.data(), std::min<size_t>(s.size(), kIdSize));
  return o;
}

int64_t NowNs() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return int64_t(ts.tv_sec) * 1000000000ll + ts.tv_nsec;
}

// Host callback of SealDescriptorAsync: runs on a HIP runtime thread once the put's copy is
// done; touches only the shared-memory store (no HIP calls allowed here).
struct SealCtx {
  Store* host;
  ObjectId id;
};
void SealCallback(void* p) {
  SealCtx* c = static_cast<SealCtx*>(p);
  try {
    c->host->Seal(c->id);
  } catch (...) {
    // aborted meanwhile (creator died / deleted before sealing): nothing to publish
  }
  c->host->Release(c->id);
  delete c;
}

// Host spill object layout: [magic][nbytes][elem_bits][nchunks][csize * nchunks] then chunks.
// csize == 0 marks a raw (uncompressed) chunk of min(kSpillChunk, remaining) bytes.
inline uint64_t SpillHdrBytes(uint64_t nchunks) { return ((4 + nchunks) * 8 + 63) & ~uint64_t(63); }
}  // namespace

std::string GpuStore::HostId(const std::string& id) {
  std::string h = id;
  h.resize(kIdSize, '\0');
  h[kIdSize - 1] = char(uint8_t(h[kIdSize - 1]) ^ 0xA5);
  h[0] = char(uint8_t(h[0]) ^ 0x5A);
  return h;
}

GpuStore::GpuStore(int device, uint64_t capacity, uint64_t slab_bytes, const std::string& shm_name,
                   bool compress_spill, double spill_threshold, uint64_t prepin_bytes)
    : device_(device), capacity_(capacity), slab_bytes_(AlignG(slab_bytes)), compress_(compress_spill),
      spill_threshold_(spill_threshold) {
  RMM_HIP_CHECK(hipSetDevice(device_));
  RMM_HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  RMM_HIP_CHECK(hipStreamCreateWithFlags(&side2_, hipStreamNonBlocking));
  for (auto& e : ev_) RMM_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (!shm_name.empty()) {
    host_.reset(Store::Attach(shm_name));
    // spill / restore DMA pins 64 MB chunks of the host segment on first use (ingest_kernels.hip)
    host_register_segment(reinterpret_cast<uintptr_t>(host_->Base()), host_->MappedSize());
  }
  st_.capacity = capacity_;
  bg_ = std::thread([this] { BackgroundSpiller(); });
  if (host_ && prepin_bytes) {
    const uintptr_t base = reinterpret_cast<uintptr_t>(host_->Base());
    const uint64_t n = std::min<uint64_t>(prepin_bytes, host_->MappedSize());
    prepin_total_ = n;
    prepin_ = std::thread([this, base, n] {
      (void)hipSetDevice(device_);
      host_prepin(base, n, &prepin_stop_, &prepin_done_);
    });
  }
}

GpuStore::~GpuStore() {
  prepin_stop_ = true;
  if (prepin_.joinable()) prepin_.join();
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  bg_cv_.notify_all();
  if (bg_.joinable()) bg_.join();
  std::lock_guard<std::mutex> x(xfer_mu_);
  std::lock_guard<std::mutex> g(mu_);
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (auto& kv : objs_)
    if (kv.second.ready) (void)hipEventDestroy(kv.second.ready);
  for (auto& s : slabs_)
    if (s && s->base) (void)hipFree(s->base);
  for (auto p : scratch_)
    if (p) (void)hipFree(p);
  if (work_) (void)hipFree(work_);
  if (spill_meta_) (void)hipFree(spill_meta_);
  for (auto e : ev_)
    if (e) (void)hipEventDestroy(e);
  if (host_) host_unregister_segment(reinterpret_cast<uintptr_t>(host_->Base()));
  if (side_) (void)hipStreamDestroy(side_);
  if (side2_) (void)hipStreamDestroy(side2_);
}

bool GpuStore::NewSlabLocked(uint64_t min_bytes) {
  bool dedicated = min_bytes > slab_bytes_;
  uint64_t sz = dedicated ? AlignG(min_bytes) : slab_bytes_;
  if (allocated_ + sz > capacity_) {
    if (allocated_ >= capacity_) return false;
    // last partial slab
    if (!dedicated && capacity_ - allocated_ >= min_bytes) sz = AlignG(capacity_ - allocated_) - kAlignG;
    else return false;
    if (sz < min_bytes) return false;
  }
  void* p = nullptr;
  if (hipMalloc(&p, sz) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  auto s = std::make_unique<Slab>();
  s->base = p;
  s->size = sz;
  s->dedicated = dedicated;
  s->free_by_off[0] = sz;
  s->free_by_size.insert({sz, 0});
  if (hipIpcGetMemHandle(&s->ipc, p) == hipSuccess) s->ipc_valid = true;
  else (void)hipGetLastError();
  allocated_ += sz;
  st_.slab_bytes_allocated = allocated_;
  for (size_t i = 0; i < slabs_.size(); i++)
    if (!slabs_[i]) {
      slabs_[i] = std::move(s);
      return true;
    }
  slabs_.push_back(std::move(s));
  return true;
}

uint64_t GpuStore::AllocLocked(Lock& lk, uint64_t nbytes, int* slab_out) {
  uint64_t need = AlignG(std::max<uint64_t>(nbytes, 1));
  for (;;) {
    // best fit across slabs
    int best = -1;
    uint64_t best_size = UINT64_MAX, best_off = 0;
    for (size_t i = 0; i < slabs_.size(); i++) {
      Slab* s = slabs_[i].get();
      if (!s) continue;
      auto it = s->free_by_size.lower_bound(need);
      if (it != s->free_by_size.end() && it->first < best_size) {
        best = int(i);
        best_size = it->first;
        best_off = it->second;
      }
    }
    if (best >= 0) {
      Slab* s = slabs_[size_t(best)].get();
      auto range = s->free_by_size.equal_range(best_size);
      for (auto it = range.first; it != range.second; ++it)
        if (it->second == best_off) {
          s->free_by_size.erase(it);
          break;
        }
      s->free_by_off.erase(best_off);
      if (best_size > need) {
        s->free_by_off[best_off + need] = best_size - need;
        s->free_by_size.insert({best_size - need, best_off + need});
      }
      s->used += need;
      st_.bytes_in_use += need;
      *slab_out = best;
      return best_off;
    }
    if (NewSlabLocked(need)) continue;
    // free empty dedicated slabs, then spill
    bool freed_slab = false;
    for (auto& s : slabs_)
      if (s && s->used == 0 && s->dedicated) {
        (void)hipFree(s->base);
        allocated_ -= s->size;
        s.reset();
        freed_slab = true;
      }
    st_.slab_bytes_allocated = allocated_;
    if (freed_slab) continue;
    if (SpillLocked(lk, need) > 0) continue;
    if (spills_in_flight_ > 0) {  // another thread is freeing memory right now: wait for it
      cv_.wait(lk);
      continue;
    }
    throw std::runtime_error("GPU object store full: cannot allocate " + std::to_string(nbytes) + " bytes");
  }
}

void GpuStore::FreeLocked(int slab, uint64_t off, uint64_t nbytes) {
  Slab* s = slabs_[size_t(slab)].get();
  uint64_t sz = AlignG(std::max<uint64_t>(nbytes, 1));
  s->used -= sz;
  st_.bytes_in_use -= sz;
  auto erase_size = [&](uint64_t size, uint64_t o) {
    auto range = s->free_by_size.equal_range(size);
    for (auto it = range.first; it != range.second; ++it)
      if (it->second == o) {
        s->free_by_size.erase(it);
        return;
      }
  };
  auto next = s->free_by_off.lower_bound(off);
  if (next != s->free_by_off.end() && next->first == off + sz) {
    sz += next->second;
    erase_size(next->second, next->first);
    next = s->free_by_off.erase(next);
  }
  if (next != s->free_by_off.begin()) {
    auto prev = std::prev(next);
    if (prev->first + prev->second == off) {
      erase_size(prev->second, prev->first);
      off = prev->first;
      sz += prev->second;
      s->free_by_off.erase(prev);
    }
  }
  s->free_by_off[off] = sz;
  s->free_by_size.insert({sz, off});
  cv_.notify_all();
}

void GpuStore::LruTouch(const std::string& id, GpuObject& o) {
  if (o.in_lru) lru_.erase(o.lru);
  lru_.push_back(id);
  o.lru = std::prev(lru_.end());
  o.in_lru = true;
}
void GpuStore::LruDrop(GpuObject& o) {
  if (o.in_lru) {
    lru_.erase(o.lru);
    o.in_lru = false;
  }
}

uint64_t GpuStore::Create(const std::string& id, uint64_t nbytes, int elem_bits) {
  Lock lk(mu_);
  RMM_HIP_CHECK(hipSetDevice(device_));
  if (objs_.count(id)) throw std::runtime_error("GPU object already exists");
  int slab;
  uint64_t off = AllocLocked(lk, nbytes, &slab);
  if (objs_.count(id)) {  // the lock was released while spilling: re-check
    FreeLocked(slab, off, nbytes);
    throw std::runtime_error("GPU object already exists");
  }
  GpuObject& o = objs_[id];
  o.slab = slab;
  o.offset = off;
  o.nbytes = nbytes;
  o.elem_bits = elem_bits;
  o.pins = 1;
  st_.num_objects++;
  st_.puts++;
  uint64_t ptr = reinterpret_cast<uint64_t>(slabs_[size_t(slab)]->base) + off;
  if (spill_threshold_ > 0 && double(st_.bytes_in_use) > spill_threshold_ * double(capacity_)) bg_cv_.notify_all();
  return ptr;
}

void GpuStore::Seal(const std::string& id, hipStream_t stream) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(id);
  if (it == objs_.end()) throw std::runtime_error("Seal: unknown GPU object");
  GpuObject& o = it->second;
  if (!o.ready) RMM_HIP_CHECK(hipEventCreateWithFlags(&o.ready, hipEventDisableTiming));
  RMM_HIP_CHECK(hipEventRecord(o.ready, stream));
  o.sealed = true;
  if (--o.pins == 0) {
    if (o.delete_pending) DeleteLocked(id);
    else LruTouch(id, o);
  }
}

uint64_t GpuStore::PutSegments(const std::string& id, const std::vector<std::pair<uint64_t, uint64_t>>& segs,
                               int elem_bits, hipStream_t stream) {
  uint64_t total = 0;
  for (auto& s : segs) total += s.second;
  uint64_t dst = Create(id, total, elem_bits);
  std::vector<CopySeg> cs;
  cs.reserve(segs.size());
  uint64_t off = 0;
  for (auto& s : segs) {
    cs.push_back({s.first, dst + off, s.second});
    off += s.second;
  }
  multi_copy(cs, stream);
  Seal(id, stream);
  return dst;
}

void GpuStore::SealDescriptorAsync(const std::string& desc_id, hipStream_t stream) {
  if (!host_) throw std::runtime_error("SealDescriptorAsync: no host store attached");
  auto* c = new SealCtx{host_.get(), ToOid(desc_id)};
  hipError_t e = hipLaunchHostFunc(stream, SealCallback, c);
  if (e != hipSuccess) {  // fall back to a synchronous seal
    (void)hipGetLastError();
    RMM_HIP_CHECK(hipStreamSynchronize(stream));
    SealCallback(c);
  }
}

void GpuStore::WaitIdleLocked(Lock& lk, const std::string& id) {
  for (;;) {
    auto it = objs_.find(id);
    if (it == objs_.end() || (!it->second.spilling && !it->second.restoring)) return;
    cv_.wait(lk);
  }
}

uint64_t GpuStore::Get(const std::string& id, hipStream_t stream) {
  Lock lk(mu_);
  RMM_HIP_CHECK(hipSetDevice(device_));
  for (;;) {
    WaitIdleLocked(lk, id);
    auto it = objs_.find(id);
    if (it == objs_.end() || it->second.delete_pending) return 0;
    GpuObject& o = it->second;
    if (o.spilled) {
      if (!RestoreOne(lk, id, &o)) throw std::runtime_error("failed to restore spilled GPU object");
      continue;  // re-validate after the lock was released
    }
    if (o.ready) RMM_HIP_CHECK(hipStreamWaitEvent(stream, o.ready, 0));
    if (o.pins++ == 0) LruDrop(o);
    st_.gets++;
    return reinterpret_cast<uint64_t>(slabs_[size_t(o.slab)]->base) + o.offset;
  }
}

void GpuStore::Release(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(id);
  if (it == objs_.end()) return;
  GpuObject& o = it->second;
  if (o.pins > 0 && --o.pins == 0) {
    if (o.delete_pending) DeleteLocked(id);
    else if (o.sealed && !o.spilled) LruTouch(id, o);
  }
}

void GpuStore::DeleteLocked(const std::string& id) {
  auto it = objs_.find(id);
  if (it == objs_.end()) return;
  GpuObject& o = it->second;
  LruDrop(o);
  if (!o.spilled) {
    // the producing copy may still be in flight: wait before recycling the memory
    if (o.ready) (void)hipEventSynchronize(o.ready);
    FreeLocked(o.slab, o.offset, o.nbytes);
  } else if (host_) {
    host_->Delete(ToOid(HostId(id)));
  }
  if (o.ready) (void)hipEventDestroy(o.ready);
  objs_.erase(it);
  st_.num_objects--;
}

bool GpuStore::Delete(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(id);
  if (it == objs_.end()) return false;
  GpuObject& o = it->second;
  if (o.pins > 0 || o.spilling || o.restoring) {
    // a zero-copy view (or a transfer) still uses the memory: free on the last Release /
    // when the transfer finishes
    if (!o.delete_pending) st_.deferred_deletes++;
    o.delete_pending = true;
    LruDrop(o);
    return true;
  }
  DeleteLocked(id);
  return true;
}

bool GpuStore::Contains(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(id);
  return it != objs_.end() && !it->second.delete_pending;
}

bool GpuStore::IsSpilled(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(id);
  return it != objs_.end() && it->second.spilled;
}

void GpuStore::Locate(const std::string& id, int* slab, uint64_t* offset, uint64_t* nbytes) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(id);
  *slab = -1;
  if (it == objs_.end() || it->second.spilled || it->second.spilling) return;
  *slab = it->second.slab;
  *offset = it->second.offset;
  *nbytes = it->second.nbytes;
}

std::string GpuStore::SlabIpcHandle(int slab) {
  std::lock_guard<std::mutex> g(mu_);
  if (slab < 0 || size_t(slab) >= slabs_.size() || !slabs_[size_t(slab)] || !slabs_[size_t(slab)]->ipc_valid)
    return std::string();
  return std::string(reinterpret_cast<const char*>(&slabs_[size_t(slab)]->ipc), sizeof(hipIpcMemHandle_t));
}

uint64_t GpuStore::SlabBase(int slab) {
  std::lock_guard<std::mutex> g(mu_);
  if (slab < 0 || size_t(slab) >= slabs_.size() || !slabs_[size_t(slab)]) return 0;
  return reinterpret_cast<uint64_t>(slabs_[size_t(slab)]->base);
}

void GpuStore::EnsureScratch() {
  if (scratch_[0]) return;
  uint64_t n16 = kSpillChunk / 2;  // worst case element count per chunk (16-bit)
  scratch_bytes_ = std::max(compress_bound(n16, 16), compress_bound(kSpillChunk / 4, 32));
  work_bytes_ = compress_workspace(n16);
  for (auto& p : scratch_) RMM_HIP_CHECK(hipMalloc(&p, scratch_bytes_));
  RMM_HIP_CHECK(hipMalloc(&work_, 2 * work_bytes_));
}

// ---------------------------------------------------------------- spill

void GpuStore::ClearStaleError(const char* where) {
  // HIP's last-error is sticky per thread: an unchecked failure of an unrelated earlier call
  // (another library on this thread) must not be reported by our kernels' launch checks
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    std::lock_guard<std::mutex> g(err_mu_);
    stale_errors_++;
    last_stale_ = std::string(where) + ": " + hipGetErrorString(e);
  }
}

namespace {
// device-placed spill chunks (SpillTransfer): RMM_SPILL_DEVICE_PLACE=1 / 0 overrides the default
bool SpillDevicePlace() {
  const char* e = std::getenv("RMM_SPILL_DEVICE_PLACE");
  return e ? std::atoi(e) != 0 : false;
}
}  // namespace

bool GpuStore::SpillTransfer(const std::string& id, const uint8_t* src, uint64_t nbytes, int elem_bits,
                             hipEvent_t ready, uint64_t* host_bytes, bool* compressed) {
  RMM_HIP_CHECK(hipSetDevice(device_));
  ClearStaleError("spill");
  uint64_t nchunks = std::max<uint64_t>(1, (nbytes + kSpillChunk - 1) / kSpillChunk);
  const bool use_c = compress_ && (elem_bits == 16 || elem_bits == 32) && nbytes >= (1u << 20);
  const uint64_t hdr = SpillHdrBytes(nchunks);
  const ObjectId hid = ToOid(HostId(id));
  bool exists = false;
  uint8_t* dst = nullptr;
  try {
    dst = host_->CreateObject(hid, hdr + nbytes, 0, kTagGpuSpill, 0, &exists);  // worst case: all raw
  } catch (const std::exception&) {
    return false;
  }
  if (exists) {
    host_->Delete(hid);
    return false;
  }
  struct AbortGuard {  // a failed transfer must not leave a half-written CREATING object behind
    Store* s;
    ObjectId id;
    bool done = false;
    ~AbortGuard() {
      if (!done) s->Abort(id);
    }
  } guard{host_.get(), hid};
  host_pin_range(dst, hdr + nbytes);
  if (use_c) EnsureScratch();
  if (ready) RMM_HIP_CHECK(hipStreamWaitEvent(side_, ready, 0));
  // Device-placed chunks (RMM_SPILL_DEVICE_PLACE=1): the compressed size of chunk c never comes back to the host
  // before chunk c is written; a copy kernel writes it at a device-resident cursor into the arena's device
  // mapping, so compression of chunk c+1 and the PCIe write of chunk c run back to back without host round trips.
  uint8_t* dst_dev = nullptr;
  if (use_c && nchunks <= kSpillMaxDeviceChunks && SpillDevicePlace()) {
    void* d0 = nullptr;
    void* d1 = nullptr;
    const uint64_t span = hdr + nbytes;
    bool ok = hipHostGetDevicePointer(&d0, dst, 0) == hipSuccess &&
              hipHostGetDevicePointer(&d1, dst + span - 1, 0) == hipSuccess &&
              static_cast<uint8_t*>(d1) - static_cast<uint8_t*>(d0) == int64_t(span - 1);
    for (uint64_t o = (64ull << 20); ok && o < span; o += (64ull << 20)) {  // contiguous across registrations
      void* dm = nullptr;
      ok = hipHostGetDevicePointer(&dm, dst + o, 0) == hipSuccess && static_cast<uint8_t*>(dm) - static_cast<uint8_t*>(d0) == int64_t(o);
    }
    (void)hipGetLastError();
    if (ok && (reinterpret_cast<uintptr_t>(src) & 15) == 0) dst_dev = static_cast<uint8_t*>(d0);
  }
  if (dst_dev) {
    if (!spill_meta_) RMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&spill_meta_), 8 * (1 + kSpillMaxDeviceChunks)));
    RMM_HIP_CHECK(hipMemsetAsync(spill_meta_, 0, 8 * (1 + nchunks), side2_));
    const uint64_t eb = uint64_t(elem_bits / 8);
    for (uint64_t c = 0; c < nchunks; c++) {
      const uint64_t len = std::min(kSpillChunk, nbytes - c * kSpillChunk);
      const uint8_t* sc = src + c * kSpillChunk;
      const int b = int(c & 1);
      const bool try_c = len % eb == 0;
      if (try_c) {
        if (c >= 2) RMM_HIP_CHECK(hipStreamWaitEvent(side_, ev_[b], 0));  // the commit that last read scratch[b]
        compress(sc, len / eb, elem_bits, scratch_[b], static_cast<uint8_t*>(work_) + uint64_t(b) * work_bytes_, side_,
                 /*readback=*/false);
      }
      RMM_HIP_CHECK(hipEventRecord(ev_[2], side_));  // orders after `ready` and this chunk's compression
      RMM_HIP_CHECK(hipStreamWaitEvent(side2_, ev_[2], 0));
      spill_commit(scratch_[b], sc, len, try_c, dst_dev + hdr, spill_meta_, spill_meta_ + 1 + c, side2_);
      RMM_HIP_CHECK(hipEventRecord(ev_[b], side2_));
    }
    std::vector<uint64_t> meta(1 + nchunks, 0);
    RMM_HIP_CHECK(hipMemcpyAsync(meta.data(), spill_meta_, 8 * (1 + nchunks), hipMemcpyDeviceToHost, side2_));
    RMM_HIP_CHECK(hipStreamSynchronize(side2_));
    RMM_HIP_CHECK(hipStreamSynchronize(side_));
    uint64_t* h = reinterpret_cast<uint64_t*>(dst);
    for (uint64_t c = 0; c < nchunks; c++) h[4 + c] = meta[1 + c];
    h[1] = nbytes;
    h[2] = uint64_t(elem_bits);
    h[3] = nchunks;
    h[0] = kSpillMagic2;  // header last
    const uint64_t doff = hdr + meta[0];
    host_->ShrinkCreating(hid, doff);
    host_->Seal(hid);
    host_->Release(hid);
    guard.done = true;
    *host_bytes = doff;
    *compressed = true;
    st_.spills_device_placed++;
    return true;
  }
  std::vector<uint64_t> csize(nchunks, 0);
  uint64_t doff = hdr;
  hipEvent_t* done = ev_;  // done[b]: the D2H that last read scratch[b]
  const uint64_t eb = use_c ? uint64_t(elem_bits / 8) : 1;
  for (uint64_t c = 0; c < nchunks; c++) {
    const uint64_t len = std::min(kSpillChunk, nbytes - c * kSpillChunk);
    const uint8_t* s = src + c * kSpillChunk;
    uint64_t cs = 0;
    const int b = int(c & 1);
    if (use_c && len % eb == 0) {
      if (c >= 2) RMM_HIP_CHECK(hipStreamWaitEvent(side_, done[b], 0));
      // ONE compression pass; compress() reads the total back (stream sync on side_)
      cs = compress(s, len / eb, elem_bits, scratch_[b], static_cast<uint8_t*>(work_) + uint64_t(b) * work_bytes_,
                    side_);
      if (cs >= len - len / 16) cs = 0;  // keep compressed only if it saves >= 6 %
    }
    if (cs) {
      RMM_HIP_CHECK(hipEventRecord(ev_[2], side_));
      RMM_HIP_CHECK(hipStreamWaitEvent(side2_, ev_[2], 0));
      dma_host_segment(dst + doff, scratch_[b], cs, false, side2_);
      RMM_HIP_CHECK(hipEventRecord(done[b], side2_));
      doff += cs;
    } else {
      RMM_HIP_CHECK(hipEventRecord(ev_[2], side_));  // orders after `ready`
      RMM_HIP_CHECK(hipStreamWaitEvent(side2_, ev_[2], 0));
      dma_host_segment(dst + doff, const_cast<uint8_t*>(s), len, false, side2_);
      doff += len;
    }
    csize[c] = cs;
  }
  RMM_HIP_CHECK(hipStreamSynchronize(side2_));
  RMM_HIP_CHECK(hipStreamSynchronize(side_));
  // header last: a reader never sees a complete header over incomplete chunks
  uint64_t* h = reinterpret_cast<uint64_t*>(dst);
  for (uint64_t c = 0; c < nchunks; c++) h[4 + c] = csize[c];
  h[1] = nbytes;
  h[2] = uint64_t(elem_bits);
  h[3] = nchunks;
  h[0] = kSpillMagic;
  host_->ShrinkCreating(hid, doff);
  host_->Seal(hid);
  host_->Release(hid);
  guard.done = true;
  *host_bytes = doff;
  *compressed = use_c;
  return true;
}

bool GpuStore::SpillOne(Lock& lk, const std::string& id) {
  if (!host_) return false;
  auto it = objs_.find(id);
  if (it == objs_.end()) return false;
  GpuObject& o = it->second;
  if (o.pins > 0 || o.spilled || o.spilling || o.restoring || !o.sealed || o.delete_pending) return false;
  // A reader in another process may hold a zero-copy view through the descriptor: the flag can
  // only be set while nobody pins the descriptor, and readers that see it take the host path.
  if (!host_->TrySetFlag(ToOid(id), kFlagGpuSpilled)) return false;
  o.spilling = true;
  LruDrop(o);
  spills_in_flight_++;
  const uint8_t* src = static_cast<uint8_t*>(slabs_[size_t(o.slab)]->base) + o.offset;
  const uint64_t nbytes = o.nbytes;
  const int bits = o.elem_bits;
  hipEvent_t ready = o.ready;
  lk.unlock();
  uint64_t host_bytes = 0;
  bool compressed = false, ok = false;
  const int64_t t0 = NowNs();
  try {
    std::lock_guard<std::mutex> x(xfer_mu_);
    ok = SpillTransfer(id, src, nbytes, bits, ready, &host_bytes, &compressed);
  } catch (const std::exception& e) {
    ok = false;
    std::lock_guard<std::mutex> g(err_mu_);
    last_error_ = e.what();
  } catch (...) {
    ok = false;
  }
  const int64_t t1 = NowNs();
  lk.lock();
  spills_in_flight_--;
  auto jt = objs_.find(id);
  if (jt == objs_.end()) {  // cannot happen (Delete defers while spilling); be safe
    cv_.notify_all();
    return ok;
  }
  GpuObject& p = jt->second;
  p.spilling = false;
  if (!ok) {
    host_->ClearFlag(ToOid(id), kFlagGpuSpilled);
    if (p.delete_pending && p.pins == 0) DeleteLocked(id);
    else if (p.pins == 0) LruTouch(id, p);
    cv_.notify_all();
    return false;
  }
  FreeLocked(p.slab, p.offset, p.nbytes);
  p.spilled = true;
  p.spill_bytes = host_bytes;
  p.spill_compressed = compressed;
  p.slab = -1;
  st_.spilled_objects++;
  st_.spilled_bytes_total += nbytes;
  st_.spilled_host_bytes_total += host_bytes;
  st_.spill_ns_total += uint64_t(t1 - t0);
  if (p.delete_pending && p.pins == 0) DeleteLocked(id);
  cv_.notify_all();
  return true;
}

uint64_t GpuStore::SpillLocked(Lock& lk, uint64_t bytes) {
  uint64_t freed = 0;
  std::vector<std::string> order(lru_.begin(), lru_.end());
  for (auto& victim : order) {
    if (freed >= bytes) break;
    auto it = objs_.find(victim);
    if (it == objs_.end()) continue;
    GpuObject& o = it->second;
    if (o.pins > 0 || o.spilled) {
      LruDrop(o);
      continue;
    }
    uint64_t n = AlignG(o.nbytes);
    if (SpillOne(lk, victim)) freed += n;
  }
  return freed;
}

uint64_t GpuStore::Spill(uint64_t bytes) {
  Lock lk(mu_);
  RMM_HIP_CHECK(hipSetDevice(device_));
  return SpillLocked(lk, bytes);
}

uint64_t GpuStore::SpillObject(const std::string& id) {
  Lock lk(mu_);
  RMM_HIP_CHECK(hipSetDevice(device_));
  auto it = objs_.find(id);
  if (it == objs_.end() || it->second.spilled || it->second.pins > 0) return 0;
  uint64_t n = it->second.nbytes;
  return SpillOne(lk, id) ? n : 0;
}

void GpuStore::SetSpillThreshold(double t) {
  {
    std::lock_guard<std::mutex> g(mu_);
    spill_threshold_ = t;
  }
  bg_cv_.notify_all();
}

void GpuStore::BackgroundSpiller() {
  (void)hipSetDevice(device_);
  Lock lk(mu_);
  while (!stop_) {
    bg_cv_.wait_for(lk, std::chrono::milliseconds(50));
    if (stop_) break;
    if (spill_threshold_ <= 0 || !host_) continue;
    const double hi = spill_threshold_ * double(capacity_);
    if (double(st_.bytes_in_use) <= hi) continue;
    // spill down to a low watermark 5 % of the capacity below the threshold
    const double lo = std::max(0.0, spill_threshold_ - 0.05) * double(capacity_);
    const uint64_t excess = uint64_t(double(st_.bytes_in_use) - lo);
    const uint64_t before = st_.spilled_objects;
    SpillLocked(lk, excess);
    st_.proactive_spills += st_.spilled_objects - before;
  }
}

// ---------------------------------------------------------------- restore

uint64_t GpuStore::RestoreTransfer(const std::string& host_id, uint8_t* dst, uint64_t nbytes, bool delete_host) {
  RMM_HIP_CHECK(hipSetDevice(device_));
  ClearStaleError("restore");
  const ObjectId hid = ToOid(host_id);
  Store::View v;
  if (!host_->Get(hid, 0, &v)) return 0;
  const uint64_t* h = reinterpret_cast<const uint64_t*>(v.data);
  if ((h[0] != kSpillMagic && h[0] != kSpillMagic2) || h[1] != nbytes) {
    host_->Release(hid);
    return 0;
  }
  const int bits = int(h[2]);
  const uint64_t nchunks = h[3];
  const uint64_t hdr = SpillHdrBytes(nchunks);
  host_pin_range(v.data, v.data_size);
  bool any_c = false;
  for (uint64_t c = 0; c < nchunks; c++) any_c |= h[4 + c] != 0;
  if (any_c) EnsureScratch();
  uint64_t soff = hdr;
  const uint64_t amask = h[0] == kSpillMagic2 ? 63 : 0;  // device-placed chunks start 64-byte aligned
  hipEvent_t* done = ev_;  // done[b]: the decompression that last read scratch[b]
  for (uint64_t c = 0; c < nchunks; c++) {
    const uint64_t len = std::min(kSpillChunk, nbytes - c * kSpillChunk);
    const uint64_t cs = h[4 + c];
    if (cs) {
      const int b = int(c & 1);
      if (c >= 2) RMM_HIP_CHECK(hipStreamWaitEvent(side2_, done[b], 0));
      dma_host_segment(const_cast<uint8_t*>(v.data) + soff, scratch_[b], cs, true, side2_);
      RMM_HIP_CHECK(hipEventRecord(ev_[2 + b], side2_));
      RMM_HIP_CHECK(hipStreamWaitEvent(side_, ev_[2 + b], 0));
      const uint64_t eb = uint64_t(bits / 8);
      decompress(scratch_[b], dst + c * kSpillChunk, len / eb, bits,
                 static_cast<uint8_t*>(work_) + uint64_t(b) * work_bytes_, side_);
      RMM_HIP_CHECK(hipEventRecord(done[b], side_));
      soff += (cs + amask) & ~amask;
    } else {
      dma_host_segment(const_cast<uint8_t*>(v.data) + soff, dst + c * kSpillChunk, len, true, side2_);
      soff += (len + amask) & ~amask;
    }
  }
  RMM_HIP_CHECK(hipStreamSynchronize(side2_));
  RMM_HIP_CHECK(hipStreamSynchronize(side_));
  host_->Release(hid);
  if (delete_host) host_->Delete(hid);
  return nbytes;
}

bool GpuStore::RestoreOne(Lock& lk, const std::string& id, GpuObject* o) {
  if (!host_) return false;
  int slab;
  const uint64_t want = o->nbytes;  // `o` may dangle once the lock is released below
  const uint64_t off = AllocLocked(lk, want, &slab);  // may spill others (lock released)
  auto it = objs_.find(id);
  if (it == objs_.end() || !it->second.spilled || it->second.restoring) {  // raced: give the memory back
    FreeLocked(slab, off, want);
    return true;
  }
  GpuObject& p = it->second;
  p.restoring = true;
  const uint64_t nbytes = p.nbytes;
  uint8_t* dst = static_cast<uint8_t*>(slabs_[size_t(slab)]->base) + off;
  lk.unlock();
  uint64_t got = 0;
  const int64_t t0 = NowNs();
  try {
    std::lock_guard<std::mutex> x(xfer_mu_);
    got = RestoreTransfer(HostId(id), dst, nbytes, true);
  } catch (const std::exception& e) {
    got = 0;
    std::lock_guard<std::mutex> g(err_mu_);
    last_error_ = e.what();
  } catch (...) {
    got = 0;
  }
  const int64_t t1 = NowNs();
  lk.lock();
  auto jt = objs_.find(id);
  GpuObject& q = jt->second;
  q.restoring = false;
  if (got != nbytes) {
    FreeLocked(slab, off, nbytes);
    // a Delete() during the transfer only marked the object: it is still spilled, so this frees
    // its host copy and the entry (nothing else would: no pins, so no Release follows)
    if (q.delete_pending && q.pins == 0) DeleteLocked(id);
    cv_.notify_all();
    return false;
  }
  q.slab = slab;
  q.offset = off;
  q.spilled = false;  // the data is in place: the transfer synchronised its streams
  // publish the new location to cross-process readers, then clear the spilled flag
  {
    Slab* sl = slabs_[size_t(slab)].get();
    ObjectId did = ToOid(id);
    host_->WithLockedData(did, [&](uint8_t* d, uint32_t) {
      GpuDesc* g = reinterpret_cast<GpuDesc*>(d);
      if (g->magic == kGpuDescMagic) {
        g->slab = slab;
        g->offset = off;
        memcpy(g->ipc, &sl->ipc, sizeof(g->ipc));
      }
    });
    host_->ClearFlag(did, kFlagGpuSpilled);
  }
  st_.restored_bytes_total += nbytes;
  st_.restore_ns_total += uint64_t(t1 - t0);
  if (q.delete_pending && q.pins == 0) DeleteLocked(id);
  else if (q.pins == 0) LruTouch(id, q);
  cv_.notify_all();
  return true;
}

uint64_t GpuStore::RestoreForeign(const std::string& host_id, uint64_t dst, uint64_t nbytes) {
  if (!host_) throw std::runtime_error("RestoreForeign: no host store attached");
  std::lock_guard<std::mutex> x(xfer_mu_);
  const int64_t t0 = NowNs();
  uint64_t n = RestoreTransfer(host_id, reinterpret_cast<uint8_t*>(dst), nbytes, false);
  std::lock_guard<std::mutex> g(mu_);
  st_.restored_bytes_total += n;
  st_.restore_ns_total += uint64_t(NowNs() - t0);
  return n;
}

std::string GpuStore::LastError() {
  std::lock_guard<std::mutex> g(err_mu_);
  if (stale_errors_) return last_error_ + " [stale errors cleared: " + std::to_string(stale_errors_) + ", last: " +
                            last_stale_ + "]";
  return last_error_;
}

GpuStats GpuStore::Stats() {
  std::lock_guard<std::mutex> g(mu_);
  GpuStats s = st_;
  s.capacity = capacity_;
  s.slab_bytes_allocated = allocated_;
  return s;
}

}  // namespace hip
}  // namespace rmm
