// HBM GPU object store implementation. See gpu_store.h.
#include "gpu_store.h"

#include <stdlib.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace rmm {
namespace hip {

namespace {
constexpr uint64_t kAlignG = 256;
constexpr uint64_t kSpillChunk = 64ull << 20;  // input bytes per compression chunk
constexpr uint64_t kSpillMagic = 0x4c4c495053555047ull;  // "GPUSPILL"
inline uint64_t AlignG(uint64_t v) { return (v + kAlignG - 1) & ~(kAlignG - 1); }

ObjectId ToOid(const std::string& s) {
  ObjectId o;
  memset(o.b, 0, kIdSize);
  memcpy(o.b, s.data(), std::min<size_t>(s.size(), kIdSize));
  return o;
}

// Page-aligned hipHostRegister of [p, p+n) so DMA goes straight to/from the shm segment.
struct HostPin {
  void* base = nullptr;
  bool ok = false;
  HostPin(void* p, uint64_t n, bool already) {
    if (already) return;
    long pg = sysconf(_SC_PAGESIZE);
    uintptr_t a = reinterpret_cast<uintptr_t>(p) & ~uintptr_t(pg - 1);
    uintptr_t e = (reinterpret_cast<uintptr_t>(p) + n + pg - 1) & ~uintptr_t(pg - 1);
    base = reinterpret_cast<void*>(a);
    ok = hipHostRegister(base, e - a, hipHostRegisterDefault) == hipSuccess;
    if (!ok) (void)hipGetLastError();
  }
  ~HostPin() {
    if (ok) (void)hipHostUnregister(base);
  }
};
}  // namespace

std::string GpuStore::HostId(const std::string& id) {
  std::string h = id;
  h.resize(kIdSize, '\0');
  h[kIdSize - 1] = char(uint8_t(h[kIdSize - 1]) ^ 0xA5);
  h[0] = char(uint8_t(h[0]) ^ 0x5A);
  return h;
}

GpuStore::GpuStore(int device, uint64_t capacity, uint64_t slab_bytes, const std::string& shm_name,
                   bool compress_spill)
    : device_(device), capacity_(capacity), slab_bytes_(AlignG(slab_bytes)), compress_(compress_spill) {
  RMM_HIP_CHECK(hipSetDevice(device_));
  RMM_HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  RMM_HIP_CHECK(hipStreamCreateWithFlags(&side2_, hipStreamNonBlocking));
  if (!shm_name.empty()) {
    host_.reset(Store::Attach(shm_name));
    // Pin the whole host segment once so every spill/restore is a straight DMA (no per-spill
    // page pinning). Falls back to per-object pinning if the segment cannot be registered.
    if (getenv("RMM_GPU_NO_HOST_REGISTER") == nullptr &&
        hipHostRegister(host_->Base(), host_->MappedSize(), hipHostRegisterDefault) == hipSuccess)
      host_registered_ = true;
    else
      (void)hipGetLastError();
  }
  st_.capacity = capacity_;
}

GpuStore::~GpuStore() {
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
  if (host_registered_) (void)hipHostUnregister(host_->Base());
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
  // reuse an empty slot if any
  for (size_t i = 0; i < slabs_.size(); i++)
    if (!slabs_[i]) {
      slabs_[i] = std::move(s);
      return true;
    }
  slabs_.push_back(std::move(s));
  return true;
}

uint64_t GpuStore::AllocLocked(uint64_t nbytes, int* slab_out) {
  uint64_t need = AlignG(std::max<uint64_t>(nbytes, 1));
  for (int attempt = 0; attempt < 3; attempt++) {
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
    if (SpillLocked(need) == 0) break;
    attempt = 0;  // progress was made; keep trying
    if (lru_.empty() && !NewSlabLocked(need)) {
      // nothing more to spill
    }
  }
  throw std::runtime_error("GPU object store full: cannot allocate " + std::to_string(nbytes) + " bytes");
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
  std::lock_guard<std::mutex> g(mu_);
  RMM_HIP_CHECK(hipSetDevice(device_));
  if (objs_.count(id)) throw std::runtime_error("GPU object already exists");
  int slab;
  uint64_t off = AllocLocked(nbytes, &slab);
  GpuObject& o = objs_[id];
  o.slab = slab;
  o.offset = off;
  o.nbytes = nbytes;
  o.elem_bits = elem_bits;
  o.pins = 1;
  st_.num_objects++;
  st_.puts++;
  return reinterpret_cast<uint64_t>(slabs_[size_t(slab)]->base) + off;
}

void GpuStore::Seal(const std::string& id, hipStream_t stream) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(id);
  if (it == objs_.end()) throw std::runtime_error("Seal: unknown GPU object");
  GpuObject& o = it->second;
  if (!o.ready) RMM_HIP_CHECK(hipEventCreateWithFlags(&o.ready, hipEventDisableTiming));
  RMM_HIP_CHECK(hipEventRecord(o.ready, stream));
  o.sealed = true;
  if (--o.pins == 0) LruTouch(id, o);
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

uint64_t GpuStore::Get(const std::string& id, hipStream_t stream) {
  std::lock_guard<std::mutex> g(mu_);
  RMM_HIP_CHECK(hipSetDevice(device_));
  auto it = objs_.find(id);
  if (it == objs_.end()) return 0;
  GpuObject& o = it->second;
  if (o.spilled) {
    if (!RestoreLocked(id, o, stream)) throw std::runtime_error("failed to restore spilled GPU object");
  }
  if (o.ready) RMM_HIP_CHECK(hipStreamWaitEvent(stream, o.ready, 0));
  if (o.pins++ == 0) LruDrop(o);
  st_.gets++;
  return reinterpret_cast<uint64_t>(slabs_[size_t(o.slab)]->base) + o.offset;
}

void GpuStore::Release(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(id);
  if (it == objs_.end()) return;
  GpuObject& o = it->second;
  if (o.pins > 0 && --o.pins == 0 && o.sealed && !o.spilled) LruTouch(id, o);
}

bool GpuStore::Delete(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(id);
  if (it == objs_.end()) return false;
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
  return true;
}

bool GpuStore::Contains(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  return objs_.count(id) > 0;
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
  if (it == objs_.end() || it->second.spilled) return;
  if (it->second.ready) (void)hipEventSynchronize(it->second.ready);
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

// Host spill object layout: [magic][nbytes][elem_bits][nchunks][csize * nchunks] then chunks.
// csize == 0 marks a raw (uncompressed) chunk of min(kSpillChunk, remaining) bytes.
bool GpuStore::SpillOneLocked(const std::string& id, GpuObject& o) {
  if (!host_) return false;
  // A reader in another process may hold a zero-copy view through the descriptor: the flag can
  // only be set while nobody pins the descriptor, and readers that see it take the host path.
  if (!host_->TrySetFlag(ToOid(id), kFlagGpuSpilled)) return false;
  bool done = false;
  struct ClearOnFail {
    Store* s; ObjectId oid; bool* done;
    ~ClearOnFail() { if (!*done) s->ClearFlag(oid, kFlagGpuSpilled); }
  } guard{host_.get(), ToOid(id), &done};
  uint8_t* src = static_cast<uint8_t*>(slabs_[size_t(o.slab)]->base) + o.offset;
  if (o.ready) RMM_HIP_CHECK(hipStreamWaitEvent(side_, o.ready, 0));
  uint64_t nchunks = (o.nbytes + kSpillChunk - 1) / kSpillChunk;
  if (nchunks == 0) nchunks = 1;
  std::vector<uint64_t> csize(nchunks, 0);
  bool use_c = compress_ && (o.elem_bits == 16 || o.elem_bits == 32) && o.nbytes >= (1u << 20);
  uint64_t payload = 0;
  if (use_c) {
    EnsureScratch();
    uint64_t eb = uint64_t(o.elem_bits / 8);
    for (uint64_t c = 0; c < nchunks; c++) {
      uint64_t len = std::min(kSpillChunk, o.nbytes - c * kSpillChunk);
      uint64_t n = len / eb;
      uint64_t cs = (len % eb == 0) ? compress(src + c * kSpillChunk, n, o.elem_bits, scratch_[0], work_, side_) : 0;
      // keep the chunk compressed only if it saves >= 6 %
      csize[c] = (cs && cs < len - len / 16) ? cs : 0;
      payload += csize[c] ? csize[c] : len;
    }
  } else {
    payload = o.nbytes;
  }
  uint64_t hdr = (4 + nchunks) * 8;
  hdr = (hdr + 63) & ~uint64_t(63);
  ObjectId hid = ToOid(HostId(id));
  bool exists = false;
  uint8_t* dst = nullptr;
  try {
    dst = host_->CreateObject(hid, hdr + payload, 0, 0x47505553u /*GPUS*/, 0, &exists);
  } catch (const std::exception&) {
    return false;
  }
  if (exists) {
    host_->Delete(hid);
    return false;
  }
  uint64_t* h = reinterpret_cast<uint64_t*>(dst);
  h[0] = kSpillMagic;
  h[1] = o.nbytes;
  h[2] = uint64_t(o.elem_bits);
  h[3] = nchunks;
  for (uint64_t c = 0; c < nchunks; c++) h[4 + c] = csize[c];
  {
    HostPin pin(dst + hdr, payload, host_registered_);
    uint64_t doff = hdr;
    hipEvent_t done[2] = {nullptr, nullptr};
    RMM_HIP_CHECK(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
    RMM_HIP_CHECK(hipEventCreateWithFlags(&done[1], hipEventDisableTiming));
    for (uint64_t c = 0; c < nchunks; c++) {
      uint64_t len = std::min(kSpillChunk, o.nbytes - c * kSpillChunk);
      if (csize[c]) {
        int b = int(c & 1);
        // scratch[b] may still be read by the D2H of chunk c-2
        if (c >= 2) RMM_HIP_CHECK(hipStreamWaitEvent(side_, done[b], 0));
        uint64_t eb = uint64_t(o.elem_bits / 8);
        uint64_t cs = compress(src + c * kSpillChunk, len / eb, o.elem_bits, scratch_[b],
                               static_cast<uint8_t*>(work_) + uint64_t(b) * work_bytes_, side_);
        if (cs != csize[c]) throw std::runtime_error("spill compression is not deterministic");
        RMM_HIP_CHECK(hipMemcpyAsync(dst + doff, scratch_[b], cs, hipMemcpyDeviceToHost, side2_));
        RMM_HIP_CHECK(hipEventRecord(done[b], side2_));
        doff += cs;
      } else {
        hipEvent_t prod;
        RMM_HIP_CHECK(hipEventCreateWithFlags(&prod, hipEventDisableTiming));
        RMM_HIP_CHECK(hipEventRecord(prod, side_));
        RMM_HIP_CHECK(hipStreamWaitEvent(side2_, prod, 0));
        RMM_HIP_CHECK(hipMemcpyAsync(dst + doff, src + c * kSpillChunk, len, hipMemcpyDeviceToHost, side2_));
        RMM_HIP_CHECK(hipEventDestroy(prod));
        doff += len;
      }
    }
    RMM_HIP_CHECK(hipStreamSynchronize(side2_));
    RMM_HIP_CHECK(hipStreamSynchronize(side_));
    (void)hipEventDestroy(done[0]);
    (void)hipEventDestroy(done[1]);
  }
  host_->Seal(hid);
  host_->Release(hid);
  FreeLocked(o.slab, o.offset, o.nbytes);
  LruDrop(o);
  o.spilled = true;
  o.spill_bytes = hdr + payload;
  o.spill_compressed = use_c;
  o.slab = -1;
  st_.spilled_objects++;
  st_.spilled_bytes_total += o.nbytes;
  st_.spilled_host_bytes_total += payload;
  done = true;
  return true;
}

uint64_t GpuStore::SpillLocked(uint64_t bytes) {
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
    if (SpillOneLocked(victim, o)) freed += n;
  }
  return freed;
}

uint64_t GpuStore::Spill(uint64_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  RMM_HIP_CHECK(hipSetDevice(device_));
  return SpillLocked(bytes);
}

uint64_t GpuStore::SpillObject(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  RMM_HIP_CHECK(hipSetDevice(device_));
  auto it = objs_.find(id);
  if (it == objs_.end() || it->second.spilled || it->second.pins > 0) return 0;
  uint64_t n = it->second.nbytes;
  return SpillOneLocked(id, it->second) ? n : 0;
}

bool GpuStore::RestoreLocked(const std::string& id, GpuObject& o, hipStream_t stream) {
  if (!host_) return false;
  ObjectId hid = ToOid(HostId(id));
  Store::View v;
  if (!host_->Get(hid, 0, &v)) return false;
  const uint64_t* h = reinterpret_cast<const uint64_t*>(v.data);
  if (h[0] != kSpillMagic || h[1] != o.nbytes) {
    host_->Release(hid);
    return false;
  }
  uint64_t nchunks = h[3];
  uint64_t hdr = ((4 + nchunks) * 8 + 63) & ~uint64_t(63);
  int slab;
  uint64_t off;
  try {
    off = AllocLocked(o.nbytes, &slab);
  } catch (...) {
    host_->Release(hid);
    throw;
  }
  uint8_t* dst = static_cast<uint8_t*>(slabs_[size_t(slab)]->base) + off;
  {
    HostPin pin(v.data + hdr, v.data_size - hdr, host_registered_);
    uint64_t soff = hdr;
    bool any_c = false;
    for (uint64_t c = 0; c < nchunks; c++) any_c |= h[4 + c] != 0;
    if (any_c) EnsureScratch();
    hipEvent_t done[2] = {nullptr, nullptr};
    RMM_HIP_CHECK(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
    RMM_HIP_CHECK(hipEventCreateWithFlags(&done[1], hipEventDisableTiming));
    for (uint64_t c = 0; c < nchunks; c++) {
      uint64_t len = std::min(kSpillChunk, o.nbytes - c * kSpillChunk);
      uint64_t cs = h[4 + c];
      if (cs) {
        int b = int(c & 1);
        if (c >= 2) RMM_HIP_CHECK(hipStreamWaitEvent(side2_, done[b], 0));
        RMM_HIP_CHECK(hipMemcpyAsync(scratch_[b], v.data + soff, cs, hipMemcpyHostToDevice, side2_));
        hipEvent_t copied;
        RMM_HIP_CHECK(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
        RMM_HIP_CHECK(hipEventRecord(copied, side2_));
        RMM_HIP_CHECK(hipStreamWaitEvent(side_, copied, 0));
        uint64_t eb = uint64_t(o.elem_bits / 8);
        decompress(scratch_[b], dst + c * kSpillChunk, len / eb, o.elem_bits,
                   static_cast<uint8_t*>(work_) + uint64_t(b) * work_bytes_, side_);
        RMM_HIP_CHECK(hipEventRecord(done[b], side_));
        RMM_HIP_CHECK(hipEventDestroy(copied));
        soff += cs;
      } else {
        RMM_HIP_CHECK(hipMemcpyAsync(dst + c * kSpillChunk, v.data + soff, len, hipMemcpyHostToDevice, side2_));
        soff += len;
      }
    }
    RMM_HIP_CHECK(hipStreamSynchronize(side2_));
    RMM_HIP_CHECK(hipStreamSynchronize(side_));
    (void)hipEventDestroy(done[0]);
    (void)hipEventDestroy(done[1]);
  }
  host_->Release(hid);
  host_->Delete(hid);
  o.slab = slab;
  o.offset = off;
  o.spilled = false;
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
  st_.restored_bytes_total += o.nbytes;
  (void)stream;
  return true;
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
