// HBM-resident GPU object store (one per process per device).
//
// North-star component with no reference equivalent: the reference pickles CUDA tensors
// through host memory (python/ray/_private/serialization.py). Here objects stay in HBM:
//  * slab arena: lazily hipMalloc'ed slabs (default 8 GiB; objects larger than a slab get a
//    dedicated slab) up to `capacity` — sized for 288 GB HBM3E;
//  * best-fit free lists per slab (256 B alignment), O(log n) alloc/free;
//  * put = one multi-segment copy kernel launch (pack) on the caller's stream;
//  * get = zero-copy device pointer, pinned until released;
//  * co-located processes open a slab once via hipIpcOpenMemHandle (dmabuf) and address
//    objects by (slab, offset);
//  * LRU spill of unpinned objects to the node's shared-memory object store on a dedicated
//    side stream, through the CDNA4 compress kernel (K4) when it pays, restore on demand.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../store/shm_store.h"

namespace rmm {
namespace hip {

struct GpuObject {
  int slab = -1;
  uint64_t offset = 0;
  uint64_t nbytes = 0;
  int elem_bits = 0;  // 16/32: compressible float data; 0: raw bytes
  int pins = 0;
  bool sealed = false;
  bool spilled = false;
  uint64_t spill_bytes = 0;  // bytes held in the host store
  bool spill_compressed = false;
  hipEvent_t ready = nullptr;  // completes when the producing copy is done
  std::list<std::string>::iterator lru;
  bool in_lru = false;
};

struct Slab {
  void* base = nullptr;
  uint64_t size = 0;
  bool dedicated = false;
  uint64_t used = 0;
  std::map<uint64_t, uint64_t> free_by_off;        // offset -> size
  std::multimap<uint64_t, uint64_t> free_by_size;  // size -> offset
  hipIpcMemHandle_t ipc{};
  bool ipc_valid = false;
};

struct GpuStats {
  uint64_t capacity, slab_bytes_allocated, bytes_in_use, num_objects;
  uint64_t spilled_objects, spilled_bytes_total, spilled_host_bytes_total, restored_bytes_total;
  uint64_t puts, gets;
};

class GpuStore {
 public:
  GpuStore(int device, uint64_t capacity, uint64_t slab_bytes, const std::string& shm_name,
           bool compress_spill);
  ~GpuStore();

  // Allocate an object and return its device pointer (unsealed, pinned by the creator).
  uint64_t Create(const std::string& id, uint64_t nbytes, int elem_bits);
  // Record that the producing work on `stream` has been enqueued; seal + unpin.
  void Seal(const std::string& id, hipStream_t stream);
  // Create + multi-segment pack copy + seal in one call.
  uint64_t PutSegments(const std::string& id, const std::vector<std::pair<uint64_t, uint64_t>>& segs,
                       int elem_bits, hipStream_t stream);
  // Pin and return the device pointer (restores spilled objects). Makes `stream` wait for the
  // producing copy. Returns 0 if unknown.
  uint64_t Get(const std::string& id, hipStream_t stream);
  void Release(const std::string& id);
  bool Delete(const std::string& id);
  bool Contains(const std::string& id);
  bool IsSpilled(const std::string& id);
  // (slab index, offset, nbytes) of a resident object, or slab = -1.
  void Locate(const std::string& id, int* slab, uint64_t* offset, uint64_t* nbytes);
  std::string SlabIpcHandle(int slab);
  uint64_t SlabBase(int slab);
  // Spill LRU objects until `bytes` are free; returns bytes freed.
  uint64_t Spill(uint64_t bytes);
  uint64_t SpillObject(const std::string& id);
  GpuStats Stats();
  int device() const { return device_; }

  // Spill-object id in the host store for a GPU object id.
  static std::string HostId(const std::string& id);

 private:
  uint64_t AllocLocked(uint64_t nbytes, int* slab);
  void FreeLocked(int slab, uint64_t off, uint64_t nbytes);
  bool NewSlabLocked(uint64_t min_bytes);
  uint64_t SpillLocked(uint64_t bytes);
  bool SpillOneLocked(const std::string& id, GpuObject& o);
  bool RestoreLocked(const std::string& id, GpuObject& o, hipStream_t stream);
  void LruTouch(const std::string& id, GpuObject& o);
  void LruDrop(GpuObject& o);
  void EnsureScratch();

  int device_;
  uint64_t capacity_;
  uint64_t slab_bytes_;
  uint64_t allocated_ = 0;
  bool compress_;
  std::vector<std::unique_ptr<Slab>> slabs_;
  std::unordered_map<std::string, GpuObject> objs_;
  std::list<std::string> lru_;  // front = least recently used
  std::mutex mu_;
  hipStream_t side_ = nullptr;   // spill / restore stream
  hipStream_t side2_ = nullptr;  // D2H copies overlapped with compression
  std::unique_ptr<Store> host_;
  bool host_registered_ = false;  // whole shm segment pinned for DMA
  // compression scratch (double buffered)
  void* scratch_[2] = {nullptr, nullptr};
  void* work_ = nullptr;
  uint64_t scratch_bytes_ = 0;
  uint64_t work_bytes_ = 0;
  GpuStats st_{};
};

}  // namespace hip
}  // namespace rmm
