// HBM-resident GPU object store (one per process per device).
//
// North-star component with no reference equivalent: the reference pickles CUDA tensors
// through host memory (python/ray/_private/serialization.py). Here objects stay in HBM:
//  * slab arena: lazily hipMalloc'ed slabs (default 8 GiB; objects larger than a slab get a
//    dedicated slab) up to `capacity` — sized for 288 GB HBM3E;
//  * best-fit free lists per slab (256 B alignment), O(log n) alloc/free;
//  * put = one multi-segment copy kernel launch (pack) on the caller's stream; the shared-memory
//    descriptor can be sealed by a stream host callback when the copy completes, so `put` never
//    blocks the host (SealDescriptorAsync);
//  * get = zero-copy device pointer, pinned until released; Delete of a pinned object is deferred
//    to the last Release;
//  * co-located processes open a slab once via hipIpcOpenMemHandle (dmabuf) and address
//    objects by (slab, offset);
//  * LRU spill of unpinned objects to the node's shared-memory object store, through the CDNA4
//    compress kernel (K4) when it pays — each chunk is compressed ONCE (size read back, then the
//    exact bytes DMA'd; the host object is allocated at its worst case and shrunk at the end,
//    header written last). The store lock is NOT held across the DMA: the victim is marked
//    `spilling`, readers of it wait on a condition variable. A background thread spills
//    proactively above `spill_threshold` of the capacity (reference: local_object_manager.cc
//    SpillObjectsOfSize driven by the object_spilling_threshold);
//  * restore on demand, also without the store lock held; processes that do not own an object
//    restore it into their own memory through RestoreForeign (pinned DMA + K4 on side streams).
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <atomic>
#include <thread>
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
  bool spilling = false;   // HBM -> host transfer in flight (store lock released)
  bool restoring = false;  // host -> HBM transfer in flight
  bool delete_pending = false;
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
  uint64_t spill_ns_total, restore_ns_total, proactive_spills, deferred_deletes;
  uint64_t spills_device_placed;  // spills whose chunks a copy kernel placed (no per-chunk host round trip)
};

class GpuStore {
 public:
  GpuStore(int device, uint64_t capacity, uint64_t slab_bytes, const std::string& shm_name,
           bool compress_spill, double spill_threshold = 0.0, uint64_t prepin_bytes = 0);
  ~GpuStore();

  // Allocate an object and return its device pointer (unsealed, pinned by the creator).
  uint64_t Create(const std::string& id, uint64_t nbytes, int elem_bits);
  // Record that the producing work on `stream` has been enqueued; seal + unpin.
  void Seal(const std::string& id, hipStream_t stream);
  // Create + multi-segment pack copy + seal in one call.
  uint64_t PutSegments(const std::string& id, const std::vector<std::pair<uint64_t, uint64_t>>& segs,
                       int elem_bits, hipStream_t stream);
  // Seal (and release the creator pin of) host-store object `desc_id` from a host callback once
  // the work enqueued on `stream` so far has completed: the descriptor of an asynchronous put.
  void SealDescriptorAsync(const std::string& desc_id, hipStream_t stream);
  // Pin and return the device pointer (restores spilled objects). Makes `stream` wait for the
  // producing copy. Returns 0 if unknown.
  uint64_t Get(const std::string& id, hipStream_t stream);
  void Release(const std::string& id);
  bool Delete(const std::string& id);
  bool Contains(const std::string& id);
  bool IsSpilled(const std::string& id);
  // (slab index, offset, nbytes) of a resident object, or slab = -1. Does not wait for the copy.
  void Locate(const std::string& id, int* slab, uint64_t* offset, uint64_t* nbytes);
  std::string SlabIpcHandle(int slab);
  uint64_t SlabBase(int slab);
  // Spill LRU objects until `bytes` are free; returns bytes freed.
  uint64_t Spill(uint64_t bytes);
  uint64_t SpillObject(const std::string& id);
  // Restore host spill object `host_id` (written by any process's GpuStore) into `dst` (device
  // memory of this store's device); blocks until the data is in place. Returns bytes restored.
  uint64_t RestoreForeign(const std::string& host_id, uint64_t dst, uint64_t nbytes);
  void SetSpillThreshold(double t);
  GpuStats Stats();
  std::string LastError();  // message of the last failed spill / restore transfer
  int device() const { return device_; }

  // Spill-object id in the host store for a GPU object id.
  static std::string HostId(const std::string& id);

 private:
  using Lock = std::unique_lock<std::mutex>;
  uint64_t AllocLocked(Lock& lk, uint64_t nbytes, int* slab);
  void FreeLocked(int slab, uint64_t off, uint64_t nbytes);
  bool NewSlabLocked(uint64_t min_bytes);
  uint64_t SpillLocked(Lock& lk, uint64_t bytes);
  // Spill one object; releases and re-acquires `lk` around the transfer. False if not spillable.
  bool SpillOne(Lock& lk, const std::string& id);
  bool RestoreOne(Lock& lk, const std::string& id, GpuObject* o);
  void DeleteLocked(const std::string& id);
  void WaitIdleLocked(Lock& lk, const std::string& id);
  void LruTouch(const std::string& id, GpuObject& o);
  void LruDrop(GpuObject& o);
  void EnsureScratch();
  // Transfers (caller holds xfer_mu_, NOT mu_).
  bool SpillTransfer(const std::string& id, const uint8_t* src, uint64_t nbytes, int elem_bits, hipEvent_t ready,
                     uint64_t* host_bytes, bool* compressed);
  uint64_t RestoreTransfer(const std::string& host_id, uint8_t* dst, uint64_t nbytes, bool delete_host);
  void BackgroundSpiller();

  int device_;
  uint64_t capacity_;
  uint64_t slab_bytes_;
  uint64_t allocated_ = 0;
  bool compress_;
  std::vector<std::unique_ptr<Slab>> slabs_;
  std::unordered_map<std::string, GpuObject> objs_;
  std::list<std::string> lru_;  // front = least recently used
  std::mutex mu_;
  std::condition_variable cv_;  // transfers finished / memory freed
  std::mutex xfer_mu_;          // one spill/restore transfer at a time (streams + scratch)
  hipStream_t side_ = nullptr;  // compression / decompression stream
  hipStream_t side2_ = nullptr; // DMA stream overlapped with (de)compression
  std::unique_ptr<Store> host_;
  // compression scratch (double buffered)
  void* scratch_[2] = {nullptr, nullptr};
  void* work_ = nullptr;
  uint64_t scratch_bytes_ = 0;
  uint64_t work_bytes_ = 0;
  uint64_t* spill_meta_ = nullptr;  // device: [host offset cursor, per-chunk compressed sizes...] (device-placed spill)
  hipEvent_t ev_[4] = {nullptr, nullptr, nullptr, nullptr};
  GpuStats st_{};
  int spills_in_flight_ = 0;
  double spill_threshold_ = 0.0;  // fraction of capacity; 0 = spill only on allocation failure
  bool stop_ = false;
  std::condition_variable bg_cv_;
  std::thread bg_;
  // background page-locking of the host arena's first prepin bytes (spill targets): a spill into
  // registered memory is one DMA; into fresh pages it first pays the pin (and page faults)
  std::thread prepin_;
  std::atomic<bool> prepin_stop_{false};
  std::atomic<uint64_t> prepin_done_{0};
  uint64_t prepin_total_ = 0;

 public:
  // (bytes of the host arena page-locked so far, bytes requested)
  std::pair<uint64_t, uint64_t> PrepinProgress() const { return {prepin_done_.load(), prepin_total_}; }

 private:
  std::mutex err_mu_;
  std::string last_error_;
  std::string last_stale_;
  uint64_t stale_errors_ = 0;
  void ClearStaleError(const char* where);
};

}  // namespace hip
}  // namespace rmm
