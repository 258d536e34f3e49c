// Shared-memory object store ("plasma" equivalent), MI355X-node edition.
//
// Parity: reference src/ray/object_manager/plasma/{store.cc,object_lifecycle_manager.cc,
// eviction_policy.cc,plasma_allocator.cc,create_request_queue.cc} and
// src/ray/raylet/local_object_manager.cc (spill / restore).
//
// Design (not a port): the reference runs plasma as a server inside the raylet and every
// client talks to it over a Unix socket (fd passing + flatbuffers). Here the WHOLE store —
// allocator state, object table, LRU list, spill bookkeeping, a process-shared robust mutex
// and condition variable — lives inside one /dev/shm segment that every process on the node
// maps. create/seal/get/release are therefore plain function calls (no IPC round trip);
// a seal broadcasts the in-segment condvar, which is what `get` waiters and the scheduler's
// dependency watcher block on. The data heap is managed by a TLSF (two-level segregated
// fit) allocator addressed by offsets, so it is valid in every mapping. The segment can be
// hipHostRegister'ed by GPU processes so spills of HBM objects DMA straight into it.
#pragma once
#include <pthread.h>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace rmm {

constexpr int kIdSize = 20;
constexpr uint64_t kAlign = 64;
constexpr uint64_t kBlockHdr = 64;
constexpr uint64_t kMinBlock = 128;
constexpr int kFL = 48;      // first-level classes (2^48 = 256 TB max block)
constexpr int kSLBits = 4;   // 16 second-level classes
constexpr int kSL = 1 << kSLBits;
constexpr uint64_t kNil = 0;

enum ObjState : uint32_t {
  kEmpty = 0,
  kCreating = 1,
  kSealed = 2,
  kSpilling = 3,   // sealed, being written to external storage (still readable)
  kSpilled = 4,    // only in external storage
  kRestoring = 5,  // being read back from external storage
  kTombstone = 6,
};

enum ObjFlags : uint32_t {
  kFlagFallback = 1u << 0,      // data lives in a per-object mmap file, not the heap
  kFlagDeletePending = 1u << 1, // delete requested while pinned
  kFlagHasSpillCopy = 1u << 2,  // an up-to-date copy exists in external storage
  kFlagError = 1u << 3,         // payload is a serialized error
  kFlagGpuSpilled = 1u << 4,    // GPU-object descriptor: HBM copy spilled to the host store
};

// Binary header of a GPU-object descriptor object (tag kTagGpu). The owning process's GPU
// store rewrites slab/offset/ipc in place when it restores a spilled object; readers only trust
// these fields while they hold a pin AND kFlagGpuSpilled is clear (both checked under the lock).
struct GpuDesc {
  uint64_t magic;  // kGpuDescMagic
  uint64_t nbytes;
  int64_t slab;
  uint64_t offset;
  int32_t device;
  int32_t owner_pid;
  uint8_t ipc[64];
  char pci_bus_id[16];
  uint64_t meta_len;  // pickled (dtype, shape, ...) follows the header
};
constexpr uint64_t kGpuDescMagic = 0x4353454455504752ull;  // "RGPUDESC"

struct ObjectId {
  uint8_t b[kIdSize];
};

struct Entry {
  uint8_t id[kIdSize];
  uint32_t state;
  uint32_t flags;
  int32_t pin_count;    // = anon_pins + the counts of this object's PinRec records
  int32_t creator_pid;
  int32_t lru_prev;  // intrusive LRU list of evictable (sealed, unpinned) entries
  int32_t lru_next;
  uint32_t in_lru;
  uint32_t user_tag;    // opaque to the store (e.g. serialization format / GPU meta)
  int32_t io_pid;       // kSpilling / kRestoring: the process doing the file IO (holds one anon pin)
  int32_t anon_pins;    // pins without a per-client record (spill / restore IO, pin-table overflow)
  uint32_t pad_;
  uint64_t offset;      // heap offset of payload (data followed by metadata)
  uint64_t data_size;
  uint64_t meta_size;
  uint64_t spill_file;  // spill file id (when kFlagHasSpillCopy / kSpilled)
  uint64_t spill_off;
  uint64_t fallback_id; // file id for kFlagFallback objects
  uint64_t create_ns;
};

// Per-client pin record (reference plasma/store.cc:323 DisconnectClient releases a dead client's
// objects; here clients are processes, so pins are recorded per (object, pid) in an open-addressing
// table inside the segment: a dead reader's pins are released by ReleaseClient(pid) or by the
// crash-recovery rebuild).
struct PinRec {
  uint8_t id[kIdSize];
  int32_t pid;
  int32_t count;
  uint32_t state;  // 0 empty, 1 live, 2 tombstone
};
constexpr uint64_t kPinCap = 1 << 16;

struct SpillFileSlot {
  uint64_t file_id;  // 0 = free
  int64_t live;      // objects still referencing this fused file
};

constexpr uint64_t kSpillSlots = 1 << 14;
constexpr uint64_t kRingCap = 1 << 16;

struct Stats {
  uint64_t bytes_in_use;
  uint64_t num_objects;
  uint64_t num_sealed;
  uint64_t bytes_spilled_total;
  uint64_t objects_spilled_total;
  uint64_t bytes_restored_total;
  uint64_t objects_restored_total;
  uint64_t spilled_bytes_current;
  uint64_t spilled_objects_current;
  uint64_t fallback_bytes_current;
  uint64_t fallback_allocs_total;
  uint64_t creates_total;
  uint64_t gets_total;
  uint64_t deletes_total;
};

struct Header {
  uint64_t magic;
  uint64_t version;
  uint64_t total_size;
  uint64_t table_off;
  uint64_t table_cap;  // power of two
  uint64_t ring_off;
  uint64_t spill_off;
  uint64_t heap_off;   // absolute offset of heap start inside the segment
  uint64_t heap_size;
  pthread_mutex_t mu;
  // The store's condition is a futex word, not a pthread_cond_t: glibc's process-shared condvar keeps
  // per-group waiter references, so a waiter SIGKILLed inside pthread_cond_timedwait leaves the next
  // broadcast waiting for it forever -- while it holds the store mutex, which hangs every process
  // (found by tests/test_chaos.py). A futex wait holds no state for the kernel to clean up.
  uint32_t cv_seq;
  uint64_t seal_seq;
  uint64_t ring_head;
  uint64_t next_file_id;
  uint64_t table_used;  // live + tombstones
  int32_t lru_head;
  int32_t lru_tail;
  // TLSF control (offsets relative to segment base)
  uint64_t fl_bitmap;
  uint32_t sl_bitmap[kFL];
  uint64_t free_heads[kFL][kSL];
  // config
  double spill_threshold;       // proactively spill when usage > threshold * heap
  uint64_t min_spill_size;      // fuse at least this many bytes per spill file
  int32_t spill_enabled;
  int32_t fallback_enabled;
  char spill_dir[2048];        // one or more directories separated by ':' (round-robin per file)
  // memory-pressure machinery (reference: plasma create_request_queue.cc, file_system_monitor.cc)
  int64_t oom_grace_ns;        // a create that cannot be satisfied waits this long (GC + spill) first
  int32_t disk_full;           // set by the node's disk monitor: no spilling / fallback files
  int32_t pad0;
  uint64_t gc_requests;        // bumped by a starved create: the node broadcasts a global GC
  uint64_t oom_waits_total;    // creates that had to wait for memory
  uint64_t oom_errors_total;   // creates that failed after the grace period
  // crash consistency: the pid holding the mutex (0 when free). A process killed inside a critical
  // section leaves its pid here; the next locker gets EOWNERDEAD and rebuilds the metadata
  // (Store::Recover), counted in recoveries_total.
  int32_t lock_pid;
  int32_t pad1;
  uint64_t recoveries_total;
  uint64_t recovered_dropped_total;  // entries the rebuild could not validate (lost objects)
  uint64_t creating_now;             // entries in kCreating (AbortCreator skips its table scan at 0)
  // per-client pins (PinRec table at pins_off, kPinCap records)
  uint64_t pins_off;
  uint64_t pins_used;                // live + tombstone records
  uint64_t pins_live;
  uint64_t pin_overflow_total;       // pins taken without a record (table full): not released on death
  uint64_t io_now;                   // entries holding a spill / restore IO pin (ReleaseClient skips its scan at 0)
  uint64_t clients_released_total;   // ReleaseClient calls that found something to release
  uint64_t client_pins_released_total;
  // integrity: a release by a process holding no pin of the object (never taken from another client's
  // record), metadata found inconsistent by a bounded walk or a heap-free check (the store rebuilt itself
  // with Recover instead of spinning under the mutex), lock waits that exceeded the watchdog period
  uint64_t unmatched_releases_total;
  uint64_t corruptions_total;
  uint64_t lock_stalls_total;
  int32_t lock_stall_pid;            // the holder the watchdog last reported
  int32_t pad2;
  Stats stats;
};

class Store {
 public:
  // Create a new segment (head process) or attach to an existing one.
  static Store* Create(const std::string& name, uint64_t size, const std::string& spill_dir,
                       double spill_threshold, uint64_t min_spill_size, bool fallback,
                       double oom_grace_s = 2.0, bool populate = false);
  // Memory-pressure controls / counters (see Header).
  void SetDiskFull(bool full);
  // automatic_object_spilling_enabled: off keeps the directories for fallback files only
  void SetSpillEnabled(bool on);
  bool DiskFull() const { return hdr_->disk_full != 0; }
  uint64_t GcRequests() const { return __atomic_load_n(&hdr_->gc_requests, __ATOMIC_ACQUIRE); }
  uint64_t OomWaits() const { return hdr_->oom_waits_total; }
  uint64_t OomErrors() const { return hdr_->oom_errors_total; }
  void SetOomGrace(double seconds);
  std::vector<std::string> SpillDirs() const;
  static Store* Attach(const std::string& name);
  ~Store();

  // Returns payload pointer or nullptr (already exists => *exists=true).
  // Throws std::runtime_error on out-of-memory when spilling/fallback cannot help.
  uint8_t* CreateObject(const ObjectId& id, uint64_t data_size, uint64_t meta_size,
                        uint32_t user_tag, uint32_t flags, bool* exists);
  void Seal(const ObjectId& id);
  void Abort(const ObjectId& id);
  // Shrink an object still being created (no metadata) to `data_size` bytes, returning the tail
  // of its heap block to the allocator. Used by writers that allocate a worst case first (the
  // GPU spill path writes a compressed stream whose size is known only at the end).
  bool ShrinkCreating(const ObjectId& id, uint64_t data_size);
  // Pins and returns pointer; waits up to timeout_ms (<0 = forever, 0 = no wait).
  // Returns nullptr on timeout.
  struct View {
    uint8_t* data = nullptr;
    uint64_t data_size = 0;
    uint64_t meta_size = 0;
    uint32_t user_tag = 0;
    uint32_t flags = 0;
  };
  bool Get(const ObjectId& id, int64_t timeout_ms, View* out);
  // Batched non-pinning readiness check: returns count of ready ids and fills ready mask.
  int Wait(const std::vector<ObjectId>& ids, int num_required, int64_t timeout_ms,
           std::vector<uint8_t>* ready);
  void Release(const ObjectId& id);
  // Delete (free) an object; deferred if pinned. Returns false if unknown.
  bool Delete(const ObjectId& id);
  bool Contains(const ObjectId& id);   // sealed / spilled
  // Set `flag` only if nobody holds a pin (returns false if pinned; true if absent).
  bool TrySetFlag(const ObjectId& id, uint32_t flag);
  void ClearFlag(const ObjectId& id, uint32_t flag);
  // Run `fn(data)` on a sealed object's payload under the store lock (in-place metadata update).
  template <typename F>
  bool WithLockedData(const ObjectId& id, F fn) {
    Lock();
    int64_t idx = Find(id);
    bool ok = idx >= 0 && E(idx)->state == kSealed && !(E(idx)->flags & kFlagFallback);
    if (ok) fn(base_ + E(idx)->offset, E(idx)->flags);
    Unlock();
    return ok;
  }
  int State(const ObjectId& id);       // ObjState or -1
  // data + metadata bytes of each object (-1 if absent), one lock acquisition for the batch
  std::vector<int64_t> Sizes(const std::vector<ObjectId>& ids);
  // Spill LRU unpinned objects until `bytes` have been freed. Returns bytes freed.
  uint64_t SpillBytes(uint64_t bytes);
  // Abort all objects still being created by `pid` (crashed creator).
  int AbortCreator(int pid);
  // A client process died: release every pin it held (gets it never released, its creator pins) and
  // roll back spills / restores it was doing (kSpilling -> kSealed, kRestoring -> kSpilled); objects
  // whose last pin this was are freed if a delete was pending, else become evictable. Returns the
  // number of pins released. Reference plasma/store.cc:323 DisconnectClient.
  int ReleaseClient(int pid);
  // Pins currently recorded for `pid` (tests / memory summary).
  int64_t PinsHeldBy(int pid);
  uint64_t PinOverflows() const { return hdr_->pin_overflow_total; }
  uint64_t UnmatchedReleases() const { return hdr_->unmatched_releases_total; }
  uint64_t Corruptions() const { return __atomic_load_n(&hdr_->corruptions_total, __ATOMIC_ACQUIRE); }
  uint64_t LockStalls() const { return __atomic_load_n(&hdr_->lock_stalls_total, __ATOMIC_ACQUIRE); }
  int LockPid() const { return __atomic_load_n(&hdr_->lock_pid, __ATOMIC_ACQUIRE); }
  // Watchdog period of the store mutex: a lock wait longer than this logs the holder's pid (once per
  // holder) and counts a stall. Process-local; 0 disables.
  static void SetLockWatchdogMs(int64_t ms);
  // Entries in kCreating (tests: a creator blocked in the create grace wait)
  uint64_t CreatingNow() const { return hdr_->creating_now; }
  // Sealed-notification ring: returns new cursor; sets overflow when the consumer fell behind.
  uint64_t PollSealed(uint64_t cursor, std::vector<ObjectId>* out, bool* overflow);
  uint64_t SealSeq();
  // Block until seal_seq != seq or timeout. Returns current seal_seq.
  uint64_t WaitSealSeq(uint64_t seq, int64_t timeout_ms);
  Stats GetStats();
  uint64_t Capacity() const { return hdr_->heap_size; }
  uint8_t* Base() const { return base_; }
  uint64_t MappedSize() const { return size_; }
  std::vector<std::pair<ObjectId, Entry>> ListObjects();
  // Allocator self-check (used by tests): verifies heap walk + free lists. Returns free bytes.
  uint64_t CheckHeap();
  void Wake();
  uint64_t Recoveries() const { return __atomic_load_n(&hdr_->recoveries_total, __ATOMIC_ACQUIRE); }
  uint64_t RecoveredDropped() const { return hdr_->recovered_dropped_total; }
  // Test hook: SIGKILL this process at crash point `p` (1 = mid heap split, 2 = mid heap merge,
  // 3 = mid table insert, 4 = mid LRU unlink), i.e. while holding the store mutex in the middle
  // of a multi-word metadata update; 5 = mid restore IO, 6 = mid spill IO (lock released, the
  // entries carry this process's IO pin); 7 = SIGSTOP inside Contains (a holder that never returns:
  // the lock watchdog reports it). 0 disables. Process-local.
  static void SetCrashPointForTest(int p);

 private:
  Store() = default;
  // All Locked* helpers require hdr_->mu held.
  void Lock();
  void Unlock();
  void OnLocked(int rc);
  // Rebuild allocator, object table, LRU list, spill-file refcounts and derived statistics from
  // the entries that validate, after `dead_pid` died holding the lock (mutex already consistent).
  void Recover(int dead_pid);
  // A bounded walk or a block check found the metadata inconsistent: count it, log it and rebuild
  // (Recover) under the lock instead of following the damage.
  void Heal(const char* why);
  // payload offset of a used heap block (in range, aligned, not marked free)
  bool UsedBlock(uint64_t payload_off) const;
  int64_t Find(const ObjectId& id);
  int64_t Insert(const ObjectId& id);
  void RemoveEntry(int64_t idx);
  Entry* E(int64_t idx) { return &table_[idx]; }
  uint64_t HeapAlloc(uint64_t n);
  void HeapFree(uint64_t payload_off);
  void HeapShrink(uint64_t payload_off, uint64_t n);
  void LruPush(int64_t idx);
  void LruRemove(int64_t idx);
  // per-client pins (lock held)
  PinRec* Pins() { return reinterpret_cast<PinRec*>(base_ + hdr_->pins_off); }
  int64_t PinFind(const uint8_t* id, int32_t pid);
  bool PinInsert(const uint8_t* id, int32_t pid, int32_t count);
  void PinRehash();
  void PinAdd(int64_t idx, int32_t pid);
  void PinDrop(int64_t idx, int32_t pid);
  void PinErase(const uint8_t* id, int32_t pid);
  void IoPin(int64_t idx);
  void IoUnpin(int64_t idx);
  void FinishUnpinned(int64_t idx);
  void FreeEntryStorage(int64_t idx);
  void DropSpillRef(uint64_t file_id);
  int64_t SpillSlot(uint64_t file_id, bool create);
  uint64_t SpillLocked(uint64_t bytes, std::vector<int64_t>* pinned_victims);
  bool RestoreLocked(int64_t idx);
  uint8_t* FallbackMap(uint64_t fid, uint64_t size, bool create);
  void FallbackUnlink(uint64_t fid);
  std::string SpillPath(uint64_t fid) const;
  std::string DirFor(uint64_t fid) const;
  std::string FallbackPath(uint64_t fid) const;
  void Broadcast();  // under the lock: bump the condition word, wake every waiter
  void CondWait(int64_t deadline_ns);
  // TLSF
  void TlsfInsert(uint64_t blk);
  void TlsfRemove(uint64_t blk);
  uint64_t TlsfFind(uint64_t size);

  std::string name_;
  uint8_t* base_ = nullptr;
  uint64_t size_ = 0;
  Header* hdr_ = nullptr;
  Entry* table_ = nullptr;
  ObjectId* ring_ = nullptr;
  SpillFileSlot* spill_ = nullptr;
  bool owner_ = false;
  // per-process cache of fallback mappings: fid -> (ptr,size)
  struct FbMap { uint64_t fid; uint8_t* ptr; uint64_t size; };
  std::vector<FbMap> fb_maps_;
  pthread_mutex_t fb_mu_ = PTHREAD_MUTEX_INITIALIZER;
};

}  // namespace rmm
