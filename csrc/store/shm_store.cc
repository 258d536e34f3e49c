// Shared-memory object store implementation. See shm_store.h for the design notes.
#include "shm_store.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <unordered_map>

namespace rmm {

namespace {

constexpr uint64_t kMagic = 0x524d4d53544f5245ull;  // "RMMSTORE"
// 6: per-client pin records, Entry.io_pid / anon_pins; 7: futex condition word; 8: integrity counters
constexpr uint64_t kVersion = 8;
constexpr uint64_t kFreeBit = 1;
constexpr uint64_t kSizeMask = ~uint64_t(kAlign - 1);

struct Blk {
  uint64_t size;       // total block bytes (multiple of 64) | kFreeBit
  uint64_t prev_phys;  // absolute offset of previous physical block, 0 if first
  uint64_t next_free;
  uint64_t prev_free;
};

inline uint64_t AlignUp(uint64_t v, uint64_t a) { return (v + a - 1) & ~(a - 1); }

inline int64_t NowNs() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return int64_t(ts.tv_sec) * 1000000000ll + ts.tv_nsec;
}

inline uint64_t HashId(const ObjectId& id) {
  uint64_t a, b;
  uint32_t c;
  memcpy(&a, id.b, 8);
  memcpy(&b, id.b + 8, 8);
  memcpy(&c, id.b + 16, 4);
  uint64_t h = a * 0x9E3779B97F4A7C15ull;
  h ^= (b + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2));
  h ^= (uint64_t(c) * 0xC2B2AE3D27D4EB4Full);
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 32;
  return h;
}

int g_crash_point = 0;

inline void CrashPoint(int p) {
  // dies holding the store mutex (test hook); point 7 stops instead (a stuck holder for the watchdog)
  if (g_crash_point == p) kill(getpid(), p == 7 ? SIGSTOP : SIGKILL);
}

// A process that has exited: no such pid, or a zombie not yet reaped by its parent (its memory and
// its store mappings are gone already).
bool ProcessGone(int pid) {
  if (pid <= 0) return true;
  if (kill(pid, 0) != 0) return errno == ESRCH;
  char path[64], buf[512];
  snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  int fd = open(path, O_RDONLY);
  if (fd < 0) return false;
  const ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return false;
  buf[n] = 0;
  const char* rp = strrchr(buf, ')');
  return rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X');
}

inline void MappingInsert(uint64_t size, int* fl, int* sl) {
  int f = 63 - __builtin_clzll(size);
  *sl = int((size >> (f - kSLBits)) ^ (uint64_t(1) << kSLBits));
  *fl = f;
}

}  // namespace

// ---------------------------------------------------------------- lifecycle

static void InitSync(Header* h) {
  pthread_mutexattr_t ma;
  pthread_mutexattr_init(&ma);
  pthread_mutexattr_setpshared(&ma, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&ma, PTHREAD_MUTEX_ROBUST);
  pthread_mutex_init(&h->mu, &ma);
  pthread_mutexattr_destroy(&ma);
  h->cv_seq = 0;
}

Store* Store::Create(const std::string& name, uint64_t size, const std::string& spill_dir,
                     double spill_threshold, uint64_t min_spill_size, bool fallback, double oom_grace_s,
                     bool populate) {
  if (spill_dir.size() >= sizeof(Header::spill_dir))
    throw std::runtime_error("spill directory list too long");
  if (size < (8ull << 20)) size = 8ull << 20;
  uint64_t table_cap = 1 << 14;
  // one slot per 4 KiB of arena (112 B each, ~2.7% overhead): small-object heavy workloads
  // (millions of tiny puts) must not run out of slots before they run out of bytes
  while (table_cap < (size >> 12) && table_cap < (1ull << 22)) table_cap <<= 1;
  uint64_t off = AlignUp(sizeof(Header), 4096);
  uint64_t table_off = off;
  off = AlignUp(off + table_cap * sizeof(Entry), 4096);
  uint64_t ring_off = off;
  off = AlignUp(off + kRingCap * sizeof(ObjectId), 4096);
  uint64_t spill_off = off;
  off = AlignUp(off + kSpillSlots * sizeof(SpillFileSlot), 4096);
  uint64_t pins_off = off;
  off = AlignUp(off + kPinCap * sizeof(PinRec), 4096);
  uint64_t heap_off = off;
  uint64_t heap_size = AlignUp(size, 4096);
  uint64_t total = heap_off + heap_size;

  int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name + ": " + strerror(errno));
  if (ftruncate(fd, off_t(total)) != 0) {
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error("ftruncate failed: " + std::string(strerror(errno)));
  }
  // populate: fault every page in now (reference preallocate_plasma_memory, plasma/dlmalloc.cc
  // MAP_POPULATE) so puts and GPU spills into the arena never pay first-touch page faults
  void* p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED | (populate ? MAP_POPULATE : 0), fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    shm_unlink(name.c_str());
    throw std::runtime_error("mmap failed: " + std::string(strerror(errno)));
  }
  Store* s = new Store();
  s->name_ = name;
  s->base_ = static_cast<uint8_t*>(p);
  s->size_ = total;
  s->owner_ = true;
  Header* h = reinterpret_cast<Header*>(p);
  memset(h, 0, sizeof(Header));
  h->total_size = total;
  h->table_off = table_off;
  h->table_cap = table_cap;
  h->ring_off = ring_off;
  h->spill_off = spill_off;
  h->pins_off = pins_off;  // records are zero (empty) from ftruncate
  h->heap_off = heap_off;
  h->heap_size = heap_size;
  h->lru_head = h->lru_tail = -1;
  h->next_file_id = 1;
  h->spill_threshold = spill_threshold;
  h->min_spill_size = min_spill_size;
  h->spill_enabled = spill_dir.empty() ? 0 : 1;
  h->fallback_enabled = (fallback && !spill_dir.empty()) ? 1 : 0;
  strncpy(h->spill_dir, spill_dir.c_str(), sizeof(h->spill_dir) - 1);
  h->oom_grace_ns = int64_t(oom_grace_s * 1e9);
  InitSync(h);
  s->hdr_ = h;
  s->table_ = reinterpret_cast<Entry*>(s->base_ + table_off);
  s->ring_ = reinterpret_cast<ObjectId*>(s->base_ + ring_off);
  s->spill_ = reinterpret_cast<SpillFileSlot*>(s->base_ + spill_off);
  // table pages are zero from ftruncate (kEmpty == 0).
  // Heap: one big free block followed by a used sentinel header.
  uint64_t first = heap_off;
  uint64_t sentinel = heap_off + heap_size - kBlockHdr;
  Blk* b = reinterpret_cast<Blk*>(s->base_ + first);
  b->size = (sentinel - first) | kFreeBit;
  b->prev_phys = 0;
  Blk* sb = reinterpret_cast<Blk*>(s->base_ + sentinel);
  sb->size = kBlockHdr;  // used
  sb->prev_phys = first;
  s->TlsfInsert(first);
  __atomic_store_n(&h->version, kVersion, __ATOMIC_RELEASE);
  __atomic_store_n(&h->magic, kMagic, __ATOMIC_RELEASE);
  return s;
}

Store* Store::Attach(const std::string& name) {
  int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open(attach) failed for " + name + ": " + strerror(errno));
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    throw std::runtime_error("fstat failed");
  }
  void* p = mmap(nullptr, size_t(st.st_size), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("mmap(attach) failed: " + std::string(strerror(errno)));
  Header* h = reinterpret_cast<Header*>(p);
  if (__atomic_load_n(&h->magic, __ATOMIC_ACQUIRE) != kMagic || h->version != kVersion) {
    munmap(p, size_t(st.st_size));
    throw std::runtime_error("object store segment " + name + " is not initialised / wrong version");
  }
  Store* s = new Store();
  s->name_ = name;
  s->base_ = static_cast<uint8_t*>(p);
  s->size_ = uint64_t(st.st_size);
  s->hdr_ = h;
  s->table_ = reinterpret_cast<Entry*>(s->base_ + h->table_off);
  s->ring_ = reinterpret_cast<ObjectId*>(s->base_ + h->ring_off);
  s->spill_ = reinterpret_cast<SpillFileSlot*>(s->base_ + h->spill_off);
  return s;
}

Store::~Store() {
  for (auto& m : fb_maps_) munmap(m.ptr, m.size);
  if (base_) munmap(base_, size_);
  if (owner_) shm_unlink(name_.c_str());
}

void Store::SetCrashPointForTest(int p) { g_crash_point = p; }

void Store::OnLocked(int rc) {
  if (rc == EOWNERDEAD) {
    // A process died inside a critical section: any multi-word update it was making (TLSF split /
    // merge, table insert, LRU links) may be half done. Rebuild every derived structure from the
    // entries that validate before anyone reads them (reference: plasma's store owns the
    // allocator, so a dead client is only a disconnect -- store.cc:323 DisconnectClient).
    const int dead = hdr_->lock_pid;
    pthread_mutex_consistent(&hdr_->mu);
    Recover(dead);
  } else if (rc != 0) {
    throw std::runtime_error("store mutex lock failed");
  }
  hdr_->lock_pid = int32_t(getpid());
}

namespace {
int64_t g_watchdog_ms = 10000;
}

void Store::SetLockWatchdogMs(int64_t ms) { g_watchdog_ms = ms; }

// Lock with a watchdog: every critical section is short (file IO and waits run with the lock dropped),
// so a wait longer than the period means a holder is stuck. Report it (pid, once per holder) and keep
// waiting -- a dead holder is handled by the robust mutex (EOWNERDEAD), a live one must finish.
void Store::Lock() {
  if (g_watchdog_ms <= 0) {
    OnLocked(pthread_mutex_lock(&hdr_->mu));
    return;
  }
  int rc = pthread_mutex_trylock(&hdr_->mu);
  if (rc != EBUSY) {
    OnLocked(rc);
    return;
  }
  int32_t reported = 0;
  for (;;) {
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    const int64_t ns = int64_t(ts.tv_nsec) + (g_watchdog_ms % 1000) * 1000000ll;
    ts.tv_sec += time_t(g_watchdog_ms / 1000 + ns / 1000000000ll);
    ts.tv_nsec = long(ns % 1000000000ll);
    rc = pthread_mutex_timedlock(&hdr_->mu, &ts);
    if (rc != ETIMEDOUT) break;
    const int32_t holder = __atomic_load_n(&hdr_->lock_pid, __ATOMIC_ACQUIRE);
    if (holder != reported) {
      reported = holder;
      __atomic_add_fetch(&hdr_->lock_stalls_total, 1, __ATOMIC_RELEASE);
      __atomic_store_n(&hdr_->lock_stall_pid, holder, __ATOMIC_RELEASE);
      fprintf(stderr, "[rmm store] pid %d: store mutex held by pid %d for more than %lld ms\n", int(getpid()),
              int(holder), (long long)g_watchdog_ms);
    }
  }
  OnLocked(rc);
}

bool Store::UsedBlock(uint64_t payload_off) const {
  const uint64_t lo = hdr_->heap_off + kBlockHdr, hi = hdr_->heap_off + hdr_->heap_size - kBlockHdr;
  if (payload_off < lo || payload_off >= hi || payload_off % kAlign != 0) return false;
  const Blk* b = reinterpret_cast<const Blk*>(base_ + payload_off - kBlockHdr);
  const uint64_t sz = b->size & kSizeMask;
  return !(b->size & kFreeBit) && sz >= kMinBlock && payload_off - kBlockHdr + sz <= hi;
}

void Store::Heal(const char* why) {
  __atomic_add_fetch(&hdr_->corruptions_total, 1, __ATOMIC_RELEASE);
  fprintf(stderr, "[rmm store] pid %d: %s; rebuilding the store metadata\n", int(getpid()), why);
  Recover(0);
}

void Store::Unlock() {
  hdr_->lock_pid = 0;
  pthread_mutex_unlock(&hdr_->mu);
}

void Store::Recover(int dead_pid) {
  const uint64_t cap = hdr_->table_cap;
  const uint64_t heap_lo = hdr_->heap_off, heap_hi = hdr_->heap_off + hdr_->heap_size - kBlockHdr;
  std::unordered_map<int, bool> seen;  // one liveness probe per pid
  auto alive = [&](int pid) {
    if (pid <= 0 || pid == dead_pid) return false;
    auto it = seen.find(pid);
    if (it != seen.end()) return it->second;
    return seen[pid] = !ProcessGone(pid);
  };
  auto resident = [](const Entry& e) {
    return !(e.flags & kFlagFallback) &&
           (e.state == kCreating || e.state == kSealed || e.state == kSpilling || e.state == kRestoring);
  };
  // 1) entries that validate
  std::vector<Entry> keep;
  uint64_t dropped = 0;
  for (uint64_t i = 0; i < cap; i++) {
    Entry e = table_[i];
    if (e.state == kEmpty || e.state == kTombstone) continue;
    bool ok = e.state <= kRestoring && e.pin_count >= 0 && e.anon_pins >= 0 &&
              e.data_size + e.meta_size <= hdr_->heap_size;
    if (ok && e.state == kCreating && !alive(e.creator_pid)) ok = false;  // its creator is gone: abort
    // a spill / restore whose IO process is gone never finishes: roll it back and drop its IO pin
    if (ok && (e.state == kSpilling || e.state == kRestoring) && e.io_pid != 0 && !alive(e.io_pid)) {
      if (e.state == kSpilling) {
        e.state = kSealed;  // the partial spill file is never referenced
      } else {
        e.state = kSpilled;  // its heap block (if any) is freed by the rebuild below (not resident)
        e.offset = 0;
      }
      e.io_pid = 0;
      if (e.anon_pins > 0) e.anon_pins--;
    }
    if (ok && resident(e)) {
      const uint64_t need = std::max(AlignUp(e.data_size + e.meta_size, kAlign) + kBlockHdr, kMinBlock);
      const bool placed = e.offset >= heap_lo + kBlockHdr && e.offset % kAlign == 0 &&
                          e.offset - kBlockHdr + need <= heap_hi;
      // a creator between its entry insert and heap allocation (or inside the unlocked fallback
      // mapping) owns no block yet: keep it, without storage
      if (!placed && (e.state == kCreating || e.state == kRestoring)) e.offset = 0;
      else if (!placed) ok = false;
    }
    if (!ok) {
      dropped++;
      continue;
    }
    e.in_lru = 0;
    e.lru_prev = e.lru_next = -1;
    keep.push_back(e);
  }
  // 2) heap-resident blocks must not overlap: keep the older entry
  std::vector<size_t> order;
  for (size_t k = 0; k < keep.size(); k++)
    if (resident(keep[k]) && keep[k].offset) order.push_back(k);
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return keep[a].offset < keep[b].offset; });
  std::vector<uint8_t> gone(keep.size(), 0);
  uint64_t end = heap_lo;
  size_t last = SIZE_MAX;
  for (size_t k : order) {
    const Entry& e = keep[k];
    const uint64_t blk = e.offset - kBlockHdr;
    if (blk < end) {
      size_t victim = (last != SIZE_MAX && keep[last].create_ns > e.create_ns) ? last : k;
      gone[victim] = 1;
      if (victim == k) continue;
    }
    end = blk + std::max(AlignUp(e.data_size + e.meta_size, kAlign) + kBlockHdr, kMinBlock);
    last = k;
  }
  // 3) object table: clean re-insert
  memset(table_, 0, cap * sizeof(Entry));
  hdr_->table_used = 0;
  hdr_->lru_head = hdr_->lru_tail = -1;
  Stats& st = hdr_->stats;
  st.num_objects = st.num_sealed = st.spilled_bytes_current = st.spilled_objects_current = 0;
  st.fallback_bytes_current = 0;
  for (uint64_t i = 0; i < kSpillSlots; i++) spill_[i].file_id = 0, spill_[i].live = 0;
  std::vector<std::pair<uint64_t, int64_t>> lru;  // (create_ns, slot)
  for (size_t k = 0; k < keep.size(); k++) {
    if (gone[k]) {
      dropped++;
      continue;
    }
    const Entry& e = keep[k];
    ObjectId o;
    memcpy(o.b, e.id, kIdSize);
    uint64_t j = HashId(o) & (cap - 1);
    while (table_[j].state != kEmpty) j = (j + 1) & (cap - 1);
    table_[j] = e;
    hdr_->table_used++;
    st.num_objects++;
    if (e.state == kSealed) st.num_sealed++;
    if (e.state == kSpilled) st.spilled_bytes_current += e.data_size + e.meta_size, st.spilled_objects_current++;
    if (e.flags & kFlagFallback) st.fallback_bytes_current += e.data_size + e.meta_size;
    if (e.flags & kFlagHasSpillCopy) {
      int64_t sl = SpillSlot(e.spill_file, true);
      if (sl >= 0) spill_[sl].live++;
    }
    if (e.state == kSealed && resident(e)) lru.push_back({e.create_ns, int64_t(j)});  // pushed if unpinned
  }
  // 3b) pins: keep the records of live clients whose object survived; every entry's pin count is
  // its anonymous pins plus its records (the records are the truth: a dead reader's pins vanish here)
  {
    PinRec* pins = Pins();
    std::vector<PinRec> recs;
    for (uint64_t i = 0; i < kPinCap; i++)
      if (pins[i].state == 1 && pins[i].count > 0 && alive(pins[i].pid)) recs.push_back(pins[i]);
    memset(pins, 0, kPinCap * sizeof(PinRec));
    hdr_->pins_used = hdr_->pins_live = 0;
    for (uint64_t i = 0; i < cap; i++)
      if (table_[i].state != kEmpty && table_[i].state != kTombstone) table_[i].pin_count = table_[i].anon_pins;
    for (auto& r : recs) {
      ObjectId o;
      memcpy(o.b, r.id, kIdSize);
      const int64_t idx = Find(o);
      if (idx < 0) continue;
      if (PinInsert(r.id, r.pid, r.count)) table_[idx].pin_count += r.count;
    }
  }
  std::sort(lru.begin(), lru.end());
  for (auto& x : lru)
    if (table_[x.second].pin_count == 0) LruPush(x.second);
  hdr_->creating_now = hdr_->io_now = 0;
  for (uint64_t i = 0; i < cap; i++) {
    hdr_->creating_now += table_[i].state == kCreating;
    hdr_->io_now += (table_[i].state == kSpilling || table_[i].state == kRestoring) && table_[i].io_pid != 0;
  }
  // 4) heap: used blocks exactly where live payloads are, every gap one free block
  hdr_->fl_bitmap = 0;
  memset(hdr_->sl_bitmap, 0, sizeof(hdr_->sl_bitmap));
  memset(hdr_->free_heads, 0, sizeof(hdr_->free_heads));
  std::vector<std::pair<uint64_t, uint64_t>> used;  // (block offset, block size)
  for (uint64_t i = 0; i < cap; i++) {
    const Entry& e = table_[i];
    if (e.state != kEmpty && e.state != kTombstone && resident(e) && e.offset)
      used.push_back({e.offset - kBlockHdr, std::max(AlignUp(e.data_size + e.meta_size, kAlign) + kBlockHdr,
                                                     kMinBlock)});
  }
  std::sort(used.begin(), used.end());
  uint64_t cur = heap_lo, prev = 0;
  st.bytes_in_use = 0;
  auto put = [&](uint64_t off, uint64_t size, bool free_blk) {
    Blk* b = reinterpret_cast<Blk*>(base_ + off);
    b->size = size | (free_blk ? kFreeBit : 0);
    b->prev_phys = prev;
    b->next_free = b->prev_free = kNil;
    if (free_blk) TlsfInsert(off);
    else st.bytes_in_use += size;
    prev = off;
  };
  for (auto& u : used) {
    if (u.first > cur) put(cur, u.first - cur, true);
    put(u.first, u.second, false);
    cur = u.first + u.second;
  }
  if (heap_hi > cur) put(cur, heap_hi - cur, true);
  Blk* sentinel = reinterpret_cast<Blk*>(base_ + heap_hi);
  sentinel->size = kBlockHdr;
  sentinel->prev_phys = prev;
  hdr_->recovered_dropped_total += dropped;
  __atomic_add_fetch(&hdr_->recoveries_total, 1, __ATOMIC_RELEASE);
  Broadcast();
}

void Store::CondWait(int64_t deadline_ns) {
  if (deadline_ns < 0) {
    // Bounded waits even for "forever" so a lost wakeup can never hang a reader.
    deadline_ns = NowNs() + 200000000ll;
  }
  // the word is read under the lock and every Broadcast bumps it under the lock, so a broadcast between
  // the unlock and the futex wait makes the wait return at once (EAGAIN): no lost wakeup
  const uint32_t v = __atomic_load_n(&hdr_->cv_seq, __ATOMIC_ACQUIRE);
  Unlock();
  const int64_t rem = deadline_ns - NowNs();
  if (rem > 0) {
    timespec rel;
    rel.tv_sec = rem / 1000000000ll;
    rel.tv_nsec = rem % 1000000000ll;
    syscall(SYS_futex, &hdr_->cv_seq, FUTEX_WAIT, v, &rel, nullptr, 0);  // shared (not _PRIVATE): cross-process
  }
  Lock();
}

void Store::Broadcast() {
  __atomic_add_fetch(&hdr_->cv_seq, 1u, __ATOMIC_RELEASE);
  syscall(SYS_futex, &hdr_->cv_seq, FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}

void Store::Wake() {
  Lock();
  Broadcast();
  Unlock();
}

// ---------------------------------------------------------------- TLSF allocator

void Store::TlsfInsert(uint64_t blk) {
  Blk* b = reinterpret_cast<Blk*>(base_ + blk);
  int fl, sl;
  MappingInsert(b->size & kSizeMask, &fl, &sl);
  uint64_t head = hdr_->free_heads[fl][sl];
  b->next_free = head;
  b->prev_free = kNil;
  if (head != kNil) reinterpret_cast<Blk*>(base_ + head)->prev_free = blk;
  hdr_->free_heads[fl][sl] = blk;
  hdr_->fl_bitmap |= (1ull << fl);
  hdr_->sl_bitmap[fl] |= (1u << sl);
}

void Store::TlsfRemove(uint64_t blk) {
  Blk* b = reinterpret_cast<Blk*>(base_ + blk);
  int fl, sl;
  MappingInsert(b->size & kSizeMask, &fl, &sl);
  if (b->prev_free != kNil) reinterpret_cast<Blk*>(base_ + b->prev_free)->next_free = b->next_free;
  if (b->next_free != kNil) reinterpret_cast<Blk*>(base_ + b->next_free)->prev_free = b->prev_free;
  if (hdr_->free_heads[fl][sl] == blk) {
    hdr_->free_heads[fl][sl] = b->next_free;
    if (b->next_free == kNil) {
      hdr_->sl_bitmap[fl] &= ~(1u << sl);
      if (hdr_->sl_bitmap[fl] == 0) hdr_->fl_bitmap &= ~(1ull << fl);
    }
  }
  b->next_free = b->prev_free = kNil;
}

uint64_t Store::TlsfFind(uint64_t size) {
  // Round up to the next class boundary so any block in the found list fits.
  int f0 = 63 - __builtin_clzll(size);
  uint64_t rounded = size + (uint64_t(1) << (f0 - kSLBits)) - 1;
  int fl, sl;
  MappingInsert(rounded, &fl, &sl);
  if (fl >= kFL) return kNil;
  uint32_t sl_map = hdr_->sl_bitmap[fl] & (~0u << sl);
  if (sl_map == 0) {
    uint64_t fl_map = (fl + 1 >= 64) ? 0 : (hdr_->fl_bitmap & (~0ull << (fl + 1)));
    if (fl_map == 0) return kNil;
    fl = __builtin_ctzll(fl_map);
    sl_map = hdr_->sl_bitmap[fl];
  }
  sl = __builtin_ctz(sl_map);
  uint64_t blk = hdr_->free_heads[fl][sl];
  if (blk != kNil) TlsfRemove(blk);
  return blk;
}

uint64_t Store::HeapAlloc(uint64_t n) {
  uint64_t need = AlignUp(n, kAlign) + kBlockHdr;
  if (need < kMinBlock) need = kMinBlock;
  uint64_t blk = TlsfFind(need);
  if (blk == kNil) return kNil;
  Blk* b = reinterpret_cast<Blk*>(base_ + blk);
  uint64_t bsize = b->size & kSizeMask;
  uint64_t rem = bsize - need;
  if (rem >= kMinBlock) {
    uint64_t nb = blk + need;
    Blk* n2 = reinterpret_cast<Blk*>(base_ + nb);
    n2->size = rem | kFreeBit;
    n2->prev_phys = blk;
    Blk* after = reinterpret_cast<Blk*>(base_ + nb + rem);
    after->prev_phys = nb;
    TlsfInsert(nb);
    bsize = need;
  }
  CrashPoint(1);  // the remainder is listed free, the block itself still carries its free bit
  b->size = bsize;  // used
  hdr_->stats.bytes_in_use += bsize;
  return blk + kBlockHdr;
}

void Store::HeapFree(uint64_t payload_off) {
  if (!UsedBlock(payload_off)) {
    // never merge from a block that is not ours (offset 0 = "no block yet" would address the segment
    // header): count it and leak nothing else
    __atomic_add_fetch(&hdr_->corruptions_total, 1, __ATOMIC_RELEASE);
    fprintf(stderr, "[rmm store] pid %d: refused to free heap offset %llu (not a used block)\n", int(getpid()),
            (unsigned long long)payload_off);
    return;
  }
  uint64_t blk = payload_off - kBlockHdr;
  Blk* b = reinterpret_cast<Blk*>(base_ + blk);
  uint64_t bsize = b->size & kSizeMask;
  hdr_->stats.bytes_in_use -= bsize;
  // merge with previous
  if (b->prev_phys != 0) {
    Blk* p = reinterpret_cast<Blk*>(base_ + b->prev_phys);
    if (p->size & kFreeBit) {
      TlsfRemove(b->prev_phys);
      CrashPoint(2);  // a free block unlisted but still marked free
      uint64_t psize = p->size & kSizeMask;
      blk = b->prev_phys;
      bsize += psize;
      b = p;
    }
  }
  // merge with next
  uint64_t nxt = blk + bsize;
  Blk* nb = reinterpret_cast<Blk*>(base_ + nxt);
  if (nb->size & kFreeBit) {
    TlsfRemove(nxt);
    bsize += nb->size & kSizeMask;
  }
  b->size = bsize | kFreeBit;
  Blk* after = reinterpret_cast<Blk*>(base_ + blk + bsize);
  after->prev_phys = blk;
  TlsfInsert(blk);
}

void Store::HeapShrink(uint64_t payload_off, uint64_t n) {
  uint64_t blk = payload_off - kBlockHdr;
  Blk* b = reinterpret_cast<Blk*>(base_ + blk);
  uint64_t bsize = b->size & kSizeMask;
  uint64_t need = AlignUp(n, kAlign) + kBlockHdr;
  if (need < kMinBlock) need = kMinBlock;
  if (bsize < need || bsize - need < kMinBlock) return;
  uint64_t rem = bsize - need;
  uint64_t nb = blk + need;
  Blk* tail = reinterpret_cast<Blk*>(base_ + nb);
  tail->prev_phys = blk;
  // coalesce the freed tail with a free physical successor
  uint64_t nxt = blk + bsize;
  Blk* nx = reinterpret_cast<Blk*>(base_ + nxt);
  if (nx->size & kFreeBit) {
    TlsfRemove(nxt);
    rem += nx->size & kSizeMask;
  }
  tail->size = rem | kFreeBit;
  reinterpret_cast<Blk*>(base_ + nb + rem)->prev_phys = nb;
  TlsfInsert(nb);
  b->size = need;
  hdr_->stats.bytes_in_use -= bsize - need;
}

bool Store::ShrinkCreating(const ObjectId& id, uint64_t data_size) {
  Lock();
  int64_t idx = Find(id);
  bool ok = idx >= 0 && E(idx)->state == kCreating && !(E(idx)->flags & kFlagFallback) &&
            E(idx)->meta_size == 0 && data_size <= E(idx)->data_size;
  if (ok) {
    HeapShrink(E(idx)->offset, data_size);
    E(idx)->data_size = data_size;
  }
  Unlock();
  return ok;
}

uint64_t Store::CheckHeap() {
  Lock();
  uint64_t off = hdr_->heap_off, end = hdr_->heap_off + hdr_->heap_size - kBlockHdr;
  uint64_t prev = 0, free_bytes = 0, used_bytes = 0, nfree = 0;
  bool ok = true;
  bool prev_free = false;
  while (off < end) {
    Blk* b = reinterpret_cast<Blk*>(base_ + off);
    uint64_t sz = b->size & kSizeMask;
    if (sz == 0 || b->prev_phys != prev) { ok = false; break; }
    bool fr = b->size & kFreeBit;
    if (fr && prev_free) { ok = false; break; }  // adjacent free blocks must be merged
    if (fr) { free_bytes += sz; nfree++; } else { used_bytes += sz; }
    prev_free = fr;
    prev = off;
    off += sz;
  }
  if (off != end) ok = false;
  uint64_t listed = 0;
  const uint64_t max_blocks = hdr_->heap_size / kMinBlock + 1;
  for (int f = 0; f < kFL && ok; f++)
    for (int s = 0; s < kSL && ok; s++)
      for (uint64_t b = hdr_->free_heads[f][s]; b != kNil && ok;
           b = reinterpret_cast<Blk*>(base_ + b)->next_free) {
        // a listed block must be a free block inside the heap; the walk is bounded (no cycle can spin)
        ok = b >= hdr_->heap_off && b < end && (reinterpret_cast<Blk*>(base_ + b)->size & kFreeBit) &&
             ++listed <= max_blocks;
      }
  // LRU list: bounded, consistent links, only evictable entries
  {
    uint64_t n = 0;
    int32_t prev_i = -1;
    for (int32_t i = hdr_->lru_head; i >= 0 && ok; i = table_[i].lru_next) {
      ok = uint64_t(i) < hdr_->table_cap && ++n <= hdr_->table_cap && table_[i].in_lru &&
           table_[i].lru_prev == prev_i && table_[i].state == kSealed && table_[i].pin_count == 0;
      prev_i = i;
      if (!ok) break;
    }
    if (ok && prev_i != hdr_->lru_tail) ok = false;
  }
  if (listed != nfree) ok = false;
  if (used_bytes != hdr_->stats.bytes_in_use) ok = false;
  Unlock();
  if (!ok) throw std::runtime_error("heap check failed");
  return free_bytes;
}

// ---------------------------------------------------------------- object table

int64_t Store::Find(const ObjectId& id) {
  uint64_t mask = hdr_->table_cap - 1;
  uint64_t i = HashId(id) & mask;
  for (uint64_t n = 0; n <= mask; n++, i = (i + 1) & mask) {
    Entry* e = &table_[i];
    if (e->state == kEmpty) return -1;
    if (e->state != kTombstone && memcmp(e->id, id.b, kIdSize) == 0) return int64_t(i);
  }
  return -1;
}

int64_t Store::Insert(const ObjectId& id) {
  uint64_t cap = hdr_->table_cap;
  uint64_t live_now = hdr_->stats.num_objects;
  // truly full (keeps >= 1/16 of the slots empty or tombstoned so probes terminate quickly);
  // the caller unlocks and reports -- never throw while holding the store mutex
  if (live_now + 1 > cap - cap / 16) return -1;
  if (hdr_->table_used + 1 > cap - cap / 8 && live_now + 1 <= cap - cap / 4) {
    // Too many tombstones: rebuild in place, keeping LRU order.
    uint64_t live = live_now;
    std::vector<Entry> keep;
    keep.reserve(live);
    std::vector<int64_t> lru_order;
    bool damaged = false;
    for (int32_t i = hdr_->lru_head; i >= 0;) {
      damaged = uint64_t(i) >= cap || lru_order.size() >= cap || !table_[i].in_lru;
      if (damaged) break;
      lru_order.push_back(i);
      i = table_[i].lru_next;
    }
    if (damaged) {
      Heal("LRU list walk exceeded the table during a rehash");  // rebuilds the table without tombstones
    } else {
      std::vector<ObjectId> lru_ids;
      for (auto i : lru_order) { ObjectId o; memcpy(o.b, table_[i].id, kIdSize); lru_ids.push_back(o); }
      for (uint64_t i = 0; i < cap; i++)
        if (table_[i].state != kEmpty && table_[i].state != kTombstone) keep.push_back(table_[i]);
      memset(table_, 0, cap * sizeof(Entry));
      hdr_->table_used = 0;
      hdr_->lru_head = hdr_->lru_tail = -1;
      for (auto& e : keep) {
        ObjectId o;
        memcpy(o.b, e.id, kIdSize);
        uint64_t mask = cap - 1, j = HashId(o) & mask;
        while (table_[j].state != kEmpty) j = (j + 1) & mask;
        table_[j] = e;
        table_[j].in_lru = 0;
        table_[j].lru_prev = table_[j].lru_next = -1;
        hdr_->table_used++;
      }
      for (auto& o : lru_ids) LruPush(Find(o));
    }
  }
  uint64_t mask = cap - 1;
  uint64_t i = HashId(id) & mask;
  int64_t tomb = -1;
  for (uint64_t n = 0; n <= mask; n++, i = (i + 1) & mask) {
    Entry* e = &table_[i];
    if (e->state == kEmpty) break;
    if (e->state == kTombstone) {
      if (tomb < 0) tomb = int64_t(i);
      continue;
    }
    if (memcmp(e->id, id.b, kIdSize) == 0) return -2 - int64_t(i);  // exists
  }
  int64_t slot = tomb >= 0 ? tomb : int64_t(i);
  if (tomb < 0) hdr_->table_used++;
  Entry* e = &table_[slot];
  memset(e, 0, sizeof(Entry));
  memcpy(e->id, id.b, kIdSize);
  CrashPoint(3);  // table_used counted, entry half written, num_objects not yet
  e->lru_prev = e->lru_next = -1;
  hdr_->stats.num_objects++;
  return slot;
}

void Store::RemoveEntry(int64_t idx) {
  Entry* e = E(idx);
  if (e->in_lru) LruRemove(idx);
  e->state = kTombstone;
  hdr_->stats.num_objects--;
}

void Store::LruPush(int64_t idx) {
  Entry* e = E(idx);
  if (e->in_lru) return;
  e->in_lru = 1;
  e->lru_next = -1;
  e->lru_prev = hdr_->lru_tail;
  if (hdr_->lru_tail >= 0) table_[hdr_->lru_tail].lru_next = int32_t(idx);
  hdr_->lru_tail = int32_t(idx);
  if (hdr_->lru_head < 0) hdr_->lru_head = int32_t(idx);
}

void Store::LruRemove(int64_t idx) {
  Entry* e = E(idx);
  if (!e->in_lru) return;
  if (e->lru_prev >= 0) table_[e->lru_prev].lru_next = e->lru_next;
  else hdr_->lru_head = e->lru_next;
  CrashPoint(4);  // the list skips the entry one way but not the other
  if (e->lru_next >= 0) table_[e->lru_next].lru_prev = e->lru_prev;
  else hdr_->lru_tail = e->lru_prev;
  e->lru_prev = e->lru_next = -1;
  e->in_lru = 0;
}

// ---------------------------------------------------------------- per-client pins

namespace {
inline uint64_t PinHash(const uint8_t* id, int32_t pid) {
  ObjectId o;
  memcpy(o.b, id, kIdSize);
  uint64_t h = HashId(o) ^ (uint64_t(uint32_t(pid)) * 0x9E3779B97F4A7C15ull);
  h ^= h >> 31;
  return h;
}
}  // namespace

int64_t Store::PinFind(const uint8_t* id, int32_t pid) {
  PinRec* P = Pins();
  const uint64_t mask = kPinCap - 1;
  uint64_t i = PinHash(id, pid) & mask;
  for (uint64_t n = 0; n <= mask; n++, i = (i + 1) & mask) {
    if (P[i].state == 0) return -1;
    if (P[i].state == 1 && P[i].pid == pid && memcmp(P[i].id, id, kIdSize) == 0) return int64_t(i);
  }
  return -1;
}

void Store::PinRehash() {
  PinRec* P = Pins();
  std::vector<PinRec> live;
  for (uint64_t i = 0; i < kPinCap; i++)
    if (P[i].state == 1) live.push_back(P[i]);
  memset(P, 0, kPinCap * sizeof(PinRec));
  hdr_->pins_used = hdr_->pins_live = 0;
  for (auto& r : live) PinInsert(r.id, r.pid, r.count);
}

// a new record (the caller checked there is none for (id, pid)); false when the table is full
bool Store::PinInsert(const uint8_t* id, int32_t pid, int32_t count) {
  if (hdr_->pins_used + 1 > kPinCap - kPinCap / 4) {
    if (hdr_->pins_live + 1 > kPinCap / 2) return false;
    PinRehash();  // mostly tombstones
  }
  PinRec* P = Pins();
  const uint64_t mask = kPinCap - 1;
  uint64_t i = PinHash(id, pid) & mask;
  while (P[i].state == 1) i = (i + 1) & mask;
  if (P[i].state == 0) hdr_->pins_used++;
  memcpy(P[i].id, id, kIdSize);
  P[i].pid = pid;
  P[i].count = count;
  P[i].state = 1;
  hdr_->pins_live++;
  return true;
}

void Store::PinAdd(int64_t idx, int32_t pid) {
  Entry* e = E(idx);
  const int64_t r = PinFind(e->id, pid);
  if (r >= 0) {
    Pins()[r].count++;
  } else if (!PinInsert(e->id, pid, 1)) {
    e->anon_pins++;  // no room for a record: this pin cannot be released on the client's death
    hdr_->pin_overflow_total++;
  }
  e->pin_count++;
}

void Store::PinErase(const uint8_t* id, int32_t pid) {
  const int64_t r = PinFind(id, pid);
  if (r < 0) return;
  Pins()[r].state = 2;
  Pins()[r].count = 0;
  hdr_->pins_live--;
}

// Release one pin of entry idx on behalf of `pid`: its own record, else an anonymous pin (a pin taken
// when the record table was full). A release by a process that holds neither (a late release after
// ReleaseClient already dropped its pins) is counted and ignored: taking another client's record would
// let the object be evicted while that client still maps it.
void Store::PinDrop(int64_t idx, int32_t pid) {
  Entry* e = E(idx);
  if (e->pin_count <= 0) return;
  PinRec* P = Pins();
  int64_t r = PinFind(e->id, pid);
  if (r < 0 && e->anon_pins > (e->io_pid != 0 ? 1 : 0)) {  // never the spill / restore IO pin
    e->anon_pins--;
    e->pin_count--;
    return;
  }
  if (r < 0) {
    hdr_->unmatched_releases_total++;
    return;
  }
  if (--P[r].count <= 0) {
    P[r].state = 2;
    P[r].count = 0;
    hdr_->pins_live--;
  }
  e->pin_count--;
}

void Store::IoPin(int64_t idx) {
  Entry* e = E(idx);
  e->anon_pins++;
  e->pin_count++;
  e->io_pid = int32_t(getpid());
  hdr_->io_now++;
}

void Store::IoUnpin(int64_t idx) {
  Entry* e = E(idx);
  if (e->anon_pins > 0) e->anon_pins--;
  if (e->pin_count > 0) e->pin_count--;
  if (e->io_pid != 0 && hdr_->io_now > 0) hdr_->io_now--;
  e->io_pid = 0;
}

// entry idx just lost its last pin: free it if a delete is pending, else make it evictable
void Store::FinishUnpinned(int64_t idx) {
  Entry* e = E(idx);
  if (e->pin_count != 0) return;
  if (e->flags & kFlagDeletePending) {
    if (e->state == kCreating) hdr_->creating_now--;
    if (e->state == kSealed) hdr_->stats.num_sealed--;
    FreeEntryStorage(idx);
    RemoveEntry(idx);
  } else if (e->state == kSealed && !(e->flags & kFlagFallback)) {
    LruPush(idx);
  }
}

// ---------------------------------------------------------------- spill files

std::vector<std::string> Store::SpillDirs() const {
  std::vector<std::string> out;
  std::string all(hdr_->spill_dir);
  size_t b = 0;
  while (b <= all.size()) {
    size_t e = all.find(':', b);
    if (e == std::string::npos) e = all.size();
    if (e > b) out.push_back(all.substr(b, e - b));
    b = e + 1;
  }
  return out;
}

// Spill / fallback files are spread round-robin over the configured directories (reference:
// python/ray/_private/external_storage.py FileSystemStorage with several directory_path entries).
std::string Store::DirFor(uint64_t fid) const {
  const char* all = hdr_->spill_dir;
  int n = 1;
  for (const char* c = all; *c; c++) n += (*c == ':');
  int k = int(fid % uint64_t(n)), i = 0;
  const char* b = all;
  for (const char* c = all;; c++) {
    if (*c == ':' || *c == 0) {
      if (i == k) return std::string(b, size_t(c - b));
      if (*c == 0) break;
      i++;
      b = c + 1;
    }
  }
  return std::string(all);
}

std::string Store::SpillPath(uint64_t fid) const {
  return DirFor(fid) + "/rmm-spill-" + std::to_string(fid) + ".bin";
}
std::string Store::FallbackPath(uint64_t fid) const {
  return DirFor(fid) + "/rmm-fallback-" + std::to_string(fid) + ".bin";
}

void Store::SetDiskFull(bool full) {
  Lock();
  hdr_->disk_full = full ? 1 : 0;
  Broadcast();
  Unlock();
}

void Store::SetSpillEnabled(bool on) {
  // spilling needs a directory: a store created without one keeps it off (fallback files are separate)
  Lock();
  hdr_->spill_enabled = (on && hdr_->spill_dir[0] != 0) ? 1 : 0;
  Broadcast();
  Unlock();
}

void Store::SetOomGrace(double seconds) {
  Lock();
  hdr_->oom_grace_ns = int64_t(seconds * 1e9);
  Unlock();
}

int64_t Store::SpillSlot(uint64_t fid, bool create) {
  uint64_t i = fid & (kSpillSlots - 1);
  for (uint64_t n = 0; n < kSpillSlots; n++, i = (i + 1) & (kSpillSlots - 1)) {
    if (spill_[i].file_id == fid) return int64_t(i);
    if (create && spill_[i].file_id == 0) {
      spill_[i].file_id = fid;
      spill_[i].live = 0;
      return int64_t(i);
    }
  }
  return -1;
}

void Store::DropSpillRef(uint64_t fid) {
  int64_t s = SpillSlot(fid, false);
  if (s < 0) return;
  if (--spill_[s].live <= 0) {
    spill_[s].file_id = 0;
    unlink(SpillPath(fid).c_str());
  }
}

uint8_t* Store::FallbackMap(uint64_t fid, uint64_t size, bool create) {
  pthread_mutex_lock(&fb_mu_);
  for (auto& m : fb_maps_)
    if (m.fid == fid) { pthread_mutex_unlock(&fb_mu_); return m.ptr; }
  std::string path = FallbackPath(fid);
  int fd = open(path.c_str(), create ? (O_CREAT | O_RDWR) : O_RDWR, 0600);
  uint8_t* ptr = nullptr;
  uint64_t msz = size ? size : 1;
  if (fd >= 0) {
    if (!create || ftruncate(fd, off_t(msz)) == 0) {
      void* p = mmap(nullptr, msz, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (p != MAP_FAILED) ptr = static_cast<uint8_t*>(p);
    }
    close(fd);
  }
  if (ptr) fb_maps_.push_back({fid, ptr, msz});
  pthread_mutex_unlock(&fb_mu_);
  return ptr;
}

void Store::FallbackUnlink(uint64_t fid) {
  pthread_mutex_lock(&fb_mu_);
  for (size_t i = 0; i < fb_maps_.size(); i++) {
    if (fb_maps_[i].fid == fid) {
      munmap(fb_maps_[i].ptr, fb_maps_[i].size);
      fb_maps_.erase(fb_maps_.begin() + long(i));
      break;
    }
  }
  pthread_mutex_unlock(&fb_mu_);
  unlink(FallbackPath(fid).c_str());
}

void Store::FreeEntryStorage(int64_t idx) {
  Entry* e = E(idx);
  if (e->flags & kFlagFallback) {
    hdr_->stats.fallback_bytes_current -= e->data_size + e->meta_size;
    FallbackUnlink(e->fallback_id);
    e->flags &= ~kFlagFallback;
  } else if (e->state == kSealed || e->state == kCreating || e->state == kSpilling) {
    // a create still waiting for memory (or mapping its fallback file with the lock dropped) owns no
    // heap block: offset 0 means "none", it is not a block to free
    if (e->offset != 0) HeapFree(e->offset);
    e->offset = 0;
    if (e->state == kCreating && e->fallback_id != 0) {
      unlink(FallbackPath(e->fallback_id).c_str());  // a fallback file reserved by a creator that died mapping it
      e->fallback_id = 0;
    }
  }
  if (e->flags & kFlagHasSpillCopy) {
    DropSpillRef(e->spill_file);
    if (e->state == kSpilled) {
      hdr_->stats.spilled_bytes_current -= e->data_size + e->meta_size;
      hdr_->stats.spilled_objects_current--;
    }
    e->flags &= ~kFlagHasSpillCopy;
  }
}

// Spill LRU victims with the lock held on entry and exit (released around file IO).
uint64_t Store::SpillLocked(uint64_t bytes, std::vector<int64_t>* /*unused*/) {
  if (!hdr_->spill_enabled || hdr_->disk_full) return 0;
  uint64_t freed = 0;
  // 1) free objects that already have an up-to-date spill copy (no IO needed)
  std::vector<ObjectId> batch;
  uint64_t batch_bytes = 0;
  uint64_t target = std::max<uint64_t>(bytes, hdr_->min_spill_size);
  const uint64_t cap = hdr_->table_cap;
  uint64_t steps = 0;
  bool damaged = false;
  for (int32_t i = hdr_->lru_head; i >= 0 && (freed < bytes || batch_bytes < target);) {
    // the LRU list links at most every slot once: a longer walk, an out-of-range link or a listed entry
    // that is not marked in_lru means the metadata is damaged -- never follow it under the mutex
    if (uint64_t(i) >= cap || ++steps > cap || !table_[i].in_lru) {
      damaged = true;
      break;
    }
    Entry* e = &table_[i];
    int32_t nxt = e->lru_next;
    if (e->state == kSealed && e->pin_count == 0 && !(e->flags & kFlagFallback)) {
      if (e->flags & kFlagHasSpillCopy) {
        LruRemove(i);
        HeapFree(e->offset);
        e->state = kSpilled;
        hdr_->stats.spilled_bytes_current += e->data_size + e->meta_size;
        hdr_->stats.spilled_objects_current++;
        freed += AlignUp(e->data_size + e->meta_size, kAlign) + kBlockHdr;
      } else if (freed + batch_bytes < bytes || batch_bytes < target) {
        ObjectId o;
        memcpy(o.b, e->id, kIdSize);
        batch.push_back(o);
        batch_bytes += AlignUp(e->data_size + e->meta_size, kAlign) + kBlockHdr;
        LruRemove(i);
        e->state = kSpilling;
        IoPin(i);
      }
    }
    i = nxt;
  }
  if (damaged) {
    for (auto& o : batch) {  // undo this walk's claims, then rebuild from the entries
      const int64_t idx = Find(o);
      if (idx < 0) continue;
      E(idx)->state = kSealed;
      IoUnpin(idx);
    }
    Heal("LRU list walk exceeded the table (cycle or bad link)");
    return freed;
  }
  if (batch.empty()) return freed;
  uint64_t fid = hdr_->next_file_id++;
  struct Item { ObjectId id; uint64_t off, len; uint8_t* src; };
  std::vector<Item> items;
  uint64_t foff = 0;
  for (auto& o : batch) {
    Entry* e = E(Find(o));
    uint64_t len = e->data_size + e->meta_size;
    items.push_back({o, foff, len, base_ + e->offset});
    foff += AlignUp(len, 4096);
  }
  Unlock();
  CrashPoint(6);  // spill IO in progress, lock released: the victims are kSpilling with this pid's IO pin
  bool ok = true;
  std::string path = SpillPath(fid);
  int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0600);
  if (fd < 0) ok = false;
  for (auto& it : items) {
    if (!ok) break;
    uint64_t done = 0;
    while (done < it.len) {
      ssize_t w = pwrite(fd, it.src + done, it.len - done, off_t(it.off + done));
      if (w <= 0) { ok = false; break; }
      done += uint64_t(w);
    }
  }
  if (fd >= 0) close(fd);
  Lock();
  if (!ok) unlink(path.c_str());
  int64_t slot = ok ? SpillSlot(fid, true) : -1;
  for (auto& it : items) {
    int64_t idx = Find(it.id);
    if (idx < 0) continue;
    Entry* e = E(idx);
    IoUnpin(idx);
    if (!ok || slot < 0) {
      e->state = kSealed;
      if (e->pin_count == 0) LruPush(idx);
      continue;
    }
    e->flags |= kFlagHasSpillCopy;
    e->spill_file = fid;
    e->spill_off = it.off;
    spill_[slot].live++;
    hdr_->stats.bytes_spilled_total += it.len;
    hdr_->stats.objects_spilled_total++;
    if (e->flags & kFlagDeletePending) {
      if (e->pin_count == 0) {
        e->state = kSealed;
        FreeEntryStorage(idx);
        RemoveEntry(idx);
        freed += AlignUp(it.len, kAlign) + kBlockHdr;
      } else {
        e->state = kSealed;
      }
      continue;
    }
    if (e->pin_count == 0) {
      HeapFree(e->offset);
      e->state = kSpilled;
      hdr_->stats.spilled_bytes_current += it.len;
      hdr_->stats.spilled_objects_current++;
      freed += AlignUp(it.len, kAlign) + kBlockHdr;
    } else {
      e->state = kSealed;  // someone pinned it meanwhile; keep in memory + spill copy
    }
  }
  if (slot >= 0 && spill_[slot].live == 0) {
    spill_[slot].file_id = 0;
    unlink(path.c_str());
  }
  Broadcast();
  return freed;
}

uint64_t Store::SpillBytes(uint64_t bytes) {
  Lock();
  uint64_t f = SpillLocked(bytes, nullptr);
  Unlock();
  return f;
}

bool Store::RestoreLocked(int64_t idx) {
  Entry* e = E(idx);
  ObjectId id;
  memcpy(id.b, e->id, kIdSize);
  uint64_t len = e->data_size + e->meta_size;
  e->state = kRestoring;
  e->offset = 0;  // no heap block yet (the allocation below may spill with the lock dropped)
  IoPin(idx);
  uint64_t off = HeapAlloc(len);
  while (off == kNil) {
    uint64_t f = SpillLocked(len, nullptr);
    off = HeapAlloc(len);
    if (off == kNil && f == 0) break;
  }
  idx = Find(id);
  if (idx < 0) {  // dropped by a rebuild while a spill had the lock released
    if (off != kNil) HeapFree(off);
    Broadcast();
    return false;
  }
  e = E(idx);
  if (off == kNil) {
    e->state = kSpilled;
    IoUnpin(idx);
    Broadcast();
    return false;
  }
  uint64_t fid = e->spill_file, foff = e->spill_off;
  uint8_t* dst = base_ + off;
  e->offset = off;  // the block is owned by this entry while the lock is dropped (crash recovery)
  Unlock();
  CrashPoint(5);  // restore IO in progress, lock released: kRestoring with this pid's IO pin
  bool ok = true;
  int fd = open(SpillPath(fid).c_str(), O_RDONLY);
  if (fd < 0) ok = false;
  uint64_t done = 0;
  while (ok && done < len) {
    ssize_t r = pread(fd, dst + done, len - done, off_t(foff + done));
    if (r <= 0) { ok = false; break; }
    done += uint64_t(r);
  }
  if (fd >= 0) close(fd);
  Lock();
  idx = Find(id);
  if (idx < 0) {
    HeapFree(off);
    Broadcast();
    return false;
  }
  e = E(idx);
  IoUnpin(idx);
  if (!ok) {
    HeapFree(off);
    e->state = kSpilled;
    Broadcast();
    return false;
  }
  e->offset = off;
  e->state = kSealed;
  hdr_->stats.spilled_bytes_current -= len;
  hdr_->stats.spilled_objects_current--;
  hdr_->stats.bytes_restored_total += len;
  hdr_->stats.objects_restored_total++;
  Broadcast();
  return true;
}

// ---------------------------------------------------------------- public API

uint8_t* Store::CreateObject(const ObjectId& id, uint64_t data_size, uint64_t meta_size,
                             uint32_t user_tag, uint32_t flags, bool* exists) {
  *exists = false;
  uint64_t len = data_size + meta_size;
  Lock();
  int64_t idx = Insert(id);
  if (idx == -1) {
    uint64_t live = hdr_->stats.num_objects;
    Unlock();
    throw std::runtime_error("ObjectStoreFullError: object table full (" + std::to_string(live) +
                             " live objects)");
  }
  if (idx <= -2) {
    *exists = true;
    Unlock();
    return nullptr;
  }
  Entry* e = E(idx);
  e->state = kCreating;
  hdr_->creating_now++;
  e->flags = flags & kFlagError;
  e->user_tag = user_tag;
  e->data_size = data_size;
  e->meta_size = meta_size;
  e->pin_count = 0;
  e->creator_pid = getpid();
  PinAdd(idx, e->creator_pid);  // the creator's pin (released after seal, or on its death)
  e->create_ns = uint64_t(NowNs());
  hdr_->stats.creates_total++;
  // proactive threshold spilling is driven by the node (SpillBytes); here only on demand.
  // Create-request queue semantics (reference plasma/create_request_queue.cc:88): when neither
  // the heap nor spilling can satisfy the request, wait — bumping gc_requests so the node
  // broadcasts a global GC, and letting in-flight spills / releases free memory — for up to
  // oom_grace_ns, then fall back to a file-backed allocation (if enabled) or fail.
  uint64_t off = HeapAlloc(len);
  int64_t wait_deadline = -1;
  bool waited = false;
  for (;;) {
    while (off == kNil && hdr_->spill_enabled && !hdr_->disk_full) {
      uint64_t f = SpillLocked(len, nullptr);
      off = HeapAlloc(len);
      if (f == 0) break;
    }
    if (off != kNil || hdr_->oom_grace_ns <= 0 || len > hdr_->heap_size) break;
    const int64_t now = NowNs();
    if (wait_deadline < 0) {
      wait_deadline = now + hdr_->oom_grace_ns;
      __atomic_add_fetch(&hdr_->gc_requests, 1, __ATOMIC_RELEASE);
      if (!waited) hdr_->oom_waits_total++;
      waited = true;
    }
    if (now >= wait_deadline) break;
    CondWait(std::min<int64_t>(wait_deadline, now + 20000000ll));  // re-check every 20 ms (or on a broadcast)
    off = HeapAlloc(len);
  }
  // the lock was dropped (spill IO, grace wait): the pending entry may have been aborted meanwhile
  auto still_mine = [&]() {
    idx = Find(id);
    return idx >= 0 && E(idx)->state == kCreating && E(idx)->creator_pid == int32_t(getpid());
  };
  if (!still_mine()) {
    if (off != kNil) HeapFree(off);
    Broadcast();
    Unlock();
    throw std::runtime_error("ObjectStoreFullError: the pending create was aborted while waiting for memory");
  }
  e = E(idx);
  uint8_t* ptr = nullptr;
  if (off != kNil) {
    e->offset = off;
    ptr = base_ + off;
  } else if (hdr_->fallback_enabled && !hdr_->disk_full) {
    uint64_t fid = hdr_->next_file_id++;
    e->fallback_id = fid;  // reserved: an abort while the file is mapped unlinks it (FreeEntryStorage)
    Unlock();
    ptr = FallbackMap(fid, len, true);
    Lock();
    if (!still_mine()) {
      FallbackUnlink(fid);
      Broadcast();
      Unlock();
      throw std::runtime_error("ObjectStoreFullError: the pending create was aborted while mapping its fallback file");
    }
    e = E(idx);
    if (ptr) {
      e->flags |= kFlagFallback;
      hdr_->stats.fallback_bytes_current += len;
      hdr_->stats.fallback_allocs_total++;
    } else {
      e->fallback_id = 0;
      unlink(FallbackPath(fid).c_str());
    }
  }
  if (!ptr) {
    PinErase(e->id, e->creator_pid);
    RemoveEntry(idx);
    hdr_->creating_now--;
    hdr_->oom_errors_total++;
    const bool disk = hdr_->disk_full != 0;
    Unlock();
    if (disk)
      throw std::runtime_error("OutOfDiskError: local disk is full: cannot spill or fall back to allocate " +
                               std::to_string(len) + " bytes (capacity " + std::to_string(hdr_->heap_size) + ")");
    throw std::runtime_error("ObjectStoreFullError: cannot allocate " + std::to_string(len) +
                             " bytes (capacity " + std::to_string(hdr_->heap_size) + ")");
  }
  Unlock();
  return ptr;
}

void Store::Seal(const ObjectId& id) {
  Lock();
  int64_t idx = Find(id);
  if (idx < 0 || E(idx)->state != kCreating) {
    Unlock();
    throw std::runtime_error("Seal: object not in creating state");
  }
  Entry* e = E(idx);
  e->state = kSealed;
  hdr_->creating_now--;
  hdr_->stats.num_sealed++;
  hdr_->seal_seq++;
  memcpy(ring_[hdr_->ring_head & (kRingCap - 1)].b, e->id, kIdSize);
  hdr_->ring_head++;
  Broadcast();
  Unlock();
}

void Store::Abort(const ObjectId& id) {
  Lock();
  int64_t idx = Find(id);
  // another process may abort a create only once its creator is gone: a live creator may be writing
  // into the block right now (it aborts its own creates itself)
  const int32_t creator = idx >= 0 ? E(idx)->creator_pid : 0;
  const bool creator_gone = creator == int32_t(getpid()) || ProcessGone(creator);
  if (idx >= 0 && E(idx)->state == kCreating && creator_gone) {
    PinErase(E(idx)->id, E(idx)->creator_pid);
    FreeEntryStorage(idx);
    RemoveEntry(idx);
    hdr_->creating_now--;
  }
  Unlock();
}

int Store::AbortCreator(int pid) {
  int n = 0;
  Lock();
  // a dead worker usually created nothing still unsealed: skip the O(table) scan then (the head
  // calls this for every worker that exits; the table has one slot per 4 KiB of arena)
  for (uint64_t i = 0; hdr_->creating_now > 0 && i < hdr_->table_cap; i++) {
    Entry* e = &table_[i];
    if (e->state == kCreating && e->creator_pid == pid) {
      PinErase(e->id, pid);
      FreeEntryStorage(int64_t(i));
      RemoveEntry(int64_t(i));
      hdr_->creating_now--;
      n++;
    }
  }
  Unlock();
  return n;
}

bool Store::Get(const ObjectId& id, int64_t timeout_ms, View* out) {
  int64_t deadline = timeout_ms < 0 ? -1 : NowNs() + timeout_ms * 1000000ll;
  int64_t restore_deadline = -1;  // a restore that found no room waits like Create does (oom_grace_ns)
  Lock();
  for (;;) {
    int64_t idx = Find(id);
    if (idx >= 0) {
      Entry* e = E(idx);
      if (e->state == kSealed || e->state == kSpilling) {
        if (e->pin_count == 0 && e->in_lru) LruRemove(idx);
        PinAdd(idx, int32_t(getpid()));
        hdr_->stats.gets_total++;
        out->data_size = e->data_size;
        out->meta_size = e->meta_size;
        out->user_tag = e->user_tag;
        out->flags = e->flags;
        if (e->flags & kFlagFallback) {
          uint64_t fid = e->fallback_id, len = e->data_size + e->meta_size;
          Unlock();
          out->data = FallbackMap(fid, len, false);
          if (!out->data) {
            Release(id);
            throw std::runtime_error("failed to map fallback object");
          }
          return true;
        }
        out->data = base_ + e->offset;
        Unlock();
        return true;
      }
      if (e->state == kSpilled) {
        if (RestoreLocked(idx)) continue;
        // no room right now: other processes' spills in flight, readers' pins and a global GC free
        // memory shortly (a concurrent map / reduce stage); wait for them like Create before failing
        const int64_t now = NowNs();
        if (restore_deadline < 0) {
          restore_deadline = now + std::max<int64_t>(hdr_->oom_grace_ns, 0);
          __atomic_add_fetch(&hdr_->gc_requests, 1, __ATOMIC_RELEASE);
          hdr_->oom_waits_total++;
        }
        if (now >= restore_deadline) {
          Unlock();
          throw std::runtime_error("ObjectStoreFullError: cannot restore spilled object");
        }
        if (deadline >= 0 && now >= deadline) {
          Unlock();
          return false;
        }
        int64_t until = std::min<int64_t>(restore_deadline, now + 20000000ll);  // re-check every 20 ms
        if (deadline >= 0) until = std::min(until, deadline);
        CondWait(until);
        continue;
      }
    }
    if (deadline >= 0 && NowNs() >= deadline) {
      Unlock();
      return false;
    }
    CondWait(deadline);
  }
}

int Store::Wait(const std::vector<ObjectId>& ids, int num_required, int64_t timeout_ms,
                std::vector<uint8_t>* ready) {
  int64_t deadline = timeout_ms < 0 ? -1 : NowNs() + timeout_ms * 1000000ll;
  ready->assign(ids.size(), 0);
  Lock();
  for (;;) {
    int n = 0;
    for (size_t i = 0; i < ids.size(); i++) {
      if (!(*ready)[i]) {
        int64_t idx = Find(ids[i]);
        if (idx >= 0) {
          uint32_t st = E(idx)->state;
          if (st == kSealed || st == kSpilling || st == kSpilled || st == kRestoring) (*ready)[i] = 1;
        }
      }
      n += (*ready)[i];
    }
    if (n >= num_required || (deadline >= 0 && NowNs() >= deadline)) {
      Unlock();
      return n;
    }
    CondWait(deadline);
  }
}

void Store::Release(const ObjectId& id) {
  Lock();
  int64_t idx = Find(id);
  if (idx < 0) { Unlock(); return; }
  PinDrop(idx, int32_t(getpid()));
  FinishUnpinned(idx);
  Unlock();
}

int Store::ReleaseClient(int pid) {
  if (pid <= 0) return 0;
  int n = 0;
  Lock();
  // 1) the client's pin records (gets never released, its creator pins of sealed objects)
  PinRec* P = Pins();
  std::vector<std::pair<ObjectId, int32_t>> drop;
  for (uint64_t i = 0; hdr_->pins_live > 0 && i < kPinCap; i++) {
    if (P[i].state == 1 && P[i].pid == pid) {
      ObjectId o;
      memcpy(o.b, P[i].id, kIdSize);
      drop.push_back({o, P[i].count});
      P[i].state = 2;
      P[i].count = 0;
      hdr_->pins_live--;
    }
  }
  for (auto& d : drop) {
    const int64_t idx = Find(d.first);
    if (idx < 0) continue;
    Entry* e = E(idx);
    e->pin_count = std::max(0, e->pin_count - d.second);
    n += d.second;
    FinishUnpinned(idx);
  }
  // 2) spills / restores it was doing with the lock dropped: roll back
  for (uint64_t i = 0; hdr_->io_now > 0 && i < hdr_->table_cap; i++) {
    Entry* e = &table_[i];
    if ((e->state != kSpilling && e->state != kRestoring) || e->io_pid != pid) continue;
    if (e->state == kRestoring) {
      if (e->offset) HeapFree(e->offset);
      e->offset = 0;
      e->state = kSpilled;
    } else {
      e->state = kSealed;
    }
    IoUnpin(int64_t(i));
    n++;
    FinishUnpinned(int64_t(i));
  }
  if (n > 0) {
    hdr_->clients_released_total++;
    hdr_->client_pins_released_total += uint64_t(n);
    Broadcast();
  }
  Unlock();
  return n;
}

int64_t Store::PinsHeldBy(int pid) {
  int64_t n = 0;
  Lock();
  PinRec* P = Pins();
  for (uint64_t i = 0; i < kPinCap; i++)
    if (P[i].state == 1 && P[i].pid == pid) n += P[i].count;
  Unlock();
  return n;
}

bool Store::Delete(const ObjectId& id) {
  Lock();
  int64_t idx = Find(id);
  if (idx < 0) { Unlock(); return false; }
  Entry* e = E(idx);
  hdr_->stats.deletes_total++;
  if (e->state == kSealed || e->state == kSpilled) {
    if (e->pin_count > 0) {
      e->flags |= kFlagDeletePending;
    } else {
      if (e->state == kSealed) hdr_->stats.num_sealed--;
      FreeEntryStorage(idx);
      RemoveEntry(idx);
    }
  } else {
    e->flags |= kFlagDeletePending;  // creating / spilling / restoring: finish first
  }
  Unlock();
  return true;
}

bool Store::Contains(const ObjectId& id) {
  Lock();
  CrashPoint(7);
  int64_t idx = Find(id);
  bool r = false;
  if (idx >= 0) {
    uint32_t st = E(idx)->state;
    r = st == kSealed || st == kSpilling || st == kSpilled || st == kRestoring;
  }
  Unlock();
  return r;
}

bool Store::TrySetFlag(const ObjectId& id, uint32_t flag) {
  Lock();
  int64_t idx = Find(id);
  bool ok = true;
  if (idx >= 0) {
    Entry* e = E(idx);
    if (e->pin_count > 0) ok = false;
    else e->flags |= flag;
  }
  Unlock();
  return ok;
}

void Store::ClearFlag(const ObjectId& id, uint32_t flag) {
  Lock();
  int64_t idx = Find(id);
  if (idx >= 0) E(idx)->flags &= ~flag;
  Unlock();
}

std::vector<int64_t> Store::Sizes(const std::vector<ObjectId>& ids) {
  std::vector<int64_t> out(ids.size(), -1);
  Lock();
  for (size_t i = 0; i < ids.size(); i++) {
    int64_t idx = Find(ids[i]);
    if (idx >= 0 && E(idx)->state != kCreating) out[i] = int64_t(E(idx)->data_size + E(idx)->meta_size);
  }
  Unlock();
  return out;
}

int Store::State(const ObjectId& id) {
  Lock();
  int64_t idx = Find(id);
  int r = idx >= 0 ? int(E(idx)->state) : -1;
  Unlock();
  return r;
}

uint64_t Store::PollSealed(uint64_t cursor, std::vector<ObjectId>* out, bool* overflow) {
  Lock();
  uint64_t head = hdr_->ring_head;
  *overflow = head - cursor > kRingCap;
  if (*overflow) cursor = head - kRingCap;
  out->reserve(head - cursor);
  for (uint64_t c = cursor; c < head; c++) out->push_back(ring_[c & (kRingCap - 1)]);
  Unlock();
  return head;
}

uint64_t Store::SealSeq() { return __atomic_load_n(&hdr_->seal_seq, __ATOMIC_ACQUIRE); }

uint64_t Store::WaitSealSeq(uint64_t seq, int64_t timeout_ms) {
  int64_t deadline = timeout_ms < 0 ? -1 : NowNs() + timeout_ms * 1000000ll;
  Lock();
  while (hdr_->seal_seq == seq) {
    if (deadline >= 0 && NowNs() >= deadline) break;
    CondWait(deadline);
  }
  uint64_t s = hdr_->seal_seq;
  Unlock();
  return s;
}

Stats Store::GetStats() {
  Lock();
  Stats s = hdr_->stats;
  Unlock();
  return s;
}

std::vector<std::pair<ObjectId, Entry>> Store::ListObjects() {
  std::vector<std::pair<ObjectId, Entry>> r;
  Lock();
  for (uint64_t i = 0; i < hdr_->table_cap; i++) {
    Entry& e = table_[i];
    if (e.state != kEmpty && e.state != kTombstone) {
      ObjectId o;
      memcpy(o.b, e.id, kIdSize);
      r.push_back({o, e});
    }
  }
  Unlock();
  return r;
}

}  // namespace rmm
