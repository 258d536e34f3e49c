// Multi-threaded stress test of the shared-memory object store, built only for the host race /
// memory checkers (tests/test_native_sanitizers.py builds it with ThreadSanitizer and with
// AddressSanitizer + UBSan). Every thread shares ONE Store mapping so the race checker sees
// every access to the segment at one address.
//
// Parity: the reference exercises plasma concurrency through
// src/ray/object_manager/plasma/test/ and python/ray/tests/test_object_spilling*.py
// (concurrent create / get / delete while spilling and restoring); this drives the same
// lifecycle paths of csrc/store/shm_store.cc directly: create -> seal -> get/release -> delete,
// proactive and explicit spilling, restore-on-get, sealed-notification polling, batched wait.
//
// Then a crash phase: for each Store::SetCrashPointForTest point a forked child attaches, and is
// SIGKILLed while holding the store mutex in the middle of a multi-word update; the parent's next
// lock recovers (Store::Recover) and the heap self-check and every surviving payload must pass.
//
// usage: store_stress <spill_dir> [threads] [iters]
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>
#include <sys/wait.h>
#include <unistd.h>

#include "../store/shm_store.h"

using rmm::ObjectId;
using rmm::Store;

namespace {

constexpr int kKeys = 384;

ObjectId Id(int key) {
  ObjectId id{};
  std::memcpy(id.b, &key, sizeof(key));
  id.b[19] = 0x5a;
  return id;
}

uint8_t Pat(int key, uint64_t i) { return static_cast<uint8_t>(key * 131 + i * 7); }

std::atomic<long> g_bad{0};
std::atomic<long> g_ops[8];

void Worker(Store* s, int tid, int iters) {
  std::mt19937_64 rng(1234 + tid);
  uint64_t cursor = 0;
  for (int it = 0; it < iters; it++) {
    int key = static_cast<int>(rng() % kKeys);
    ObjectId id = Id(key);
    int r = static_cast<int>(rng() % 100);
    if (r < 30) {
      uint64_t n = 64 + rng() % (key % 4 == 0 ? (512u << 10) : (16u << 10));
      bool exists = false;
      uint8_t* p = nullptr;
      try {
        p = s->CreateObject(id, n, 0, 0, 0, &exists);
      } catch (const std::runtime_error&) {
        g_ops[7]++;  // out of memory even after spilling: legal under this pressure
        continue;
      }
      if (!p || exists) continue;
      for (uint64_t i = 0; i < n; i++) p[i] = Pat(key, i);
      s->Seal(id);
      s->Release(id);  // creator's pin (plasma semantics: the creator releases after seal)
      g_ops[0]++;
    } else if (r < 62) {
      Store::View v;
      bool got = false;
      try {
        got = s->Get(id, 0, &v);
      } catch (const std::runtime_error&) {
        g_ops[7]++;  // restore of a spilled object found no room: legal under this pressure
      }
      if (got) {
        // sealed payloads never change while pinned (spill keeps the heap copy readable,
        // restore rewrites the bytes before the object is visible again)
        uint64_t n = v.data_size;
        if (n && (v.data[0] != Pat(key, 0) || v.data[n - 1] != Pat(key, n - 1) ||
                  v.data[n / 2] != Pat(key, n / 2)))
          g_bad++;
        s->Release(id);
        g_ops[1]++;
      }
    } else if (r < 76) {
      s->Delete(id);
      g_ops[2]++;
    } else if (r < 82) {
      (void)s->Contains(id);
      (void)s->State(id);
    } else if (r < 88) {
      std::vector<ObjectId> ids;
      for (int k = 0; k < 4; k++) ids.push_back(Id(static_cast<int>(rng() % kKeys)));
      std::vector<uint8_t> ready;
      s->Wait(ids, 4, 0, &ready);
      (void)s->Sizes(ids);
      g_ops[3]++;
    } else if (r < 91) {
      s->SpillBytes(1u << 20);
      g_ops[4]++;
    } else if (r < 96) {
      std::vector<ObjectId> out;
      bool overflow = false;
      cursor = s->PollSealed(cursor, &out, &overflow);
      g_ops[5]++;
    } else {
      (void)s->GetStats();
      (void)s->ListObjects();
      g_ops[6]++;
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <spill_dir> [threads] [iters]\n", argv[0]);
    return 2;
  }
  int threads = argc > 2 ? std::atoi(argv[2]) : 6;
  int iters = argc > 3 ? std::atoi(argv[3]) : 4000;
  std::string name = "/rmm_stress_" + std::to_string(getpid());
  // 24 MiB arena against up to ~100 x 512 KiB live objects: creates spill, gets restore
  Store* s = Store::Create(name, 24ull << 20, argv[1], 0.8, 1u << 20, /*fallback=*/false,
                           /*oom_grace_s=*/0.05);
  std::atomic<bool> stop{false};
  std::thread waiter([&] {
    uint64_t seq = s->SealSeq();
    while (!stop.load()) seq = s->WaitSealSeq(seq, 5);
  });
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; t++) ts.emplace_back(Worker, s, t, iters);
  for (auto& t : ts) t.join();
  stop = true;
  s->Wake();
  waiter.join();

  // ---- crash phase: a client killed inside the critical section, the parent recovers
  long crash_bad = 0;
  for (int point = 1; point <= 4; point++) {
    ObjectId a = Id(10000 + point * 4), b = Id(10001 + point * 4), c = Id(10002 + point * 4),
             d = Id(10003 + point * 4);
    for (ObjectId x : {a, b, c}) {
      bool ex = false;
      uint8_t* p = s->CreateObject(x, 4096, 0, 0, 0, &ex);
      if (p) {
        std::memset(p, 0x3c, 4096);
        s->Seal(x);
        s->Release(x);
      }
    }
    s->Delete(a);
    pid_t pid = fork();
    if (pid == 0) {
      Store* cs = Store::Attach(name);
      Store::SetCrashPointForTest(point);
      bool ex = false;
      Store::View v;
      if (point == 1 || point == 3) (void)cs->CreateObject(d, 2048, 0, 0, 0, &ex);
      else if (point == 2) cs->Delete(b);  // merges with the free block `a` left
      else (void)cs->Get(c, 0, &v);        // unpins from the LRU list
      _exit(3);                            // crash point not reached
    }
    int status = 0;
    waitpid(pid, &status, 0);
    const uint64_t rec = s->Recoveries();
    if (point == 2 && WIFEXITED(status) && WEXITSTATUS(status) == 3) {
      // the merge point needs `a` to sit right before `b`; the stress phase's leftovers decide the
      // layout, so when they were not neighbours the crash point is not reached (nothing to recover)
      std::printf("crash point 2: a and b not neighbours in this layout (skipped)\n");
      for (ObjectId x : {a, b, c, d}) s->Delete(x);
      continue;
    }
    if (!(WIFSIGNALED(status) && WTERMSIG(status) == SIGKILL)) {
      crash_bad++;
      std::printf("crash point %d: child not killed (status %d)\n", point, status);
    }
    (void)s->Contains(c);  // first lock after the kill: EOWNERDEAD -> Recover
    if (s->Recoveries() != rec + 1) {
      crash_bad++;
      std::printf("crash point %d: no recovery\n", point);
    }
    try {
      s->CheckHeap();
    } catch (const std::runtime_error&) {
      crash_bad++;
      std::printf("crash point %d: heap check failed\n", point);
    }
    Store::View v;
    if (s->Get(c, 0, &v)) {
      if (v.data_size != 4096 || v.data[0] != 0x3c || v.data[4095] != 0x3c) crash_bad++;
      s->Release(c);
    } else {
      crash_bad++;
    }
    for (ObjectId x : {a, b, c, d}) s->Delete(x);  // the final num_objects == 0 check catches leaks
  }
  std::printf("crash phase: recoveries=%lu dropped=%lu bad=%ld\n", (unsigned long)s->Recoveries(),
              (unsigned long)s->RecoveredDropped(), crash_bad);
  g_bad += crash_bad;

  // ---- client-death phase: a reader SIGKILLed while it holds pins (no lock held), then one killed
  // inside a restore's and a spill's file IO (lock released); ReleaseClient releases / rolls back
  long client_bad = 0;
  {
    ObjectId r0 = Id(20000), r1 = Id(20001), r2 = Id(20002);
    for (ObjectId x : {r0, r1, r2}) {
      bool ex = false;
      uint8_t* p = s->CreateObject(x, 8192, 0, 0, 0, &ex);
      if (p) {
        std::memset(p, 0x5a, 8192);
        s->Seal(x);
        s->Release(x);
      }
    }
    // (a) reader holds three pins and dies
    pid_t pid = fork();
    if (pid == 0) {
      Store* cs = Store::Attach(name);
      Store::View v;
      for (ObjectId x : {r0, r1, r2}) (void)cs->Get(x, 1000, &v);
      kill(getpid(), SIGKILL);
      _exit(3);
    }
    int status = 0;
    waitpid(pid, &status, 0);
    if (s->PinsHeldBy(pid) != 3) client_bad++;
    for (ObjectId x : {r0, r1}) s->Delete(x);  // deferred: the dead reader still pins them
    if (s->State(r0) != rmm::kSealed) client_bad++;
    if (s->ReleaseClient(pid) != 3) client_bad++;
    if (s->State(r0) != -1 || s->State(r1) != -1 || s->State(r2) != rmm::kSealed) client_bad++;
    // (b) killed inside a restore's file IO: r2 stuck kRestoring until its IO pin is released
    s->SpillBytes(1ull << 40);
    if (s->State(r2) == rmm::kSpilled) {
      pid = fork();
      if (pid == 0) {
        Store* cs = Store::Attach(name);
        Store::SetCrashPointForTest(5);
        Store::View v;
        (void)cs->Get(r2, 1000, &v);
        _exit(3);
      }
      waitpid(pid, &status, 0);
      if (s->State(r2) != rmm::kRestoring) client_bad++;
      if (s->ReleaseClient(pid) != 1 || s->State(r2) != rmm::kSpilled) client_bad++;
    }
    // (c) killed inside a spill's file IO: its victims (r3 has no spill copy yet, so it needs IO) stuck
    // kSpilling until rolled back
    Store::View v;
    if (!s->Get(r2, 1000, &v) || v.data[0] != 0x5a || v.data[8191] != 0x5a) client_bad++;
    s->Release(r2);
    ObjectId r3 = Id(20003);
    {
      bool ex = false;
      uint8_t* p = s->CreateObject(r3, 8192, 0, 0, 0, &ex);
      if (p) {
        std::memset(p, 0x5b, 8192);
        s->Seal(r3);
        s->Release(r3);
      }
    }
    pid = fork();
    if (pid == 0) {
      Store* cs = Store::Attach(name);
      Store::SetCrashPointForTest(6);
      cs->SpillBytes(1ull << 40);
      _exit(3);
    }
    waitpid(pid, &status, 0);
    if (s->State(r3) != rmm::kSpilling) client_bad++;
    if (s->ReleaseClient(pid) < 1 || s->State(r3) != rmm::kSealed) client_bad++;
    if (!s->Get(r3, 1000, &v) || v.data[0] != 0x5b || v.data[8191] != 0x5b) client_bad++;
    s->Release(r3);
    try {
      s->CheckHeap();
    } catch (const std::runtime_error&) {
      client_bad++;
    }
    s->Delete(r2);
    s->Delete(r3);
  }
  std::printf("client-death phase: bad=%ld\n", client_bad);
  g_bad += client_bad;

  // ---- dead waiting creator: a create blocked in the grace wait (entry kCreating, no heap block yet)
  // is SIGKILLed; AbortCreator must free nothing (round 5: it freed heap offset 0 and corrupted the
  // segment header), the heap check passes and other creates proceed
  long waiter_bad = 0;
  {
    s->SetOomGrace(30.0);
    s->SpillBytes(1ull << 40);  // the stress phase's leftovers go to disk: only pinned bytes stay
    std::vector<ObjectId> held;
    for (int k = 0; k < 64; k++) {  // fill the arena with objects this process keeps pinned
      ObjectId x = Id(30000 + k);
      bool ex = false;
      uint8_t* p = nullptr;
      try {
        p = s->CreateObject(x, 1u << 20, 0, 0, 0, &ex);
      } catch (const std::runtime_error&) {
        break;
      }
      if (!p) break;
      std::memset(p, 0x6c, 1u << 20);
      s->Seal(x);  // the creator pin stays: nothing can spill
      held.push_back(x);
      if (s->GetStats().bytes_in_use + (2u << 20) > s->Capacity()) break;
    }
    const uint64_t free_before = s->CheckHeap();
    const uint64_t waits0 = s->OomWaits();
    pid_t pid = fork();
    if (pid == 0) {
      Store* cs = Store::Attach(name);
      bool ex = false;
      try {
        (void)cs->CreateObject(Id(39999), 8u << 20, 0, 0, 0, &ex);
      } catch (const std::runtime_error&) {
      }
      _exit(3);
    }
    for (int t = 0; t < 3000 && !(s->CreatingNow() == 1 && s->OomWaits() > waits0); t++) usleep(10000);
    if (s->CreatingNow() != 1 || s->OomWaits() <= waits0) waiter_bad++;
    kill(pid, SIGKILL);
    int status = 0;
    waitpid(pid, &status, 0);
    if (s->AbortCreator(pid) != 1) waiter_bad++;
    try {
      if (s->CheckHeap() != free_before) waiter_bad++;
    } catch (const std::runtime_error&) {
      waiter_bad++;
    }
    if (s->Corruptions() != 0 || s->CreatingNow() != 0) waiter_bad++;
    for (ObjectId x : held) {
      s->Release(x);
      s->Delete(x);
    }
    s->SetOomGrace(0.05);
    bool ex = false;
    uint8_t* p = s->CreateObject(Id(39998), 8u << 20, 0, 0, 0, &ex);
    if (!p) waiter_bad++;
    else {
      s->Seal(Id(39998));
      s->Release(Id(39998));
      s->Delete(Id(39998));
    }
  }
  std::printf("dead-waiting-creator phase: bad=%ld\n", waiter_bad);
  g_bad += waiter_bad;

  uint64_t free_before = s->CheckHeap();
  for (int k = 0; k < kKeys; k++) s->Delete(Id(k));
  uint64_t free_after = s->CheckHeap();
  rmm::Stats st = s->GetStats();
  std::printf("ops create=%ld get=%ld delete=%ld wait=%ld spill=%ld poll=%ld stats=%ld oom=%ld\n",
              g_ops[0].load(), g_ops[1].load(), g_ops[2].load(), g_ops[3].load(), g_ops[4].load(),
              g_ops[5].load(), g_ops[6].load(), g_ops[7].load());
  std::printf("spilled=%lu restored=%lu free_before=%lu free_after=%lu in_use=%lu objects=%lu bad=%ld\n",
              (unsigned long)st.objects_spilled_total, (unsigned long)st.objects_restored_total,
              (unsigned long)free_before, (unsigned long)free_after, (unsigned long)st.bytes_in_use,
              (unsigned long)st.num_objects, g_bad.load());
  bool ok = g_bad.load() == 0 && st.num_objects == 0 && st.bytes_in_use == 0 && g_ops[0] > 0 &&
            g_ops[1] > 0;
  delete s;
  std::printf(ok ? "STRESS OK\n" : "STRESS FAILED\n");
  return ok ? 0 : 1;
}
