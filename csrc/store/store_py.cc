// pybind11 bindings for the shared-memory object store + the serialized-object layout
// (pickle-5 payload followed by 64-byte aligned out-of-band buffers) + a parallel memcpy.
//
// Parity: reference python/ray/_raylet.pyx (Plasma put/get, `parallel_memcopy`),
// python/ray/_private/serialization.py (out-of-band buffer layout).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>

#include "shm_store.h"

namespace py = pybind11;
using namespace rmm;

namespace {

// ------------------------------------------------------------ parallel memcpy pool
class CopyPool {
 public:
  explicit CopyPool(int n) {
    for (int i = 0; i < n; i++) threads_.emplace_back([this] { Loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  int size() const { return int(threads_.size()); }
  // Copy `n` bytes using the pool + calling thread.
  void Copy(uint8_t* dst, const uint8_t* src, size_t n) {
    const size_t kMin = 4u << 20;
    int parts = int(std::min<size_t>(threads_.size() + 1, n / kMin));
    if (parts <= 1) {
      memcpy(dst, src, n);
      return;
    }
    size_t chunk = ((n / size_t(parts)) + 63) & ~size_t(63);
    std::atomic<int> remaining(parts - 1);
    std::mutex dm;
    std::condition_variable dcv;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int p = 1; p < parts; p++) {
        size_t off = size_t(p) * chunk;
        size_t len = off >= n ? 0 : std::min(chunk, n - off);
        jobs_.push_back([=, &remaining, &dm, &dcv] {
          if (len) memcpy(dst + off, src + off, len);
          if (remaining.fetch_sub(1) == 1) {
            std::lock_guard<std::mutex> g2(dm);
            dcv.notify_all();
          }
        });
      }
    }
    cv_.notify_all();
    memcpy(dst, src, std::min(chunk, n));
    std::unique_lock<std::mutex> lk(dm);
    dcv.wait(lk, [&] { return remaining.load() == 0; });
  }

 private:
  void Loop() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !jobs_.empty(); });
        if (stop_ && jobs_.empty()) return;
        job = std::move(jobs_.back());
        jobs_.pop_back();
      }
      job();
    }
  }
  std::vector<std::thread> threads_;
  std::vector<std::function<void()>> jobs_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

CopyPool* g_pool = nullptr;
CopyPool& Pool() {
  if (!g_pool) {
    unsigned hw = std::thread::hardware_concurrency();
    int n = int(std::max(1u, std::min(8u, hw / 2)));
    g_pool = new CopyPool(n);
  }
  return *g_pool;
}

ObjectId ToId(const py::bytes& b) {
  std::string s = b;
  if (s.size() != kIdSize) throw std::invalid_argument("object id must be 20 bytes");
  ObjectId o;
  memcpy(o.b, s.data(), kIdSize);
  return o;
}
ObjectId ToIdView(const char* p, size_t n) {
  if (n != kIdSize) throw std::invalid_argument("object id must be 20 bytes");
  ObjectId o;
  memcpy(o.b, p, kIdSize);
  return o;
}

struct PyStore;

// A pinned view of an object's payload. Releases the pin when garbage collected.
struct Pinned {
  std::shared_ptr<Store> store;
  ObjectId id;
  uint8_t* ptr;
  uint64_t size;
  bool writable;
  bool released = false;
  ~Pinned() {
    if (released || !store) return;
    // the store mutex may be contended (or, in a bug, stuck): never wait for it holding the GIL
    if (PyGILState_Check() && !_Py_IsFinalizing()) {
      py::gil_scoped_release nogil;
      store->Release(id);
    } else {
      store->Release(id);
    }
  }
};

constexpr uint64_t kLayoutMagic = 0x314e4c5941594f52ull;

inline uint64_t A64(uint64_t v) { return (v + 63) & ~uint64_t(63); }

struct PyStore {
  std::shared_ptr<Store> s;
};

py::dict StatsDict(const Stats& st, uint64_t cap) {
  py::dict d;
  d["capacity"] = cap;
  d["bytes_in_use"] = st.bytes_in_use;
  d["num_objects"] = st.num_objects;
  d["bytes_spilled_total"] = st.bytes_spilled_total;
  d["objects_spilled_total"] = st.objects_spilled_total;
  d["bytes_restored_total"] = st.bytes_restored_total;
  d["objects_restored_total"] = st.objects_restored_total;
  d["spilled_bytes_current"] = st.spilled_bytes_current;
  d["spilled_objects_current"] = st.spilled_objects_current;
  d["fallback_bytes_current"] = st.fallback_bytes_current;
  d["fallback_allocs_total"] = st.fallback_allocs_total;
  d["creates_total"] = st.creates_total;
  d["gets_total"] = st.gets_total;
  d["deletes_total"] = st.deletes_total;
  return d;
}

}  // namespace

PYBIND11_MODULE(_store, m) {
  m.doc() = "Shared-memory object store (native)";
  m.attr("ID_SIZE") = kIdSize;

  py::class_<Pinned, std::shared_ptr<Pinned>>(m, "PinnedBuffer", py::buffer_protocol())
      .def_buffer([](Pinned& p) -> py::buffer_info {
        return py::buffer_info(p.ptr, 1, py::format_descriptor<uint8_t>::format(), 1,
                               {py::ssize_t(p.size)}, {py::ssize_t(1)}, !p.writable);
      })
      .def_property_readonly("size", [](Pinned& p) { return p.size; })
      .def_property_readonly("address", [](Pinned& p) { return reinterpret_cast<uintptr_t>(p.ptr); })
      .def("release", [](Pinned& p) {
        if (!p.released) {
          p.released = true;
          py::gil_scoped_release nogil;
          p.store->Release(p.id);
        }
      })
      // hand the pin over to native code that releases it later (e.g. a HIP host callback that
      // seals a GPU-object descriptor once the device copy has completed)
      .def("disown", [](Pinned& p) { p.released = true; });

  py::class_<PyStore>(m, "ObjectStore")
      .def_static(
          "create_segment",
          [](const std::string& name, uint64_t size, const std::string& spill_dir,
             double spill_threshold, uint64_t min_spill_size, bool fallback, double oom_grace_s,
             bool populate) {
            PyStore ps;
            ps.s.reset(Store::Create(name, size, spill_dir, spill_threshold, min_spill_size, fallback,
                                     oom_grace_s, populate));
            return ps;
          },
          py::arg("name"), py::arg("size"), py::arg("spill_dir") = "",
          py::arg("spill_threshold") = 0.8, py::arg("min_spill_size") = 100ull << 20,
          py::arg("fallback") = true, py::arg("oom_grace_s") = 2.0, py::arg("populate") = false)
      .def_static("attach",
                  [](const std::string& name) {
                    PyStore ps;
                    ps.s.reset(Store::Attach(name));
                    return ps;
                  })
      .def("create",
           [](PyStore& self, py::bytes oid, uint64_t data_size, uint64_t meta_size, uint32_t tag,
              bool error) -> py::object {
             ObjectId id = ToId(oid);
             bool exists = false;
             uint8_t* p;
             {
               py::gil_scoped_release nogil;
               p = self.s->CreateObject(id, data_size, meta_size, tag, error ? kFlagError : 0, &exists);
             }
             if (exists) return py::none();
             auto pin = std::make_shared<Pinned>();
             pin->store = self.s;
             pin->id = id;
             pin->ptr = p;
             pin->size = data_size + meta_size;
             pin->writable = true;
             return py::cast(pin);
           },
           py::arg("oid"), py::arg("data_size"), py::arg("meta_size") = 0, py::arg("tag") = 0,
           py::arg("error") = false)
      .def("seal", [](PyStore& self, py::bytes oid) {
        ObjectId id = ToId(oid);
        py::gil_scoped_release nogil;
        self.s->Seal(id);
      })
      .def("abort", [](PyStore& self, py::bytes oid) {
        ObjectId id = ToId(oid);
        py::gil_scoped_release nogil;
        self.s->Abort(id);
      })
      // Serialize-and-seal: pickle payload + out-of-band buffers in one shot.
      // Layout: [magic u64][nbuf u64][pickle_len u64][buf_len u64 * nbuf] pad64
      //         [pickle] pad64 [buf0] pad64 [buf1] ...
      .def(
          "put_serialized",
          [](PyStore& self, py::bytes oid, py::buffer pickled, py::list buffers, uint32_t tag,
             bool error) -> bool {
            ObjectId id = ToId(oid);
            std::vector<py::buffer_info> infos;
            infos.reserve(buffers.size());
            py::buffer_info pinfo = pickled.request();
            for (auto b : buffers) infos.push_back(py::reinterpret_borrow<py::buffer>(b).request());
            uint64_t nbuf = infos.size();
            uint64_t hdr = A64(8 * (3 + nbuf));
            uint64_t total = hdr + A64(uint64_t(pinfo.size * pinfo.itemsize));
            for (auto& bi : infos) total += A64(uint64_t(bi.size * bi.itemsize));
            bool exists = false;
            {
              py::gil_scoped_release nogil;
              uint8_t* p = self.s->CreateObject(id, total, 0, tag, error ? kFlagError : 0, &exists);
              if (exists) return false;
              uint64_t* h = reinterpret_cast<uint64_t*>(p);
              h[0] = kLayoutMagic;
              h[1] = nbuf;
              h[2] = uint64_t(pinfo.size * pinfo.itemsize);
              for (uint64_t i = 0; i < nbuf; i++) h[3 + i] = uint64_t(infos[i].size * infos[i].itemsize);
              uint64_t off = hdr;
              memcpy(p + off, pinfo.ptr, size_t(h[2]));
              off += A64(h[2]);
              for (uint64_t i = 0; i < nbuf; i++) {
                Pool().Copy(p + off, static_cast<const uint8_t*>(infos[i].ptr), size_t(h[3 + i]));
                off += A64(h[3 + i]);
              }
              self.s->Seal(id);
              self.s->Release(id);
            }
            return true;
          },
          py::arg("oid"), py::arg("pickled"), py::arg("buffers"), py::arg("tag") = 0,
          py::arg("error") = false)
      // Returns (pickle_mv, [buffer_mv...], tag, is_error) or None on timeout.
      .def(
          "get_serialized",
          [](PyStore& self, py::bytes oid, int64_t timeout_ms) -> py::object {
            ObjectId id = ToId(oid);
            Store::View v;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = self.s->Get(id, timeout_ms, &v);
            }
            if (!ok) return py::none();
            auto pin = std::make_shared<Pinned>();
            pin->store = self.s;
            pin->id = id;
            pin->ptr = v.data;
            pin->size = v.data_size + v.meta_size;
            pin->writable = false;
            py::object owner = py::cast(pin);
            py::memoryview whole = py::memoryview(py::reinterpret_steal<py::object>(
                PyMemoryView_FromObject(owner.ptr())));
            uint64_t* h = reinterpret_cast<uint64_t*>(v.data);
            if (v.data_size < 24 || h[0] != kLayoutMagic) {
              // raw object (not written by put_serialized)
              return py::make_tuple(whole, py::list(), v.user_tag, bool(v.flags & kFlagError), true);
            }
            uint64_t nbuf = h[1];
            uint64_t off = A64(8 * (3 + nbuf));
            py::object getitem = whole.attr("__getitem__");
            py::object pick = getitem(py::slice(py::int_(off), py::int_(off + h[2]), py::none()));
            off += A64(h[2]);
            py::list bufs;
            for (uint64_t i = 0; i < nbuf; i++) {
              bufs.append(getitem(py::slice(py::int_(off), py::int_(off + h[3 + i]), py::none())));
              off += A64(h[3 + i]);
            }
            return py::make_tuple(pick, bufs, v.user_tag, bool(v.flags & kFlagError), false);
          },
          py::arg("oid"), py::arg("timeout_ms") = -1)
      .def(
          "get_raw",
          [](PyStore& self, py::bytes oid, int64_t timeout_ms) -> py::object {
            ObjectId id = ToId(oid);
            Store::View v;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = self.s->Get(id, timeout_ms, &v);
            }
            if (!ok) return py::none();
            auto pin = std::make_shared<Pinned>();
            pin->store = self.s;
            pin->id = id;
            pin->ptr = v.data;
            pin->size = v.data_size + v.meta_size;
            pin->writable = false;
            return py::make_tuple(py::cast(pin), v.data_size, v.meta_size, v.user_tag,
                                  bool(v.flags & kFlagError), v.flags);
          },
          py::arg("oid"), py::arg("timeout_ms") = -1)
      .def(
          "wait",
          [](PyStore& self, std::vector<py::bytes> oids, int num_required, int64_t timeout_ms) {
            std::vector<ObjectId> ids;
            ids.reserve(oids.size());
            for (auto& o : oids) ids.push_back(ToId(o));
            std::vector<uint8_t> ready;
            {
              py::gil_scoped_release nogil;
              self.s->Wait(ids, num_required, timeout_ms, &ready);
            }
            std::vector<bool> r(ready.begin(), ready.end());
            return r;
          },
          py::arg("oids"), py::arg("num_required"), py::arg("timeout_ms") = -1)
      .def("release", [](PyStore& self, py::bytes oid) {
        ObjectId id = ToId(oid);
        py::gil_scoped_release nogil;
        self.s->Release(id);
      })
      .def("delete",
           [](PyStore& self, std::vector<py::bytes> oids) {
             std::vector<ObjectId> ids;
             for (auto& o : oids) ids.push_back(ToId(o));
             py::gil_scoped_release nogil;
             int n = 0;
             for (auto& i : ids) n += self.s->Delete(i) ? 1 : 0;
             return n;
           })
      .def("contains", [](PyStore& self, py::bytes oid) {
        ObjectId id = ToId(oid);
        py::gil_scoped_release nogil;
        return self.s->Contains(id);
      })
      .def("state", [](PyStore& self, py::bytes oid) {
        ObjectId id = ToId(oid);
        py::gil_scoped_release nogil;
        return self.s->State(id);
      })
      .def("sizes", [](PyStore& self, const std::vector<py::bytes>& oids) {
        std::vector<ObjectId> ids;
        ids.reserve(oids.size());
        for (auto& o : oids) ids.push_back(ToId(o));
        py::gil_scoped_release nogil;
        return self.s->Sizes(ids);
      })
      .def("spill",
           [](PyStore& self, uint64_t bytes) {
             py::gil_scoped_release nogil;
             return self.s->SpillBytes(bytes);
           })
      .def("abort_creator", [](PyStore& self, int pid) {
        py::gil_scoped_release nogil;
        return self.s->AbortCreator(pid);
      })
      .def("release_client", [](PyStore& self, int pid) {
        py::gil_scoped_release nogil;
        return self.s->ReleaseClient(pid);
      })
      .def("pins_held_by", [](PyStore& self, int pid) {
        py::gil_scoped_release nogil;
        return self.s->PinsHeldBy(pid);
      })
      .def("pin_overflows", [](PyStore& self) { return self.s->PinOverflows(); })
      .def("poll_sealed",
           [](PyStore& self, uint64_t cursor) {
             std::vector<ObjectId> out;
             bool overflow = false;
             uint64_t c;
             {
               py::gil_scoped_release nogil;
               c = self.s->PollSealed(cursor, &out, &overflow);
             }
             py::list l;
             for (auto& o : out) l.append(py::bytes(reinterpret_cast<const char*>(o.b), kIdSize));
             return py::make_tuple(c, l, overflow);
           })
      .def("seal_seq", [](PyStore& self) { return self.s->SealSeq(); })
      .def("wait_seal_seq",
           [](PyStore& self, uint64_t seq, int64_t timeout_ms) {
             py::gil_scoped_release nogil;
             return self.s->WaitSealSeq(seq, timeout_ms);
           })
      .def("wake", [](PyStore& self) {
        py::gil_scoped_release nogil;
        self.s->Wake();
      })
      .def("stats", [](PyStore& self) {
        Stats st;
        {
          py::gil_scoped_release nogil;
          st = self.s->GetStats();
        }
        return StatsDict(st, self.s->Capacity());
      })
      .def("capacity", [](PyStore& self) { return self.s->Capacity(); })
      .def("set_disk_full", [](PyStore& self, bool full) {
        py::gil_scoped_release nogil;
        self.s->SetDiskFull(full);
      })
      .def("disk_full", [](PyStore& self) { return self.s->DiskFull(); })
      .def("set_spill_enabled", [](PyStore& self, bool on) {
        py::gil_scoped_release nogil;
        self.s->SetSpillEnabled(on);
      })
      .def("gc_requests", [](PyStore& self) { return self.s->GcRequests(); })
      .def("set_oom_grace", [](PyStore& self, double s) {
        py::gil_scoped_release nogil;
        self.s->SetOomGrace(s);
      })
      .def("spill_dirs", [](PyStore& self) { return self.s->SpillDirs(); })
      .def("oom_stats", [](PyStore& self) {
        py::dict d;
        d["oom_waits_total"] = self.s->OomWaits();
        d["oom_errors_total"] = self.s->OomErrors();
        d["gc_requests"] = self.s->GcRequests();
        d["disk_full"] = self.s->DiskFull();
        return d;
      })
      .def("base_address", [](PyStore& self) { return reinterpret_cast<uintptr_t>(self.s->Base()); })
      .def("mapped_size", [](PyStore& self) { return self.s->MappedSize(); })
      .def("check_heap", [](PyStore& self) {
        py::gil_scoped_release nogil;
        return self.s->CheckHeap();
      })
      .def("recoveries", [](PyStore& self) { return self.s->Recoveries(); })
      .def("integrity", [](PyStore& self) {
        py::dict d;
        d["corruptions_total"] = self.s->Corruptions();
        d["lock_stalls_total"] = self.s->LockStalls();
        d["unmatched_releases_total"] = self.s->UnmatchedReleases();
        d["pin_overflow_total"] = self.s->PinOverflows();
        d["recoveries_total"] = self.s->Recoveries();
        d["lock_pid"] = self.s->LockPid();
        d["creating_now"] = self.s->CreatingNow();
        return d;
      })
      .def("creating_now", [](PyStore& self) { return self.s->CreatingNow(); })
      .def_static("set_lock_watchdog_ms", &rmm::Store::SetLockWatchdogMs)
      .def("recovered_dropped", [](PyStore& self) { return self.s->RecoveredDropped(); })
      .def_static("set_crash_point_for_test", &rmm::Store::SetCrashPointForTest)
      .def("list_objects", [](PyStore& self) {
        py::list out;
        static const char* names[] = {"EMPTY", "CREATING", "SEALED", "SPILLING", "SPILLED", "RESTORING", "TOMBSTONE"};
        std::vector<std::pair<ObjectId, Entry>> objs;
        {
          py::gil_scoped_release nogil;
          objs = self.s->ListObjects();
        }
        for (auto& pr : objs) {
          py::dict d;
          d["object_id"] = py::bytes(reinterpret_cast<const char*>(pr.first.b), kIdSize);
          d["state"] = names[pr.second.state < 7 ? pr.second.state : 0];
          d["size"] = pr.second.data_size + pr.second.meta_size;
          d["pin_count"] = pr.second.pin_count;
          d["creator_pid"] = pr.second.creator_pid;
          d["fallback"] = bool(pr.second.flags & kFlagFallback);
          d["has_spill_copy"] = bool(pr.second.flags & kFlagHasSpillCopy);
          d["delete_pending"] = bool(pr.second.flags & kFlagDeletePending);
          d["tag"] = pr.second.user_tag;
          out.append(d);
        }
        return out;
      });

  m.attr("FLAG_GPU_SPILLED") = uint32_t(kFlagGpuSpilled);
  m.attr("GPU_DESC_MAGIC") = kGpuDescMagic;
  m.attr("GPU_DESC_SIZE") = sizeof(GpuDesc);
  m.def("parallel_memcpy",
        [](py::buffer dst, py::buffer src) {
          auto d = dst.request(true);
          auto s = src.request();
          size_t n = size_t(s.size * s.itemsize);
          if (size_t(d.size * d.itemsize) < n) throw std::invalid_argument("dst too small");
          py::gil_scoped_release nogil;
          Pool().Copy(static_cast<uint8_t*>(d.ptr), static_cast<const uint8_t*>(s.ptr), n);
        });
  m.def("copy_threads", [] { return Pool().size() + 1; });
}
