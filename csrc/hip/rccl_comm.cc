// RCCL communicator owned by the framework (not by torch.distributed): graph-capturable
// collectives on a caller-chosen HIP stream.
//
// Why not ProcessGroupNCCL: its watchdog thread queries the events of every collective, and on
// ROCm it aborts the process when a collective was captured into a HIP graph ("operation not
// permitted on an event last recorded in a capturing stream", measured on MI355X with torch
// 2.10 / RCCL 2.26, tools/rccl_same_gpu_probe.py). The PPO learner wants its gradient all-reduces
// INSIDE the per-minibatch graph, forked onto a comm stream next to the trunk backward, so it
// drives RCCL directly: ncclAllReduce / ncclBroadcast enqueue on the stream they are given and are
// legal inside stream capture.
//
// The library is the librccl the process already has loaded (torch links it); it is opened by path
// with dlopen, so this extension has no link-time RCCL dependency and loads on CPU-only hosts.
#include "rccl_comm.h"

#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace rmm::hip {
namespace {

struct Api {
  void* lib = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
  decltype(&ncclGetVersion) version = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
};

std::mutex g_mu;
Api g_api;

template <typename F>
void Sym(void* lib, const char* name, F* out) {
  void* p = dlsym(lib, name);
  if (!p) throw std::runtime_error(std::string("RCCL symbol missing: ") + name);
  *out = reinterpret_cast<F>(p);
}

const Api& A() {
  if (!g_api.lib) throw std::runtime_error("RCCL not loaded: call rccl_load(path) first");
  return g_api;
}

void Check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    const char* s = g_api.err ? g_api.err(r) : "?";
    throw std::runtime_error(std::string(what) + " failed: " + s + " (" + std::to_string(int(r)) + ")");
  }
}

}  // namespace

int rccl_load(const std::string& path) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_api.lib) {
    int v = 0;
    g_api.version(&v);
    return v;
  }
  // the copy torch already mapped when the path matches: one RCCL instance per process
  void* lib = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!lib) throw std::runtime_error(std::string("dlopen ") + path + ": " + dlerror());
  Api a;
  a.lib = lib;
  Sym(lib, "ncclGetUniqueId", &a.get_unique_id);
  Sym(lib, "ncclCommInitRank", &a.init_rank);
  Sym(lib, "ncclAllReduce", &a.all_reduce);
  Sym(lib, "ncclBroadcast", &a.broadcast);
  Sym(lib, "ncclCommDestroy", &a.destroy);
  Sym(lib, "ncclCommAbort", &a.abort);
  Sym(lib, "ncclGetErrorString", &a.err);
  Sym(lib, "ncclGetVersion", &a.version);
  Sym(lib, "ncclCommGetAsyncError", &a.async_error);
  g_api = a;
  int v = 0;
  g_api.version(&v);
  return v;
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  Check(A().get_unique_id(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

RcclComm::RcclComm(const std::string& uid, int nranks, int rank, int device) : nranks_(nranks), rank_(rank) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("RcclComm: unique id must be 128 bytes");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("RcclComm: bad rank / nranks");
  ncclUniqueId id;
  memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  RMM_HIP_CHECK(hipSetDevice(device));
  Check(A().init_rank(&comm_, nranks, id, rank), "ncclCommInitRank");
}

RcclComm::~RcclComm() {
  if (comm_ && g_api.lib) (void)g_api.destroy(comm_);
}

void RcclComm::AllReduce(uint64_t send, uint64_t recv, uint64_t count, int dtype, int op, uint64_t stream) {
  if (!comm_) throw std::runtime_error("RcclComm: communicator closed");
  Check(A().all_reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), size_t(count),
                       ncclDataType_t(dtype), ncclRedOp_t(op), comm_, reinterpret_cast<hipStream_t>(stream)),
        "ncclAllReduce");
}

void RcclComm::Broadcast(uint64_t send, uint64_t recv, uint64_t count, int dtype, int root, uint64_t stream) {
  if (!comm_) throw std::runtime_error("RcclComm: communicator closed");
  Check(A().broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), size_t(count),
                      ncclDataType_t(dtype), root, comm_, reinterpret_cast<hipStream_t>(stream)),
        "ncclBroadcast");
}

std::string RcclComm::AsyncError() {
  if (!comm_) return "";
  ncclResult_t r = ncclSuccess;
  Check(A().async_error(comm_, &r), "ncclCommGetAsyncError");
  return r == ncclSuccess ? std::string() : std::string(A().err(r));
}

void RcclComm::Abort() {
  if (comm_) {
    (void)A().abort(comm_);
    comm_ = nullptr;
  }
}

void RcclComm::Destroy() {
  if (comm_) {
    Check(A().destroy(comm_), "ncclCommDestroy");
    comm_ = nullptr;
  }
}

}  // namespace rmm::hip
