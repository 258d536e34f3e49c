// pybind11 bindings for the CDNA4 kernels and the HBM GPU object store.
// Tensors cross the boundary as raw device pointers + the caller's hipStream_t (from
// torch.cuda.current_stream().cuda_stream); results come back zero-copy as DLPack capsules.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>

#include "common.h"
#include "gpu_store.h"
#include "kernels.h"
#include "peer_allreduce.h"
#include "rccl_comm.h"
#include "rollout_loop.h"

namespace py = pybind11;
using namespace rmm::hip;

namespace {

inline hipStream_t S(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }
template <typename T>
inline T* P(uint64_t p) {
  return reinterpret_cast<T*>(p);
}

// [master, m1, m2, grad, wbf16, n, hp, step_ctr, bump, nbump, bump_next] (empty: no Adam workgroups);
// pointers already offset to the range start, bump_next = 0 for the in-place ticket bump
AdamTail adam_tail(const std::vector<uint64_t>& v, float grad_scale) {
  AdamTail at;
  if (v.empty()) return at;
  if (v.size() != 11 && v.size() != 14) throw std::invalid_argument("adam tail: 11 (+3 split) fields");
  if (v[0])  // master == 0: counters only (no linear Adam workgroups)
    for (int k : {0, 1, 2, 3, 4, 6, 7})
      if (v[k] == 0) throw std::invalid_argument("adam tail: null buffer");
  at.master = v[0] ? P<float>(v[0]) : nullptr;
  at.m1 = P<float>(v[1]);
  at.m2 = P<float>(v[2]);
  at.grad = P<const void>(v[3]);
  at.wbf16 = P<void>(v[4]);
  at.n = int64_t(v[5]);
  at.hp = P<const float>(v[6]);
  at.step_ctr = P<const int64_t>(v[7]);
  at.bump = v[8] ? P<int64_t>(v[8]) : nullptr;
  at.nbump = int(v[9]);
  at.bump_next = v[10] ? P<int64_t>(v[10]) : nullptr;
  at.grad_scale = grad_scale;
  if (v.size() == 14 && v[11]) {  // [.., part, rs, K]: gradients from the K12 row-split partials
    at.part = P<const float>(v[11]);
    at.rs = int(v[12]);
    at.K = int64_t(v[13]);
  }
  return at;
}

// [grad_base, master, m1, m2, wbf16, hp, step_ctr, bump, nbump, done] (empty: plain gradient stores)
FusedAdam fused_adam(const std::vector<uint64_t>& v) {
  FusedAdam fa;
  if (v.empty()) return fa;
  if (v.size() != 10) throw std::invalid_argument("fused adam: 10 fields");
  for (int k : {0, 1, 2, 3, 4, 5, 6})
    if (v[k] == 0) throw std::invalid_argument("fused adam: null buffer");
  if (v[7] && (v[8] <= 0 || v[9] == 0)) throw std::invalid_argument("fused adam: bump needs nbump and done");
  fa.grad_base = P<const void>(v[0]);
  fa.master = P<float>(v[1]);
  fa.m1 = P<float>(v[2]);
  fa.m2 = P<float>(v[3]);
  fa.wbf16 = P<void>(v[4]);
  fa.hp = P<const float>(v[5]);
  fa.step_ctr = P<const int64_t>(v[6]);
  fa.bump = v[7] ? P<int64_t>(v[7]) : nullptr;
  fa.nbump = int(v[8]);
  fa.done = v[9] ? P<uint32_t>(v[9]) : nullptr;
  return fa;
}

using XP = std::pair<uint64_t, uint64_t>;  // split pair (hi_ptr, lo_ptr)
X3In xin(const XP& p) { return X3In{reinterpret_cast<const void*>(p.first), reinterpret_cast<const void*>(p.second)}; }
X3Out xout(const XP& p) { return X3Out{reinterpret_cast<void*>(p.first), reinterpret_cast<void*>(p.second)}; }

// ---- minimal DLPack ABI (stable C ABI, v0.x "dltensor" capsule)
struct DLDevice {
  int32_t device_type;
  int32_t device_id;
};
struct DLDataType {
  uint8_t code;
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLROCM = 10;

struct Ctx {
  std::vector<int64_t> shape, strides;
  std::shared_ptr<GpuStore> store;
  std::string id;
  PyObject* callback = nullptr;
};

void dl_deleter(DLManagedTensor* t) {
  Ctx* c = static_cast<Ctx*>(t->manager_ctx);
  if (c->store) c->store->Release(c->id);
  if (c->callback) {
    py::gil_scoped_acquire gil;
    PyObject* r = PyObject_CallObject(c->callback, nullptr);
    if (!r) PyErr_Clear();
    Py_XDECREF(r);
    Py_DECREF(c->callback);
  }
  delete c;
  delete t;
}

void capsule_destructor(PyObject* cap) {
  // only delete if never consumed (consumer renames to "used_dltensor")
  if (PyCapsule_IsValid(cap, "dltensor")) {
    auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
    if (t && t->deleter) t->deleter(t);
  }
}

py::object make_dlpack(uint64_t ptr, std::vector<int64_t> shape, int code, int bits, int device,
                       std::shared_ptr<GpuStore> store, const std::string& id, py::object callback) {
  auto* t = new DLManagedTensor();
  auto* c = new Ctx();
  c->shape = std::move(shape);
  c->strides.resize(c->shape.size());
  int64_t st = 1;
  for (int i = int(c->shape.size()) - 1; i >= 0; i--) {
    c->strides[size_t(i)] = st;
    st *= c->shape[size_t(i)];
  }
  c->store = std::move(store);
  c->id = id;
  if (!callback.is_none()) {
    c->callback = callback.ptr();
    Py_INCREF(c->callback);
  }
  t->dl_tensor.data = reinterpret_cast<void*>(ptr);
  t->dl_tensor.device = {kDLROCM, device};
  t->dl_tensor.ndim = int32_t(c->shape.size());
  t->dl_tensor.dtype = {uint8_t(code), uint8_t(bits), 1};
  t->dl_tensor.shape = c->shape.data();
  t->dl_tensor.strides = c->strides.data();
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = c;
  t->deleter = dl_deleter;
  return py::reinterpret_steal<py::object>(PyCapsule_New(t, "dltensor", capsule_destructor));
}

}  // namespace

// adam (the x3 tail Adam): [master, m1, m2, grad, whi, wlo, n_trunk, n, hp, step_ctr, bump, nbump, done, bump_next
// (, grad2: the K12x second row part's dense + heads gradients)]; empty = no Adam
X3Adam x3_adam_args(const std::vector<uint64_t>& adam, float grad_scale, const char* who) {
  X3Adam xa;
  if (adam.empty()) return xa;
  if (adam.size() != 14 && adam.size() != 15) throw std::invalid_argument(std::string(who) + ": adam needs 14 or 15 fields");
  if (adam.size() == 15 && adam[14]) {
    if (adam[14] & 15) throw std::invalid_argument(std::string(who) + ": grad2 must be 16-byte aligned");
    xa.grad2 = P<const float>(adam[14]);
  }
  xa.master = P<float>(adam[0]), xa.m1 = P<float>(adam[1]), xa.m2 = P<float>(adam[2]);
  xa.grad = P<const float>(adam[3]), xa.whi = P<void>(adam[4]), xa.wlo = P<void>(adam[5]);
  xa.n_trunk = int64_t(adam[6]), xa.n = int64_t(adam[7]);
  xa.hp = P<const float>(adam[8]), xa.step_ctr = P<const int64_t>(adam[9]);
  xa.bump = adam[10] ? P<int64_t>(adam[10]) : nullptr, xa.nbump = int(adam[11]);
  xa.done = adam[12] ? P<uint32_t>(adam[12]) : nullptr, xa.bump_next = adam[13] ? P<int64_t>(adam[13]) : nullptr;
  xa.grad_scale = grad_scale;
  return xa;
}

PYBIND11_MODULE(_hip, m) {
  m.doc() = "CDNA4 (gfx950) kernels + HBM GPU object store";

  m.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return n;
  });
  m.def("device_synchronize", [] {
    py::gil_scoped_release nogil;
    RMM_HIP_CHECK(hipDeviceSynchronize());
  });
  m.def("stream_synchronize", [](uint64_t s) {
    py::gil_scoped_release nogil;
    RMM_HIP_CHECK(hipStreamSynchronize(S(s)));
  });
  m.def("arch", [](int dev) {
    hipDeviceProp_t p;
    RMM_HIP_CHECK(hipGetDeviceProperties(&p, dev));
    return std::string(p.gcnArchName);
  });

  // ---------------------------------------------------------------- kernels
  m.def("multi_copy",
        [](const std::vector<std::tuple<uint64_t, uint64_t, uint64_t>>& segs, uint64_t stream) {
          std::vector<CopySeg> cs;
          cs.reserve(segs.size());
          for (auto& s : segs) cs.push_back({std::get<0>(s), std::get<1>(s), std::get<2>(s)});
          multi_copy(cs, S(stream));
        });
  m.def("gather_rows", [](uint64_t in, uint64_t idx, uint64_t out, int64_t rows, int64_t row_bytes,
                          uint64_t stream, uint64_t ctr, int64_t period) {
    gather_rows(P<const void>(in), P<const int64_t>(idx), P<void>(out), rows, row_bytes, S(stream),
                ctr ? P<const int64_t>(ctr) : nullptr, period);
  }, py::arg("in"), py::arg("idx"), py::arg("out"), py::arg("rows"), py::arg("row_bytes"), py::arg("stream"),
     py::arg("ctr") = 0, py::arg("period") = 1);
  m.def("frames_to_nhwc_bf16", [](uint64_t src, uint64_t idx, uint64_t dst, int64_t B, int64_t C, int64_t H,
                                  int64_t W, float scale, uint64_t stream, uint64_t ctr, int64_t period) {
    frames_to_nhwc_bf16(P<const uint8_t>(src), idx ? P<const int64_t>(idx) : nullptr, P<void>(dst), B, C, H, W,
                        scale, S(stream), ctr ? P<const int64_t>(ctr) : nullptr, period);
  }, py::arg("src"), py::arg("idx"), py::arg("dst"), py::arg("B"), py::arg("C"), py::arg("H"), py::arg("W"),
     py::arg("scale"), py::arg("stream"), py::arg("ctr") = 0, py::arg("period") = 1);
  m.def("frames_to_nhwc_f32", [](uint64_t src, uint64_t idx, uint64_t dst, int64_t B, int64_t C, int64_t H,
                                 int64_t W, float scale, uint64_t stream, uint64_t ctr, int64_t period) {
    frames_to_nhwc_f32(P<const uint8_t>(src), idx ? P<const int64_t>(idx) : nullptr, P<float>(dst), B, C, H, W, scale,
                       S(stream), ctr ? P<const int64_t>(ctr) : nullptr, period);
  }, py::arg("src"), py::arg("idx"), py::arg("dst"), py::arg("B"), py::arg("C"), py::arg("H"), py::arg("W"),
     py::arg("scale"), py::arg("stream"), py::arg("ctr") = 0, py::arg("period") = 1);
  m.def("gae", [](uint64_t rew, uint64_t val, uint64_t done, uint64_t last, uint64_t adv, uint64_t ret,
                  int64_t T, int64_t B, float gamma, float lam, uint64_t stream) {
    gae(P<const float>(rew), P<const float>(val), P<const float>(done), P<const float>(last), P<float>(adv),
        P<float>(ret), T, B, gamma, lam, S(stream));
  });
  m.def("compress_bound", &compress_bound);
  m.def("compress_workspace", &compress_workspace);
  m.def("compress", [](uint64_t src, uint64_t n, int bits, uint64_t dst, uint64_t ws, uint64_t stream) {
    py::gil_scoped_release nogil;
    return compress(P<const void>(src), n, bits, P<void>(dst), P<void>(ws), S(stream));
  });
  m.def("decompress", [](uint64_t src, uint64_t dst, uint64_t n, int bits, uint64_t ws, uint64_t stream) {
    decompress(P<const void>(src), P<void>(dst), n, bits, P<void>(ws), S(stream));
  });
  m.def("scan_u16", [](uint64_t in, uint64_t out, uint64_t n, uint64_t ws, uint64_t stream) {
    scan_u16(P<const uint16_t>(in), P<uint64_t>(out), n, P<void>(ws), S(stream));
  });
  m.def("ppo_loss", [](uint64_t logp_new, uint64_t logp_old, uint64_t adv, uint64_t v_new, uint64_t v_tgt,
                       uint64_t ent, uint64_t g_logp, uint64_t g_v, uint64_t g_ent, uint64_t stats, int64_t n,
                       float clip, float vf_clip, float vf_coeff, float ent_coeff, uint64_t stream) {
    ppo_loss_fwd(P<const float>(logp_new), P<const float>(logp_old), P<const float>(adv), P<const float>(v_new),
                 nullptr, P<const float>(v_tgt), P<const float>(ent), P<float>(g_logp), P<float>(g_v),
                 P<float>(g_ent), P<float>(stats), n, clip, vf_clip, vf_coeff, ent_coeff, S(stream));
  });

  m.def("ppo_cat_loss", [](bool fwd, uint64_t logits, bool logits_bf16, uint64_t old_logits, uint64_t actions,
                           uint64_t old_logp, uint64_t adv, uint64_t values, bool values_bf16, uint64_t vtgt,
                           uint64_t coef, uint64_t stats, uint64_t gout, uint64_t g_logits, uint64_t g_values,
                           int64_t N, int A, uint64_t stream) {
    ppo_cat_loss(fwd, P<const void>(logits), logits_bf16, P<const float>(old_logits), P<const int64_t>(actions),
                 P<const float>(old_logp), P<const float>(adv), P<const void>(values), values_bf16, P<const float>(vtgt),
                 P<const float>(coef), P<float>(stats), P<const float>(gout), P<void>(g_logits), P<void>(g_values), N,
                 A, S(stream));
  });
  m.def("adam_flat", [](uint64_t master, uint64_t m1, uint64_t m2, uint64_t grad, bool grad_bf16, uint64_t wbf16,
                        uint64_t hp, float grad_scale, int64_t n, uint64_t stream, uint64_t step_ctr, uint64_t bump,
                        int nbump, uint64_t done, uint64_t scale_ptr, int max_blocks, uint64_t bump_next,
                        uint64_t wlo) {
    adam_flat(P<float>(master), P<float>(m1), P<float>(m2), P<const void>(grad), grad_bf16,
              wbf16 ? P<void>(wbf16) : nullptr, P<const float>(hp), grad_scale, n, S(stream),
              step_ctr ? P<const int64_t>(step_ctr) : nullptr, bump ? P<int64_t>(bump) : nullptr, nbump,
              done ? P<uint32_t>(done) : nullptr, scale_ptr ? P<const float>(scale_ptr) : nullptr, max_blocks,
              bump_next ? P<int64_t>(bump_next) : nullptr, wlo ? P<void>(wlo) : nullptr);
  }, py::arg("master"), py::arg("m1"), py::arg("m2"), py::arg("grad"), py::arg("grad_bf16"), py::arg("wbf16"),
     py::arg("hp"), py::arg("grad_scale"), py::arg("n"), py::arg("stream"), py::arg("step_ctr") = 0,
     py::arg("bump") = 0, py::arg("nbump") = 0, py::arg("done") = 0, py::arg("scale_ptr") = 0,
     py::arg("max_blocks") = 0, py::arg("bump_next") = 0, py::arg("wlo") = 0);
  m.def("grad_clip_workspace_floats", &grad_clip_workspace_floats);
  m.def("ingest_gae", [](uint64_t raw, uint64_t boot, uint64_t blocks, int nblocks, int A, float gamma, float lam,
                         uint64_t cols, uint64_t stats, uint64_t stream) {
    ingest_gae(P<const float>(raw), P<const float>(boot), P<const IngestBlock>(blocks), nblocks, A, gamma, lam,
               P<float>(cols), P<double>(stats), S(stream));
  });
  m.def("vtrace", [](uint64_t blogp, uint64_t tlogp, uint64_t rew, uint64_t val, uint64_t done, uint64_t boot,
                     int64_t T, int64_t B, float gamma, float clip_rho, float clip_pg_rho, float lam, uint64_t vs,
                     uint64_t pg, uint64_t stream) {
    vtrace(P<const float>(blogp), P<const float>(tlogp), P<const float>(rew), P<const float>(val),
           P<const float>(done), P<const float>(boot), T, B, gamma, clip_rho, clip_pg_rho, lam, P<float>(vs),
           P<float>(pg), S(stream));
  });
  m.def("ingest_block_bytes",[] { return int(sizeof(IngestBlock)); });
  m.def("standardize_col", [](uint64_t cols, int64_t N, int C, int col, uint64_t stats, uint64_t stream) {
    standardize_col(P<float>(cols), N, C, col, P<const double>(stats), S(stream));
  });
  m.def("host_register_segment", [](uint64_t base, uint64_t size) { host_register_segment(base, size); });
  m.def("h2d_from_segment", [](uint64_t dst, uint64_t src, uint64_t n, uint64_t stream) {
    py::gil_scoped_release nogil;
    return h2d_from_segment(P<void>(dst), P<const void>(src), n, S(stream));
  });
  m.def("host_unregister_all", [] { host_unregister_all(); });
  m.def("host_unregister_segment", [](uint64_t base) { host_unregister_segment(base); });
  m.def("h2d_stats", [] { return h2d_stats(); });
  m.def("host_register_last_error", [] { return host_register_last_error(); });
  m.def("grad_clip_coef", [](uint64_t grad, bool grad_bf16, int64_t n, float grad_scale, float max_norm,
                             uint64_t ws, uint64_t out, uint64_t stream) {
    grad_clip_coef(P<const void>(grad), grad_bf16, n, grad_scale, max_norm, P<float>(ws), P<float>(out), S(stream));
  });
  m.def("bump_done_words", &bump_done_words);
  m.def("ppo_heads_loss", [](bool bwd, uint64_t heads, uint64_t cols, uint64_t coef, uint64_t acc, uint64_t gout,
                             uint64_t g_heads, int64_t N, int A, uint64_t stream) {
    ppo_heads_loss(bwd, P<const void>(heads), P<const float>(cols), P<const float>(coef), P<float>(acc),
                   P<const float>(gout), P<void>(g_heads), N, A, S(stream));
  });
  m.def("sample_store", [](uint64_t logits, bool logits_bf16, uint64_t values, bool values_bf16, uint64_t t_ptr,
                           uint64_t ctr, uint32_t seed, uint64_t act, uint64_t logp, uint64_t vf, uint64_t lout,
                           uint64_t act_now, int64_t B, int A, uint64_t stream, int64_t ldl, int64_t ldv) {
    sample_store(P<const void>(logits), logits_bf16, P<const void>(values), values_bf16, P<const int64_t>(t_ptr),
                 P<const int64_t>(ctr), seed, P<int64_t>(act), P<float>(logp), P<float>(vf), P<float>(lout),
                 P<int64_t>(act_now), B, A, S(stream), ldl, ldv);
  }, py::arg("logits"), py::arg("logits_bf16"), py::arg("values"), py::arg("values_bf16"), py::arg("t_ptr"),
     py::arg("ctr"), py::arg("seed"), py::arg("act"), py::arg("logp"), py::arg("vf"), py::arg("lout"),
     py::arg("act_now"), py::arg("B"), py::arg("A"), py::arg("stream"), py::arg("ldl") = 0, py::arg("ldv") = 0);

  // device-visible address of pinned (hipHostMalloc / registered) host memory; throws if unmapped,
  // so a kernel is never handed a host pointer the GPU cannot reach
  m.def("host_device_pointer", [](uint64_t host_ptr) {
    void* d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, P<void>(host_ptr), 0);
    if (e != hipSuccess || d == nullptr) {
      (void)hipGetLastError();
      throw std::runtime_error(std::string("host_device_pointer: not mapped pinned memory: ") + hipGetErrorString(e));
    }
    return reinterpret_cast<uint64_t>(d);
  }, py::arg("host_ptr"));
  // native hybrid rollout loop: groups = [(graph_exec, stream, pools, t, step, seed, n, A, episode_len, act,
  // new_frames, rew, done, ep_rew, ep_len[, gate release counter])], all raw addresses; returns finished
  // (return, length) episodes
  m.def("hybrid_rollout", [](const std::vector<std::vector<uint64_t>>& groups, int64_t T, int threads, bool spin) {
    std::vector<RolloutGroup> G;
    for (const auto& v : groups) {
      if (v.size() != 15 && v.size() != 16) throw std::invalid_argument("hybrid_rollout: 15 or 16 fields per group");
      RolloutGroup g;
      g.exec = reinterpret_cast<hipGraphExec_t>(v[0]);
      g.stream = S(v[1]);
      g.env.pools = P<const uint8_t>(v[2]);
      g.env.t = P<int64_t>(v[3]);
      g.env.step = P<uint64_t>(v[4]);
      g.env.seed = v[5];
      g.env.n = int64_t(v[6]);
      g.env.num_actions = int64_t(v[7]);
      g.env.episode_len = int64_t(v[8]);
      g.act = P<const int64_t>(v[9]);
      g.new_frames = P<uint8_t>(v[10]);
      g.rew = P<float>(v[11]);
      g.done = P<float>(v[12]);
      g.ep_rew = P<double>(v[13]);
      g.ep_len = P<int64_t>(v[14]);
      g.release = v.size() > 15 && v[15] ? P<int64_t>(v[15]) : nullptr;
      if (g.env.n <= 0 || g.env.num_actions <= 0 || g.env.episode_len <= 0)
        throw std::invalid_argument("hybrid_rollout: bad env shape");
      G.push_back(g);
    }
    py::gil_scoped_release nogil;
    return hybrid_rollout(G, T, threads, spin);
  }, py::arg("groups"), py::arg("T"), py::arg("threads") = 1, py::arg("spin") = false);
  m.def("hybrid_rollout_phases", &hybrid_rollout_phases);
  m.def("launch_overhead_probe", [](int n, uint64_t stream) {
    py::gil_scoped_release nogil;
    return launch_overhead_probe(n, S(stream));
  }, py::arg("n"), py::arg("stream"));
  // the native loop over ONE group with direct kernel launches per step (no graph): `group` =
  // hybrid_rollout's 15 fields (exec ignored), weights / strides / bufs as hybrid_rollout_server,
  // k16_done = K16's zero-initialised completion counter
  m.def("hybrid_rollout_direct", [](const std::vector<uint64_t>& v, const std::vector<uint64_t>& wts,
                                    std::vector<int64_t> w1s, std::vector<int64_t> w2s,
                                    const std::vector<uint64_t>& bufs, int64_t B, int slices, int A1, uint32_t seed,
                                    uint64_t k16_done, int64_t T, int threads, bool spin, uint64_t host_seq,
                                    uint64_t host_seq_dev, uint64_t release, uint64_t release_dev, uint64_t gate_err,
                                    int gate_parts, int gate_timeout_ms, bool fused_heads) {
    // fp32 policy: 16 weights (8 hi planes, then the 8 lo planes) and a 12th buffer (the h2 lo plane)
    const bool x3 = wts.size() == 16;
    if (fused_heads && (!x3 || B > 64))
      throw std::invalid_argument("hybrid_rollout_direct: fused K13x + K16x needs the fp32 policy and B <= 64");
    if (v.size() < 15 || (wts.size() != 8 && !x3) || bufs.size() < size_t(x3 ? 12 : 11) || w1s.size() != 4 ||
        w2s.size() != 4 || !k16_done)
      throw std::invalid_argument("hybrid_rollout_direct: 15 group fields, 8 (16) weights, 11 (12) buffers, 4+4 strides, done");
    RolloutGroup g;
    g.stream = S(v[1]);
    g.env.pools = P<const uint8_t>(v[2]);
    g.env.t = P<int64_t>(v[3]);
    g.env.step = P<uint64_t>(v[4]);
    g.env.seed = v[5];
    g.env.n = int64_t(v[6]);
    g.env.num_actions = int64_t(v[7]);
    g.env.episode_len = int64_t(v[8]);
    g.act = P<const int64_t>(v[9]);
    g.new_frames = P<uint8_t>(v[10]);
    g.rew = P<float>(v[11]);
    g.done = P<float>(v[12]);
    g.ep_rew = P<double>(v[13]);
    g.ep_len = P<int64_t>(v[14]);
    if (g.env.n != B) throw std::invalid_argument("hybrid_rollout_direct: env count != B");
    RolloutServerArgs a;
    a.W1 = P<const void>(wts[0]);
    a.b1 = P<const void>(wts[1]);
    a.W2 = P<const void>(wts[2]);
    a.b2 = P<const void>(wts[3]);
    a.Wd = P<const void>(wts[4]);
    a.bd = P<const void>(wts[5]);
    a.Wh = P<const void>(wts[6]);
    a.bh = P<const void>(wts[7]);
    for (int k = 0; k < 4; k++) a.w1s[k] = w1s[k], a.w2s[k] = w2s[k];
    a.stack = P<uint8_t>(bufs[0]);
    a.nf = P<const uint8_t>(bufs[1]);
    a.rows = P<uint8_t>(bufs[2]);
    a.h2 = P<void>(bufs[3]);
    a.hpart = P<float>(bufs[4]);
    a.act = P<int64_t>(bufs[5]);
    a.logp = P<float>(bufs[6]);
    a.vf = P<float>(bufs[7]);
    a.lout = P<float>(bufs[8]);
    a.act_now = P<int64_t>(bufs[9]);
    a.ctr_t = P<int64_t>(bufs[10]);
    a.B = B;
    a.S = slices;
    a.A1 = A1;
    a.seed = seed;
    if (x3) {
      a.x3 = true;
      a.W1lo = P<const void>(wts[8]);
      a.b1lo = P<const void>(wts[9]);
      a.W2lo = P<const void>(wts[10]);
      a.b2lo = P<const void>(wts[11]);
      a.Wdlo = P<const void>(wts[12]);
      a.bdlo = P<const void>(wts[13]);
      a.Whlo = P<const void>(wts[14]);
      a.bhlo = P<const void>(wts[15]);
      a.h2lo = P<void>(bufs[11]);
    }
    a.fused_heads = fused_heads;
    g.direct = &a;
    g.k16_done = P<unsigned int>(k16_done);
    if ((host_seq == 0) != (host_seq_dev == 0))
      throw std::invalid_argument("hybrid_rollout_direct: host_seq needs its device view and vice versa");
    g.host_seq = host_seq ? P<int64_t>(host_seq) : nullptr;
    g.host_seq_dev = host_seq_dev ? P<int64_t>(host_seq_dev) : nullptr;
    // in-kernel step gate (the fp32 K10x only: the bf16 K10 push does not gate, so it would read stale frames)
    if (release || release_dev || gate_err) {
      if (!x3 || !release || !release_dev || !gate_err)
        throw std::invalid_argument("hybrid_rollout_direct: the step gate needs the fp32 policy, the pinned release "
                                    "counter, its device view and an error word");
      g.release = P<int64_t>(release);
      a.gate = P<const int64_t>(release_dev);
      a.gate_err = P<int>(gate_err);
      if (gate_parts < 1 || gate_parts > B) throw std::invalid_argument("hybrid_rollout_direct: 1 <= gate_parts <= B");
      g.gate_parts = gate_parts;
      if (gate_timeout_ms < 1) throw std::invalid_argument("hybrid_rollout_direct: gate_timeout_ms >= 1");
      a.gate_timeout_ms = gate_timeout_ms;
    }
    std::vector<RolloutGroup> G{g};
    py::gil_scoped_release nogil;
    return hybrid_rollout(G, T, threads, spin);
  }, py::arg("group"), py::arg("weights"), py::arg("w1s"), py::arg("w2s"), py::arg("bufs"), py::arg("B"), py::arg("S"),
     py::arg("A1"), py::arg("seed"), py::arg("k16_done"), py::arg("T"), py::arg("threads") = 1, py::arg("spin") = false,
     py::arg("host_seq") = 0, py::arg("host_seq_dev") = 0, py::arg("release") = 0, py::arg("release_dev") = 0,
     py::arg("gate_err") = 0, py::arg("gate_parts") = 1, py::arg("gate_timeout_ms") = 2000,
     py::arg("fused_heads") = false);
  // K21 persistent rollout server over one group: `group` = hybrid_rollout's 15 group fields (exec
  // ignored); weights = [W1, b1, W2, b2, Wd, bd, Wh, bh]; bufs = [stack, nf, rows, h2, hpart, act,
  // logp, vf, lout, act_now, ctr_t]
  m.def("hybrid_rollout_server", [](const std::vector<uint64_t>& v, const std::vector<uint64_t>& wts,
                                    std::vector<int64_t> w1s, std::vector<int64_t> w2s,
                                    const std::vector<uint64_t>& bufs, int64_t B, int64_t T, int slices, int A1,
                                    uint32_t seed, int threads, int workgroups, double go_timeout,
                                    double barrier_timeout, double wait_timeout) {
    if (v.size() < 15 || wts.size() != 8 || (bufs.size() != 11 && bufs.size() != 12) || w1s.size() != 4 ||
        w2s.size() != 4)
      throw std::invalid_argument("hybrid_rollout_server: 15 group fields, 8 weights, 11 (+prof) buffers, 4+4 strides");
    RolloutGroup g;
    g.stream = S(v[1]);
    g.env.pools = P<const uint8_t>(v[2]);
    g.env.t = P<int64_t>(v[3]);
    g.env.step = P<uint64_t>(v[4]);
    g.env.seed = v[5];
    g.env.n = int64_t(v[6]);
    g.env.num_actions = int64_t(v[7]);
    g.env.episode_len = int64_t(v[8]);
    g.act = P<const int64_t>(v[9]);
    g.new_frames = P<uint8_t>(v[10]);
    g.rew = P<float>(v[11]);
    g.done = P<float>(v[12]);
    g.ep_rew = P<double>(v[13]);
    g.ep_len = P<int64_t>(v[14]);
    if (g.env.n != B) throw std::invalid_argument("hybrid_rollout_server: env count != B");
    RolloutServerArgs a;
    a.W1 = P<const void>(wts[0]);
    a.b1 = P<const void>(wts[1]);
    a.W2 = P<const void>(wts[2]);
    a.b2 = P<const void>(wts[3]);
    a.Wd = P<const void>(wts[4]);
    a.bd = P<const void>(wts[5]);
    a.Wh = P<const void>(wts[6]);
    a.bh = P<const void>(wts[7]);
    for (int k = 0; k < 4; k++) a.w1s[k] = w1s[k], a.w2s[k] = w2s[k];
    a.stack = P<uint8_t>(bufs[0]);
    a.nf = P<const uint8_t>(bufs[1]);
    a.rows = P<uint8_t>(bufs[2]);
    a.h2 = P<void>(bufs[3]);
    a.hpart = P<float>(bufs[4]);
    a.act = P<int64_t>(bufs[5]);
    a.logp = P<float>(bufs[6]);
    a.vf = P<float>(bufs[7]);
    a.lout = P<float>(bufs[8]);
    a.act_now = P<int64_t>(bufs[9]);
    a.ctr_t = P<int64_t>(bufs[10]);
    a.prof = bufs.size() > 11 && bufs[11] ? P<uint64_t>(bufs[11]) : nullptr;
    a.B = B;
    a.S = slices;
    a.A1 = A1;
    a.seed = seed;
    a.workgroups = workgroups;
    a.go_timeout_s = go_timeout;
    a.barrier_timeout_s = barrier_timeout;
    py::gil_scoped_release nogil;
    return hybrid_rollout_server(g, a, T, threads, wait_timeout);
  }, py::arg("group"), py::arg("weights"), py::arg("w1s"), py::arg("w2s"), py::arg("bufs"), py::arg("B"), py::arg("T"),
     py::arg("S"), py::arg("A1"), py::arg("seed"), py::arg("threads") = 1, py::arg("workgroups") = 0,
     py::arg("go_timeout") = 20.0, py::arg("barrier_timeout") = 5.0, py::arg("wait_timeout") = 30.0);
  m.def("step_gate", [](uint64_t host_release, uint64_t dev_seq, int64_t max_polls, uint64_t err, uint64_t stream) {
    step_gate(P<const int64_t>(host_release), P<int64_t>(dev_seq), max_polls, P<int>(err), S(stream));
  });
  m.def("frame_push", [](uint64_t stack, uint64_t new_frames, uint64_t buf_obs, uint64_t t_ptr, int64_t B, int64_t hw,
                         uint64_t stream) {
    frame_push(P<uint8_t>(stack), P<const uint8_t>(new_frames), buf_obs ? P<uint8_t>(buf_obs) : nullptr,
               t_ptr ? P<const int64_t>(t_ptr) : nullptr, B, hw, S(stream));
  }, py::arg("stack"), py::arg("new_frames"), py::arg("buf_obs"), py::arg("t_ptr"), py::arg("B"), py::arg("hw"),
     py::arg("stream"));
  m.def("synth_env_step", [](uint64_t frames, uint64_t pool, uint64_t actions, uint64_t tenv, uint64_t ctr_t,
                             uint64_t buf_obs, uint64_t buf_rew, uint64_t buf_done, uint32_t seed, int episode_len,
                             int64_t B, uint64_t stream, uint64_t bump, uint64_t done) {
    synth_env_step(P<uint8_t>(frames), P<const uint8_t>(pool), P<const int64_t>(actions), P<int32_t>(tenv),
                   P<const int64_t>(ctr_t), buf_obs ? P<uint8_t>(buf_obs) : nullptr, P<float>(buf_rew),
                   P<float>(buf_done), seed, episode_len, B, S(stream), bump ? P<int64_t>(bump) : nullptr,
                   done ? P<uint32_t>(done) : nullptr);
  }, py::arg("frames"), py::arg("pool"), py::arg("actions"), py::arg("tenv"), py::arg("ctr_t"), py::arg("buf_obs"),
     py::arg("buf_rew"), py::arg("buf_done"), py::arg("seed"), py::arg("episode_len"), py::arg("B"), py::arg("stream"),
     py::arg("bump") = 0, py::arg("done") = 0);
  m.def("bias_relu_fwd", [](uint64_t y, uint64_t bias, int64_t M, int C, bool relu, uint64_t stream) {
    bias_relu_fwd(P<void>(y), P<const void>(bias), M, C, relu, S(stream));
  });
  m.def("bias_relu_bwd_partials", &bias_relu_bwd_partials);
  m.def("mask_colsum", [](uint64_t dy, uint64_t y, uint64_t dpre, uint64_t db, int64_t M, int C, bool relu,
                          uint64_t stream) {
    mask_colsum(P<const void>(dy), y ? P<const void>(y) : nullptr, dpre ? P<void>(dpre) : nullptr, P<void>(db), M, C,
                relu, S(stream));
  });
  m.def("bias_relu_bwd", [](uint64_t dy, uint64_t y, uint64_t dpre, uint64_t db, uint64_t partial, int64_t M, int C,
                            bool relu, uint64_t stream) {
    bias_relu_bwd(P<const void>(dy), P<const void>(y), P<void>(dpre), P<void>(db), P<float>(partial), M, C, relu,
                  S(stream));
  });

  m.def("nature_trunk_fwd", [](uint64_t obs, uint64_t idx, uint64_t ctr, int64_t period, int64_t B, uint64_t W1,
                               std::vector<int64_t> w1s, uint64_t b1, uint64_t W2, std::vector<int64_t> w2s,
                               uint64_t b2, uint64_t h1, uint64_t h2, uint64_t stream, int dbg) {
    if (w1s.size() != 4 || w2s.size() != 4) throw std::invalid_argument("nature_trunk_fwd: 4 strides per weight");
    nature_trunk_fwd(P<const uint8_t>(obs), idx ? P<const int64_t>(idx) : nullptr,
                     ctr ? P<const int64_t>(ctr) : nullptr, period, B, P<const void>(W1), w1s.data(),
                     P<const void>(b1), P<const void>(W2), w2s.data(), P<const void>(b2), h1 ? P<void>(h1) : nullptr,
                     P<void>(h2), S(stream), dbg);
  }, py::arg("obs"), py::arg("idx"), py::arg("ctr"), py::arg("period"), py::arg("B"), py::arg("W1"), py::arg("w1s"),
     py::arg("b1"), py::arg("W2"), py::arg("w2s"), py::arg("b2"), py::arg("h1"), py::arg("h2"), py::arg("stream"),
     py::arg("dbg") = 0);
  m.def("nature_trunk_fwd_push", [](uint64_t stack, uint64_t nf, uint64_t rows, uint64_t t_ptr, int64_t B, uint64_t W1,
                                    std::vector<int64_t> w1s, uint64_t b1, uint64_t W2, std::vector<int64_t> w2s,
                                    uint64_t b2, uint64_t h2, uint64_t stream) {
    if (w1s.size() != 4 || w2s.size() != 4) throw std::invalid_argument("nature_trunk_fwd_push: 4 strides per weight");
    nature_trunk_fwd_push(P<uint8_t>(stack), P<const uint8_t>(nf), rows ? P<uint8_t>(rows) : nullptr,
                          t_ptr ? P<const int64_t>(t_ptr) : nullptr, B, P<const void>(W1), w1s.data(), P<const void>(b1),
                          P<const void>(W2), w2s.data(), P<const void>(b2), P<void>(h2), S(stream));
  });
  m.def("nature_trunk_fwd_push_rows", [](uint64_t rows, int64_t T, uint64_t nf, uint64_t t_ptr, int64_t B, uint64_t W1,
                                         std::vector<int64_t> w1s, uint64_t b1, uint64_t W2, std::vector<int64_t> w2s,
                                         uint64_t b2, uint64_t h2, uint64_t stream) {
    if (w1s.size() != 4 || w2s.size() != 4) throw std::invalid_argument("nature_trunk_fwd_push_rows: 4 strides per weight");
    nature_trunk_fwd_push_rows(P<uint8_t>(rows), T, P<const uint8_t>(nf), P<const int64_t>(t_ptr), B, P<const void>(W1),
                               w1s.data(), P<const void>(b1), P<const void>(W2), w2s.data(), P<const void>(b2), P<void>(h2),
                               S(stream));
  });
  m.def("nature_trunk_partial_floats", &nature_trunk_partial_floats);
  m.def("dense_relu_fwd", [](uint64_t x, uint64_t w, uint64_t b, int64_t M, int64_t K, int N, uint64_t y,
                             uint64_t stream) {
    dense_relu_fwd(P<const void>(x), P<const void>(w), P<const void>(b), M, K, N, P<void>(y), S(stream));
  });
  m.def("dense_heads_fwd", [](uint64_t hidden, uint64_t wh, uint64_t bh, int64_t M, int A1, uint64_t heads,
                              uint64_t stream) {
    dense_heads_fwd(P<const void>(hidden), P<const void>(wh), P<const void>(bh), M, A1, P<void>(heads), S(stream));
  });
  m.def("partition_groups", &partition_groups);
  m.def("partition_hist", [](uint64_t keys, int64_t n, int R, int mode, uint64_t counts, uint64_t stream) {
    partition_hist(P<const int64_t>(keys), n, R, mode, P<int64_t>(counts), S(stream));
  });
  m.def("partition_scatter", [](uint64_t keys, uint64_t vals, int64_t n, int64_t row_bytes, int R, int mode,
                                uint64_t offsets, uint64_t out_keys, uint64_t out_vals, uint64_t stream) {
    partition_scatter(P<const int64_t>(keys), vals ? P<const void>(vals) : nullptr, n, row_bytes, R, mode,
                      P<const int64_t>(offsets), P<int64_t>(out_keys), out_vals ? P<void>(out_vals) : nullptr,
                      S(stream));
  });
  m.def("dense_heads_bwd", [](uint64_t dz, int A1, uint64_t wh, uint64_t y, uint64_t x, uint64_t w, int64_t M,
                              int64_t K, uint64_t dx, uint64_t dw, uint64_t db, uint64_t dwh, uint64_t dbh,
                              uint64_t scratch, uint64_t stream, bool dpre_ready, std::vector<uint64_t> adam,
                              bool defer_finalize, int split) {
    dense_heads_bwd(P<const void>(dz), A1, P<const void>(wh), P<const void>(y), P<const void>(x), P<const void>(w), M,
                    K, P<void>(dx), P<void>(dw), P<void>(db), P<void>(dwh), P<void>(dbh), P<void>(scratch),
                    S(stream), dpre_ready, fused_adam(adam), defer_finalize, split);
  }, py::arg("dz"), py::arg("A1"), py::arg("wh"), py::arg("y"), py::arg("x"), py::arg("w"), py::arg("M"), py::arg("K"),
     py::arg("dx"), py::arg("dw"), py::arg("db"), py::arg("dwh"), py::arg("dbh"), py::arg("scratch"), py::arg("stream"),
     py::arg("dpre_ready") = false, py::arg("adam") = std::vector<uint64_t>{}, py::arg("defer_finalize") = false, py::arg("split") = -1);
  m.def("dense_split_plan", [](int64_t M, int64_t K, int split, uint64_t stream) {
    const DenseSplitPlan p = dense_split_plan(M, K, split, S(stream));
    return py::make_tuple(reinterpret_cast<uint64_t>(p.part), p.rs, p.groups);
  }, py::arg("M"), py::arg("K"), py::arg("split"), py::arg("stream"));
  m.def("dense_heads_sample", [](uint64_t hidden, uint64_t wh, uint64_t bh, uint64_t t_ptr, uint64_t ctr,
                                 uint32_t seed, uint64_t act, uint64_t logp, uint64_t vf, uint64_t lout,
                                 uint64_t act_now, int64_t B, int A1, uint64_t stream, uint64_t done, uint64_t hpart,
                                 int nslices, uint64_t hb) {
    dense_heads_sample(P<const void>(hidden), P<const void>(wh), P<const void>(bh), P<const int64_t>(t_ptr),
                       P<const int64_t>(ctr), seed, P<int64_t>(act), P<float>(logp), P<float>(vf), P<float>(lout),
                       P<int64_t>(act_now), B, A1, S(stream), P<unsigned int>(done), P<const float>(hpart), nslices,
                       P<const void>(hb));
  }, py::arg("hidden"), py::arg("wh"), py::arg("bh"), py::arg("t_ptr"), py::arg("ctr"), py::arg("seed"), py::arg("act"),
     py::arg("logp"), py::arg("vf"), py::arg("lout"), py::arg("act_now"), py::arg("B"), py::arg("A1"),
     py::arg("stream"), py::arg("done") = 0, py::arg("hpart") = 0, py::arg("S") = 0, py::arg("hb") = 0);
  m.def("dense_fwd_part_slices", &dense_fwd_part_slices);
  m.def("dense_fwd_part", [](uint64_t x, uint64_t w, int64_t M, int64_t K, int N, uint64_t part, int nslices,
                             uint64_t stream) {
    dense_fwd_part(P<const void>(x), P<const void>(w), M, K, N, P<float>(part), nslices, S(stream));
  });
  m.def("dense_heads_ppo", [](uint64_t hidden, uint64_t wh, uint64_t bh, uint64_t cols, uint64_t coef, uint64_t acc,
                              uint64_t gout, int64_t M, int A1, uint64_t dz, uint64_t dpre, uint64_t stream,
                              uint64_t cidx, uint64_t ctr, int64_t period, uint64_t hpart, int nslices, uint64_t hb,
                              uint64_t hid_out) {
    dense_heads_ppo(P<const void>(hidden), P<const void>(wh), P<const void>(bh), P<const float>(cols),
                    P<const float>(coef), P<float>(acc), P<const float>(gout), M, A1, P<void>(dz), P<void>(dpre),
                    S(stream), P<const int64_t>(cidx), P<const int64_t>(ctr), period, P<const float>(hpart), nslices,
                    P<const void>(hb), P<void>(hid_out));
  }, py::arg("hidden"), py::arg("wh"), py::arg("bh"), py::arg("cols"), py::arg("coef"), py::arg("acc"),
     py::arg("gout"), py::arg("M"), py::arg("A1"), py::arg("dz"), py::arg("dpre"), py::arg("stream"),
     py::arg("cidx") = 0, py::arg("ctr") = 0, py::arg("period") = 1, py::arg("hpart") = 0, py::arg("S") = 0,
     py::arg("hb") = 0, py::arg("hid_out") = 0);
  m.def("nature_trunk_bwd", [](uint64_t obs, uint64_t idx, uint64_t ctr, int64_t period, int64_t B, uint64_t W2,
                               std::vector<int64_t> w2s, uint64_t h1, uint64_t h2, uint64_t dh2, uint64_t partial,
                               uint64_t dW1, std::vector<int64_t> w1s, uint64_t db1, uint64_t dW2, uint64_t db2,
                               uint64_t stream, int dbg, std::vector<uint64_t> adam, std::vector<uint64_t> tail,
                               float tail_scale, std::vector<uint64_t> fin) {
    DenseFinalize df;
    if (!fin.empty()) {  // [part, rs, groups, K, A1, dw, db, dwh, dbh]
      if (fin.size() != 9 && fin.size() != 10) throw std::invalid_argument("nature_trunk_bwd: fin = 9 (+group0) fields");
      df.group0 = fin.size() > 9 ? int(fin[9]) : 0;
      df.part = P<const float>(fin[0]);
      df.rs = int(fin[1]);
      df.groups = int(fin[2]);
      df.K = int64_t(fin[3]);
      df.A1 = int(fin[4]);
      df.dw = P<void>(fin[5]);
      df.db = P<void>(fin[6]);
      df.dwh = P<void>(fin[7]);
      df.dbh = P<void>(fin[8]);
    }
    if (w1s.size() != 4 || w2s.size() != 4) throw std::invalid_argument("nature_trunk_bwd: 4 strides per weight");
    nature_trunk_bwd(P<const uint8_t>(obs), idx ? P<const int64_t>(idx) : nullptr,
                     ctr ? P<const int64_t>(ctr) : nullptr, period, B, P<const void>(W2), w2s.data(),
                     P<const void>(h1), P<const void>(h2), P<const void>(dh2), P<float>(partial), P<void>(dW1),
                     w1s.data(), P<void>(db1), P<void>(dW2), P<void>(db2), S(stream), dbg, fused_adam(adam),
                     adam_tail(tail, tail_scale), df);
  }, py::arg("obs"), py::arg("idx"), py::arg("ctr"), py::arg("period"), py::arg("B"), py::arg("W2"), py::arg("w2s"),
     py::arg("h1"), py::arg("h2"), py::arg("dh2"), py::arg("partial"), py::arg("dW1"), py::arg("w1s"), py::arg("db1"),
     py::arg("dW2"), py::arg("db2"), py::arg("stream"), py::arg("dbg") = 0, py::arg("adam") = std::vector<uint64_t>{},
     py::arg("tail") = std::vector<uint64_t>{}, py::arg("tail_scale") = 1.0f, py::arg("fin") = std::vector<uint64_t>{});

  // ---------------------------------------------------------------- split-bf16 (fp32-level) kernels
  // a split pair crosses as (hi_ptr, lo_ptr); (0, 0) = absent
  m.def("x3_probe_set", [](uint64_t ts) { x3_probe_set(reinterpret_cast<uint64_t*>(ts)); }, py::arg("ts"));
  m.def("x3_split", [](uint64_t src, uint64_t hi, uint64_t lo, int64_t n, uint64_t stream) {
    x3_split(P<const float>(src), P<void>(hi), P<void>(lo), n, S(stream));
  });
  m.def("x3_trunk_fwd", [](uint64_t obs, uint64_t idx, uint64_t ctr, int64_t period, int64_t B, XP W1,
                           std::vector<int64_t> w1s, XP b1, XP W2, std::vector<int64_t> w2s, XP b2, XP h1, XP h2,
                           uint64_t stream, uint64_t cols, uint64_t cols_out, int ncols) {
    if (w1s.size() != 4 || w2s.size() != 4) throw std::invalid_argument("x3_trunk_fwd: 4 strides per weight");
    x3_trunk_fwd(P<const uint8_t>(obs), idx ? P<const int64_t>(idx) : nullptr, ctr ? P<const int64_t>(ctr) : nullptr,
                 period, B, xin(W1), w1s.data(), xin(b1), xin(W2), w2s.data(), xin(b2), xout(h1), xout(h2), S(stream),
                 cols ? P<const float>(cols) : nullptr, cols_out ? P<float>(cols_out) : nullptr, ncols);
  }, py::arg("obs"), py::arg("idx"), py::arg("ctr"), py::arg("period"), py::arg("B"), py::arg("W1"), py::arg("w1s"),
     py::arg("b1"), py::arg("W2"), py::arg("w2s"), py::arg("b2"), py::arg("h1"), py::arg("h2"), py::arg("stream"),
     py::arg("cols") = 0, py::arg("cols_out") = 0, py::arg("ncols") = 0);
  m.def("x3_trunk_fwd_push", [](uint64_t stack, uint64_t nf, uint64_t rows, uint64_t t_ptr, int64_t B, XP W1,
                                std::vector<int64_t> w1s, XP b1, XP W2, std::vector<int64_t> w2s, XP b2, XP h2,
                                uint64_t stream) {
    if (w1s.size() != 4 || w2s.size() != 4) throw std::invalid_argument("x3_trunk_fwd_push: 4 strides per weight");
    x3_trunk_fwd_push(P<uint8_t>(stack), P<const uint8_t>(nf), rows ? P<uint8_t>(rows) : nullptr,
                      t_ptr ? P<const int64_t>(t_ptr) : nullptr, B, xin(W1), w1s.data(), xin(b1), xin(W2), w2s.data(),
                      xin(b2), xout(h2), S(stream));
  });
  m.def("x3_trunk_partial_floats", &x3_trunk_partial_floats);
  m.def("x3_trunk_bwd", [](uint64_t obs, uint64_t idx, uint64_t ctr, int64_t period, int64_t B, XP W2,
                           std::vector<int64_t> w2s, XP h1, uint64_t h2hi, XP dh2, XP dpre1, uint64_t partial,
                           uint64_t dW1, std::vector<int64_t> w1s, uint64_t db1, uint64_t dW2, uint64_t db2,
                           uint64_t stream, std::vector<uint64_t> adam, float grad_scale, bool dense_separate) {
    if (w1s.size() != 4 || w2s.size() != 4) throw std::invalid_argument("x3_trunk_bwd: 4 strides per weight");
    const X3Adam xa = x3_adam_args(adam, grad_scale, "x3_trunk_bwd");
    x3_trunk_bwd(P<const uint8_t>(obs), idx ? P<const int64_t>(idx) : nullptr, ctr ? P<const int64_t>(ctr) : nullptr,
                 period, B, xin(W2), w2s.data(), xin(h1), P<const void>(h2hi), xin(dh2), xout(dpre1), P<float>(partial),
                 P<float>(dW1), w1s.data(), P<float>(db1), P<float>(dW2), P<float>(db2), S(stream), xa, dense_separate);
  }, py::arg("obs"), py::arg("idx"), py::arg("ctr"), py::arg("period"), py::arg("B"), py::arg("W2"), py::arg("w2s"),
     py::arg("h1"), py::arg("h2hi"), py::arg("dh2"), py::arg("dpre1"), py::arg("partial"), py::arg("dW1"),
     py::arg("w1s"), py::arg("db1"), py::arg("dW2"), py::arg("db2"), py::arg("stream"),
     py::arg("adam") = std::vector<uint64_t>{}, py::arg("grad_scale") = 1.0f, py::arg("dense_separate") = false);
  // the tail Adam's dense + heads range alone (same adam fields; the counters are not advanced here)
  m.def("x3_dense_adam", [](std::vector<uint64_t> adam, float grad_scale, uint64_t stream) {
    x3_dense_adam(x3_adam_args(adam, grad_scale, "x3_dense_adam"), S(stream));
  }, py::arg("adam"), py::arg("grad_scale"), py::arg("stream"));
  m.def("x3_dense_fwd_part_slices", &x3_dense_fwd_part_slices);
  m.def("x3_dense_fwd_part", [](XP x, XP w, int64_t M, int64_t K, int N, uint64_t part, int nslices, uint64_t stream) {
    x3_dense_fwd_part(xin(x), xin(w), M, K, N, P<float>(part), nslices, S(stream));
  });
  m.def("x3_heads_ppo", [](uint64_t hpart, int nslices, XP hb, XP wh, XP bh, uint64_t cols, uint64_t coef, uint64_t acc,
                           uint64_t gout, int64_t M, int A1, XP dz, XP dpre, XP hid, uint64_t stream, uint64_t cidx,
                           uint64_t ctr, int64_t period, bool acc_slab) {
    x3_heads_ppo(P<const float>(hpart), nslices, xin(hb), xin(wh), xin(bh), P<const float>(cols), P<const float>(coef),
                 P<float>(acc), P<const float>(gout), M, A1, xout(dz), xout(dpre), xout(hid), S(stream),
                 cidx ? P<const int64_t>(cidx) : nullptr, ctr ? P<const int64_t>(ctr) : nullptr, period, acc_slab);
  }, py::arg("hpart"), py::arg("S"), py::arg("hb"), py::arg("wh"), py::arg("bh"), py::arg("cols"), py::arg("coef"),
     py::arg("acc"), py::arg("gout"), py::arg("M"), py::arg("A1"), py::arg("dz"), py::arg("dpre"), py::arg("hid"),
     py::arg("stream"), py::arg("cidx") = 0, py::arg("ctr") = 0, py::arg("period") = 1, py::arg("acc_slab") = false);
  m.def("x3_heads_ppo_groups", &x3_heads_ppo_groups, py::arg("M"));
  m.def("x3_heads_sample", [](uint64_t hpart, int nslices, XP hb, XP wh, XP bh, uint64_t t_ptr, uint64_t ctr,
                              uint32_t seed, uint64_t act, uint64_t logp, uint64_t vf, uint64_t lout, uint64_t act_now,
                              int64_t B, int A1, uint64_t stream, uint64_t done, uint64_t host_seq) {
    x3_heads_sample(P<const float>(hpart), nslices, xin(hb), xin(wh), xin(bh), P<const int64_t>(t_ptr),
                    P<const int64_t>(ctr), seed, P<int64_t>(act), P<float>(logp), P<float>(vf), P<float>(lout),
                    P<int64_t>(act_now), B, A1, S(stream), done ? P<unsigned int>(done) : nullptr,
                    host_seq ? P<int64_t>(host_seq) : nullptr);
  }, py::arg("hpart"), py::arg("S"), py::arg("hb"), py::arg("wh"), py::arg("bh"), py::arg("t_ptr"), py::arg("ctr"),
     py::arg("seed"), py::arg("act"), py::arg("logp"), py::arg("vf"), py::arg("lout"), py::arg("act_now"), py::arg("B"),
     py::arg("A1"), py::arg("stream"), py::arg("done") = 0, py::arg("host_seq") = 0);
  m.def("x3_dense_heads_sample", [](XP x, XP w, int64_t M, int64_t K, uint64_t part, int nslices, XP hb, XP wh, XP bh,
                                    uint64_t t_ptr, uint64_t ctr, uint32_t seed, uint64_t act, uint64_t logp, uint64_t vf,
                                    uint64_t lout, uint64_t act_now, int A1, uint64_t stream, uint64_t done,
                                    uint64_t host_seq) {
    x3_dense_heads_sample(xin(x), xin(w), M, K, P<float>(part), nslices, xin(hb), xin(wh), xin(bh),
                          P<const int64_t>(t_ptr), P<const int64_t>(ctr), seed, P<int64_t>(act), P<float>(logp),
                          P<float>(vf), P<float>(lout), P<int64_t>(act_now), A1, S(stream), P<unsigned int>(done),
                          host_seq ? P<int64_t>(host_seq) : nullptr);
  }, py::arg("x"), py::arg("w"), py::arg("M"), py::arg("K"), py::arg("part"), py::arg("S"), py::arg("hb"), py::arg("wh"),
     py::arg("bh"), py::arg("t_ptr"), py::arg("ctr"), py::arg("seed"), py::arg("act"), py::arg("logp"), py::arg("vf"),
     py::arg("lout"), py::arg("act_now"), py::arg("A1"), py::arg("stream"), py::arg("done"), py::arg("host_seq") = 0);
  m.def("x3_dense_heads_bwd", [](XP dz, int A1, XP y, XP x, XP w, XP dpre, int64_t M, int64_t K, XP dx, uint64_t dw,
                                 uint64_t db, uint64_t dwh, uint64_t dbh, uint64_t stream, int rs, uint64_t dw2,
                                 uint64_t db2, uint64_t dwh2, uint64_t dbh2) {
    x3_dense_heads_bwd(xin(dz), A1, xin(y), xin(x), xin(w), xin(dpre), M, K, xout(dx), P<float>(dw), P<float>(db),
                       P<float>(dwh), P<float>(dbh), S(stream), rs, dw2 ? P<float>(dw2) : nullptr,
                       db2 ? P<float>(db2) : nullptr, dwh2 ? P<float>(dwh2) : nullptr, dbh2 ? P<float>(dbh2) : nullptr);
  }, py::arg("dz"), py::arg("A1"), py::arg("y"), py::arg("x"), py::arg("w"), py::arg("dpre"), py::arg("M"), py::arg("K"),
     py::arg("dx"), py::arg("dw"), py::arg("db"), py::arg("dwh"), py::arg("dbh"), py::arg("stream"), py::arg("rs") = 1,
     py::arg("dw2") = 0, py::arg("db2") = 0, py::arg("dwh2") = 0, py::arg("dbh2") = 0);

  // ---------------------------------------------------------------- IPC
  m.def("ipc_open", [](py::bytes handle, int device) {
    std::string h = handle;
    if (h.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("bad IPC handle size");
    hipIpcMemHandle_t mh;
    memcpy(&mh, h.data(), sizeof(mh));
    RMM_HIP_CHECK(hipSetDevice(device));
    void* p = nullptr;
    RMM_HIP_CHECK(hipIpcOpenMemHandle(&p, mh, hipIpcMemLazyEnablePeerAccess));
    return reinterpret_cast<uint64_t>(p);
  });
  m.def("ipc_close", [](uint64_t p) { RMM_HIP_CHECK(hipIpcCloseMemHandle(reinterpret_cast<void*>(p))); });
  // Canonical PCI address "dddd:bb:dd.f" of a visible device: identifies a physical GPU across
  // processes whose HIP_VISIBLE_DEVICES differ (a local device index does not).
  m.def("pci_bus_id", [](int device) {
    char buf[64] = {0};
    RMM_HIP_CHECK(hipDeviceGetPCIBusId(buf, int(sizeof(buf)), device));
    std::string s(buf);
    for (auto& ch : s) ch = char(tolower(ch));
    return s;
  });
  m.def("can_access_peer", [](int dev, int peer) {
    int ok = 0;
    if (hipDeviceCanAccessPeer(&ok, dev, peer) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return ok != 0;
  });
  m.def("memcpy_async", [](uint64_t dst, uint64_t src, uint64_t n, uint64_t stream) {
    RMM_HIP_CHECK(hipMemcpyAsync(P<void>(dst), P<const void>(src), n, hipMemcpyDefault, S(stream)));
  });
  m.def("host_register", [](uint64_t p, uint64_t n) {
    return hipHostRegister(P<void>(p), n, hipHostRegisterDefault) == hipSuccess;
  });
  m.def("host_unregister", [](uint64_t p) { return hipHostUnregister(P<void>(p)) == hipSuccess; });

  // DLPack capsule over device memory. dtype code: 0 int, 1 uint, 2 float, 4 bfloat.
  m.def("dlpack", [](uint64_t ptr, std::vector<int64_t> shape, int code, int bits, int device, py::object cb) {
    return make_dlpack(ptr, std::move(shape), code, bits, device, nullptr, std::string(), cb);
  }, py::arg("ptr"), py::arg("shape"), py::arg("code"), py::arg("bits"), py::arg("device"),
     py::arg("release") = py::none());

  // ---------------------------------------------------------------- GPU object store
  py::class_<GpuStore, std::shared_ptr<GpuStore>>(m, "GpuStore")
      .def(py::init<int, uint64_t, uint64_t, const std::string&, bool, double, uint64_t>(), py::arg("device"),
           py::arg("capacity"), py::arg("slab_bytes") = 8ull << 30, py::arg("shm_name") = "",
           py::arg("compress_spill") = true, py::arg("spill_threshold") = 0.0, py::arg("prepin_bytes") = 0)
      .def("prepin_progress", [](GpuStore& s) { return s.PrepinProgress(); })
      .def("seal_descriptor_async", [](GpuStore& s, py::bytes desc_id, uint64_t stream) {
        s.SealDescriptorAsync(std::string(desc_id), S(stream));
      })
      .def("restore_foreign", [](GpuStore& s, py::bytes host_id, uint64_t dst, uint64_t nbytes) {
        std::string hid = host_id;
        py::gil_scoped_release nogil;
        return s.RestoreForeign(hid, dst, nbytes);
      })
      .def("set_spill_threshold", &GpuStore::SetSpillThreshold)
      .def("last_error", &GpuStore::LastError)
      .def("create", [](GpuStore& s, py::bytes id, uint64_t n, int bits) {
        return s.Create(std::string(id), n, bits);
      })
      .def("seal", [](GpuStore& s, py::bytes id, uint64_t stream) { s.Seal(std::string(id), S(stream)); })
      .def("put_segments",
           [](GpuStore& s, py::bytes id, const std::vector<std::pair<uint64_t, uint64_t>>& segs, int bits,
              uint64_t stream) {
             std::string sid = id;
             py::gil_scoped_release nogil;
             return s.PutSegments(sid, segs, bits, S(stream));
           })
      .def("get", [](GpuStore& s, py::bytes id, uint64_t stream) {
        std::string sid = id;
        py::gil_scoped_release nogil;
        return s.Get(sid, S(stream));
      })
      .def("release", [](GpuStore& s, py::bytes id) { s.Release(std::string(id)); })
      .def("delete", [](GpuStore& s, py::bytes id) {
        std::string sid = id;
        py::gil_scoped_release nogil;
        return s.Delete(sid);
      })
      .def("contains", [](GpuStore& s, py::bytes id) { return s.Contains(std::string(id)); })
      .def("is_spilled", [](GpuStore& s, py::bytes id) { return s.IsSpilled(std::string(id)); })
      .def("locate", [](GpuStore& s, py::bytes id) {
        int slab;
        uint64_t off = 0, n = 0;
        s.Locate(std::string(id), &slab, &off, &n);
        return py::make_tuple(slab, off, n);
      })
      .def("slab_ipc_handle", [](GpuStore& s, int slab) { return py::bytes(s.SlabIpcHandle(slab)); })
      .def("slab_base", &GpuStore::SlabBase)
      .def("spill", [](GpuStore& s, uint64_t bytes) {
        py::gil_scoped_release nogil;
        return s.Spill(bytes);
      })
      .def("spill_object", [](GpuStore& s, py::bytes id) {
        std::string sid = id;
        py::gil_scoped_release nogil;
        return s.SpillObject(sid);
      })
      .def_static("host_id", [](py::bytes id) { return py::bytes(GpuStore::HostId(std::string(id))); })
      .def_property_readonly("device", &GpuStore::device)
      .def("stats", [](GpuStore& s) {
        GpuStats st = s.Stats();
        py::dict d;
        d["capacity"] = st.capacity;
        d["slab_bytes_allocated"] = st.slab_bytes_allocated;
        d["bytes_in_use"] = st.bytes_in_use;
        d["num_objects"] = st.num_objects;
        d["spilled_objects"] = st.spilled_objects;
        d["spilled_bytes_total"] = st.spilled_bytes_total;
        d["spilled_host_bytes_total"] = st.spilled_host_bytes_total;
        d["restored_bytes_total"] = st.restored_bytes_total;
        d["puts"] = st.puts;
        d["gets"] = st.gets;
        d["spill_s_total"] = double(st.spill_ns_total) * 1e-9;
        d["restore_s_total"] = double(st.restore_ns_total) * 1e-9;
        d["proactive_spills"] = st.proactive_spills;
        d["deferred_deletes"] = st.deferred_deletes;
        d["spills_device_placed"] = st.spills_device_placed;
        return d;
      });

  // Zero-copy DLPack view of a GPU-store object; the pin is released when the tensor dies.
  m.def("store_dlpack", [](std::shared_ptr<GpuStore> s, py::bytes id, std::vector<int64_t> shape, int code,
                           int bits, uint64_t stream) {
    std::string sid = id;
    uint64_t ptr;
    {
      py::gil_scoped_release nogil;
      ptr = s->Get(sid, S(stream));
    }
    if (!ptr) throw std::runtime_error("GPU object not found");
    return make_dlpack(ptr, std::move(shape), code, bits, s->device(), s, sid, py::none());
  });

  // ---------------------------------------------------------------- peer-memory all-reduce (xGMI / hipIPC)
  m.def("peer_occupancy", [](int device) {
    const PeerOccupancy o = PeerKernelOccupancy(device);
    py::dict d;
    d["cus"] = o.cus;
    d["allreduce_per_cu"] = o.allreduce_per_cu;
    d["zero1_per_cu"] = o.zero1_per_cu;
    return d;
  });
  py::class_<PeerAllReduce, std::shared_ptr<PeerAllReduce>>(m, "PeerAllReduce")
      .def(py::init<int, int, int, uint64_t, int, double>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("cap_bytes") = 8ull << 20, py::arg("nblocks") = 64, py::arg("timeout_s") = 30.0)
      .def("handles", [](const PeerAllReduce& c) { return py::bytes(c.Handles()); })
      .def("open", [](PeerAllReduce& c, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (const auto& h : hs) v.emplace_back(std::string(h));
        c.Open(v);
      })
      .def("all_reduce", &PeerAllReduce::AllReduce, py::arg("buf"), py::arg("count"), py::arg("dtype"),
           py::arg("stream"), py::arg("algo") = 0)
      .def("all_reduce_adam",
           [](PeerAllReduce& c, uint64_t grad, uint64_t count, int dtype, uint64_t stream, uint64_t master, uint64_t m1,
              uint64_t m2, uint64_t whi, uint64_t wlo, uint64_t hp, float grad_scale, uint64_t step_ctr, uint64_t bump,
              int nbump, uint64_t done, uint64_t bump_next) {
             PeerAllReduce::AdamArgs z{P<float>(master), P<float>(m1), P<float>(m2), reinterpret_cast<void*>(whi),
                                       reinterpret_cast<void*>(wlo), P<const float>(hp), grad_scale,
                                       step_ctr ? P<const int64_t>(step_ctr) : nullptr,
                                       bump ? P<int64_t>(bump) : nullptr, nbump,
                                       done ? P<uint32_t>(done) : nullptr, bump_next ? P<int64_t>(bump_next) : nullptr};
             c.AllReduceAdam(grad, count, dtype, stream, z);
           },
           py::arg("grad"), py::arg("count"), py::arg("dtype"), py::arg("stream"), py::arg("master"), py::arg("m1"),
           py::arg("m2"), py::arg("whi"), py::arg("wlo") = 0, py::arg("hp") = 0, py::arg("grad_scale") = 1.0f,
           py::arg("step_ctr") = 0, py::arg("bump") = 0, py::arg("nbump") = 0, py::arg("done") = 0,
           py::arg("bump_next") = 0)
      .def("mask_unowned", &PeerAllReduce::MaskUnowned, py::arg("buf"), py::arg("count"), py::arg("dtype"),
           py::arg("stream"))
      .def("error", &PeerAllReduce::Error)
      .def("clear_error", &PeerAllReduce::ClearError)
      .def("set_timeout", &PeerAllReduce::set_timeout)
      .def("close", &PeerAllReduce::Close)
      .def_property_readonly("launches", &PeerAllReduce::launches)
      .def_property_readonly("world", &PeerAllReduce::world)
      .def_property_readonly("rank", &PeerAllReduce::rank)
      .def_property_readonly("nblocks", &PeerAllReduce::nblocks)
      .def_property_readonly("cap_bytes", &PeerAllReduce::cap_bytes)
      .def_property_readonly("uncached_signals", &PeerAllReduce::uncached_signals)
      .def_property_readonly("alloc_attempts", &PeerAllReduce::alloc_attempts);

  // ---------------------------------------------------------------- RCCL (framework-owned communicator)
  m.def("rccl_load", &rccl_load, py::arg("path"));
  m.def("rccl_unique_id", [] { return py::bytes(rccl_unique_id()); });
  m.attr("NCCL_FLOAT32") = int(ncclFloat32);
  m.attr("NCCL_BFLOAT16") = int(ncclBfloat16);
  m.attr("NCCL_FLOAT16") = int(ncclFloat16);
  m.attr("NCCL_INT32") = int(ncclInt32);
  m.attr("NCCL_INT64") = int(ncclInt64);
  m.attr("NCCL_UINT8") = int(ncclUint8);
  m.attr("NCCL_FLOAT64") = int(ncclFloat64);
  m.attr("NCCL_SUM") = int(ncclSum);
  m.attr("NCCL_PROD") = int(ncclProd);
  m.attr("NCCL_MAX") = int(ncclMax);
  m.attr("NCCL_MIN") = int(ncclMin);
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int nranks, int rank, int device) {
             std::string u = uid;
             py::gil_scoped_release nogil;  // blocks until every rank has joined
             return std::make_shared<RcclComm>(u, nranks, rank, device);
           }),
           py::arg("uid"), py::arg("nranks"), py::arg("rank"), py::arg("device"))
      .def("all_reduce", &RcclComm::AllReduce, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"),
           py::arg("op"), py::arg("stream"))
      .def("broadcast", &RcclComm::Broadcast, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"),
           py::arg("root"), py::arg("stream"))
      .def("async_error", &RcclComm::AsyncError)
      .def("abort", &RcclComm::Abort)
      .def("destroy", &RcclComm::Destroy)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("rank", &RcclComm::rank);
}
