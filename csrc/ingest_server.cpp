// Native Ape-X ingest service on the GPU: the device-independent core (csrc/host/ingest_core.h:
// rings -> pinned staging sets -> learner-stream-ordered H2D copies + PER insert + size word,
// semantics and threading documented there) bound to HIP, plus its Python binding. The same
// core runs under ThreadSanitizer with a fake device (csrc/host/tests/ingest_stress.cpp).
// The reference's actor is the worker's own episode loop feeding a Python deque
// (/root/reference/src/dqn_agent.py:72-106, src/replay_memory.py:22-23).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "host/ingest_core.h"
#include "include/dqn_kernels.h"

namespace {

#define HIPCK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)

struct HipDev {
  using Event = hipEvent_t;
  int device = 0;
  hipStream_t stream = nullptr;      // the learner stream

  void bind() { HIPCK(hipSetDevice(device)); }
  void* host_alloc(size_t b) {
    void* p = nullptr;
    HIPCK(hipHostMalloc(&p, b, hipHostMallocDefault));
    return p;
  }
  void host_free(void* p) { hipHostFree(p); }
  void* dev_alloc(size_t b) {
    void* p = nullptr;
    HIPCK(hipMalloc(&p, b));
    return p;
  }
  void dev_free(void* p) { hipFree(p); }
  Event event_create() {
    Event e;
    HIPCK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }
  void event_destroy(Event e) { hipEventDestroy(e); }
  void event_record(Event e) { HIPCK(hipEventRecord(e, stream)); }
  void event_sync(Event e) { HIPCK(hipEventSynchronize(e)); }
  void h2d(void* dst, const void* src, size_t b) { HIPCK(hipMemcpyAsync(dst, src, b, hipMemcpyHostToDevice, stream)); }
  void per_insert(float* sum, float* mn, float* maxp, const int32_t* idx, int n, int P) {
    launch_sumtree_set(sum, mn, maxp, idx, maxp, 0.f, 0.f, 1, n, P, stream);
  }
};

class IngestServer {
 public:
  // rings: int64 [n] ring addresses; states: int32 [n][words] per-actor ingest state (zeroed);
  // dev: [frames, sidx, nidx, act, rew, done, gam, size] device pointers of the replay;
  // per: [sum, min, max_p, P] (P = 0: uniform replay); cursors: [f_next, t_next, size];
  // cfg: [k, nstep, HW, capacity, num_frames, stage_cap, nsets, flush_min, flush_max_us, device, cpu]
  IngestServer(int64_t rings, int64_t n, int64_t states, int64_t words, double gamma, std::vector<int64_t> dev,
               std::vector<int64_t> per, std::vector<int64_t> cursors, std::vector<int64_t> cfg, int64_t learner_stream) {
    if (dev.size() != 8 || per.size() != 4 || cursors.size() != 3 || cfg.size() != 11)
      throw std::runtime_error("IngestServer: argument sizes");
    dqn_ingest::DevPtrs d{reinterpret_cast<uint8_t*>(dev[0]), reinterpret_cast<int32_t*>(dev[1]),
                          reinterpret_cast<int32_t*>(dev[2]), reinterpret_cast<int32_t*>(dev[3]),
                          reinterpret_cast<float*>(dev[4]),   reinterpret_cast<float*>(dev[5]),
                          reinterpret_cast<float*>(dev[6]),   reinterpret_cast<int32_t*>(dev[7]),
                          reinterpret_cast<float*>(per[0]),   reinterpret_cast<float*>(per[1]),
                          reinterpret_cast<float*>(per[2]),   (int)per[3]};
    dqn_ingest::Config c;
    c.k = (int)cfg[0];
    c.nstep = (int)cfg[1];
    c.hw = cfg[2];
    c.capacity = cfg[3];
    c.num_frames = cfg[4];
    c.stage_cap = cfg[5];
    c.nsets = (int)cfg[6];
    c.flush_min = cfg[7];
    c.flush_max_us = cfg[8];
    c.cpu = (int)cfg[10];
    dev_.device = (int)cfg[9];
    dev_.stream = reinterpret_cast<hipStream_t>(learner_stream);
    core_ = std::make_unique<dqn_ingest::IngestCore<HipDev>>(dev_, reinterpret_cast<const int64_t*>(rings), n,
                                                             reinterpret_cast<int32_t*>(states), words, gamma, d,
                                                             cursors[0], cursors[1], cursors[2], c);
  }

  void start() {
    dev_.bind();
    core_->start();
  }
  void stop() { core_->stop(); }

  pybind11::tuple cursors() const {
    int64_t f, t, sz;
    core_->cursors(&f, &t, &sz);
    return pybind11::make_tuple(f, t, sz);
  }

  // (consumed records, env frames, episodes, flushes, replay size, error)
  pybind11::tuple stats() const {
    auto s = core_->stats();
    return pybind11::make_tuple(s.consumed, s.frames, s.episodes, s.flushes, s.size, s.err);
  }

  pybind11::list pop_returns() {
    pybind11::list out;
    for (float r : core_->pop_returns()) out.append(r);
    return out;
  }

 private:
  HipDev dev_;
  std::unique_ptr<dqn_ingest::IngestCore<HipDev>> core_;
};

}  // namespace

void register_ingest_server(pybind11::module_& m) {
  pybind11::class_<IngestServer>(m, "IngestServer", pybind11::module_local())
      .def(pybind11::init<int64_t, int64_t, int64_t, int64_t, double, std::vector<int64_t>, std::vector<int64_t>,
                          std::vector<int64_t>, std::vector<int64_t>, int64_t>())
      .def("start", &IngestServer::start)
      .def("stop", &IngestServer::stop, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("cursors", &IngestServer::cursors)
      .def("stats", &IngestServer::stats)
      .def("pop_returns", &IngestServer::pop_returns);
}
