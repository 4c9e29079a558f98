// Native Ape-X inference service on the GPU: the device-independent core (csrc/host/infer_core.h:
// mailboxes -> pinned batch -> H2D -> the bucket's inference graph -> D2H -> respond; semantics
// and threading documented there) bound to HIP graphs captured once per batch-size bucket by the
// Python side, plus its binding. The same core runs under ThreadSanitizer with a fake device
// (csrc/host/tests/infer_stress.cpp).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "host/infer_core.h"

namespace {

#define HIPCK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)

struct HipInferDev {
  int device = 0;
  hipStream_t st = nullptr;
  std::vector<hipGraphExec_t> execs;     // [bucket]

  void bind() {
    HIPCK(hipSetDevice(device));
    int lo = 0, hi = 0;
    HIPCK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIPCK(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, hi));     // highest priority
  }
  void unbind() {
    if (st) hipStreamDestroy(st);
    st = nullptr;
  }
  void h2d(void* dst, const void* src, size_t b) { HIPCK(hipMemcpyAsync(dst, src, b, hipMemcpyHostToDevice, st)); }
  void launch(int64_t bucket) { HIPCK(hipGraphLaunch(execs[bucket], st)); }
  void d2h(void* dst, const void* src, size_t b) { HIPCK(hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToHost, st)); }
  void sync() { HIPCK(hipStreamSynchronize(st)); }
};

class InferServer {
 public:
  // region: mailbox region (n slots of state_bytes); pin_in [n][state_bytes] pinned host;
  // dev_in [n][state_bytes] device (the graphs' input); dev_out int32 [n] device (their
  // output); pin_out int32 [n] pinned host. gap_us: pause after a served batch.
  InferServer(int64_t region, int64_t n, int64_t state_bytes, int64_t pin_in, int64_t dev_in, int64_t dev_out,
              int64_t pin_out, int64_t device, int64_t gap_us) {
    dev_.device = (int)device;
    dev_.execs.assign(n + 1, nullptr);
    core_ = std::make_unique<dqn_infer::InferCore<HipInferDev>>(
        dev_, reinterpret_cast<uint8_t*>(region), n, state_bytes, reinterpret_cast<uint8_t*>(pin_in),
        reinterpret_cast<void*>(dev_in), reinterpret_cast<void*>(dev_out), reinterpret_cast<int32_t*>(pin_out), gap_us);
  }

  // graph for batches of up to m rows
  void set_graph(int64_t m, int64_t exec) {
    core_->set_bucket(m);
    dev_.execs[m] = reinterpret_cast<hipGraphExec_t>(exec);
  }
  void set_cpu(int64_t cpu) { core_->set_cpu((int)cpu); }
  void start() { core_->start(); }
  void stop() { core_->stop(); }

  pybind11::tuple stats() const {
    auto s = core_->stats();
    return pybind11::make_tuple(s.served, s.calls, s.err);
  }

 private:
  HipInferDev dev_;
  std::unique_ptr<dqn_infer::InferCore<HipInferDev>> core_;
};

}  // namespace

void register_infer_server(pybind11::module_& m) {
  // module_local: every extension variant (_C, _C_f16, _C_f32) registers its own copy and one
  // process may load several of them
  pybind11::class_<InferServer>(m, "InferServer", pybind11::module_local())
      .def(pybind11::init<int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t>())
      .def("set_graph", &InferServer::set_graph)
      .def("set_cpu", &InferServer::set_cpu)
      .def("start", &InferServer::start)
      .def("stop", &InferServer::stop, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("stats", &InferServer::stats);
}
