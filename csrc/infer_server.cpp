// Native Ape-X inference service: a C++ thread that answers the CPU actors' mailboxes
// (csrc/host/mailbox.cpp) with HIP graphs captured once per batch-size bucket by the Python
// side (the whole greedy-action forward: states -> Q -> argmax -> int32 actions). Per batch:
// collect into pinned memory, one H2D copy, hipGraphLaunch, one D2H copy, stream sync,
// respond -- no Python and no GIL, so the learner thread keeps the interpreter to itself.
// The reference answers each actor with a batch-1 session.run against the PS parameters
// (/root/reference/src/dqn_agent.py:155-189).
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <pybind11/pybind11.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <thread>
#include <vector>

#include "include/dqn_host.h"

namespace {

#define HIPCK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)

class InferServer {
 public:
  // region: mailbox region (n slots of state_bytes); pin_in [n][state_bytes] pinned host;
  // dev_in [n][state_bytes] device (the graphs' input); dev_out int32 [n] device (their
  // output); pin_out int32 [n] pinned host. gap_us: pause after a served batch.
  InferServer(int64_t region, int64_t n, int64_t state_bytes, int64_t pin_in, int64_t dev_in, int64_t dev_out,
              int64_t pin_out, int64_t device, int64_t gap_us)
      : region_(reinterpret_cast<uint8_t*>(region)), n_(n), sb_(state_bytes),
        pin_in_(reinterpret_cast<uint8_t*>(pin_in)), dev_in_(reinterpret_cast<void*>(dev_in)),
        dev_out_(reinterpret_cast<void*>(dev_out)), pin_out_(reinterpret_cast<int32_t*>(pin_out)),
        device_(static_cast<int>(device)), gap_us_(gap_us), execs_(n + 1, nullptr), ids_(n), seq_(n) {}

  ~InferServer() { stop(); }

  // graph for batches of up to m rows (the next bucket up serves smaller batches: its extra
  // rows hold stale states whose actions are discarded)
  void set_graph(int64_t m, int64_t exec) {
    if (m < 1 || m > n_) throw std::runtime_error("set_graph: bucket size");
    if (running_) throw std::runtime_error("set_graph while running");
    execs_[m] = reinterpret_cast<hipGraphExec_t>(exec);
  }

  // pin the serving thread to one CPU (-1: no pinning); before start()
  void set_cpu(int64_t cpu) { cpu_ = (int)cpu; }

  void start() {
    if (running_) return;
    bucket_.assign(n_ + 1, 0);                      // bucket lookup table: smallest graph >= m
    int64_t next = 0;
    for (int64_t m = n_; m >= 1; --m) {
      if (execs_[m] != nullptr) next = m;
      bucket_[m] = next;
    }
    if (bucket_[n_] == 0) throw std::runtime_error("InferServer: no graph covers the full batch");
    stop_ = false;
    running_ = true;
    th_ = std::thread([this] { run(); });
  }

  void stop() {
    if (!running_) return;
    stop_ = true;
    th_.join();
    running_ = false;
  }

  pybind11::tuple stats() const {
    return pybind11::make_tuple((int64_t)served_.load(), (int64_t)calls_.load(), err_);
  }

 private:
  void run() {
    try {
      HIPCK(hipSetDevice(device_));
      if (cpu_ >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cpu_, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);   // (best effort)
      }
      int lo = 0, hi = 0;
      HIPCK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      hipStream_t st;
      HIPCK(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, hi));   // highest priority
      while (!stop_.load(std::memory_order_relaxed) && !dqn_mbox_stopped(region_)) {
        const int64_t m = dqn_mbox_collect(region_, n_, sb_, pin_in_, ids_.data(), seq_.data(), n_);
        if (m == 0) {
          std::this_thread::sleep_for(std::chrono::microseconds(50));
          continue;
        }
        const int64_t g = bucket_[m];
        HIPCK(hipMemcpyAsync(dev_in_, pin_in_, (size_t)(m * sb_), hipMemcpyHostToDevice, st));
        HIPCK(hipGraphLaunch(execs_[g], st));
        HIPCK(hipMemcpyAsync(pin_out_, dev_out_, (size_t)m * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        dqn_mbox_respond(region_, sb_, ids_.data(), seq_.data(), pin_out_, m);
        served_ += m;
        calls_ += 1;
        if (gap_us_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(gap_us_));
      }
      hipStreamDestroy(st);
    } catch (const std::exception& e) {
      err_ = e.what();
    }
  }

  uint8_t* region_;
  int64_t n_, sb_;
  uint8_t* pin_in_;
  void* dev_in_;
  void* dev_out_;
  int32_t* pin_out_;
  int device_;
  int cpu_ = -1;
  int64_t gap_us_;
  std::vector<hipGraphExec_t> execs_;
  std::vector<int64_t> bucket_;
  std::vector<int32_t> ids_;
  std::vector<uint64_t> seq_;
  std::thread th_;
  std::atomic<bool> stop_{false};
  bool running_ = false;
  std::atomic<int64_t> served_{0}, calls_{0};
  std::string err_;
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
