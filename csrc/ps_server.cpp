// Native server thread of the asynchronous parameter server over xGMI (parallel/async_ps.py
// XgmiPSServer, the reference's default training mode: every worker's gradient is applied to
// the PS-held variables as it arrives, /root/reference/src/network.py:184-202, src/main.py:105-129).
//
// The thread polls the workers' push words in the host-shared control page (written by the
// workers' GPUs with system-scope release stores) and answers each push, in arrival order, by
// launching that worker's captured HIP graph on the PS stream: the fused optimizer reading the
// worker's gradient slot in place, then the snapshot + step copy and the done word (echoing the
// push number; async_ps.hip ps_publish_kernel). No Python and no GIL in the loop, no host sync
// per update. A stop request answers each worker's next push with the STOP status instead.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <thread>
#include <immintrin.h>
#include <sched.h>
#include <vector>

namespace {

#define HIPCK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)

constexpr uint64_t kBye = 15;                // push kind: the worker leaves (async_ps.py _BYE)

class PsServer {
 public:
  // ctl: host address of the control page; stride: bytes per worker (push word at 0); workers
  // 1..nworkers; stream: the PS stream (hipStream_t) the graphs replay on
  PsServer(int64_t ctl, int64_t nworkers, int64_t stride, int64_t stream, int64_t device)
      : ctl_(reinterpret_cast<const uint8_t*>(ctl)), nw_((int)nworkers), stride_(stride),
        stream_(reinterpret_cast<hipStream_t>(stream)), device_((int)device),
        apply_(nworkers + 1, nullptr), stop_g_(nworkers + 1, nullptr), per_(nworkers + 1, 0) {
    if (ctl == 0 || nworkers < 1 || stride < 64) throw std::runtime_error("PsServer: arguments");
  }

  ~PsServer() {
    try {
      wait();
    } catch (...) {
    }
  }

  void set_graphs(int64_t w, int64_t apply_exec, int64_t stop_exec) {
    if (w < 1 || w > nw_ || running_) throw std::runtime_error("PsServer.set_graphs: worker / running");
    apply_[w] = reinterpret_cast<hipGraphExec_t>(apply_exec);
    stop_g_[w] = reinterpret_cast<hipGraphExec_t>(stop_exec);
  }

  // seen: the push number already answered per worker (1 = the initial pull)
  void start(int64_t max_updates, int64_t seen) {
    if (running_) return;
    for (int w = 1; w <= nw_; ++w)
      if (apply_[w] == nullptr || stop_g_[w] == nullptr) throw std::runtime_error("PsServer: graphs missing");
    max_updates_ = max_updates;
    seen0_ = (uint64_t)seen;
    stop_ = false;
    running_ = true;
    th_ = std::thread([this] { run(); });
  }

  void request_stop() { stop_.store(true, std::memory_order_relaxed); }

  // Quiesce for a consistent host-side read of the PS state (a checkpoint snapshot): the thread
  // stops launching at the top of its loop, drains the PS stream and acknowledges; pushes that
  // arrive meanwhile stay in their push words and are answered after resume(). Returns once
  // paused (or once the thread has exited). Called with the GIL released.
  void pause() {
    pause_req_.store(true, std::memory_order_release);
    while (running_ && !done_.load() && !paused_.load(std::memory_order_acquire))
      std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  // returns once the thread has left its pause (or exited): a pause() right after this cannot see
  // the previous pause's stale paused_ == true and return while the thread goes on launching
  void resume() {
    pause_req_.store(false, std::memory_order_release);
    while (running_ && !done_.load() && paused_.load(std::memory_order_acquire))
      std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  int64_t pauses() const { return pauses_.load(); }

  // join (GIL released by the binding); returns the number of applied pushes
  int64_t wait() {
    if (running_) {
      th_.join();
      running_ = false;
      if (!err_.empty()) throw std::runtime_error("PsServer: " + err_);
    }
    return updates_.load();
  }

  int64_t updates() const { return updates_.load(std::memory_order_relaxed); }
  bool running() const { return running_ && !done_.load(); }

  // (updates, per-worker updates [index = worker], stopped workers, busy seconds); after wait()
  pybind11::tuple stats() const {
    if (running_) throw std::runtime_error("PsServer.stats() before wait()");
    std::vector<int64_t> per(per_.begin(), per_.end());
    return pybind11::make_tuple(updates_.load(), per, (int64_t)stopped_workers_, busy_s_);
  }
  // seconds since serving started at every kMarkEvery-th launched update (steady-state rate windows);
  // after wait()
  std::vector<double> marks() const {
    if (running_) throw std::runtime_error("PsServer.marks() before wait()");
    return marks_;
  }
  static constexpr int kMarkEvery = 64;

 private:
  uint64_t push_word(int w) const {
    return __atomic_load_n(reinterpret_cast<const uint64_t*>(ctl_ + (int64_t)w * stride_), __ATOMIC_ACQUIRE);
  }

  void run() {
    try {
      HIPCK(hipSetDevice(device_));
      std::vector<uint64_t> seen(nw_ + 1, seen0_);
      std::vector<char> active(nw_ + 1, 1);
      int nactive = nw_;
      const auto t0 = std::chrono::steady_clock::now();
      uint32_t idle = 0;
      while (nactive > 0 && !(max_updates_ > 0 && updates_.load() >= max_updates_)) {
        if (pause_req_.load(std::memory_order_acquire)) {
          HIPCK(hipStreamSynchronize(stream_));            // every launched update has landed
          paused_.store(true, std::memory_order_release);
          pauses_.fetch_add(1);
          while (pause_req_.load(std::memory_order_acquire))
            std::this_thread::sleep_for(std::chrono::microseconds(20));
          paused_.store(false, std::memory_order_release);
        }
        bool got = false;
        for (int w = 1; w <= nw_; ++w) {
          if (!active[w]) continue;
          const uint64_t v = push_word(w);
          const uint64_t s = v >> 4, kind = v & 15;
          if (s <= seen[w]) continue;
          got = true;
          seen[w] = s;
          if (kind == kBye) {
            active[w] = 0;
            --nactive;
            continue;
          }
          if (stop_.load(std::memory_order_relaxed)) {
            HIPCK(hipGraphLaunch(stop_g_[w], stream_));
            active[w] = 0;
            --nactive;
            ++stopped_workers_;
            continue;
          }
          HIPCK(hipGraphLaunch(apply_[w], stream_));       // arrival order: one stream
          per_[w] += 1;
          if ((updates_.fetch_add(1, std::memory_order_relaxed) + 1) % kMarkEvery == 0)
            marks_.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        // idle: spin (a 2 us sleep_for slept ~60 us under the kernel's timer slack -- a push then waited
        // that long to be seen); a yield every 256 empty polls keeps the core shareable
        if (!got) {
          _mm_pause();
          if ((++idle & 255) == 0) sched_yield();
        } else {
          idle = 0;
        }
      }
      HIPCK(hipStreamSynchronize(stream_));
      busy_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } catch (const std::exception& e) {
      err_ = e.what();
    }
    done_ = true;
  }

  const uint8_t* ctl_;
  int nw_;
  int64_t stride_;
  hipStream_t stream_;
  int device_;
  std::vector<hipGraphExec_t> apply_, stop_g_;
  std::vector<int64_t> per_;
  int64_t max_updates_ = 0;
  uint64_t seen0_ = 1;
  int stopped_workers_ = 0;
  double busy_s_ = 0.0;
  std::vector<double> marks_;
  std::atomic<int64_t> updates_{0};
  std::atomic<bool> stop_{false}, done_{false}, pause_req_{false}, paused_{false};
  std::atomic<int64_t> pauses_{0};
  bool running_ = false;
  std::thread th_;
  std::string err_;
};

}  // namespace

void register_ps_server(pybind11::module_& m) {
  pybind11::class_<PsServer>(m, "PsServer", pybind11::module_local())
      .def(pybind11::init<int64_t, int64_t, int64_t, int64_t, int64_t>())
      .def("set_graphs", &PsServer::set_graphs)
      .def("start", &PsServer::start)
      .def("request_stop", &PsServer::request_stop)
      .def("pause", &PsServer::pause, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("resume", &PsServer::resume)
      .def("pauses", &PsServer::pauses)
      .def("wait", &PsServer::wait, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("updates", &PsServer::updates)
      .def("running", &PsServer::running)
      .def("stats", &PsServer::stats)
      .def("marks", &PsServer::marks);
}
