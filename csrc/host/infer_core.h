// Ape-X inference service core: the thread that answers the CPU actors' mailboxes
// (mailbox.cpp) with the greedy actions of a batch-size-bucketed inference graph. Per batch:
// collect into pinned memory, one H2D copy, the bucket's graph, one D2H copy, a stream sync,
// respond. Device-independent so it runs under ThreadSanitizer with a fake device
// (csrc/host/tests/infer_stress.cpp) and on the GPU (csrc/infer_server.cpp, HIP graphs).
// The reference answers each actor with a batch-1 session.run against the PS parameters
// (/root/reference/src/dqn_agent.py:155-189).
//
// Threads: start() spawns the serving thread; stats() may be called from any thread while it
// runs; stop() joins it.
//
// Dev provides:
//   void bind();                    (serving thread start: device + its own stream)
//   void unbind();                  (serving thread end)
//   void h2d(void* dst, const void* src, size_t bytes);
//   void launch(int64_t bucket);    (the bucket's graph: dev_in -> dev_out)
//   void d2h(void* dst, const void* src, size_t bytes);
//   void sync();
#pragma once
#include <pthread.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../include/dqn_host.h"

namespace dqn_infer {

template <class Dev>
class InferCore {
 public:
  // region: mailbox region (n slots of state_bytes); pin_in [n][state_bytes] pinned host;
  // dev_in [n][state_bytes] device (the graphs' input); dev_out int32 [n] device (their output);
  // pin_out int32 [n] pinned host. gap_us: pause after a served batch.
  InferCore(Dev& dev, uint8_t* region, int64_t n, int64_t state_bytes, uint8_t* pin_in, void* dev_in, void* dev_out,
            int32_t* pin_out, int64_t gap_us)
      : dev_(dev), region_(region), n_(n), sb_(state_bytes), pin_in_(pin_in), dev_in_(dev_in), dev_out_(dev_out),
        pin_out_(pin_out), gap_us_(gap_us), has_(n + 1, 0), ids_(n), seq_(n) {}

  ~InferCore() {
    try {
      stop();
    } catch (...) {
    }
  }

  InferCore(const InferCore&) = delete;
  InferCore& operator=(const InferCore&) = delete;

  // a graph serves batches of up to m rows (the next bucket up serves smaller batches: its extra
  // rows hold stale states whose actions are discarded)
  void set_bucket(int64_t m) {
    if (m < 1 || m > n_) throw std::runtime_error("set_graph: bucket size");
    if (running_) throw std::runtime_error("set_graph while running");
    has_[m] = 1;
  }

  void set_cpu(int cpu) { cpu_ = cpu; }

  void start() {
    if (running_) return;
    bucket_.assign(n_ + 1, 0);                      // bucket lookup table: smallest graph >= m
    int64_t next = 0;
    for (int64_t m = n_; m >= 1; --m) {
      if (has_[m]) next = m;
      bucket_[m] = next;
    }
    if (bucket_[n_] == 0) throw std::runtime_error("InferServer: no graph covers the full batch");
    stop_.store(false);
    running_ = true;
    th_ = std::thread([this] { run(); });
  }

  void stop() {
    if (!running_) return;
    stop_.store(true);
    th_.join();
    running_ = false;
  }

  struct Stats {
    int64_t served, calls;
    std::string err;
  };
  Stats stats() const {
    Stats s{served_.load(), calls_.load(), {}};
    std::lock_guard<std::mutex> g(err_mu_);
    s.err = err_;
    return s;
  }

 private:
  void run() {
    try {
      dev_.bind();
      if (cpu_ >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cpu_, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);   // (best effort)
      }
      while (!stop_.load(std::memory_order_relaxed) && !dqn_mbox_stopped(region_)) {
        const int64_t m = dqn_mbox_collect(region_, n_, sb_, pin_in_, ids_.data(), seq_.data(), n_);
        if (m == 0) {
          std::this_thread::sleep_for(std::chrono::microseconds(50));
          continue;
        }
        dev_.h2d(dev_in_, pin_in_, (size_t)(m * sb_));
        dev_.launch(bucket_[m]);
        dev_.d2h(pin_out_, dev_out_, (size_t)m * sizeof(int32_t));
        dev_.sync();
        dqn_mbox_respond(region_, sb_, ids_.data(), seq_.data(), pin_out_, m);
        served_ += m;
        calls_ += 1;
        if (gap_us_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(gap_us_));
      }
      dev_.unbind();
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(err_mu_);
      err_ = e.what();
    }
  }

  Dev& dev_;
  uint8_t* region_;
  int64_t n_, sb_;
  uint8_t* pin_in_;
  void* dev_in_;
  void* dev_out_;
  int32_t* pin_out_;
  int64_t gap_us_;
  int cpu_ = -1;
  std::vector<char> has_;
  std::vector<int64_t> bucket_;
  std::vector<int32_t> ids_;
  std::vector<uint64_t> seq_;
  std::thread th_;
  std::atomic<bool> stop_{false};
  bool running_ = false;             // owner thread only
  std::atomic<int64_t> served_{0}, calls_{0};
  mutable std::mutex err_mu_;
  std::string err_;
};

}  // namespace dqn_infer
