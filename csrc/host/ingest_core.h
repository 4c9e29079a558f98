// Ape-X ingest service core: the thread that moves the CPU actors' transition records from
// their SPSC rings (spsc_ring.cpp) into the replay, independent of the device runtime so the
// same code runs under ThreadSanitizer on the host (csrc/host/tests/ingest_stress.cpp, a fake
// device whose "stream" is a worker thread) and on the GPU (csrc/ingest_server.cpp, HIP).
//
// Per staging set (pinned host memory, several in rotation):
//   dqn_apex_ingest per actor ring (frames, frame-slot stacks, n-step fold: apex_ingest.cpp)
//   -> on flush: the H2D copies of the frame range and the transition columns (wrap-split), the
//      PER insert at max priority and the new size into the device size word, all submitted ON
//      THE LEARNER STREAM: in stream order with every learner graph, so no learner launch can
//      sample a half-overwritten slot or race the sum-tree insert (a side stream ordered by
//      events is not enough: launches the learner thread submits between the two events would
//      run beside the copies).
// A staging set is refilled only after its copies completed (its event). Semantics match
// DeviceReplay.ingest_rings + flush (replay/device.py), which the Python path keeps.
//
// Threads: start() spawns the ingest thread; stats() / pop_returns() may be called from any
// thread while it runs (atomics / a mutex); stop() joins it after a final drain + flush; the
// replay cursors are handed back (cursors()) only after stop().
//
// Dev (the device runtime) provides:
//   void bind();                                   (ingest thread start: select the device)
//   void* host_alloc(size_t); void host_free(void*);       pinned host memory
//   void* dev_alloc(size_t);  void dev_free(void*);
//   using Event; Event event_create(); void event_destroy(Event);
//   void event_record(Event); void event_sync(Event);       on / for the learner stream
//   void h2d(void* dst, const void* src, size_t bytes);     async, learner-stream ordered
//   void per_insert(float* sum, float* mn, float* maxp, const int32_t* idx_dev, int n, int P);
#pragma once
#include <sched.h>
#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../include/dqn_host.h"

namespace dqn_ingest {

struct Config {
  int k = 4, nstep = 1;
  int64_t hw = 0, capacity = 0, num_frames = 0, stage_cap = 1024;
  int nsets = 6;
  int64_t flush_min = 256, flush_max_us = 5000;
  int cpu = -1;                      // pin the ingest thread (-1: no pinning)
};

struct DevPtrs {                     // the replay's device columns
  uint8_t* frames;
  int32_t *sidx, *nidx, *act;
  float *rew, *done, *gam;
  int32_t* size;
  float *sum = nullptr, *mn = nullptr, *maxp = nullptr;   // PER sum-tree (P = 0: uniform)
  int P = 0;
};

template <class Dev>
class IngestCore {
 public:
  using Event = typename Dev::Event;

  // rings: n ring base addresses; states: [n][words] per-actor ingest state (zeroed);
  // cursors: the replay's host cursors [f_next, t_next, size] at hand-over
  IngestCore(Dev& dev, const int64_t* rings, int64_t n, int32_t* states, int64_t words, double gamma,
             const DevPtrs& d, int64_t f_next, int64_t t_next, int64_t size, const Config& cfg)
      : dev_(dev), rings_(rings), n_(n), states_(states), words_(words), gamma_(gamma), d_(d), cfg_(cfg),
        f_next_(f_next), t_next_(t_next), size_(size) {
    if (cfg.k < 1 || cfg.nstep < 1 || cfg.hw < 1 || cfg.capacity < 1 || cfg.num_frames < 1 ||
        cfg.stage_cap < cfg.nstep + 1 || cfg.nsets < 2 || n < 1)
      throw std::runtime_error("IngestServer: bad configuration");
    frames_cap_ = 2 * cfg.stage_cap + cfg.k + 8;    // every record writes one frame, a reset one more
    size_pub_.store(size_);
  }

  ~IngestCore() {
    try {
      stop();
    } catch (...) {
    }
    free_sets();
  }

  IngestCore(const IngestCore&) = delete;
  IngestCore& operator=(const IngestCore&) = delete;

  void start() {
    if (running_) return;
    alloc_sets();
    stop_.store(false);
    running_ = true;
    th_ = std::thread([this] { run(); });
  }

  // stops the thread after a final drain + flush
  void stop() {
    if (running_) {
      stop_.store(true);
      th_.join();
      running_ = false;
    }
  }

  bool running() const { return running_; }

  // the replay cursors [f_next, t_next, size]: hand-back to DeviceReplay after stop()
  void cursors(int64_t* f_next, int64_t* t_next, int64_t* size) const {
    if (running_) throw std::runtime_error("IngestServer.cursors() while running");
    *f_next = f_next_;
    *t_next = t_next_;
    *size = size_;
  }

  struct Stats {
    int64_t consumed, frames, episodes, flushes, size;
    std::string err;
  };
  Stats stats() const {
    Stats s{consumed_.load(), frames_.load(), episodes_.load(), flushes_.load(), size_pub_.load(), {}};
    std::lock_guard<std::mutex> g(err_mu_);
    s.err = err_;
    return s;
  }

  // episode returns ended since the last call
  std::vector<float> pop_returns() {
    std::lock_guard<std::mutex> g(ret_mu_);
    std::vector<float> out;
    out.swap(returns_);
    return out;
  }

 private:
  struct StageSet {
    uint8_t* frames = nullptr;       // pinned [frames_cap][HW]
    int32_t* sidx = nullptr;         // pinned [cap][k]
    int32_t* cols = nullptr;         // pinned: nidx [cap] | act [cap] | rew [cap] | done [cap] | gam [cap] | size
    int32_t* pidx = nullptr;         // pinned [cap]: PER leaf indices
    int32_t* pidx_dev = nullptr;     // device [cap]
    Event done{};
    bool has_event = false;
    bool busy = false;
    int64_t nf = 0, nt = 0;
    int64_t f_first = 0;             // replay frame slot of staged frame 0
  };

  void alloc_sets() {
    if (!sets_.empty()) return;
    const int64_t C = cfg_.stage_cap;
    sets_.resize(cfg_.nsets);
    for (auto& s : sets_) {
      s.frames = static_cast<uint8_t*>(dev_.host_alloc((size_t)(frames_cap_ * cfg_.hw)));
      s.sidx = static_cast<int32_t*>(dev_.host_alloc(sizeof(int32_t) * (size_t)(C * cfg_.k)));
      s.cols = static_cast<int32_t*>(dev_.host_alloc(sizeof(int32_t) * (size_t)(5 * C + 1)));
      s.pidx = static_cast<int32_t*>(dev_.host_alloc(sizeof(int32_t) * (size_t)C));
      s.pidx_dev = static_cast<int32_t*>(dev_.dev_alloc(sizeof(int32_t) * (size_t)C));
      s.done = dev_.event_create();
      s.has_event = true;
    }
  }

  void free_sets() {
    for (auto& s : sets_) {
      if (s.has_event && s.busy) dev_.event_sync(s.done);
      if (s.frames) dev_.host_free(s.frames);
      if (s.sidx) dev_.host_free(s.sidx);
      if (s.cols) dev_.host_free(s.cols);
      if (s.pidx) dev_.host_free(s.pidx);
      if (s.pidx_dev) dev_.dev_free(s.pidx_dev);
      if (s.has_event) dev_.event_destroy(s.done);
    }
    sets_.clear();
  }

  StageSet& acquire(int i) {         // wait until set i's previous copies completed
    StageSet& s = sets_[i];
    if (s.busy) {
      dev_.event_sync(s.done);
      s.busy = false;
    }
    s.nf = s.nt = 0;
    s.f_first = f_next_;
    return s;
  }

  template <typename T>
  void ring_copy(T* dst, int64_t cap, int64_t first, const T* src, int64_t n, int64_t row) {
    const int64_t end = first + n;
    if (end <= cap) {
      dev_.h2d(dst + first * row, src, sizeof(T) * (size_t)(n * row));
    } else {
      const int64_t a = cap - first;
      dev_.h2d(dst + first * row, src, sizeof(T) * (size_t)(a * row));
      dev_.h2d(dst, src + a * row, sizeof(T) * (size_t)((n - a) * row));
    }
  }

  void flush(StageSet& s) {
    if (s.nf == 0 && s.nt == 0) return;
    const int64_t C = cfg_.stage_cap, cap = cfg_.capacity;
    if (s.nf) ring_copy(d_.frames, cfg_.num_frames, s.f_first, s.frames, s.nf, cfg_.hw);
    const int64_t n = s.nt;
    if (n) {
      const int64_t first = t_next_;
      ring_copy(d_.sidx, cap, first, s.sidx, n, (int64_t)cfg_.k);
      ring_copy(d_.nidx, cap, first, s.cols, n, 1);
      ring_copy(d_.act, cap, first, s.cols + C, n, 1);
      ring_copy(d_.rew, cap, first, reinterpret_cast<const float*>(s.cols + 2 * C), n, 1);
      ring_copy(d_.done, cap, first, reinterpret_cast<const float*>(s.cols + 3 * C), n, 1);
      ring_copy(d_.gam, cap, first, reinterpret_cast<const float*>(s.cols + 4 * C), n, 1);
      t_next_ = (first + n) % cap;
      size_ = std::min(cap, size_ + n);
      if (d_.P > 0) {                                    // new transitions enter at max priority
        for (int64_t i = 0; i < n; ++i) s.pidx[i] = (int32_t)((first + i) % cap);
        dev_.h2d(s.pidx_dev, s.pidx, sizeof(int32_t) * (size_t)n);
        dev_.per_insert(d_.sum, d_.mn, d_.maxp, s.pidx_dev, (int)n, d_.P);
      }
      int32_t* sw = s.cols + 5 * C;
      *sw = (int32_t)size_;
      dev_.h2d(d_.size, sw, sizeof(int32_t));
    }
    dev_.event_record(s.done);                         // (the staging set is reusable after it)
    s.busy = true;
    size_pub_.store(size_, std::memory_order_relaxed);
    flushes_ += 1;
  }

  void run() {
    try {
      dev_.bind();
      if (cfg_.cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cfg_.cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);   // (best effort)
      }
      const int64_t C = cfg_.stage_cap;
      int cur = 0;
      StageSet* s = &acquire(cur);
      int64_t first_actor = 0;
      auto last_flush = std::chrono::steady_clock::now();
      std::vector<float> rets(1024);
      bool final_pass = false;
      for (;;) {
        if (stop_.load(std::memory_order_relaxed)) final_pass = true;   // drain what is there, once
        int64_t consumed = 0;
        bool full = false;
        for (int64_t j = 0; j < n_; ++j) {
          const int64_t a = (first_actor + j) % n_;
          DqnIngestStage st{s->frames, frames_cap_, s->nf, s->sidx, s->cols, s->cols + C,
                            reinterpret_cast<float*>(s->cols + 2 * C), reinterpret_cast<float*>(s->cols + 3 * C),
                            reinterpret_cast<float*>(s->cols + 4 * C), C, s->nt, f_next_, cfg_.num_frames};
          DqnIngestOut out{};
          dqn_apex_ingest(reinterpret_cast<uint8_t*>(rings_[a]), -1, states_ + a * words_, cfg_.k, cfg_.nstep,
                          gamma_, cfg_.hw, &st, rets.data(), (int64_t)rets.size(), &out);
          s->nf = st.nf;
          s->nt = st.nt;
          f_next_ = st.f_next;
          consumed += out.consumed;
          frames_ += out.frames;
          episodes_ += out.episodes;
          if (out.n_returns > 0) {
            std::lock_guard<std::mutex> g(ret_mu_);
            for (int64_t i = 0; i < out.n_returns; ++i) returns_.push_back(rets[i]);
            if (returns_.size() > 4096) returns_.erase(returns_.begin(), returns_.end() - 4096);
          }
          if (out.stage_full) {
            full = true;
            first_actor = a;                 // resume with this actor after the flush
            break;
          }
        }
        consumed_ += consumed;
        const auto now = std::chrono::steady_clock::now();
        const int64_t waited = std::chrono::duration_cast<std::chrono::microseconds>(now - last_flush).count();
        if (full || s->nt >= cfg_.flush_min || (s->nt > 0 && waited >= cfg_.flush_max_us) ||
            (final_pass && s->nt + s->nf)) {
          flush(*s);
          last_flush = now;
          cur = (cur + 1) % cfg_.nsets;
          s = &acquire(cur);
        }
        if (!full) first_actor = (first_actor + 1) % n_;
        if (final_pass && !full) break;
        if (consumed == 0 && !full) std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
      for (auto& t : sets_)
        if (t.busy) {
          dev_.event_sync(t.done);
          t.busy = false;
        }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(err_mu_);
      err_ = e.what();
    }
  }

  Dev& dev_;
  const int64_t* rings_;
  int64_t n_;
  int32_t* states_;
  int64_t words_;
  double gamma_;
  DevPtrs d_;
  Config cfg_;
  int64_t f_next_, t_next_, size_;   // ingest thread only while running
  int64_t frames_cap_ = 0;
  std::vector<StageSet> sets_;
  std::thread th_;
  std::atomic<bool> stop_{false};
  bool running_ = false;             // owner thread only
  std::atomic<int64_t> consumed_{0}, frames_{0}, episodes_{0}, flushes_{0}, size_pub_{0};
  mutable std::mutex err_mu_;
  std::mutex ret_mu_;
  std::vector<float> returns_;
  std::string err_;
};

}  // namespace dqn_ingest
