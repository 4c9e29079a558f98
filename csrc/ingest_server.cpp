// Native Ape-X ingest service: a C++ thread that moves the CPU actors' transition records from
// their SPSC rings (csrc/host/spsc_ring.cpp) into the HBM replay, so the learner's Python thread
// only replays learner graphs. Per staging set (pinned host memory, several in rotation):
//   dqn_apex_ingest per actor ring (frames, frame-slot stacks, n-step fold: apex_ingest.cpp)
//   -> on flush: the H2D copies of the frame range and the transition columns (wrap-split), the
//      PER insert at max priority and the new size into the device size word, all submitted ON
//      THE LEARNER STREAM: in stream order with every learner graph, so no learner launch can
//      sample a half-overwritten slot or race the sum-tree insert (a side stream ordered by
//      events is not enough: launches the learner thread submits between the two events would
//      run beside the copies). Copies from pinned memory are cheap to submit; the learner
//      thread keeps submitting its graphs meanwhile (HIP serialises submissions per stream).
// A staging set is refilled only after its copies completed (its event). Semantics match
// DeviceReplay.ingest_rings + flush (replay/device.py), which the Python path keeps.
// The reference's actor is the worker's own episode loop feeding a Python deque
// (/root/reference/src/dqn_agent.py:72-106, src/replay_memory.py:22-23).
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "include/dqn_host.h"
#include "include/dqn_kernels.h"

namespace {

#define HIPCK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)

struct StageSet {
  uint8_t* frames = nullptr;         // pinned [frames_cap][HW]
  int32_t* sidx = nullptr;           // pinned [cap][k]
  int32_t* cols = nullptr;           // pinned: nidx [cap] | act [cap] | rew [cap] | done [cap] | gam [cap] | size
  int32_t* pidx = nullptr;           // pinned [cap]: PER leaf indices
  int32_t* pidx_dev = nullptr;       // device [cap]
  hipEvent_t done = nullptr;
  bool busy = false;
  int64_t nf = 0, nt = 0;
  int64_t f_first = 0;               // replay frame slot of staged frame 0
};

class IngestServer {
 public:
  // rings: int64 [n] ring addresses; states: int32 [n][words] per-actor ingest state (zeroed);
  // dev: [frames, sidx, nidx, act, rew, done, gam, size] device pointers of the replay;
  // per: [sum, min, max_p, P] (P = 0: uniform replay); cursors: [f_next, t_next, size];
  // cfg: [k, nstep, HW, capacity, num_frames, stage_cap, nsets, flush_min, flush_max_us, device, cpu]
  IngestServer(int64_t rings, int64_t n, int64_t states, int64_t words, double gamma, std::vector<int64_t> dev,
               std::vector<int64_t> per, std::vector<int64_t> cursors, std::vector<int64_t> cfg, int64_t learner_stream)
      : rings_(reinterpret_cast<const int64_t*>(rings)), n_(n), states_(reinterpret_cast<int32_t*>(states)),
        words_(words), gamma_(gamma), learner_(reinterpret_cast<hipStream_t>(learner_stream)) {
    if (dev.size() != 8 || per.size() != 4 || cursors.size() != 3 || cfg.size() != 11)
      throw std::runtime_error("IngestServer: argument sizes");
    frames_d_ = reinterpret_cast<uint8_t*>(dev[0]);
    sidx_d_ = reinterpret_cast<int32_t*>(dev[1]);
    nidx_d_ = reinterpret_cast<int32_t*>(dev[2]);
    act_d_ = reinterpret_cast<int32_t*>(dev[3]);
    rew_d_ = reinterpret_cast<float*>(dev[4]);
    done_d_ = reinterpret_cast<float*>(dev[5]);
    gam_d_ = reinterpret_cast<float*>(dev[6]);
    size_d_ = reinterpret_cast<int32_t*>(dev[7]);
    sum_ = reinterpret_cast<float*>(per[0]);
    mn_ = reinterpret_cast<float*>(per[1]);
    maxp_ = reinterpret_cast<float*>(per[2]);
    P_ = (int)per[3];
    f_next_ = cursors[0];
    t_next_ = cursors[1];
    size_ = cursors[2];
    k_ = (int)cfg[0];
    nstep_ = (int)cfg[1];
    hw_ = cfg[2];
    cap_ = cfg[3];
    num_frames_ = cfg[4];
    stage_cap_ = cfg[5];
    nsets_ = (int)cfg[6];
    flush_min_ = cfg[7];
    flush_max_us_ = cfg[8];
    device_ = (int)cfg[9];
    cpu_ = (int)cfg[10];
    if (k_ < 1 || nstep_ < 1 || hw_ < 1 || cap_ < 1 || stage_cap_ < nstep_ + 1 || nsets_ < 2 || n_ < 1)
      throw std::runtime_error("IngestServer: bad configuration");
    frames_cap_ = 2 * stage_cap_ + k_ + 8;    // every record writes one frame, a reset one more
    size_pub_.store(size_);
  }

  ~IngestServer() {
    try {
      stop();
    } catch (...) {
    }
    free_sets();
  }

  void start() {
    if (running_) return;
    HIPCK(hipSetDevice(device_));
    alloc_sets();
    stop_ = false;
    running_ = true;
    th_ = std::thread([this] { run(); });
  }

  // stops the thread after a final drain + flush (GIL released by the binding)
  void stop() {
    if (running_) {
      stop_ = true;
      th_.join();
      running_ = false;
    }
  }

  // the replay cursors [f_next, t_next, size] (hand-back to DeviceReplay after stop())
  pybind11::tuple cursors() const {
    if (running_) throw std::runtime_error("IngestServer.cursors() while running");
    return pybind11::make_tuple(f_next_, t_next_, size_);
  }

  // (consumed records, env frames, episodes, flushes, replay size, error)
  pybind11::tuple stats() const {
    return pybind11::make_tuple((int64_t)consumed_.load(), (int64_t)frames_.load(), (int64_t)episodes_.load(),
                                (int64_t)flushes_.load(), (int64_t)size_pub_.load(), err_);
  }

  // episode returns ended since the last call
  pybind11::list pop_returns() {
    std::lock_guard<std::mutex> g(ret_mu_);
    pybind11::list out;
    for (float r : returns_) out.append(r);
    returns_.clear();
    return out;
  }

 private:
  void alloc_sets() {
    if (!sets_.empty()) return;
    sets_.resize(nsets_);
    for (auto& s : sets_) {
      HIPCK(hipHostMalloc(reinterpret_cast<void**>(&s.frames), (size_t)(frames_cap_ * hw_), hipHostMallocDefault));
      HIPCK(hipHostMalloc(reinterpret_cast<void**>(&s.sidx), sizeof(int32_t) * (size_t)(stage_cap_ * k_),
                          hipHostMallocDefault));
      HIPCK(hipHostMalloc(reinterpret_cast<void**>(&s.cols), sizeof(int32_t) * (size_t)(5 * stage_cap_ + 1),
                          hipHostMallocDefault));
      HIPCK(hipHostMalloc(reinterpret_cast<void**>(&s.pidx), sizeof(int32_t) * (size_t)stage_cap_,
                          hipHostMallocDefault));
      HIPCK(hipMalloc(reinterpret_cast<void**>(&s.pidx_dev), sizeof(int32_t) * (size_t)stage_cap_));
      HIPCK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    }
  }

  void free_sets() {
    for (auto& s : sets_) {
      if (s.done) hipEventSynchronize(s.done);
      if (s.frames) hipHostFree(s.frames);
      if (s.sidx) hipHostFree(s.sidx);
      if (s.cols) hipHostFree(s.cols);
      if (s.pidx) hipHostFree(s.pidx);
      if (s.pidx_dev) hipFree(s.pidx_dev);
      if (s.done) hipEventDestroy(s.done);
    }
    sets_.clear();
  }

  StageSet& acquire(int i) {         // wait until set i's previous copies completed
    StageSet& s = sets_[i];
    if (s.busy) {
      HIPCK(hipEventSynchronize(s.done));
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
      HIPCK(hipMemcpyAsync(dst + first * row, src, sizeof(T) * (size_t)(n * row), hipMemcpyHostToDevice, learner_));
    } else {
      const int64_t a = cap - first;
      HIPCK(hipMemcpyAsync(dst + first * row, src, sizeof(T) * (size_t)(a * row), hipMemcpyHostToDevice, learner_));
      HIPCK(hipMemcpyAsync(dst, src + a * row, sizeof(T) * (size_t)((n - a) * row), hipMemcpyHostToDevice, learner_));
    }
  }

  void flush(StageSet& s) {
    if (s.nf == 0 && s.nt == 0) return;
    if (s.nf) ring_copy(frames_d_, num_frames_, s.f_first, s.frames, s.nf, hw_);
    const int64_t n = s.nt;
    if (n) {
      const int64_t first = t_next_;
      const int32_t* nidx = s.cols;
      const int32_t* act = s.cols + stage_cap_;
      const float* rew = reinterpret_cast<const float*>(s.cols + 2 * stage_cap_);
      const float* done = reinterpret_cast<const float*>(s.cols + 3 * stage_cap_);
      const float* gam = reinterpret_cast<const float*>(s.cols + 4 * stage_cap_);
      ring_copy(sidx_d_, cap_, first, s.sidx, n, k_);
      ring_copy(nidx_d_, cap_, first, nidx, n, 1);
      ring_copy(act_d_, cap_, first, act, n, 1);
      ring_copy(rew_d_, cap_, first, rew, n, 1);
      ring_copy(done_d_, cap_, first, done, n, 1);
      ring_copy(gam_d_, cap_, first, gam, n, 1);
      t_next_ = (first + n) % cap_;
      size_ = std::min(cap_, size_ + n);
      if (P_ > 0) {                                      // new transitions enter at max priority
        for (int64_t i = 0; i < n; ++i) s.pidx[i] = (int32_t)((first + i) % cap_);
        HIPCK(hipMemcpyAsync(s.pidx_dev, s.pidx, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, learner_));
        launch_sumtree_set(sum_, mn_, maxp_, s.pidx_dev, maxp_, 0.f, 0.f, 1, (int)n, P_, learner_);
      }
      int32_t* sw = s.cols + 5 * stage_cap_;
      *sw = (int32_t)size_;
      HIPCK(hipMemcpyAsync(size_d_, sw, sizeof(int32_t), hipMemcpyHostToDevice, learner_));
    }
    HIPCK(hipEventRecord(s.done, learner_));            // (the staging set is reusable after it)
    s.busy = true;
    size_pub_.store(size_, std::memory_order_relaxed);
    flushes_ += 1;
  }

  void run() {
    try {
      HIPCK(hipSetDevice(device_));
      if (cpu_ >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cpu_, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);   // (best effort)
      }
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
          DqnIngestStage st{s->frames, frames_cap_, s->nf, s->sidx, s->cols, s->cols + stage_cap_,
                            reinterpret_cast<float*>(s->cols + 2 * stage_cap_),
                            reinterpret_cast<float*>(s->cols + 3 * stage_cap_),
                            reinterpret_cast<float*>(s->cols + 4 * stage_cap_), stage_cap_, s->nt, f_next_,
                            num_frames_};
          DqnIngestOut out{};
          dqn_apex_ingest(reinterpret_cast<uint8_t*>(rings_[a]), -1, states_ + a * words_, k_, nstep_, gamma_, hw_,
                          &st, rets.data(), (int64_t)rets.size(), &out);
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
        const int64_t waited =
            std::chrono::duration_cast<std::chrono::microseconds>(now - last_flush).count();
        if (full || s->nt >= flush_min_ || (s->nt > 0 && waited >= flush_max_us_) || (final_pass && s->nt + s->nf)) {
          flush(*s);
          last_flush = now;
          cur = (cur + 1) % nsets_;
          s = &acquire(cur);
        }
        if (!full) first_actor = (first_actor + 1) % n_;
        if (final_pass && !full) break;
        if (consumed == 0 && !full) std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
      for (auto& t : sets_)
        if (t.busy) HIPCK(hipEventSynchronize(t.done));
    } catch (const std::exception& e) {
      err_ = e.what();
    }
  }

  const int64_t* rings_;
  int64_t n_;
  int32_t* states_;
  int64_t words_;
  double gamma_;
  hipStream_t learner_;
  uint8_t* frames_d_;
  int32_t *sidx_d_, *nidx_d_, *act_d_, *size_d_;
  float *rew_d_, *done_d_, *gam_d_;
  float *sum_, *mn_, *maxp_;
  int P_;
  int64_t f_next_, t_next_, size_;
  int k_, nstep_;
  int64_t hw_, cap_, num_frames_, stage_cap_, frames_cap_;
  int nsets_;
  int64_t flush_min_, flush_max_us_;
  int device_, cpu_;
  std::vector<StageSet> sets_;
  std::thread th_;
  std::atomic<bool> stop_{false};
  bool running_ = false;
  std::atomic<int64_t> consumed_{0}, frames_{0}, episodes_{0}, flushes_{0}, size_pub_{0};
  std::mutex ret_mu_;
  std::vector<float> returns_;
  std::string err_;
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
