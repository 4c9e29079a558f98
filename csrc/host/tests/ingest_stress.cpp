// Stress test of the Ape-X ingest service's threading (csrc/host/ingest_core.h), built with
// -fsanitize=thread by tests/test_apex.py: the same IngestCore the GPU binding
// runs (csrc/ingest_server.cpp), on a fake device whose "learner stream" is a worker thread
// executing the queued H2D copies / PER inserts / event markers late and in order.
//
// Covered: actor threads producing into their SPSC rings under back-pressure; the ingest thread
// draining them into rotating staging sets while the stream thread still reads earlier sets
// (a set is refilled only after its event); the owner thread polling stats() / pop_returns()
// during the run; stop() with its final drain + flush; the cursor hand-back after stop().
// Exits non-zero on a lost / duplicated / mismatched transition or cursor; TSAN reports races.
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../ingest_core.h"

namespace {

struct FakeDev {
  using Event = int;
  struct Op {
    int kind;                          // 0 copy, 1 marker, 2 PER insert
    void* dst;
    const void* src;
    size_t bytes;
    uint64_t ticket;
    float* sum;
    const int32_t* idx;
    int n;
  };
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<Op> q;
  uint64_t submitted = 0, completed = 0;
  std::vector<uint64_t> ev_ticket;
  bool quit = false;
  std::thread worker;
  std::atomic<int64_t> copies{0}, inserts{0};

  FakeDev() {
    worker = std::thread([this] { run(); });
  }
  ~FakeDev() {
    {
      std::lock_guard<std::mutex> g(mu);
      quit = true;
    }
    cv_work.notify_all();
    worker.join();
  }
  void run() {
    std::mt19937 rng(7);
    for (;;) {
      Op op;
      {
        std::unique_lock<std::mutex> g(mu);
        cv_work.wait(g, [&] { return quit || !q.empty(); });
        if (q.empty()) return;
        op = q.front();
        q.pop_front();
      }
      if (rng() % 8 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));   // a slow copy
      if (op.kind == 0) {
        std::memcpy(op.dst, op.src, op.bytes);
        copies++;
      } else if (op.kind == 2) {
        for (int i = 0; i < op.n; ++i) op.sum[op.idx[i]] += 1.f;      // "at max priority": count inserts
        inserts += op.n;
      }
      {
        std::lock_guard<std::mutex> g(mu);
        completed = op.ticket;
      }
      cv_done.notify_all();
    }
  }
  void push(Op op) {
    {
      std::lock_guard<std::mutex> g(mu);
      op.ticket = ++submitted;
      q.push_back(op);
    }
    cv_work.notify_one();
  }

  void bind() {}
  void* host_alloc(size_t b) { return std::calloc(1, b); }
  void host_free(void* p) { std::free(p); }
  void* dev_alloc(size_t b) { return std::calloc(1, b); }
  void dev_free(void* p) { std::free(p); }
  Event event_create() {
    std::lock_guard<std::mutex> g(mu);
    ev_ticket.push_back(0);
    return (int)ev_ticket.size() - 1;
  }
  void event_destroy(Event) {}
  void event_record(Event e) {
    std::lock_guard<std::mutex> g(mu);
    Op op{1, nullptr, nullptr, 0, ++submitted, nullptr, nullptr, 0};
    ev_ticket[e] = op.ticket;
    q.push_back(op);
    cv_work.notify_one();
  }
  void event_sync(Event e) {
    std::unique_lock<std::mutex> g(mu);
    const uint64_t t = ev_ticket[e];
    cv_done.wait(g, [&] { return completed >= t; });
  }
  void h2d(void* dst, const void* src, size_t b) { push(Op{0, dst, src, b, 0, nullptr, nullptr, 0}); }
  void per_insert(float* sum, float*, float*, const int32_t* idx, int n, int) {
    push(Op{2, nullptr, nullptr, 0, 0, sum, idx, n});
  }
};

struct Header {                        // actors/apex.py HEADER
  uint8_t kind, done;
  uint16_t pad;
  int32_t action;
  float reward, ret;
};

constexpr int kHW = 16, kK = 4, kN = 3;
constexpr int64_t kRec = sizeof(Header) + kHW;

void stamp(uint8_t* obs, int actor, uint32_t count) {
  std::memset(obs, actor, kHW);
  std::memcpy(obs + 4, &count, 4);
}
int frame_actor(const uint8_t* f) { return f[0]; }
uint32_t frame_count(const uint8_t* f) {
  uint32_t c;
  std::memcpy(&c, f + 4, 4);
  return c;
}

}  // namespace

int main() {
  const int n = 6, episodes = 120;
  // per actor: episodes with 3..40 steps each (fixed seeds: the totals are known in advance)
  std::vector<std::vector<int>> lens(n);
  int64_t steps = 0, resets = 0;
  for (int a = 0; a < n; ++a) {
    std::mt19937 r(100 + a);
    for (int e = 0; e < episodes; ++e) {
      lens[a].push_back(3 + (int)(r() % 38));
      steps += lens[a].back();
      resets += 1;
    }
  }
  const int64_t frames_total = steps + resets;
  std::vector<std::vector<uint8_t>> rings(n);
  std::vector<int64_t> ring_ptrs(n);
  for (int a = 0; a < n; ++a) {
    rings[a].resize(dqn_ring_bytes(64, kRec));                  // small rings: back-pressure
    dqn_ring_init(rings[a].data(), 64, kRec);
    ring_ptrs[a] = (int64_t)rings[a].data();
  }
  const int64_t words = kK + 1 + kN * kK + 2 * kN;
  std::vector<int32_t> states(n * words, 0);
  const int64_t cap = steps + 16, nfr = frames_total + 16;     // no wrap: contents checkable
  std::vector<uint8_t> frames(nfr * kHW);
  std::vector<int32_t> sidx(cap * kK), nidx(cap), act(cap), size_word(1);
  std::vector<float> rew(cap), done(cap), gam(cap), sum(cap, 0.f), mn(1), maxp(1, 1.f);
  dqn_ingest::DevPtrs d{frames.data(), sidx.data(), nidx.data(), act.data(), rew.data(), done.data(), gam.data(),
                        size_word.data(), sum.data(), mn.data(), maxp.data(), (int)cap};
  dqn_ingest::Config cfg;
  cfg.k = kK;
  cfg.nstep = kN;
  cfg.hw = kHW;
  cfg.capacity = cap;
  cfg.num_frames = nfr;
  cfg.stage_cap = 96;                                           // many flushes, full-stage breaks
  cfg.nsets = 3;
  cfg.flush_min = 40;
  cfg.flush_max_us = 300;
  int bad = 0;
  int64_t polled_returns = 0;
  {
    FakeDev dev;
    dqn_ingest::IngestCore<FakeDev> core(dev, ring_ptrs.data(), n, states.data(), words, 0.99, d, 0, 0, 0, cfg);
    core.start();
    std::vector<std::thread> actors;
    for (int a = 0; a < n; ++a) {
      actors.emplace_back([&, a] {
        uint8_t rec[kRec];
        Header h{};
        uint32_t count = 0;
        auto push = [&] {
          std::memcpy(rec, &h, sizeof(h));
          stamp(rec + sizeof(h), a, count++);
          while (dqn_ring_push(rings[a].data(), rec, 1) != 1) std::this_thread::yield();
        };
        for (int len : lens[a]) {
          h = Header{0, 0, 0, 0, 0.f, NAN};
          push();
          for (int t = 0; t < len; ++t) {
            const bool last = t + 1 == len;
            h = Header{1, (uint8_t)last, 0, (int32_t)(count % 5), 1.f, last ? (float)len : NAN};
            push();
          }
        }
      });
    }
    // the owner thread polls the counters while the service runs
    const int64_t records = frames_total;
    for (;;) {
      auto s = core.stats();
      polled_returns += (int64_t)core.pop_returns().size();
      if (!s.err.empty()) {
        std::printf("ingest error: %s\n", s.err.c_str());
        bad++;
        break;
      }
      if (s.consumed >= records) break;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    for (auto& t : actors) t.join();
    core.stop();
    polled_returns += (int64_t)core.pop_returns().size();
    int64_t f, t, sz;
    core.cursors(&f, &t, &sz);
    auto s = core.stats();
    if (f != frames_total || t != steps || sz != steps || s.frames != steps || s.episodes != n * episodes ||
        polled_returns != n * episodes || size_word[0] != steps || dev.inserts.load() != steps) {
      std::printf("cursor mismatch: f %lld/%lld t %lld/%lld size %lld word %d frames %lld episodes %lld returns %lld "
                  "inserts %lld\n",
                  (long long)f, (long long)frames_total, (long long)t, (long long)steps, (long long)sz, size_word[0],
                  (long long)s.frames, (long long)s.episodes, (long long)polled_returns,
                  (long long)dev.inserts.load());
      bad++;
    }
  }
  // contents: every transition's next frame and last stacked frame belong to one actor, in order
  int64_t dones = 0;
  for (int64_t i = 0; i < steps; ++i) {
    const uint8_t* fn = frames.data() + (int64_t)nidx[i] * kHW;
    const uint8_t* fl = frames.data() + (int64_t)sidx[i * kK + kK - 1] * kHW;
    if (frame_actor(fn) != frame_actor(fl) || frame_count(fn) <= frame_count(fl) || sum[i] != 1.f) {
      if (bad < 10)
        std::printf("transition %lld: next (%d,%u) last (%d,%u) inserts %.0f\n", (long long)i, frame_actor(fn),
                    frame_count(fn), frame_actor(fl), frame_count(fl), sum[i]);
      bad++;
    }
    dones += done[i] == 1.f;
  }
  const int64_t want_dones = [&] {     // n-step: the last min(n, len) steps of an episode are done
    int64_t c = 0;
    for (auto& v : lens)
      for (int len : v) c += std::min(len, kN);
    return c;
  }();
  if (dones != want_dones) {
    std::printf("done flags %lld, want %lld\n", (long long)dones, (long long)want_dones);
    bad++;
  }
  std::printf("ingest transitions %lld, frames %lld, errors %d\n", (long long)steps, (long long)frames_total, bad);
  return bad ? 1 : 0;
}
