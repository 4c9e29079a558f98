// Stress test of the Ape-X inference service's threading (csrc/host/infer_core.h), built with
// -fsanitize=thread by tests/test_apex.py: the InferCore the GPU binding runs
// (csrc/infer_server.cpp) on a fake device whose stream is a worker thread (H2D copy, a "graph"
// computing action = state[0] + 1 for the bucket's rows, D2H copy, completed late and in order).
// Actor threads post requests through the mailboxes and check every answer; the owner thread
// polls stats() while it runs; stop(). Exits non-zero on a wrong / missing answer; TSAN reports
// any data race.
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../infer_core.h"

namespace {

struct FakeInferDev {
  int64_t sb = 0;                       // state bytes
  uint8_t* dev_in = nullptr;
  int32_t* dev_out = nullptr;
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<std::function<void()>> q;
  uint64_t submitted = 0, completed = 0;
  bool quit = false;
  std::thread worker;

  FakeInferDev() {
    worker = std::thread([this] {
      std::mt19937 rng(3);
      for (;;) {
        std::function<void()> op;
        {
          std::unique_lock<std::mutex> g(mu);
          cv_work.wait(g, [&] { return quit || !q.empty(); });
          if (q.empty()) return;
          op = std::move(q.front());
          q.pop_front();
        }
        if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 100));
        op();
        {
          std::lock_guard<std::mutex> g(mu);
          completed += 1;
        }
        cv_done.notify_all();
      }
    });
  }
  ~FakeInferDev() {
    {
      std::lock_guard<std::mutex> g(mu);
      quit = true;
    }
    cv_work.notify_all();
    worker.join();
  }
  void push(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu);
      q.push_back(std::move(f));
      submitted += 1;
    }
    cv_work.notify_one();
  }
  void bind() {}
  void unbind() {}
  void h2d(void* dst, const void* src, size_t b) { push([=] { std::memcpy(dst, src, b); }); }
  void d2h(void* dst, const void* src, size_t b) { push([=] { std::memcpy(dst, src, b); }); }
  void launch(int64_t bucket) {
    push([=] {
      for (int64_t i = 0; i < bucket; ++i) dev_out[i] = (int32_t)dev_in[i * sb] + 1;
    });
  }
  void sync() {
    std::unique_lock<std::mutex> g(mu);
    const uint64_t want = submitted;
    cv_done.wait(g, [&] { return completed >= want; });
  }
};

}  // namespace

int main() {
  const int64_t n = 6, sb = 32, rounds = 2000;
  std::vector<uint8_t> region(dqn_mbox_region_bytes(n, sb));
  dqn_mbox_init(region.data(), n, sb);
  std::vector<uint8_t> pin_in(n * sb), dev_in(n * sb);
  std::vector<int32_t> dev_out(n), pin_out(n);
  int bad = 0;
  int64_t polled = 0;
  {
    FakeInferDev dev;
    dev.sb = sb;
    dev.dev_in = dev_in.data();
    dev.dev_out = dev_out.data();
    dqn_infer::InferCore<FakeInferDev> core(dev, region.data(), n, sb, pin_in.data(), dev_in.data(), dev_out.data(),
                                            pin_out.data(), 0);
    for (int64_t m : {1, 2, 4, 6}) core.set_bucket(m);
    core.start();
    std::vector<std::thread> actors;
    std::vector<int> errs(n, 0);
    for (int64_t a = 0; a < n; ++a) {
      actors.emplace_back([&, a] {
        uint8_t st[32];
        for (int64_t r = 0; r < rounds; ++r) {
          std::memset(st, (int)((a * 11 + r) % 200), sb);
          const int64_t act = dqn_mbox_request(region.data(), a, sb, st, -1);
          if (act != (int64_t)((a * 11 + r) % 200) + 1) ++errs[a];
        }
      });
    }
    for (;;) {                                      // the owner thread polls the counters
      auto s = core.stats();
      polled = s.served;
      if (!s.err.empty()) {
        std::printf("serve error: %s\n", s.err.c_str());
        bad++;
        break;
      }
      if (s.served >= n * rounds) break;
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    for (auto& t : actors) t.join();
    dqn_mbox_set_stop(region.data(), 1);
    core.stop();
    for (int e : errs) bad += e;
    auto s = core.stats();
    if (s.served != n * rounds) {
      std::printf("served %lld of %lld\n", (long long)s.served, (long long)(n * rounds));
      bad++;
    }
    polled = s.served;
  }
  std::printf("infer served %lld, errors %d\n", (long long)polled, bad);
  return bad ? 1 : 0;
}
