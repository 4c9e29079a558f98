// Stress test of the host runtime's cross-thread protocols, built with
// -fsanitize=thread by tests/test_apex.py: one producer and one
// consumer hammer an SPSC ring; actor threads and a server thread exchange
// requests through the mailbox region. Exits non-zero on any lost, duplicated
// or reordered record / mismatched action; TSAN reports any data race.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/dqn_host.h"

static int ring_test() {
  const uint64_t cap = 64, rec = 24, N = 200000;
  std::vector<uint8_t> buf(dqn_ring_bytes(cap, rec));
  dqn_ring_init(buf.data(), cap, rec);
  int bad = 0;
  std::thread prod([&] {
    uint8_t r[24];
    for (uint64_t i = 0; i < N;) {
      std::memcpy(r, &i, 8);
      std::memset(r + 8, (int)(i & 0xff), 16);
      if (dqn_ring_push(buf.data(), r, 1) == 1) ++i; else std::this_thread::yield();
    }
  });
  std::thread cons([&] {
    uint8_t out[24 * 16];
    for (uint64_t want = 0; want < N;) {
      const int64_t m = dqn_ring_pop(buf.data(), out, 16);
      for (int64_t j = 0; j < m; ++j, ++want) {
        uint64_t got;
        std::memcpy(&got, out + j * 24, 8);
        if (got != want || out[j * 24 + 8 + 15] != (uint8_t)(want & 0xff)) ++bad;
      }
      if (m == 0) std::this_thread::yield();
    }
  });
  prod.join();
  cons.join();
  return bad;
}

static int mailbox_test() {
  const int64_t n = 4, sb = 32, rounds = 3000;
  std::vector<uint8_t> region(dqn_mbox_region_bytes(n, sb));
  dqn_mbox_init(region.data(), n, sb);
  int bad = 0;
  std::vector<std::thread> actors;
  std::vector<int> errs(n, 0);
  for (int64_t a = 0; a < n; ++a) {
    actors.emplace_back([&, a] {
      uint8_t st[32];
      for (int64_t r = 0; r < rounds; ++r) {
        std::memset(st, (int)((a * 7 + r) & 0xff), sb);
        const int64_t act = dqn_mbox_request(region.data(), a, sb, st, -1);
        if (act != (int64_t)((a * 7 + r) & 0xff) + 1) ++errs[a];   // server echoes state[0] + 1
      }
    });
  }
  std::thread server([&] {
    std::vector<uint8_t> states(n * sb);
    std::vector<int32_t> ids(n), acts(n);
    std::vector<uint64_t> seq(n);
    int64_t served = 0;
    while (served < n * rounds) {
      const int64_t m = dqn_mbox_collect(region.data(), n, sb, states.data(), ids.data(), seq.data(), n);
      for (int64_t j = 0; j < m; ++j) {
        for (int64_t b = 1; b < sb; ++b)
          if (states[j * sb + b] != states[j * sb]) ++bad;              // torn state
        acts[j] = states[j * sb] + 1;
      }
      dqn_mbox_respond(region.data(), sb, ids.data(), seq.data(), acts.data(), m);
      served += m;
      if (m == 0) std::this_thread::yield();
    }
  });
  for (auto& t : actors) t.join();
  server.join();
  for (int e : errs) bad += e;
  return bad;
}

int main() {
  const int r = ring_test(), m = mailbox_test();
  std::printf("ring errors %d, mailbox errors %d\n", r, m);
  return (r || m) ? 1 : 0;
}
