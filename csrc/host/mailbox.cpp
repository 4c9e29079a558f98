// Actor <-> inference-server mailboxes in shared memory (Ape-X batched inference).
//
// Reference: every actor step runs its own batch-1 `session.run(q_output)`
// against parameters fetched from the PS (/root/reference/src/dqn_agent.py:184-189,
// SURVEY M1). Here CPU actor processes post their state into a mailbox slot and
// the learner process answers ALL pending slots with one batched GPU forward.
//
// Region layout: [0] stop flag (u64) [64..] N slots of `stride` bytes:
//   slot + 0    req  (u64, written by the actor, release)
//   slot + 64   resp (u64, written by the server, release)
//   slot + 128  action (i32) , slot + 132 reserved
//   slot + 192  state bytes
// An actor owns its slot's state/req words; the server owns resp/action.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>

#include "../include/dqn_host.h"

namespace {
constexpr size_t kStop = 0, kSlots = 64, kReq = 0, kResp = 64, kAct = 128, kState = 192;
inline uint64_t* w64(uint8_t* p) { return reinterpret_cast<uint64_t*>(p); }
inline uint8_t* slot(uint8_t* region, int64_t i, int64_t stride) { return region + kSlots + (size_t)i * stride; }
}  // namespace

size_t dqn_mbox_region_bytes(int64_t n, int64_t state_bytes) {
  return kSlots + (size_t)n * dqn_mbox_stride(state_bytes);
}

int64_t dqn_mbox_stride(int64_t state_bytes) { return (int64_t)((kState + state_bytes + 63) / 64 * 64); }

void dqn_mbox_init(uint8_t* region, int64_t n, int64_t state_bytes) {
  std::memset(region, 0, dqn_mbox_region_bytes(n, state_bytes));
  // (published to other threads/processes by their creation, which happens after init)
}

void dqn_mbox_set_stop(uint8_t* region, int64_t v) { __atomic_store_n(w64(region + kStop), (uint64_t)v, __ATOMIC_RELEASE); }
int64_t dqn_mbox_stopped(uint8_t* region) { return (int64_t)__atomic_load_n(w64(region + kStop), __ATOMIC_ACQUIRE); }

int64_t dqn_mbox_request(uint8_t* region, int64_t i, int64_t state_bytes, const uint8_t* state, int64_t timeout_us) {
  const int64_t stride = dqn_mbox_stride(state_bytes);
  uint8_t* s = slot(region, i, stride);
  const uint64_t seq = __atomic_load_n(w64(s + kReq), __ATOMIC_RELAXED) + 1;
  std::memcpy(s + kState, state, (size_t)state_bytes);
  __atomic_store_n(w64(s + kReq), seq, __ATOMIC_RELEASE);           // publish the state
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spins = 0;; ++spins) {
    if (__atomic_load_n(w64(s + kResp), __ATOMIC_ACQUIRE) == seq)   // action visible after this
      return *reinterpret_cast<const int32_t*>(s + kAct);
    if (dqn_mbox_stopped(region)) return -2;
    if (spins > 256) {
      if (timeout_us >= 0 &&
          std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count() >
              timeout_us)
        return -1;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
}

int64_t dqn_mbox_collect(uint8_t* region, int64_t n, int64_t state_bytes, uint8_t* out_states, int32_t* out_ids,
                         uint64_t* out_seq, int64_t max_batch) {
  const int64_t stride = dqn_mbox_stride(state_bytes);
  int64_t m = 0;
  for (int64_t i = 0; i < n && m < max_batch; ++i) {
    uint8_t* s = slot(region, i, stride);
    const uint64_t req = __atomic_load_n(w64(s + kReq), __ATOMIC_ACQUIRE);   // state visible after this
    const uint64_t resp = __atomic_load_n(w64(s + kResp), __ATOMIC_RELAXED);
    if (req == resp) continue;
    std::memcpy(out_states + (size_t)m * state_bytes, s + kState, (size_t)state_bytes);
    out_ids[m] = (int32_t)i;
    out_seq[m] = req;
    ++m;
  }
  return m;
}

void dqn_mbox_respond(uint8_t* region, int64_t state_bytes, const int32_t* ids, const uint64_t* seq,
                      const int32_t* actions, int64_t m) {
  const int64_t stride = dqn_mbox_stride(state_bytes);
  for (int64_t j = 0; j < m; ++j) {
    uint8_t* s = slot(region, ids[j], stride);
    *reinterpret_cast<int32_t*>(s + kAct) = actions[j];
    __atomic_store_n(w64(s + kResp), seq[j], __ATOMIC_RELEASE);     // action published
  }
}
