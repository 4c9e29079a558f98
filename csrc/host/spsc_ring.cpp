// Lock-free single-producer / single-consumer ring over a caller-provided
// byte buffer (e.g. POSIX shared memory): CPU actor processes push fixed-size
// transition records, the learner drains them in bulk and ships them to the
// HBM replay with one pinned H2D copy. Replaces the reference's in-process
// deque appends (/root/reference/src/replay_memory.py:11-23).
//
// Layout: [0] head (u64, written by producer) [64] tail (u64, written by
// consumer) [128] capacity (u64) [136] record bytes (u64) [192..] records.
#include <atomic>
#include <cstdint>
#include <cstring>

#include "../include/dqn_host.h"

namespace {
constexpr size_t kHead = 0, kTail = 64, kCap = 128, kRec = 136, kData = 192;
inline uint64_t* u64(uint8_t* b, size_t off) { return reinterpret_cast<uint64_t*>(b + off); }
}  // namespace

size_t dqn_ring_bytes(uint64_t capacity, uint64_t record_bytes) { return kData + capacity * record_bytes; }

void dqn_ring_init(uint8_t* buf, uint64_t capacity, uint64_t record_bytes) {
  __atomic_store_n(u64(buf, kHead), 0, __ATOMIC_RELAXED);
  __atomic_store_n(u64(buf, kTail), 0, __ATOMIC_RELAXED);
  *u64(buf, kCap) = capacity;
  *u64(buf, kRec) = record_bytes;
  // (published to other threads/processes by their creation, which happens after init)
}

int64_t dqn_ring_push(uint8_t* buf, const uint8_t* recs, int64_t n) {
  const uint64_t cap = *u64(buf, kCap), rb = *u64(buf, kRec);
  const uint64_t head = __atomic_load_n(u64(buf, kHead), __ATOMIC_RELAXED);
  const uint64_t tail = __atomic_load_n(u64(buf, kTail), __ATOMIC_ACQUIRE);
  const uint64_t space = cap - (head - tail);
  const uint64_t m = (uint64_t)n < space ? (uint64_t)n : space;
  for (uint64_t i = 0; i < m; ++i)
    std::memcpy(buf + kData + ((head + i) % cap) * rb, recs + i * rb, rb);
  __atomic_store_n(u64(buf, kHead), head + m, __ATOMIC_RELEASE);
  return (int64_t)m;
}

int64_t dqn_ring_pop(uint8_t* buf, uint8_t* out, int64_t max_n) {
  const uint64_t cap = *u64(buf, kCap), rb = *u64(buf, kRec);
  const uint64_t tail = __atomic_load_n(u64(buf, kTail), __ATOMIC_RELAXED);
  const uint64_t head = __atomic_load_n(u64(buf, kHead), __ATOMIC_ACQUIRE);
  const uint64_t avail = head - tail;
  const uint64_t m = (uint64_t)max_n < avail ? (uint64_t)max_n : avail;
  for (uint64_t i = 0; i < m; ++i)
    std::memcpy(out + i * rb, buf + kData + ((tail + i) % cap) * rb, rb);
  __atomic_store_n(u64(buf, kTail), tail + m, __ATOMIC_RELEASE);
  return (int64_t)m;
}

int64_t dqn_ring_size(uint8_t* buf) {
  return (int64_t)(__atomic_load_n(u64(buf, kHead), __ATOMIC_ACQUIRE) -
                   __atomic_load_n(u64(buf, kTail), __ATOMIC_ACQUIRE));
}

const uint8_t* dqn_ring_peek(uint8_t* buf, uint64_t* tail, uint64_t* avail, uint64_t* cap, uint64_t* rec_bytes) {
  *cap = *u64(buf, kCap);
  *rec_bytes = *u64(buf, kRec);
  *tail = __atomic_load_n(u64(buf, kTail), __ATOMIC_RELAXED);
  *avail = __atomic_load_n(u64(buf, kHead), __ATOMIC_ACQUIRE) - *tail;
  return buf + kData;
}

void dqn_ring_release(uint8_t* buf, uint64_t n) {
  const uint64_t tail = __atomic_load_n(u64(buf, kTail), __ATOMIC_RELAXED);
  __atomic_store_n(u64(buf, kTail), tail + n, __ATOMIC_RELEASE);
}
