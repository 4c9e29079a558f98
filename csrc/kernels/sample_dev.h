// Uniform sampling WITHOUT replacement of B transition indices out of n, shared by the
// standalone sampler (replay.hip, one 1024-lane workgroup) and the Nature trunk's fused
// sampling (trunk.hip: every (sample, instance) workgroup re-derives the whole batch, so
// no launch and no cross-workgroup exchange is needed). Deterministic in (seed, ctr, n,
// B): every caller gets the same indices.
//
// Reference: python `random.sample(deque, B)` (/root/reference/src/replay_memory.py:44).
#pragma once
#include "common.h"
#include "../include/dqn_nets_k.h"

namespace dqn {

struct SampleLds {          // LDS scratch (any 16-byte aligned region of >= 8.3 KB)
  int32_t cand[1024];
  uint32_t used[2048];      // 65536-bit bitmap of the serial fix-up
  int any_dup, fix_needed;
};

// Lane i < B (B <= blockDim.x <= 1024) returns its index; lanes >= B return -1. Every
// thread of the block must call it (it has barriers).
DQN_DEV int32_t draw_distinct(uint64_t seed, uint64_t ctr, uint32_t n, int B, SampleLds& s) {
  const int i = threadIdx.x;
  uint32_t attempt = 0;
  auto draw = [&]() -> int32_t {
    u32x4 r = philox(seed, ctr, (uint32_t)i, attempt++);
    return (int32_t)(((uint64_t)r.x * n) >> 32);
  };
  int32_t v = (i < B) ? draw() : -1;
  const bool distinct_possible = n >= (uint32_t)B;
  for (int round = 0; round < 64; ++round) {
    s.cand[i] = v;
    if (i == 0) s.any_dup = 0;
    __syncthreads();
    bool dup = false;
    if (i < B && distinct_possible) {
      for (int j = 0; j < i; ++j) dup |= (s.cand[j] == v);
    }
    if (dup) s.any_dup = 1;
    __syncthreads();
    if (!s.any_dup) break;
    if (dup) v = draw();
    __syncthreads();
  }
  // Rejection stalls when B is close to n (coupon collector): resolve what is
  // left serially with an LDS bitmap (only reachable for small n).
  if (i == 0) s.fix_needed = 0;
  s.cand[i] = v;
  __syncthreads();
  bool dup = false;
  if (i < B && distinct_possible) {
    for (int j = 0; j < i; ++j) dup |= (s.cand[j] == v);
    if (dup) s.fix_needed = 1;
  }
  __syncthreads();
  if (s.fix_needed && n <= 65536u) {
    for (int w = i; w < 2048; w += blockDim.x) s.used[w] = 0;
    __syncthreads();
    if (i < B && !dup) atomicOr(&s.used[v >> 5], 1u << (v & 31));
    __syncthreads();
    if (i == 0) {
      for (int j = 0; j < B; ++j) {
        bool dj = false;
        for (int q = 0; q < j; ++q) dj |= (s.cand[q] == s.cand[j]);
        if (!dj) continue;
        uint32_t c = (uint32_t)s.cand[j];
        while (s.used[c >> 5] & (1u << (c & 31))) c = (c + 1) % n;
        s.used[c >> 5] |= 1u << (c & 31);
        s.cand[j] = (int32_t)c;
      }
    }
    __syncthreads();
    if (i < B) v = s.cand[i];
  }
  return v;
}

// Per-sample outputs of transition tr as sample b (index, scalars, s / s' slot rows; k = 4)
DQN_DEV void write_sample_slots(const TrunkSample& s, int b, int32_t tr, int4 st, int32_t nx) {
  s.idx_out[b] = tr;
  s.a_out[b] = s.actions[tr];
  s.r_out[b] = s.rewards[tr];
  s.d_out[b] = s.dones[tr];
  s.g_out[b] = s.gammas[tr];
  reinterpret_cast<int4*>(s.st_slots)[b] = st;
  reinterpret_cast<int4*>(s.nx_slots)[b] = make_int4(st.y, st.z, st.w, nx);
}

}  // namespace dqn
