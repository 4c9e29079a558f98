// Device-side actor step pieces shared by the standalone actor kernel
// (actor.hip, E blocks) and the fused acting path of the head kernel
// (qnet.hip: Q tile -> eps-greedy -> env step -> replay append in ONE launch).
#pragma once
#include "common.h"
#include "../include/dqn_nets_k.h"

namespace dqn {

DQN_DEV void write_random_frame(uint8_t* dst, int HW, uint64_t seed, uint64_t ctr, uint32_t salt, int tid, int nth) {
  // 16 bytes per philox call; 84x84 = 7056 = 441 * 16
  const int n16 = HW / 16;
  for (int i = tid; i < n16; i += nth) {
    u32x4 r = philox(seed, ctr, (uint32_t)i, salt);
    *reinterpret_cast<uint4*>(dst + (int64_t)i * 16) = make_uint4(r.x, r.y, r.z, r.w);
  }
  for (int i = n16 * 16 + tid; i < HW; i += nth) dst[i] = (uint8_t)(i * 131u + salt);
}

// Env e's decision + replay append (one thread). Returns done; frame slots via refs.
DQN_DEV int actor_env_step(const ActorArgs& a, const float* qe, int e, int64_t t0, int64_t f0, float eps0,
                           float eps_min, float decay, uint64_t seed, uint64_t ctr, int& fslot, int& rslot) {
  fslot = (int)((f0 + 2 * e) % a.F);
  rslot = (int)((f0 + 2 * e + 1) % a.F);
  // reference: eps decays BEFORE each roll (dqn_agent.py:162-174); env e rolls the (e+1)-th time
  float eps = eps0;
  for (int i = 0; i <= e && eps > eps_min; ++i) eps -= decay;
  u32x4 r = philox(seed ^ 0xA5A5A5A5ull, ctr, (uint32_t)e, 1u);
  int act;
  if (u01(r.x) < eps) {
    act = (int)(((uint64_t)r.y * (uint32_t)a.A) >> 32);
  } else {
    act = 0;
    float best = qe[0];
    for (int i = 1; i < a.A; ++i) if (qe[i] > best) { best = qe[i]; act = i; }
  }
  const float u = u01(r.z);
  const float reward = u < 0.01f ? 1.f : (u < 0.02f ? -1.f : 0.f);
  const int done = u01(r.w) < a.p_done ? 1 : 0;
  const int t = (int)((t0 + e) % a.C);
  int32_t* st = a.stacks + (int64_t)e * a.K;
  for (int c = 0; c < a.K; ++c) a.state_idx[(int64_t)t * a.K + c] = st[c];
  a.next_idx[t] = fslot;
  a.actions[t] = act;
  a.rewards[t] = reward;
  a.dones[t] = (float)done;
  a.gammas[t] = a.gamma;
  if (done) {
    for (int c = 0; c < a.K; ++c) st[c] = rslot;     // new episode: reset frame duplicated k times
  } else {
    for (int c = 0; c + 1 < a.K; ++c) st[c] = st[c + 1];
    st[a.K - 1] = fslot;
  }
  return done;
}

DQN_DEV void actor_advance(const ActorArgs& a, int64_t t0, int64_t f0, int64_t size0, float eps0, float eps_min,
                           float decay, uint64_t ctr) {
  float eps = eps0;
  for (int i = 0; i < a.E && eps > eps_min; ++i) eps -= decay;
  a.eps[0] = eps;
  a.cursor[0] = (t0 + a.E) % a.C;
  a.cursor[1] = (f0 + 2 * a.E) % a.F;
  const int64_t ns = size0 + a.E < a.C ? size0 + a.E : a.C;
  a.cursor[2] = ns;
  a.size_dev[0] = (int32_t)ns;
  a.rng[1] = (int64_t)(ctr + 1);
  a.frames_done[0] += a.E;
}

// Whole actor step for all E envs inside ONE workgroup; q = [E][A] (LDS or global).
DQN_DEV void actor_step_block(const ActorArgs& a, const float* q, int* s_done /* LDS [E] */) {
  const int tid = threadIdx.x, nth = blockDim.x;
  const int64_t t0 = a.cursor[0], f0 = a.cursor[1], size0 = a.cursor[2];
  const float eps0 = a.eps[0], eps_min = a.eps[1], decay = a.eps[2];
  const uint64_t seed = (uint64_t)a.rng[0], ctr = (uint64_t)a.rng[1];
  __syncthreads();
  for (int e = tid; e < a.E; e += nth) {
    int fs, rs;
    s_done[e] = actor_env_step(a, q + e * a.A, e, t0, f0, eps0, eps_min, decay, seed, ctr, fs, rs);
  }
  __syncthreads();
  for (int e = 0; e < a.E; ++e) {
    const int fslot = (int)((f0 + 2 * e) % a.F), rslot = (int)((f0 + 2 * e + 1) % a.F);
    write_random_frame(a.frames + (int64_t)fslot * a.HW, a.HW, seed, ctr, 0x100u + 2u * e, tid, nth);
    if (s_done[e]) write_random_frame(a.frames + (int64_t)rslot * a.HW, a.HW, seed, ctr, 0x101u + 2u * e, tid, nth);
  }
  __syncthreads();
  if (tid == 0) actor_advance(a, t0, f0, size0, eps0, eps_min, decay, ctr);
}

}  // namespace dqn
