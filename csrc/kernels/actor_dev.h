// Device-side actor step pieces shared by the standalone actor kernel
// (actor.hip, E blocks) and the fused acting path of the head kernel
// (qnet.hip: Q tile -> eps-greedy -> env step -> replay append in ONE launch).
#pragma once
#include "common.h"
#include "sumtree_dev.h"
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
                           float eps_min, float decay, uint64_t seed, uint64_t ctr, int& fslot, int& rslot,
                           const int32_t* st_pre = nullptr) {
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
  const int done = u01(r.w) < a.p_done ? 1 : 0;          // == actor_done(a, seed, ctr, e)
  const int t = (int)((t0 + e) % a.C);
  int32_t* st = a.stacks + (int64_t)e * a.K;
  DQN_ASSERT(a.K >= 1 && a.K <= 4);
  int32_t cur[4];                                        // K <= 4 (frames_per_state, host-checked)
  for (int c = 0; c < a.K; ++c) cur[c] = st_pre != nullptr ? st_pre[c] : st[c];
  for (int c = 0; c < a.K; ++c) a.state_idx[(int64_t)t * a.K + c] = cur[c];
  a.next_idx[t] = fslot;
  a.actions[t] = act;
  a.rewards[t] = reward;
  a.dones[t] = (float)done;
  a.gammas[t] = a.gamma;
  if (done) {
    for (int c = 0; c < a.K; ++c) st[c] = rslot;     // new episode: reset frame duplicated k times
  } else {
    for (int c = 0; c + 1 < a.K; ++c) st[c] = cur[c + 1];
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

DQN_DEV void actor_advance(const ActorArgs& a, int64_t t0, int64_t f0, int64_t size0, float eps0, float eps_min,
                           float decay, uint64_t ctr, int64_t frames_done0) {
  float eps = eps0;
  for (int i = 0; i < a.E && eps > eps_min; ++i) eps -= decay;
  a.eps[0] = eps;
  a.cursor[0] = (t0 + a.E) % a.C;
  a.cursor[1] = (f0 + 2 * a.E) % a.F;
  const int64_t ns = size0 + a.E < a.C ? size0 + a.E : a.C;
  a.cursor[2] = ns;
  a.size_dev[0] = (int32_t)ns;
  a.rng[1] = (int64_t)(ctr + 1);
  a.frames_done[0] = frames_done0 + a.E;
}

// The actor's step state (cursor, eps schedule, rng): loaded up front so a caller can
// issue these loads before unrelated work (the fused head's Q tiles) and hide them.
struct ActorPre {
  int64_t t0, f0, size0, frames_done;
  float eps0, eps_min, decay;
  uint64_t seed, ctr;
  int32_t st[4];                 // this thread's env stack (thread e < E), K <= 4
};

DQN_DEV ActorPre actor_prefetch(const ActorArgs& a) {
  ActorPre p;
  p.t0 = a.cursor[0]; p.f0 = a.cursor[1]; p.size0 = a.cursor[2];
  p.eps0 = a.eps[0]; p.eps_min = a.eps[1]; p.decay = a.eps[2];
  p.seed = (uint64_t)a.rng[0]; p.ctr = (uint64_t)a.rng[1];
  p.frames_done = threadIdx.x == 0 ? a.frames_done[0] : 0;
  const int e = threadIdx.x;
  for (int c = 0; c < 4; ++c) p.st[c] = (e < a.E && c < a.K) ? a.stacks[(int64_t)e * a.K + c] : 0;
  return p;
}

// env e's episode end this step: the same draw actor_env_step makes (any thread can ask)
DQN_DEV bool actor_done(const ActorArgs& a, uint64_t seed, uint64_t ctr, int e) {
  const u32x4 r = philox(seed ^ 0xA5A5A5A5ull, ctr, (uint32_t)e, 1u);
  return u01(r.w) < a.p_done;
}

// Whole actor step for all E envs inside ONE workgroup; q = [E][A] (LDS or global, visible
// to every thread on entry). No barrier inside: every thread re-derives the envs' episode
// ends from the rng instead of waiting on the deciding threads, so the replay / frame
// stores are never waited for (a __syncthreads would drain them, ~us per barrier).
DQN_DEV void actor_step_block(const ActorArgs& a, const float* q, void* lds_scratch, const ActorPre& p) {
  // lds_scratch: >= sizeof(SumtreeLds) bytes of dead LDS (prioritized replay's tree insert)
  const int tid = threadIdx.x, nth = blockDim.x;
  for (int e = tid; e < a.E; e += nth) {
    int fs, rs;
    actor_env_step(a, q + e * a.A, e, p.t0, p.f0, p.eps0, p.eps_min, p.decay, p.seed, p.ctr, fs, rs,
                   e == tid ? p.st : nullptr);
  }
  for (int e = 0; e < a.E; ++e) {
    const int fslot = (int)((p.f0 + 2 * e) % a.F), rslot = (int)((p.f0 + 2 * e + 1) % a.F);
    write_random_frame(a.frames + (int64_t)fslot * a.HW, a.HW, p.seed, p.ctr, 0x100u + 2u * e, tid, nth);
    if (actor_done(a, p.seed, p.ctr, e))
      write_random_frame(a.frames + (int64_t)rslot * a.HW, a.HW, p.seed, p.ctr, 0x101u + 2u * e, tid, nth);
  }
  if (tid == 0) actor_advance(a, p.t0, p.f0, p.size0, p.eps0, p.eps_min, p.decay, p.ctr, p.frames_done);
  if (a.tsum != nullptr)           // PER: the E new transitions enter with the running max priority
    sumtree_update_wave(a.tsum, a.tmin, a.tmaxp, nullptr, nullptr, 0.f, 0.f, 1, a.E, a.tP, a.tlevels,
                        *reinterpret_cast<SumtreeLds*>(lds_scratch), (int)(p.t0 % a.C), a.C);
}

DQN_DEV void actor_step_block(const ActorArgs& a, const float* q, void* lds_scratch) {
  actor_step_block(a, q, lds_scratch, actor_prefetch(a));
}

// Fused acting with ONE ENV PER WORKGROUP (the head kernels' acting blocks), in two parts so
// the caller can put its Q computation in between:
//   actor_env_frames  env e's new frame (+ reset frame): they depend only on the rng state,
//                     never on Q, so every thread writes them while the Q loads are in flight;
//   actor_env_finish  thread 0 decides + appends from qe (env e's Q row, visible to thread 0),
//                     and the LAST block to arrive (ticket) advances the actor state (every
//                     block read it at its start) and, PER, inserts the E new transitions.
// flag / st: block LDS scratch.
DQN_DEV void actor_env_frames(const ActorArgs& x, int e, const ActorPre& pre) {
  const int tid = threadIdx.x, nth = blockDim.x;
  const int fslot = (int)((pre.f0 + 2 * e) % x.F), rslot = (int)((pre.f0 + 2 * e + 1) % x.F);
  write_random_frame(x.frames + (int64_t)fslot * x.HW, x.HW, pre.seed, pre.ctr, 0x100u + 2u * e, tid, nth);
  if (actor_done(x, pre.seed, pre.ctr, e))
    write_random_frame(x.frames + (int64_t)rslot * x.HW, x.HW, pre.seed, pre.ctr, 0x101u + 2u * e, tid, nth);
}

DQN_DEV void actor_env_finish(const ActorArgs& x, const float* qe, int e, const ActorPre& pre, const int32_t* st_e,
                              int* flag, SumtreeLds& st) {
  const int tid = threadIdx.x;
  if (tid == 0) {
    int fs, rs;
    actor_env_step(x, qe, e, pre.t0, pre.f0, pre.eps0, pre.eps_min, pre.decay, pre.seed, pre.ctr, fs, rs, st_e);
    const int tk = __hip_atomic_fetch_add(x.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = tk == x.E - 1 ? 1 : 0;
    if (*flag) {
      actor_advance(x, pre.t0, pre.f0, pre.size0, pre.eps0, pre.eps_min, pre.decay, pre.ctr);
      __hip_atomic_store(x.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (x.tsum != nullptr) {          // PER: the last block inserts the E new transitions at max priority
    __syncthreads();
    if (*flag) sumtree_update_wave(x.tsum, x.tmin, x.tmaxp, nullptr, nullptr, 0.f, 0.f, 1, x.E, x.tP, x.tlevels, st,
                                   (int)(pre.t0 % x.C), x.C);
  }
}

}  // namespace dqn
