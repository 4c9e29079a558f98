// Device actor step: epsilon-greedy action selection + synthetic Atari env
// step + replay append, for E environments, in ONE launch (block e = env e).
//
// Reference actor step (/root/reference/src/dqn_agent.py:84-101): decay eps,
// roll dice, batch-1 forward via session.run, argmax on the host, env.step,
// cv2 resize, np.stack, deque append — all host-side per frame. Here the
// forward for all E envs is one batched device forward and this kernel does
// the rest without leaving the GPU, so the actor can live inside a HIP graph.
//
// Replay cursor (device-resident): cursor[0] = next transition slot,
// cursor[1] = next frame slot, cursor[2] = size. Each call consumes E
// transition slots and 2E frame slots (next frame + a reserved reset frame),
// matching the replay's frame-ring bound F >= 2C + k. The LAST block to finish
// advances the cursor, the epsilon state and the RNG counter (arrival ticket).
#include "common.h"
#include "../include/dqn_kernels.h"

namespace dqn {

struct ActorArgs {
  const float* q;          // [E, A] online Q of the current states
  uint8_t* frames;         // [F, HW]
  int32_t* stacks;         // [E, K] frame slots of each env's current state
  int64_t* cursor;         // [3]
  int32_t* size_dev;       // [1]
  int32_t* state_idx;      // [C, K]
  int32_t* next_idx;       // [C]
  int32_t* actions;        // [C]
  float* rewards;          // [C]
  float* dones;            // [C]
  float* gammas;           // [C]
  float* eps;              // [3]: eps, eps_min, decay
  int64_t* rng;            // [2]
  int32_t* ticket;         // [1]
  int64_t* frames_done;    // [1] env-frame counter
  int E, A, K, HW, C, F;
  float gamma, p_done;
};

DQN_DEV void write_random_frame(uint8_t* dst, int HW, uint64_t seed, uint64_t ctr, uint32_t salt) {
  // 16 bytes per philox call; HW is a multiple of 16 for 84x84 (7056 = 441*16)
  const int n16 = HW / 16;
  for (int i = threadIdx.x; i < n16; i += blockDim.x) {
    u32x4 r = philox(seed, ctr, (uint32_t)i, salt);
    *reinterpret_cast<uint4*>(dst + (int64_t)i * 16) = make_uint4(r.x, r.y, r.z, r.w);
  }
  for (int i = n16 * 16 + threadIdx.x; i < HW; i += blockDim.x) dst[i] = (uint8_t)(i * 131u + salt);
}

__global__ void __launch_bounds__(256) actor_step_kernel(ActorArgs a) {
  __shared__ int s_done;
  const int e = blockIdx.x;
  const int64_t t0 = a.cursor[0], f0 = a.cursor[1], size0 = a.cursor[2];
  const float eps0 = a.eps[0], eps_min = a.eps[1], decay = a.eps[2];
  const uint64_t seed = (uint64_t)a.rng[0], ctr = (uint64_t)a.rng[1];
  const int fslot = (int)((f0 + 2 * e) % a.F);
  const int rslot = (int)((f0 + 2 * e + 1) % a.F);
  if (threadIdx.x == 0) {
    // reference: eps decays BEFORE each roll (dqn_agent.py:162-174); env e rolls (e+1)-th
    float eps = eps0;
    for (int i = 0; i <= e && eps > eps_min; ++i) eps -= decay;
    u32x4 r = philox(seed ^ 0xA5A5A5A5ull, ctr, (uint32_t)e, 1u);
    int act;
    if (u01(r.x) < eps) {
      act = (int)(((uint64_t)r.y * (uint32_t)a.A) >> 32);
    } else {
      const float* qe = a.q + (int64_t)e * a.A;
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
    s_done = done;
  }
  __syncthreads();
  write_random_frame(a.frames + (int64_t)fslot * a.HW, a.HW, seed, ctr, 0x100u + 2u * e);
  if (s_done) write_random_frame(a.frames + (int64_t)rslot * a.HW, a.HW, seed, ctr, 0x101u + 2u * e);
  __syncthreads();
  if (threadIdx.x == 0) {
    // relaxed ticket: the last block only writes the cursor/eps/rng words that
    // every block read at its start (see optim.hip for the same pattern)
    const int tk = __hip_atomic_fetch_add(a.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == (int)gridDim.x - 1) {
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
      __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Build the uint8 NHWC state stacks [E, H, W, K] of the actors' current states.
__global__ void stack_states_kernel(const uint8_t* __restrict__ frames, const int32_t* __restrict__ stacks,
                                    uint8_t* __restrict__ out, int E, int HW, int K) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= E * HW) return;
  const int e = t / HW, p = t - e * HW;
  for (int c = 0; c < K; ++c) out[(int64_t)t * K + c] = frames[(int64_t)stacks[e * K + c] * HW + p];
}

}  // namespace dqn

using namespace dqn;

void launch_actor_step(const float* q, uint8_t* frames, int32_t* stacks, int64_t* cursor, int32_t* size_dev,
                       int32_t* state_idx, int32_t* next_idx, int32_t* actions, float* rewards, float* dones,
                       float* gammas, float* eps, int64_t* rng, int32_t* ticket, int64_t* frames_done, int E,
                       int A, int K, int HW, int C, int F, float gamma, float p_done, hipStream_t st) {
  ActorArgs a{q, frames, stacks, cursor, size_dev, state_idx, next_idx, actions, rewards, dones, gammas,
              eps, rng, ticket, frames_done, E, A, K, HW, C, F, gamma, p_done};
  hipLaunchKernelGGL(actor_step_kernel, dim3(E), dim3(256), 0, st, a);
}

void launch_stack_states(const uint8_t* frames, const int32_t* stacks, uint8_t* out, int E, int HW, int K,
                         hipStream_t st) {
  const int total = E * HW;
  hipLaunchKernelGGL(stack_states_kernel, dim3((total + 255) / 256), dim3(256), 0, st, frames, stacks, out, E, HW,
                     K);
}
