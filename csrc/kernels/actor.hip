// Device actor step: epsilon-greedy action selection + synthetic Atari env
// step + replay append, for E environments.
//
// Reference actor step (/root/reference/src/dqn_agent.py:84-101): decay eps,
// roll dice, batch-1 forward via session.run, argmax on the host, env.step,
// cv2 resize, np.stack, deque append — all host-side per frame. Here the
// forward for all E envs is one batched device forward and the rest runs on
// the GPU, so the actor can live inside a HIP graph. For small E the step is
// fused into the head kernel (qnet.hip, HeadArgs::has_actor); this standalone
// kernel (block e = env e) serves large env batches.
//
// Replay cursor (device-resident): cursor[0] = next transition slot,
// cursor[1] = next frame slot, cursor[2] = size. Each call consumes E
// transition slots and 2E frame slots (next frame + a reserved reset frame),
// matching the replay's frame-ring bound F >= 2C + k. The LAST block to finish
// advances the cursor, the epsilon state and the RNG counter (arrival ticket).
#include "actor_dev.h"
#include "../include/dqn_kernels.h"

namespace dqn {

__global__ void __launch_bounds__(256) actor_step_kernel(ActorArgs a) {
  __shared__ int s_done;
  const int e = blockIdx.x;
  const int64_t t0 = a.cursor[0], f0 = a.cursor[1], size0 = a.cursor[2];
  const float eps0 = a.eps[0], eps_min = a.eps[1], decay = a.eps[2];
  const uint64_t seed = (uint64_t)a.rng[0], ctr = (uint64_t)a.rng[1];
  int fslot = (int)((f0 + 2 * e) % a.F), rslot = (int)((f0 + 2 * e + 1) % a.F);
  if (threadIdx.x == 0)
    s_done = actor_env_step(a, a.q + (int64_t)e * a.A, e, t0, f0, eps0, eps_min, decay, seed, ctr, fslot, rslot);
  __syncthreads();
  write_random_frame(a.frames + (int64_t)fslot * a.HW, a.HW, seed, ctr, 0x100u + 2u * e, threadIdx.x, blockDim.x);
  if (s_done)
    write_random_frame(a.frames + (int64_t)rslot * a.HW, a.HW, seed, ctr, 0x101u + 2u * e, threadIdx.x, blockDim.x);
  __syncthreads();
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    // relaxed ticket: the last block only writes the cursor/eps/rng words that
    // every block read at its start (see optim.hip for the same pattern)
    const int tk = __hip_atomic_fetch_add(a.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = tk == (int)gridDim.x - 1 ? 1 : 0;
    if (s_last) {
      actor_advance(a, t0, f0, size0, eps0, eps_min, decay, ctr);
      __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (a.tsum != nullptr) {           // PER: the last block inserts the E new transitions at max priority
    __shared__ SumtreeLds L;
    __syncthreads();
    if (s_last) sumtree_update_wave(a.tsum, a.tmin, a.tmaxp, nullptr, nullptr, 0.f, 0.f, 1, a.E, a.tP, a.tlevels, L,
                                    (int)(t0 % a.C), a.C);
  }
}

// Build the uint8 NHWC state stacks [E, H, W, K] of the actors' current states
// (only needed by executors that do not read the frame ring directly).
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
