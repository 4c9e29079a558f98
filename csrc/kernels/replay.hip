// HBM replay kernels: uniform sampling without replacement + frame-stack gather.
//
// Reference: python `random.sample(deque, B)` + tuple partition + numpy stack
// + feed_dict H2D (/root/reference/src/replay_memory.py:31-45,
// /root/reference/src/dqn_agent.py:113-129,249-253). Here the sample is one
// workgroup (B <= 1024 lanes, Philox4x32-10, counter advanced on the device so
// graph replays draw fresh numbers) and the gather rebuilds the uint8 k-frame
// stacks straight from the frame ring (frames stored once, not per state).
#include "common.h"
#include "../include/dqn_kernels.h"

#include "sample_dev.h"

namespace dqn {

DQN_DEV void write_sample_outputs(const SampleOut& so, int i, int tr) {
  if (so.st_slots == nullptr) return;
  so.a_out[i] = so.actions[tr];
  so.r_out[i] = so.rewards[tr];
  so.d_out[i] = so.dones[tr];
  so.g_out[i] = so.gammas[tr];
  const int K = so.K;
  for (int c = 0; c < K; ++c) {
    const int v = so.state_idx[(int64_t)tr * K + c];
    so.st_slots[i * K + c] = v;
    if (c > 0) so.nx_slots[i * K + c - 1] = v;
  }
  so.nx_slots[i * K + K - 1] = so.next_idx[tr];
}

__global__ void __launch_bounds__(1024)
sample_uniform_kernel(const int32_t* __restrict__ size_p, int64_t* __restrict__ rng,
                      int32_t* __restrict__ out, int B, SampleOut so) {
  __shared__ SampleLds sl;
  const int i = threadIdx.x;
  const uint32_t n = (uint32_t)max(size_p[0], 1);
  const uint64_t seed = (uint64_t)rng[0];
  const uint64_t ctr = (uint64_t)rng[1];
  const int32_t v = draw_distinct(seed, ctr, n, B, sl);
  if (i < B) {
    DQN_ASSERT(v >= 0 && (uint32_t)v < n);
    out[i] = v;
    write_sample_outputs(so, i, v);
  }
  if (i == 0) rng[1] = (int64_t)(ctr + 1);
}

// frames: [F, H, W] u8; state_idx: [C, k] i32; next_idx: [C] i32; idx: [B]
// outputs s, ns: [B, H, W, k] u8 (NHWC, channel = frame in the stack).
template <int K>
__global__ void gather_frames_kernel(const uint8_t* __restrict__ frames, const int32_t* __restrict__ state_idx,
                                     const int32_t* __restrict__ next_idx, const int32_t* __restrict__ idx,
                                     uint8_t* __restrict__ s, uint8_t* __restrict__ ns, int B, int HW,
                                     GatherScalars sc) {
  // one thread = 4 consecutive pixels of one sample, both stacks
  const int groups = HW / 4;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (sc.a_out != nullptr && t < B) {        // per-sample scalars ride along
    const int tr = idx[t];
    sc.a_out[t] = sc.actions[tr];
    sc.r_out[t] = sc.rewards[tr];
    sc.d_out[t] = sc.dones[tr];
    sc.g_out[t] = sc.gammas[tr];
  }
  if (t >= B * groups) return;
  const int b = t / groups, g = t - b * groups;
  const int tr = idx[b];
  int slots[K + 1];
#pragma unroll
  for (int c = 0; c < K; ++c) slots[c] = state_idx[(int64_t)tr * K + c];
  slots[K] = next_idx[tr];
#pragma unroll
  for (int c = 0; c <= K; ++c) DQN_ASSERT(slots[c] >= 0);
  uint32_t px[K + 1];
#pragma unroll
  for (int c = 0; c <= K; ++c)
    px[c] = *reinterpret_cast<const uint32_t*>(frames + (int64_t)slots[c] * HW + g * 4);
  // transpose (K+1) frames x 4 pixels -> per pixel K channels
  uint8_t* ds = s + ((int64_t)b * HW + g * 4) * K;
  uint8_t* dn = ns + ((int64_t)b * HW + g * 4) * K;
  if constexpr (K == 4) {
    uint32_t ws[4], wn[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      ws[p] = wn[p] = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        ws[p] |= ((px[c] >> (8 * p)) & 0xffu) << (8 * c);
        wn[p] |= ((px[c + 1] >> (8 * p)) & 0xffu) << (8 * c);
      }
    }
    *reinterpret_cast<uint4*>(ds) = make_uint4(ws[0], ws[1], ws[2], ws[3]);
    *reinterpret_cast<uint4*>(dn) = make_uint4(wn[0], wn[1], wn[2], wn[3]);
  } else {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
      for (int c = 0; c < K; ++c) {
        ds[p * K + c] = (uint8_t)(px[c] >> (8 * p));
        dn[p * K + c] = (uint8_t)(px[c + 1] >> (8 * p));
      }
    }
  }
}

}  // namespace dqn

using namespace dqn;

void launch_replay_sample_uniform(const int32_t* size, int64_t* rng, int32_t* out, int B, const SampleOut& so,
                                  hipStream_t st) {
  hipLaunchKernelGGL(sample_uniform_kernel, dim3(1), dim3(1024), 0, st, size, rng, out, B, so);
}

void launch_replay_gather_frames(const uint8_t* frames, const int32_t* state_idx, const int32_t* next_idx,
                                 const int32_t* idx, uint8_t* s, uint8_t* ns, int B, int HW, int K,
                                 const GatherScalars& sc, hipStream_t st) {
  const int total = B * (HW / 4);
  dim3 grid((total + 255) / 256), block(256);
  switch (K) {
    case 1: hipLaunchKernelGGL(gather_frames_kernel<1>, grid, block, 0, st, frames, state_idx, next_idx, idx, s, ns, B, HW, sc); break;
    case 2: hipLaunchKernelGGL(gather_frames_kernel<2>, grid, block, 0, st, frames, state_idx, next_idx, idx, s, ns, B, HW, sc); break;
    case 3: hipLaunchKernelGGL(gather_frames_kernel<3>, grid, block, 0, st, frames, state_idx, next_idx, idx, s, ns, B, HW, sc); break;
    case 4: hipLaunchKernelGGL(gather_frames_kernel<4>, grid, block, 0, st, frames, state_idx, next_idx, idx, s, ns, B, HW, sc); break;
    default: break;  // host checks K in [1, 4]
  }
}
