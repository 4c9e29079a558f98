// Prioritized-replay sum-tree / min-tree kernels (Schaul et al. 2016).
// Tree layout: f32[2P], root at 1, leaf i at P + i (see replay/sumtree.py).
#include "common.h"
#include "sumtree_dev.h"
#include "../include/dqn_kernels.h"

namespace dqn {

// ONE workgroup. Leaves are written first, then each level's parents are
// recomputed from their children with a workgroup barrier between levels, so
// lanes whose paths merge write identical values (duplicates in the batch are
// last-writer-wins on the leaf, exact on every ancestor).
__global__ void __launch_bounds__(1024)
sumtree_set_kernel(float* __restrict__ sum, float* __restrict__ mn, float* __restrict__ maxp,
                   const int32_t* __restrict__ idx, const float* __restrict__ td, float alpha, float eps,
                   int use_max, int n, int P, int levels) {
  __shared__ float red[16];
  const int t = threadIdx.x;
  // phase 1: leaves (+ running max of p^alpha)
  float local_max = 0.f;
  const float mp = maxp[0];
  for (int i = t; i < n; i += blockDim.x) {
    float p = use_max ? mp : powf(fabsf(td[i]) + eps, alpha);
    local_max = fmaxf(local_max, p);
    const int leaf = P + idx[i];
    sum[leaf] = p;
    mn[leaf] = p;
  }
  if (!use_max) {
    float m = wave_max(local_max);
    if ((t & 63) == 0) red[t >> 6] = m;
  }
  __syncthreads();
  if (!use_max && t == 0) {
    float m = red[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) m = fmaxf(m, red[w]);
    maxp[0] = fmaxf(mp, m);
  }
  // phase 2: ancestors, level by level
  for (int l = 1; l <= levels; ++l) {
    for (int i = t; i < n; i += blockDim.x) {
      const int node = (P + idx[i]) >> l;
      const float a = sum[2 * node], b = sum[2 * node + 1];
      const float c = mn[2 * node], d = mn[2 * node + 1];
      sum[node] = a + b;
      mn[node] = fminf(c, d);
    }
    __syncthreads();
  }
}

// B <= 64: one wave, see sumtree_update_wave (sumtree_dev.h)
__global__ void __launch_bounds__(64)
sumtree_set_wave_kernel(float* __restrict__ sum, float* __restrict__ mn, float* __restrict__ maxp,
                        const int32_t* __restrict__ idx, const float* __restrict__ td, float alpha, float eps,
                        int use_max, int n, int P, int levels) {
  __shared__ SumtreeLds L;
  sumtree_update_wave(sum, mn, maxp, idx, td, alpha, eps, use_max, n, P, levels, L);
}

// Stratified proportional sampling; w_i = (N p_i)^-beta / (N p_min)^-beta.
__global__ void __launch_bounds__(1024) sumtree_sample_kernel(const float* __restrict__ sum, const float* __restrict__ mn,
                                      int64_t* __restrict__ rng, const int32_t* __restrict__ size_p,
                                      const float* __restrict__ beta_p, int32_t* __restrict__ idx_out,
                                      float* __restrict__ w_out, int B, int P, SampleOut so,
                                      const int64_t* __restrict__ sched_step, float beta0, float beta_steps) {
  const int i = threadIdx.x;
  const uint64_t seed = (uint64_t)rng[0], ctr = (uint64_t)rng[1];
  if (i < B) {
    // annealed IS exponent from the device global_step (no host math, no extra launches):
    // beta = min(1, beta0 + (1 - beta0) * step / steps)
    const float beta = sched_step != nullptr
        ? fminf(1.f, beta0 + (1.f - beta0) * (float)sched_step[0] / beta_steps) : beta_p[0];
    per_sample_lane(sum, mn, seed, ctr, size_p[0], i, B, P, beta, idx_out, w_out, so);
  }
  __syncthreads();                      // every lane has read the counter
  if (threadIdx.x == 0) rng[1] = (int64_t)(ctr + 1);
}

}  // namespace dqn

using namespace dqn;

void launch_sumtree_set(float* sum, float* mn, float* maxp, const int32_t* idx, const float* td, float alpha,
                        float eps, int use_max, int n, int P, hipStream_t st) {
  int levels = 0;
  while ((1 << levels) < P) ++levels;
  if (n <= 64 && levels <= kMaxLevels) {
    hipLaunchKernelGGL(sumtree_set_wave_kernel, dim3(1), dim3(64), 0, st, sum, mn, maxp, idx, td, alpha, eps,
                       use_max, n, P, levels);
    return;
  }
  hipLaunchKernelGGL(sumtree_set_kernel, dim3(1), dim3(1024), 0, st, sum, mn, maxp, idx, td, alpha, eps,
                     use_max, n, P, levels);
}

void launch_sumtree_sample(const float* sum, const float* mn, int64_t* rng, const int32_t* size,
                           const float* beta, int32_t* idx_out, float* w_out, int B, int P, const SampleOut& so,
                           const int64_t* sched_step, float beta0, float beta_steps, hipStream_t st) {
  // one workgroup (host guarantees B <= 1024) so the rng counter update is ordered
  hipLaunchKernelGGL(sumtree_sample_kernel, dim3(1), dim3(1024), 0, st, sum, mn, rng, size, beta,
                     idx_out, w_out, B, P, so, sched_step, beta0, beta_steps);
}
