// Prioritized-replay sum-tree / min-tree kernels (Schaul et al. 2016).
// Tree layout: f32[2P], root at 1, leaf i at P + i (see replay/sumtree.py).
#include "common.h"
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

// Stratified proportional sampling; w_i = (N p_i)^-beta / (N p_min)^-beta.
__global__ void __launch_bounds__(1024) sumtree_sample_kernel(const float* __restrict__ sum, const float* __restrict__ mn,
                                      int64_t* __restrict__ rng, const int32_t* __restrict__ size_p,
                                      const float* __restrict__ beta_p, int32_t* __restrict__ idx_out,
                                      float* __restrict__ w_out, int B, int P, SampleOut so) {
  const int i = threadIdx.x;
  const uint64_t seed = (uint64_t)rng[0], ctr = (uint64_t)rng[1];
  if (i < B) {
    const float total = sum[1];
    u32x4 r = philox(seed ^ 0x5bd1e995ull, ctr, (uint32_t)i, 0x7u);
    float u = ((float)i + u01(r.x)) * (total / (float)B);
    int node = 1;
    while (node < P) {
      const int left = 2 * node;
      const float ls = sum[left];
      const bool right = (u >= ls) && (sum[left + 1] > 0.f);
      u = right ? u - ls : u;
      node = right ? left + 1 : left;
    }
    const int n = max(size_p[0], 1);
    int leaf = min(node - P, n - 1);
    DQN_ASSERT(leaf >= 0 && node >= P && node < 2 * P);
    idx_out[i] = leaf;
    const float beta = beta_p[0];
    const float p = sum[P + leaf] / total;
    const float pmin = mn[1] / total;
    w_out[i] = powf((float)n * p, -beta) / powf((float)n * pmin, -beta);
    if (so.st_slots != nullptr) {
      so.a_out[i] = so.actions[leaf];
      so.r_out[i] = so.rewards[leaf];
      so.d_out[i] = so.dones[leaf];
      so.g_out[i] = so.gammas[leaf];
      const int K = so.K;
      for (int c = 0; c < K; ++c) {
        const int v = so.state_idx[(int64_t)leaf * K + c];
        so.st_slots[i * K + c] = v;
        if (c > 0) so.nx_slots[i * K + c - 1] = v;
      }
      so.nx_slots[i * K + K - 1] = so.next_idx[leaf];
    }
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
  hipLaunchKernelGGL(sumtree_set_kernel, dim3(1), dim3(1024), 0, st, sum, mn, maxp, idx, td, alpha, eps,
                     use_max, n, P, levels);
}

void launch_sumtree_sample(const float* sum, const float* mn, int64_t* rng, const int32_t* size,
                           const float* beta, int32_t* idx_out, float* w_out, int B, int P, const SampleOut& so,
                           hipStream_t st) {
  // one workgroup (host guarantees B <= 1024) so the rng counter update is ordered
  hipLaunchKernelGGL(sumtree_sample_kernel, dim3(1), dim3(1024), 0, st, sum, mn, rng, size, beta,
                     idx_out, w_out, B, P, so);
}
