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

// B <= 64 (the Atari minibatch): ONE wave and no level barriers. Lanes are ranked by
// (leaf, batch position) through LDS, duplicates collapse onto the last batch position
// (last-writer-wins, as in the level-synchronous kernel). Every sibling value the climb
// needs is loaded up front in one batch of independent loads; a sibling that is itself on
// an updated path is the adjacent active lane in sorted order and comes over a lane
// shuffle instead. Then each level is pure ALU + shuffles; stores are fire-and-forget.
constexpr int kMaxLevels = 30;

__global__ void __launch_bounds__(64)
sumtree_set_wave_kernel(float* __restrict__ sum, float* __restrict__ mn, float* __restrict__ maxp,
                        const int32_t* __restrict__ idx, const float* __restrict__ td, float alpha, float eps,
                        int use_max, int n, int P, int levels) {
  __shared__ uint64_t keys[64];
  __shared__ uint64_t sk[64];
  __shared__ float sv[64];
  const int lane = threadIdx.x;
  const bool valid = lane < n;
  const float mp = maxp[0];
  float p = 0.f;
  if (valid) p = use_max ? mp : powf(fabsf(td[lane]) + eps, alpha);
  if (!use_max) {
    const float m = wave_max(valid ? p : 0.f);
    if (lane == 0) maxp[0] = fmaxf(mp, m);
  }
  // unique keys (the lane breaks ties); padding lanes sort last with leaf field 0xffffffff
  const uint64_t key = ((uint64_t)(valid ? (uint32_t)idx[lane] : 0xffffffffu) << 6) | (uint64_t)lane;
  keys[lane] = key;
  __syncthreads();
  int rank = 0;
  for (int j = 0; j < 64; ++j) rank += keys[j] < key ? 1 : 0;
  sk[rank] = key;
  sv[rank] = p;
  __syncthreads();
  const uint64_t k = sk[lane];
  const float v0 = sv[lane];
  const bool ok = (k >> 6) != 0xffffffffull;
  const int leaf = ok ? (int)(k >> 6) : 0;
  // last lane of each equal-leaf run = the latest batch position: it owns the leaf
  const uint64_t kn = lane < 63 ? sk[lane + 1] : ~0ull;
  bool act = ok && (lane == 63 || (kn >> 6) != (k >> 6));
  int c = P + leaf;
  float sib_s[kMaxLevels], sib_m[kMaxLevels];
#pragma unroll
  for (int l = 0; l < kMaxLevels; ++l) {
    if (l < levels && act) {
      const int sb = (c >> l) ^ 1;
      sib_s[l] = sum[sb];
      sib_m[l] = mn[sb];
    } else {
      sib_s[l] = 0.f;
      sib_m[l] = INFINITY;
    }
  }
  float vs = v0, vm = v0;
  if (act) {
    sum[c] = vs;
    mn[c] = vm;
  }
#pragma unroll
  for (int l = 0; l < kMaxLevels; ++l) {
    if (l >= levels) break;                                 // uniform
    const uint64_t am = __ballot(act);
    // nearest active lanes below / above
    const uint64_t below = am & ((1ull << lane) - 1ull);
    const uint64_t above = lane < 63 ? am & ~((2ull << lane) - 1ull) : 0ull;
    const int lo = below ? 63 - __clzll((long long)below) : lane;
    const int hi = above ? __ffsll((long long)above) - 1 : lane;
    const int nlo = __shfl(c, lo, 64), nhi = __shfl(c, hi, 64);
    const float slo = __shfl(vs, lo, 64), shi = __shfl(vs, hi, 64);
    const float mlo = __shfl(vm, lo, 64), mhi = __shfl(vm, hi, 64);
    const bool right = c & 1;
    const int sib = c ^ 1;
    float os = sib_s[l], om = sib_m[l];
    bool sib_act = false;
    if (right && below && nlo == sib) { os = slo; om = mlo; sib_act = true; }
    if (!right && above && nhi == sib) { os = shi; om = mhi; sib_act = true; }
    const float ps = right ? os + vs : vs + os;
    const float pm = fminf(vm, om);
    // the left sibling of an active pair carries on; the right one retires
    if (right && sib_act) act = false;
    c >>= 1;
    vs = ps;
    vm = pm;
    if (act) {
      sum[c] = vs;
      mn[c] = vm;
    }
  }
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
    // annealed IS exponent from the device global_step (no host math, no extra launches):
    // beta = min(1, beta0 + (1 - beta0) * step / steps)
    const float beta = sched_step != nullptr
        ? fminf(1.f, beta0 + (1.f - beta0) * (float)sched_step[0] / beta_steps) : beta_p[0];
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
