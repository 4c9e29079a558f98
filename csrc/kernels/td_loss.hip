// Fused TD-loss kernels: Q(s,a) gather, bootstrap target, loss, dL/dQ and
// per-sample priorities in ONE launch.
//
// Reference: host-side max over target Q (/root/reference/src/dqn_agent.py:120-122),
// python loop for y and one-hot actions (:224-253), then
// reduce_sum(q*onehot) / reduce_mean(squared_difference) in the graph
// (/root/reference/src/network.py:149-150). Extensions: Huber, Double DQN,
// per-sample n-step discount, PER importance weights, C51 projection.
#include "common.h"
#include "../include/dqn_kernels.h"

namespace dqn {

// One workgroup, one lane per sample (B <= 1024). Q rows are fp32 [B, A].
__global__ void __launch_bounds__(1024)
td_loss_scalar_kernel(const float* __restrict__ q, const float* __restrict__ qn_t,
                      const float* __restrict__ qn_o, const int32_t* __restrict__ act,
                      const float* __restrict__ rew, const float* __restrict__ done,
                      const float* __restrict__ gam, const float* __restrict__ wts,
                      float* __restrict__ loss_out, float* __restrict__ dq, float* __restrict__ prio,
                      int B, int A, int huber, float delta) {
  __shared__ float red[16];
  const int b = threadIdx.x;
  float contrib = 0.f;
  if (b < B) {
    const float* sel = (qn_o != nullptr ? qn_o : qn_t) + (int64_t)b * A;
    int best = 0;
    float bv = sel[0];
    for (int a = 1; a < A; ++a) {
      const float v = sel[a];
      if (v > bv) { bv = v; best = a; }
    }
    const float nxt = qn_t[(int64_t)b * A + best];
    const float y = rew[b] + gam[b] * (1.f - done[b]) * nxt;
    const int a_t = act[b];
    const float d = q[(int64_t)b * A + a_t] - y;
    const float w = wts != nullptr ? wts[b] : 1.f;
    float per, dper;
    if (huber) {
      const float ad = fabsf(d);
      per = ad <= delta ? 0.5f * d * d : delta * (ad - 0.5f * delta);
      dper = ad <= delta ? d : copysignf(delta, d);
    } else {
      per = d * d;
      dper = 2.f * d;
    }
    contrib = w * per;
    const float gsc = w * dper / (float)B;
    for (int a = 0; a < A; ++a) dq[(int64_t)b * A + a] = (a == a_t) ? gsc : 0.f;
    prio[b] = fabsf(d);
  }
  const float s = wave_sum(contrib);
  if ((b & 63) == 0) red[b >> 6] = s;
  __syncthreads();
  if (b == 0) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    loss_out[0] = t / (float)B;
  }
}

// C51 (Bellemare et al. 2017). One wave per sample (lane = atom, N <= 64),
// 16 waves per workgroup looping over the batch; logits fp32 [B, A, N].
__global__ void __launch_bounds__(1024)
td_loss_c51_kernel(const float* __restrict__ lg, const float* __restrict__ lgn_t,
                   const float* __restrict__ lgn_o, const int32_t* __restrict__ act,
                   const float* __restrict__ rew, const float* __restrict__ done,
                   const float* __restrict__ gam, const float* __restrict__ wts,
                   float* __restrict__ loss_out, float* __restrict__ dlg, float* __restrict__ prio,
                   int B, int A, int N, float vmin, float vmax) {
  __shared__ float red[16];
  __shared__ float mproj[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const float dz = (vmax - vmin) / (float)(N - 1);
  const bool on = lane < N;
  const float z = vmin + dz * (float)lane;
  float acc = 0.f;
  for (int b = wv; b < B; b += nw) {
    // greedy next action by expected value of the selector distribution
    const float* sel = (lgn_o != nullptr ? lgn_o : lgn_t) + (int64_t)b * A * N;
    int best = 0;
    float bq = -INFINITY;
    for (int a = 0; a < A; ++a) {
      const float x = on ? sel[a * N + lane] : -INFINITY;
      const float m = wave_max(x);
      const float e = on ? __expf(x - m) : 0.f;
      const float den = wave_sum(e);
      const float qv = wave_sum(e * z) / den;
      if (qv > bq) { bq = qv; best = a; }
    }
    // target distribution p_next = softmax(target logits[b, best])
    const float xt = on ? lgn_t[((int64_t)b * A + best) * N + lane] : -INFINITY;
    const float mt = wave_max(xt);
    const float et = on ? __expf(xt - mt) : 0.f;
    const float pn = et / wave_sum(et);
    // projection of r + gamma*z onto the support (scatter through LDS)
    mproj[wv][lane] = 0.f;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    const float tz = fminf(fmaxf(rew[b] + gam[b] * (1.f - done[b]) * z, vmin), vmax);
    const float bpos = (tz - vmin) / dz;
    const float lo = floorf(bpos), hi = ceilf(bpos);
    if (on) {
      const int l = (int)lo, u = (int)hi;
      const float eq = (l == u) ? 1.f : 0.f;
      atomicAdd(&mproj[wv][l], pn * (hi - bpos + eq));
      atomicAdd(&mproj[wv][u], pn * (bpos - lo));
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    const float m = on ? mproj[wv][lane] : 0.f;
    // cross-entropy against log_softmax(online logits[b, a])
    const int a_t = act[b];
    const float xo = on ? lg[((int64_t)b * A + a_t) * N + lane] : -INFINITY;
    const float mo = wave_max(xo);
    const float eo = on ? __expf(xo - mo) : 0.f;
    const float so = wave_sum(eo);
    const float logp = on ? (xo - mo - __logf(so)) : 0.f;
    const float ce = -wave_sum(m * logp);
    const float w = wts != nullptr ? wts[b] : 1.f;
    // dCE/dlogits = softmax - m (sum m = 1), scaled by w / B
    const float g = on ? (eo / so - m) * w / (float)B : 0.f;
    float* drow = dlg + (int64_t)b * A * N;
    for (int a = 0; a < A; ++a)
      if (on) drow[a * N + lane] = (a == a_t) ? g : 0.f;
    if (lane == 0) prio[b] = ce;
    acc += (lane == 0) ? w * ce : 0.f;
  }
  const float s = wave_sum(acc);
  if (lane == 0) red[wv] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += red[i];
    loss_out[0] = t / (float)B;
  }
}

}  // namespace dqn

using namespace dqn;

void launch_td_loss_scalar(const float* q, const float* qn_t, const float* qn_o, const int32_t* act,
                           const float* rew, const float* done, const float* gam, const float* wts,
                           float* loss, float* dq, float* prio, int B, int A, int huber, float delta,
                           hipStream_t st) {
  hipLaunchKernelGGL(td_loss_scalar_kernel, dim3(1), dim3(1024), 0, st, q, qn_t, qn_o, act, rew, done, gam,
                     wts, loss, dq, prio, B, A, huber, delta);
}

void launch_td_loss_c51(const float* lg, const float* lgn_t, const float* lgn_o, const int32_t* act,
                        const float* rew, const float* done, const float* gam, const float* wts, float* loss,
                        float* dlg, float* prio, int B, int A, int N, float vmin, float vmax, hipStream_t st) {
  hipLaunchKernelGGL(td_loss_c51_kernel, dim3(1), dim3(1024), 0, st, lg, lgn_t, lgn_o, act, rew, done, gam, wts,
                     loss, dlg, prio, B, A, N, vmin, vmax);
}
