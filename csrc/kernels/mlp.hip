// Fused MLP Q-network kernels: the reference `SimpleNetwork`
// (/root/reference/src/network.py:258-313: in -> 20 tanh -> 20 tanh -> A affine)
// and any small dense chain (<= 4 layers, widths <= 64), fp32 end to end.
//
// The reference runs this net as separate TF ops per layer plus a host round trip
// for the target maxima (/root/reference/src/dqn_agent.py:120-122). Here ONE workgroup
// does the whole SGD-step gradient: online forward on s (activations kept in LDS),
// target forward on s' (+ online forward on s' for Double DQN), TD loss (MSE or Huber,
// PER weights, per-sample n-step discount), backward to the per-layer deltas, and the
// weight/bias gradients reduced over the batch into an LDS accumulator, written once.
// Widths of 20 are far below an MFMA tile, so this is lane-per-sample fp32 FMA work:
// the kernel is latency-bound and the point is doing it in one launch.
#include "common.h"
#include "../include/dqn_kernels.h"

namespace dqn {

namespace {

DQN_DEV float act_fn(int kind, float z) {
  return kind == 1 ? tanhf(z) : (kind == 2 ? fmaxf(z, 0.f) : z);
}
DQN_DEV float act_grad(int kind, float h) {     // derivative from the OUTPUT h
  return kind == 1 ? (1.f - h * h) : (kind == 2 ? (h > 0.f ? 1.f : 0.f) : 1.f);
}

// Forward of one sample through all layers. in: [fin0] (row in LDS or global), rows:
// layer outputs written to out[l] (stride per layer); w/b from `P` (flat params, LDS or global).
// Returns nothing; the last layer's output row holds Q.
template <typename PT>
DQN_DEV void forward_row(const MlpArgs& a, const PT* P, const float* in, float* const* out) {
  const float* h = in;
  for (int l = 0; l < a.L; ++l) {
    const PT* W = P + a.w_off[l];
    const PT* bb = P + a.b_off[l];
    const int fi = a.fin[l], fo = a.fout[l];
    float* o = out[l];
    for (int j = 0; j < fo; ++j) {
      float z = (float)bb[j];
      for (int i = 0; i < fi; ++i) z = fmaf(h[i], (float)W[i * fo + j], z);
      o[j] = act_fn(a.act[l], z);
    }
    h = o;
  }
}

}  // namespace

// Inference: one lane per sample, params from global (L1-resident), q_out [B, A].
// LDS row per lane: [x (fin0) | ping (sw) | pong (sw)].
__global__ void __launch_bounds__(kMlpThreads) mlp_fwd_kernel(MlpArgs a) {
  extern __shared__ float lds[];
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int D0 = a.fin[0];
  float* row = lds + (long)threadIdx.x * (D0 + 2 * a.sw + 1);
  for (int i = 0; i < D0; ++i) row[i] = a.x[(long)b * D0 + i] * a.in_scale;
  float* outs[kMlpMaxLayers];
  for (int l = 0; l < a.L; ++l) outs[l] = row + D0 + (l & 1) * a.sw;
  forward_row(a, a.w_on, row, outs);
  const float* q = outs[a.L - 1];
  for (int j = 0; j < a.A; ++j) a.q_out[(long)b * a.A + j] = q[j];
}

// Training: ONE workgroup of kMlpThreads lanes, samples in chunks of kMlpThreads.
// LDS: online params [P] | grad accumulator [P] | per-chunk rows:
//   H   [CH][Hs]  x (scaled), then every layer's output (post-activation)
//   D   [CH][Ds]  every layer's delta dL/dz (reused as scratch for the s' forwards)
__global__ void __launch_bounds__(kMlpThreads) mlp_train_kernel(MlpArgs a) {
  extern __shared__ float lds[];
  const int t = threadIdx.x;
  const int P = a.P;
  float* Pw = lds;
  float* G = lds + P;
  float* H = G + P;
  float* D = H + (long)kMlpThreads * a.Hs;
  __shared__ float red[kMlpThreads / 64];
  for (int i = t; i < P; i += kMlpThreads) {
    Pw[i] = a.w_on[i];
    G[i] = 0.f;
  }
  __syncthreads();
  // row offsets of each layer inside H / D
  int hoff[kMlpMaxLayers + 1], doff[kMlpMaxLayers];
  hoff[0] = 0;
  for (int l = 0; l < a.L; ++l) hoff[l + 1] = hoff[l] + a.fin[l];
  {
    int o = 0;
    for (int l = 0; l < a.L; ++l) { doff[l] = o; o += a.fout[l]; }
  }
  const int A = a.A;
  float loss_acc = 0.f;
  for (int c0 = 0; c0 < a.B; c0 += kMlpThreads) {
    const int b = c0 + t;
    const int nb = min(kMlpThreads, a.B - c0);
    float* h = H + (long)t * a.Hs;
    float* d = D + (long)t * a.Ds;
    if (b < a.B) {
      // ---- s' forwards (scratch = my D row, ping-pong): target max (Double: argmax by online)
      const int D0 = a.fin[0];
      for (int i = 0; i < D0; ++i) h[i] = a.xn[(long)b * D0 + i] * a.in_scale;
      float* sc[kMlpMaxLayers];
      for (int l = 0; l < a.L; ++l) sc[l] = d + (l & 1) * a.sw;
      int best = 0;
      if (a.double_dqn) {
        forward_row(a, Pw, h, sc);
        const float* qo = sc[a.L - 1];
        float bv = qo[0];
        for (int j = 1; j < A; ++j) if (qo[j] > bv) { bv = qo[j]; best = j; }
      }
      forward_row(a, a.w_tg, h, sc);
      const float* qt = sc[a.L - 1];
      if (!a.double_dqn) {
        float bv = qt[0];
        for (int j = 1; j < A; ++j) if (qt[j] > bv) { bv = qt[j]; best = j; }
      }
      const float qnext = qt[best];
      const float y = a.rew[b] + a.gam[b] * (1.f - a.done[b]) * qnext;
      // ---- online forward on s, activations kept
      for (int i = 0; i < D0; ++i) h[i] = a.x[(long)b * D0 + i] * a.in_scale;
      float* outs[kMlpMaxLayers];
      for (int l = 0; l < a.L; ++l) outs[l] = h + hoff[l + 1];
      forward_row(a, Pw, h, outs);
      const int at = a.act_idx[b];
      const float dd = outs[a.L - 1][at] - y;
      const float w = a.wts != nullptr ? a.wts[b] : 1.f;
      float per, dper;
      if (a.huber) {
        const float ad = fabsf(dd);
        per = ad <= a.delta ? 0.5f * dd * dd : a.delta * (ad - 0.5f * a.delta);
        dper = ad <= a.delta ? dd : copysignf(a.delta, dd);
      } else {
        per = dd * dd;
        dper = 2.f * dd;
      }
      loss_acc += w * per;
      a.prio[b] = fabsf(dd);
      // ---- backward to the deltas (output layer is affine)
      float* dl = d + doff[a.L - 1];
      for (int j = 0; j < A; ++j) dl[j] = (j == at) ? w * dper / (float)a.B : 0.f;
      for (int l = a.L - 1; l >= 1; --l) {
        const float* W = Pw + a.w_off[l];
        const int fi = a.fin[l], fo = a.fout[l];
        const float* dn = d + doff[l];
        float* dp = d + doff[l - 1];
        const float* hp = h + hoff[l];          // output of layer l-1
        for (int i = 0; i < fi; ++i) {
          float s = 0.f;
          for (int j = 0; j < fo; ++j) s = fmaf(dn[j], W[i * fo + j], s);
          dp[i] = s * act_grad(a.act[l - 1], hp[i]);
        }
      }
    }
    __syncthreads();
    // ---- weight / bias gradients of this chunk: G[p] += sum_b in[b][i] * delta[b][j]
    for (int l = 0; l < a.L; ++l) {
      const int fi = a.fin[l], fo = a.fout[l];
      for (int p = t; p < fi * fo + fo; p += kMlpThreads) {
        float s = 0.f;
        if (p < fi * fo) {
          const int i = p / fo, j = p - i * fo;
          for (int bb = 0; bb < nb; ++bb) s = fmaf(H[(long)bb * a.Hs + hoff[l] + i], D[(long)bb * a.Ds + doff[l] + j], s);
          G[a.w_off[l] + p] += s;
        } else {
          const int j = p - fi * fo;
          for (int bb = 0; bb < nb; ++bb) s += D[(long)bb * a.Ds + doff[l] + j];
          G[a.b_off[l] + j] += s;
        }
      }
    }
    __syncthreads();
  }
  // ---- write gradients (param ranges only; padding between tensors stays zero)
  for (int l = 0; l < a.L; ++l) {
    const int fi = a.fin[l], fo = a.fout[l];
    for (int p = t; p < fi * fo; p += kMlpThreads) a.grad[a.w_off[l] + p] = G[a.w_off[l] + p];
    for (int j = t; j < fo; j += kMlpThreads) a.grad[a.b_off[l] + j] = G[a.b_off[l] + j];
  }
  const float s = wave_sum(loss_acc);
  if ((t & 63) == 0) red[t >> 6] = s;
  __syncthreads();
  if (t == 0) {
    float tot = 0.f;
    for (int i = 0; i < kMlpThreads / 64; ++i) tot += red[i];
    a.loss[0] = tot / (float)a.B;
  }
}

}  // namespace dqn

size_t mlp_train_lds_bytes(const dqn::MlpArgs& a) {
  return sizeof(float) * (2 * (size_t)a.P + (size_t)dqn::kMlpThreads * (a.Hs + a.Ds));
}

int launch_mlp(const dqn::MlpArgs& a, int train, hipStream_t st) {
  if (a.L < 1 || a.L > dqn::kMlpMaxLayers || a.B < 1) return 1;
  for (int l = 0; l < a.L; ++l)
    if (a.fin[l] < 1 || a.fin[l] > dqn::kMlpMaxWidth || a.fout[l] < 1 || a.fout[l] > dqn::kMlpMaxWidth) return 2;
  if (a.fout[a.L - 1] != a.A) return 3;
  if (a.sw < a.fout[0] || 2 * a.sw > a.Ds) return 5;
  for (int l = 0; l < a.L; ++l) if (a.fout[l] > a.sw) return 5;
  if (!train) {
    const size_t lds = sizeof(float) * dqn::kMlpThreads * (a.fin[0] + 2 * a.sw + 1);
    hipLaunchKernelGGL(dqn::mlp_fwd_kernel, dim3((a.B + dqn::kMlpThreads - 1) / dqn::kMlpThreads),
                       dim3(dqn::kMlpThreads), lds, st, a);
    return 0;
  }
  const size_t lds = mlp_train_lds_bytes(a);
  if (lds > 160 * 1024) return 4;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dqn::mlp_train_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(dqn::mlp_train_kernel, dim3(1), dim3(dqn::kMlpThreads), lds, st, a);
  return 0;
}
