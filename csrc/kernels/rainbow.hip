// Rainbow pieces of the HIP executor: the C51 distributional head and the
// factorised-Gaussian noisy-layer parameter mix / gradient split.
//
// Reference: the reference has scalar heads only (/root/reference/src/network.py:401-409);
// C51 (Bellemare et al. 2017) and noisy nets (Fortunato et al. 2018) are the
// BASELINE.json config-5 extensions. Torch oracles: dist_dqn_amd/models/losses.py
// (c51_loss, categorical_projection) and models/torch_net.py (_dense with noise).
//
//   c51_train_kernel  training head, one wave64 per sample (lanes = atoms, N <= 64) on the
//                     precomputed igemm logits: dueling combine, Double-DQN action choice,
//                     categorical projection (per-wave LDS row), cross-entropy loss /
//                     priorities, and dL/dlogits as the bf16 dZ rows the dH igemm and the
//                     output layer's grouped weight-gradient members consume.
//   c51_infer_kernel  acting / q_values: Q = sum_n p_n z_n -> q_out / fused actor step.
//   noisy_mix_kernel  eff = mu + sigma * f(eps_in) f(eps_out)^T (f(x) = sgn(x) sqrt|x|),
//                     plain copy for deterministic tensors: the executor packs
//                     and reads the effective parameters from `eff`.
//   noisy_grad_kernel dL/dsigma = dL/dW_eff * f(eps_in) f(eps_out)^T (bias: * f(eps_out));
//                     the conv/dense backward writes dL/dW_eff into the mu slots.
#include "common.h"
#include "actor_dev.h"
#include "../include/dqn_nets_k.h"

namespace dqn {

typedef __attribute__((ext_vector_type(8))) act_t bfx8;

DQN_DEV bfx8 rz8() {
  bfx8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (act_t)0.f;
  return z;
}

// Row layout of the precomputed logits (one igemm over the combined output layer): KD floats
// per row = [plain / advantage logits (NO) | pad | dueling value logits (atoms) at VO | pad],
// VO = NO rounded up to 32 (the same columns as the dL/dlogits rows of dout16).
DQN_DEV_HOST_INLINE int c51_vo(const HeadArgs& a) { return (a.A * a.atoms + 31) / 32 * 32; }
DQN_DEV_HOST_INLINE int c51_kd(const HeadArgs& a) {
  return c51_vo(a) + (a.dueling ? (a.atoms + 31) / 32 * 32 : 0);
}

// logits of one instance from the precomputed igemm outputs (global fp32) into LDS
DQN_DEV void c51_load_logits(const HeadArgs& a, int inst, float* lg, float* vl, int tid, int nth, int B) {
  const int NA = a.atoms, NO = a.A * NA, KD = c51_kd(a), VO = c51_vo(a);
  const float* src = a.lgi[inst];
  for (int t = tid; t < B * NO; t += nth) lg[t] = src[(t / NO) * KD + t % NO];
  if (a.dueling)
    for (int t = tid; t < B * NA; t += nth) vl[t] = src[(t / NA) * KD + VO + t % NA];
}

DQN_DEV float c51_z(const HeadArgs& a, int n) {
  return a.vmin + (a.vmax - a.vmin) * (float)n / (float)(a.atoms - 1);
}

// dueling combine per atom, then in-place softmax of every (b, a) row: SIXTEEN LANES PER
// ROW (one DPP row; atom n = l16 + 16 i, i < 4, so atoms <= 64), max / sum reductions on
// DPP row ops (no LDS crossbar); q[b][i] = sum_n p_n z_n (action values: acting / q_values).
DQN_DEV void c51_softmax(const HeadArgs& a, float* lg, const float* vl, float* q, int tid, int nth, int B) {
  const int A = a.A, NA = a.atoms, NO = A * NA;
  if (a.dueling) {
    for (int t = tid; t < B * NA; t += nth) {
      const int b = t / NA, n = t - b * NA;
      float mean = 0.f;
      for (int i = 0; i < A; ++i) mean += lg[b * NO + i * NA + n];
      mean /= (float)A;
      const float v = vl[b * NA + n] - mean;
      for (int i = 0; i < A; ++i) lg[b * NO + i * NA + n] += v;
    }
    __syncthreads();
  }
  const int l16 = tid & 15;
  for (int row = tid >> 4; row < B * A; row += nth >> 4) {     // uniform per 16-lane group
    const int b = row / A, i = row - b * A;
    float* r = lg + b * NO + i * NA;
    float x[4];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = l16 + 16 * u;
      x[u] = n < NA ? r[n] : -INFINITY;
      mx = fmaxf(mx, x[u]);
    }
    mx = row16_max(mx);
    float e[4], s = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      e[u] = l16 + 16 * u < NA ? __expf(x[u] - mx) : 0.f;
      s += e[u];
    }
    s = row16_sum(s);
    const float inv = 1.f / s;
    float qs = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = l16 + 16 * u;
      if (n < NA) {
        const float p = e[u] * inv;
        r[n] = p;
        qs += p * c51_z(a, n);
      }
    }
    qs = row16_sum(qs);
    if (l16 == 0) q[row] = qs;
  }
  __syncthreads();
}

// LDS (floats) of the one-block softmax paths: logits [B][NO], value logits [B][NA], Q [B][A]
DQN_DEV_HOST_INLINE size_t c51_rows_floats(const HeadArgs& a, int rows) {
  return (size_t)rows * ((size_t)a.A * a.atoms + a.atoms + a.A);
}

// Acting / q_values: one block, Q = sum_n p_n z_n of every row -> q_out / fused actor step.
__global__ void __launch_bounds__(1024) c51_infer_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int B = a.B, NO = a.A * a.atoms;
  float* lg = sm;
  float* vl = lg + B * NO;
  float* q = vl + B * a.atoms;
  c51_load_logits(a, 0, lg, vl, threadIdx.x, blockDim.x, B);
  __syncthreads();
  c51_softmax(a, lg, vl, q, threadIdx.x, blockDim.x, B);
  if (a.q_out != nullptr)
    for (int t = threadIdx.x; t < B * a.A; t += blockDim.x) a.q_out[t] = q[t];
  if (a.has_actor) actor_step_block(a.actor, q, lg);       // (the probabilities are dead after q)
}

// ---------------------------------------------------------------- C51 training head
// ONE WAVE PER SAMPLE, lanes = atoms (N <= 64), every reduction on DPP rows + readlanes:
//   * all of the sample's logits loads (selection / target / online instances, every action
//     row + dueling value row) issued up front, from the igemm outputs;
//   * dueling combine per atom, per-action softmax of the selection instance -> Q -> a*
//     (Double DQN: online net on s'; else the target net);
//   * target distribution of a*, projected onto the support: two LDS float atomics per atom
//     into the wave's own 64-float row (a wave's LDS ops complete in order: no barrier);
//   * online log-softmax of the taken action, cross-entropy (= the priority), and
//     dL/dlogits = w/B (p - m) as act_t (loss-scaled) rows of dout16 [B][KD]: plain /
//     advantage logits in [0, NO) (dueling: times (i == a) - 1/A), value in [VO, VO + N).
// dout16 is the A operand of the dH igemm (dH = dout16 . [W | Wv]^T, ReLU-masked by h) and
// the dZ operand of the output layer's grouped weight-gradient members; its pad columns are
// never written (zero from allocation). Per-block loss partials go to loss_parts[block]
// (summed by the fc dgrad launch). Fused acting: one more block per env (c51_act_env_block).
constexpr int kC51Waves = 8, kC51Threads = 64 * kC51Waves, kC51MaxParts = 64;

// Fused acting, one block per env e (training launch): env e's logits rows -> wave 0 (lanes =
// atoms) -> Q row in LDS, while every thread writes the env's new frames (rng-only); then the
// decision / replay append and, in the last block to arrive, the actor state advance.
template <int AM>
DQN_DEV void c51_act_env_block(const HeadArgs& a, int e, SumtreeLds& st) {
  __shared__ float qs[32];
  __shared__ int flag;
  const ActorArgs& x = a.actor;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int A = a.A, NA = a.atoms, NO = A * NA;
  int64_t* prof = (a.prof != nullptr && tid == 0 && e == 0) ? a.prof : nullptr;
  if (prof) prof[16] = (int64_t)__builtin_amdgcn_s_memtime();
  const ActorPre pre = actor_prefetch(x);
  int32_t st_e[4] = {0, 0, 0, 0};                    // env e's frame stack (thread 0)
  if (tid == 0)
    for (int c = 0; c < 4; ++c) st_e[c] = x.stacks[(int64_t)e * x.K + min(c, x.K - 1)];
  const bool on = lane < NA;
  const int ln = on ? lane : 0;
  float xr[AM], v = 0.f;
  if (wave == 0) {                                   // the Q row's loads first ...
    const float* row = a.act_lgi + (int64_t)e * c51_kd(a);
#pragma unroll
    for (int i = 0; i < AM; ++i) xr[i] = row[min(i, A - 1) * NA + ln];
    v = a.dueling ? row[c51_vo(a) + ln] : 0.f;
  }
  actor_env_frames(x, e, pre);                       // ... the frames under their latency
  if (prof) prof[17] = (int64_t)__builtin_amdgcn_s_memtime();
  if (wave == 0) {
    if (a.dueling) {
      float mean = 0.f;
#pragma unroll
      for (int i = 0; i < AM; ++i) mean += i < A ? xr[i] : 0.f;
      v -= mean / (float)A;
    }
    const float z = c51_z(a, ln);
#pragma unroll
    for (int i = 0; i < AM; ++i) {
      const float xi = xr[i] + v;
      const float m = wave_max_dpp(on ? xi : -INFINITY);
      const float ex = on ? __expf(xi - m) : 0.f;
      const float qi = wave_sum_dpp(ex * z) / wave_sum_dpp(ex);
      if (lane == 0 && i < A) qs[i] = qi;
    }
  }
  __syncthreads();
  if (prof) prof[18] = (int64_t)__builtin_amdgcn_s_memtime();
  actor_env_finish(x, qs, e, pre, st_e, &flag, st);
  if (prof) prof[19] = (int64_t)__builtin_amdgcn_s_memtime();
}

DQN_DEV_HOST_INLINE int c51_learn_blocks(int B) {
  const int n = (B + kC51Waves - 1) / kC51Waves;
  return n < kC51MaxParts ? n : kC51MaxParts;
}

template <int AM>
__global__ void __launch_bounds__(kC51Threads) c51_train_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nlearn = (int)gridDim.x - (a.act_E > 0 ? a.act_E : 0);
  if ((int)blockIdx.x >= nlearn) {
    c51_act_env_block<AM>(a, (int)blockIdx.x - nlearn, *reinterpret_cast<SumtreeLds*>(sm));
    return;
  }
  const int B = a.B, A = a.A, NA = a.atoms, NO = A * NA;
  const int VO = c51_vo(a), KD = c51_kd(a);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool on = lane < NA;
  const int ln = on ? lane : 0;                 // clamped: loads of idle lanes stay in bounds
  const bool dbl = a.lgi[2] != nullptr;
  const float* lsel = a.lgi[dbl ? 2 : 1];       // action choice on s'
  const float* ltgt = a.lgi[1];                 // target distribution (same buffer without Double DQN)
  const float* lon = a.lgi[0];

  const float dz = (a.vmax - a.vmin) / (float)(NA - 1);
  const float z = c51_z(a, ln);
  const float inva = a.dueling ? 1.f / (float)A : 0.f;
  act_t* dout = reinterpret_cast<act_t*>(a.dq16);
  __shared__ float mrow[kC51Waves][64];          // per-wave projected target distribution
  // optional s_memtime phase stamps of learner block 0, wave 0 (scripts/probe_head.py)
  int64_t* prof = (a.prof != nullptr && blockIdx.x == 0 && wave == 0 && lane == 0) ? a.prof : nullptr;
#define C51_MARK(i) if (prof) prof[i] = (int64_t)__builtin_amdgcn_s_memtime()
  C51_MARK(0);
  float contrib = 0.f;
  for (int b = blockIdx.x * kC51Waves + wave; b < B; b += nlearn * kC51Waves) {
    float xs[AM], xt[AM], xo[AM];
    const int64_t r0 = (int64_t)b * KD + ln;
#pragma unroll
    for (int i = 0; i < AM; ++i) {
      const int ii = i < A ? i : 0;
      xs[i] = lsel[r0 + ii * NA];
      xt[i] = ltgt[r0 + ii * NA];
      xo[i] = lon[r0 + ii * NA];
    }
    const int64_t v0 = (int64_t)b * KD + (a.dueling ? VO : 0) + ln;   // (no dueling: an ignored in-row load)
    float vs = lsel[v0], vt = ltgt[v0], vo = lon[v0];
    const int act = a.act[b];
    const float rw = a.rew[b], gm = a.gam[b] * (1.f - a.done[b]);
    const float w = a.wts != nullptr ? a.wts[b] : 1.f;
    if (a.dueling) {                            // x_i += v - mean_j x_j, per atom
      float ms = 0.f, mt = 0.f, mo = 0.f;
#pragma unroll
      for (int i = 0; i < AM; ++i)
        if (i < A) { ms += xs[i]; mt += xt[i]; mo += xo[i]; }
      vs -= ms * inva; vt -= mt * inva; vo -= mo * inva;
#pragma unroll
      for (int i = 0; i < AM; ++i) { xs[i] += vs; xt[i] += vt; xo[i] += vo; }
    }
    // 1. action choice: Q_i = sum_n softmax(x_i)_n z_n, first maximum wins
    int best = 0;
    float bq = -INFINITY;
#pragma unroll
    for (int i = 0; i < AM; ++i) {            // (no early exit: the AM reduction chains interleave)
      const float m = wave_max_dpp(on ? xs[i] : -INFINITY);
      const float e = on ? __expf(xs[i] - m) : 0.f;
      const float qi = wave_sum_dpp(e * z) / wave_sum_dpp(e);
      if (i < A && qi > bq) { bq = qi; best = i; }
    }
    C51_MARK(1);
    // 2. target distribution of a* (register select: no dynamic register indexing)
    float xa = xt[0], xb = xo[0];
#pragma unroll
    for (int i = 1; i < AM; ++i) {
      if (i == best) xa = xt[i];
      if (i == act) xb = xo[i];
    }
    float pt;
    {
      const float m = wave_max_dpp(on ? xa : -INFINITY);
      const float e = on ? __expf(xa - m) : 0.f;
      pt = e / wave_sum_dpp(e);
    }
    C51_MARK(2);
    // 3. projection onto the support: each atom's mass to its floor / ceil neighbours through
    //    LDS float atomics into this wave's own row (in-order within the wave: no barrier)
    const float tz = fminf(fmaxf(rw + gm * z, a.vmin), a.vmax);
    const float bj = fminf((tz - a.vmin) / dz, (float)(NA - 1));
    float* mr = mrow[wave];
    mr[lane] = 0.f;
    if (on) {
      const float lo = floorf(bj), hi = ceilf(bj);
      atomicAdd(&mr[(int)lo], pt * (hi - bj + (lo == hi ? 1.f : 0.f)));
      atomicAdd(&mr[(int)hi], pt * (bj - lo));
    }
    const float mj = mr[lane];
    C51_MARK(3);
    // 4. online log-softmax of the taken action, cross-entropy, dL/dlogits
    const float m = wave_max_dpp(on ? xb : -INFINITY);
    const float e = on ? __expf(xb - m) : 0.f;
    const float s = wave_sum_dpp(e);
    const float logp = xb - m - __logf(s);
    const float ce = -wave_sum_dpp(on ? mj * logp : 0.f);
    const float dl = w / (float)B * (e / s - mj) * kLossScale;
    if (lane == 0) a.prio[b] = ce;
    contrib += w * ce;
    act_t* drow = dout + (int64_t)b * KD;
    if (on) {
#pragma unroll
      for (int i = 0; i < AM; ++i)
        if (i < A) drow[i * NA + lane] = (act_t)(dl * ((i == act ? 1.f : 0.f) - inva));
      if (a.dueling) drow[VO + lane] = (act_t)dl;
    }
    C51_MARK(4);
  }
  __shared__ float red[kC51Waves];
  if (lane == 0) red[wave] = contrib;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kC51Waves; ++i) t += red[i];
    a.loss_parts[blockIdx.x] = t;
  }
  C51_MARK(5);
#undef C51_MARK
}

// ------------------------------------------------------------------ noisy nets
DQN_DEV float fnoise(float x) { return copysignf(sqrtf(fabsf(x)), x); }

// Standard normals for the factorised noise: Box-Muller over Philox4x32-10 keyed by the run
// seed rng[0] at counter rng[1] (4 normals per Philox call) -> out0[0, n) then out1[0, n).
// Same seed on every DP rank -> the same noise everywhere (the fused optimizer derives the
// sigma gradients from the all-reduced mu gradients with it). ONE block: the counter bump
// after the barrier is ordered after every lane's read; graph-capturable (no host state).
__global__ void __launch_bounds__(1024) noise_normal_kernel(float* __restrict__ out0, float* __restrict__ out1,
                                                            int n, int64_t* __restrict__ rng) {
  const uint64_t seed = (uint64_t)rng[0], ctr = (uint64_t)rng[1];
  const int total = out1 != nullptr ? 2 * n : n;
  for (int q = threadIdx.x; 4 * q < total; q += blockDim.x) noise_normals4(out0, out1, n, seed, ctr, q);
  __syncthreads();
  if (threadIdx.x == 0) rng[1] = (int64_t)(ctr + 1);
}

__global__ void __launch_bounds__(256) noisy_mix_kernel(const float* __restrict__ flat, float* __restrict__ eff,
                                                        const float* __restrict__ noise,
                                                        const NoisyJob* __restrict__ jobs) {
  const NoisyJob j = jobs[blockIdx.y];
  const int n = j.K * j.N;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
    float v = flat[j.mu_off + t];
    if (j.sigma_off >= 0 && noise != nullptr) {
      const int k = t / j.N, c = t - k * j.N;
      const float fin = j.ein_off >= 0 ? fnoise(noise[j.ein_off + k]) : 1.f;
      v += flat[j.sigma_off + t] * fin * fnoise(noise[j.eout_off + c]);
    }
    eff[j.mu_off + t] = v;
  }
}

__global__ void __launch_bounds__(256) noisy_grad_kernel(float* __restrict__ grad, const float* __restrict__ noise,
                                                         const NoisyJob* __restrict__ jobs) {
  const NoisyJob j = jobs[blockIdx.y];
  if (j.sigma_off < 0) return;
  const int n = j.K * j.N;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
    const int k = t / j.N, c = t - k * j.N;
    const float fin = j.ein_off >= 0 ? fnoise(noise[j.ein_off + k]) : 1.f;
    grad[j.sigma_off + t] = grad[j.mu_off + t] * fin * fnoise(noise[j.eout_off + c]);
  }
}

}  // namespace dqn

using namespace dqn;

size_t c51_head_lds_bytes(const HeadArgs& a) {
  // training: the acting blocks' PER insert scratch (the rest is static); infer: B logits rows,
  // whose (dead) probabilities the fused actor's PER tree insert reuses.
  if (!a.infer) return a.act_E > 0 && a.actor.tsum != nullptr ? sizeof(SumtreeLds) : 0;   // acting blocks
  const size_t n = c51_rows_floats(a, a.B) * sizeof(float);
  return a.has_actor && a.actor.tsum != nullptr && n < sizeof(SumtreeLds) ? sizeof(SumtreeLds) : n;
}

int c51_train_blocks(const HeadArgs& a) { return c51_learn_blocks(a.B); }

void launch_c51_head(const HeadArgs& a, hipStream_t st) {
  const size_t lds = c51_head_lds_bytes(a);
  if (a.infer) {
    hipLaunchKernelGGL(c51_infer_kernel, dim3(1), dim3(1024), lds, st, a);
    return;
  }
  const dim3 grid(c51_learn_blocks(a.B) + (a.act_E > 0 ? a.act_E : 0));   // learner blocks + one per env
#define C51K(AM) hipLaunchKernelGGL(c51_train_kernel<AM>, grid, dim3(kC51Threads), lds, st, a)
  if (a.A <= 4) C51K(4);
  else if (a.A <= 8) C51K(8);
  else if (a.A <= 18) C51K(18);
  else C51K(32);
#undef C51K
}

void launch_noisy_mix(const float* flat, float* eff, const float* noise, const NoisyJob* jobs, int njobs,
                      int max_elems, hipStream_t st) {
  int g = (max_elems + 255) / 256;
  g = g < 1 ? 1 : (g > 512 ? 512 : g);
  hipLaunchKernelGGL(noisy_mix_kernel, dim3(g, njobs), dim3(256), 0, st, flat, eff, noise, jobs);
}

void launch_noise_normal(float* out0, float* out1, int n, int64_t* rng, hipStream_t st) {
  hipLaunchKernelGGL(noise_normal_kernel, dim3(1), dim3(1024), 0, st, out0, out1, n, rng);
}

void launch_noisy_grad(float* grad, const float* noise, const NoisyJob* jobs, int njobs, int max_elems,
                       hipStream_t st) {
  int g = (max_elems + 255) / 256;
  g = g < 1 ? 1 : (g > 512 ? 512 : g);
  hipLaunchKernelGGL(noisy_grad_kernel, dim3(g, njobs), dim3(256), 0, st, grad, noise, jobs);
}
