// Fused multi-tensor optimizer over the flat parameter buffer (TF-0.x exact).
//
// Reference: tf.train.{GradientDescent,Momentum,RMSProp,Adam,Adagrad,Adadelta,Ftrl}
// Optimizer.minimize() colocated with the variables on the parameter server
// (/root/reference/src/network.py:159-203) — one ApplyX op per variable plus
// the separate L2 term in the loss (network.py:151-152,311,407).
//
// Here: ONE launch for all parameters; float4 vector loads; per element
//   g = grad * grad_scale (+ reg * w for flat[:reg_end])   -- 1/world DP averaging folded in
// then the TF update rule. Adam's beta powers (TF non-slot variables) are
// read by every block and advanced by the LAST block to finish (arrival
// ticket), together with global_step, so no extra launch is needed.
#include "common.h"
#include "../include/dqn_kernels.h"

namespace dqn {

struct OptHP {
  float lr, reg, grad_scale;
  float momentum, rho, rms_mom, rms_eps, b1, b2, adam_eps, ad_rho, ad_eps;
  int reg_end;
};

// Contraction is pinned off in the update math so every kernel that inlines it
// (optim_kernel's float4 loop, optim_pack_kernel's tiles) rounds identically:
// with fp-contract=fast the backend fuses differently per call site.
DQN_DEV float opt_grad(float g, float w, bool reg, const OptHP& h) {
#pragma clang fp contract(off)
  float x = g * h.grad_scale;
  if (reg) x += h.reg * w;
  return x;
}

template <int OP>
DQN_DEV void update_one(float& w, float g, float& s0, float& s1, const OptHP& h, float lr_t) {
#pragma clang fp contract(off)
  if constexpr (OP == 0) {            // sgd
    w -= h.lr * g;
  } else if constexpr (OP == 1) {     // momentum (non-Nesterov)
    s0 = h.momentum * s0 + g;
    w -= h.lr * s0;
  } else if constexpr (OP == 2) {     // rmsprop: ms (init 1), mom
    s0 = h.rho * s0 + (1.f - h.rho) * g * g;
    s1 = h.rms_mom * s1 + h.lr * g / sqrtf(s0 + h.rms_eps);
    w -= s1;
  } else if constexpr (OP == 3) {     // adam (TF epsilon-hat form)
    s0 = h.b1 * s0 + (1.f - h.b1) * g;
    s1 = h.b2 * s1 + (1.f - h.b2) * g * g;
    w -= lr_t * s0 / (sqrtf(s1) + h.adam_eps);
  } else if constexpr (OP == 4) {     // adagrad (accumulator init 0.1)
    s0 += g * g;
    w -= h.lr * g / sqrtf(s0);
  } else if constexpr (OP == 5) {     // adadelta
    s0 = h.ad_rho * s0 + (1.f - h.ad_rho) * g * g;
    const float upd = sqrtf(s1 + h.ad_eps) / sqrtf(s0 + h.ad_eps) * g;
    s1 = h.ad_rho * s1 + (1.f - h.ad_rho) * upd * upd;
    w -= h.lr * upd;
  } else {                            // ftrl (lr_power -0.5, l1 = l2 = 0)
    const float na = s0 + g * g;
    s1 += g - (sqrtf(na) - sqrtf(s0)) / h.lr * w;
    const float quad = sqrtf(na) / h.lr;
    w = fabsf(s1) > 0.f ? -s1 / quad : 0.f;
    s0 = na;
  }
}

template <int OP>
__global__ void __launch_bounds__(256)
optim_kernel(float* __restrict__ w, const float* __restrict__ grad, float* __restrict__ s0,
             float* __restrict__ s1, float* __restrict__ beta_pow, int64_t* __restrict__ step,
             int32_t* __restrict__ ticket, OptHP h, int n4, float* __restrict__ tgt, int tfreq) {
  float lr_t = h.lr;
  // fused hard target sync: this update makes global_step s+1; the reference copies
  // target <- online after the train step when (s+1) % target_update_freq == 0
  const bool sync = tgt != nullptr && step != nullptr && ((step[0] + 1) % tfreq) == 0;
  float4* T = reinterpret_cast<float4*>(tgt);
  if constexpr (OP == 3) {
    const float b1p = beta_pow[0], b2p = beta_pow[1];
    lr_t = h.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  }
  float4* W = reinterpret_cast<float4*>(w);
  const float4* G = reinterpret_cast<const float4*>(grad);
  float4* S0 = reinterpret_cast<float4*>(s0);
  float4* S1 = reinterpret_cast<float4*>(s1);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    float4 wv = W[i], gv = G[i];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if constexpr (OP != 0) a = S0[i];
    if constexpr (OP == 2 || OP == 3 || OP == 5 || OP == 6) b = S1[i];
    const bool reg = (i * 4) < h.reg_end;       // reg_end is a multiple of 64
    float ww[4] = {wv.x, wv.y, wv.z, wv.w}, gg[4] = {gv.x, gv.y, gv.z, gv.w};
    float aa[4] = {a.x, a.y, a.z, a.w}, bb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      update_one<OP>(ww[j], opt_grad(gg[j], ww[j], reg, h), aa[j], bb[j], h, lr_t);
    }
    const float4 nw = make_float4(ww[0], ww[1], ww[2], ww[3]);
    W[i] = nw;
    if (sync) T[i] = nw;
    if constexpr (OP != 0) S0[i] = make_float4(aa[0], aa[1], aa[2], aa[3]);
    if constexpr (OP == 2 || OP == 3 || OP == 5 || OP == 6) S1[i] = make_float4(bb[0], bb[1], bb[2], bb[3]);
  }
  // last block advances global_step and (Adam) the beta powers. Every block
  // read beta_pow above, before its ticket add, so the update cannot race.
  if (threadIdx.x == 0) {
    // relaxed: the last arriver only WRITES beta_pow/step; every block's read of
    // beta_pow completed (value consumed in the loop) before its ticket add.
    // (An acq_rel agent atomic here costs an L2 writeback + invalidate per block.)
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (int)gridDim.x - 1) {
      if (step) step[0] += 1;
      if constexpr (OP == 3) {
        beta_pow[0] *= h.b1;
        beta_pow[1] *= h.b2;
      }
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}


// ------------------------------------------------------------- update + pack
// The optimizer step fused with the executor's weight packing: a workgroup owns
// a 32 (k) x 64 (n) tile of a weight matrix (TF layout [K][N]), updates it in
// registers (8 consecutive n per thread), writes fp32 weights + slots back, and
// emits the tile's bf16 MFMA fragments straight away:
//   * forward fragments ([K/32][N/16][64][8]: 8 consecutive k per lane) through
//     one LDS transpose of the tile;
//   * dgrad fragments (dense transpose, or conv (tap, co) x ci) directly from the
//     thread's registers: their 8 consecutive K' ARE 8 consecutive n of one row.
// Elementwise items (biases, ...) carry an optional fp32 copy into the packed
// buffer (the concatenated fc bias). Same ticket as optim_kernel; the hard target
// sync writes the target's fp32 master and packed fragments under the predicate.
typedef __attribute__((ext_vector_type(8))) act_t bfx8;

constexpr int kTicketSubs = 16, kTicketStride = 32;    // hierarchical ticket: int32 words

struct UpdJob {
  int kind;                      // 0 = tile, 1 = elementwise chunk
  int src_off, K, N, k0, n0;     // tile: tensor offset / shape / origin; elem: offset, count (K)
  int fwd_off, fwd_N16, fwd_nt_off, fwd_ks_off;   // forward fragments (elem: fp32 copy offset or -1)
  int dg_mode, dg_off, dg_N16, dg_nt_off, dg_ks_off, dg_cin;   // dgrad: 0 none, 1 conv, 2 dense
};

template <int OP>
DQN_DEV void upd8(float* w, const float* g, float* a, float* b, int k0flat, int reg_end, const OptHP& h,
                  float lr_t, bool* ok) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (!ok[j]) continue;
    update_one<OP>(w[j], opt_grad(g[j], w[j], k0flat + j < reg_end, h), a[j], b[j], h, lr_t);
  }
}

template <int OP>
__global__ void __launch_bounds__(256)
optim_pack_kernel(float* __restrict__ W, const float* __restrict__ G, float* __restrict__ S0, float* __restrict__ S1,
                  float* __restrict__ beta_pow, int64_t* __restrict__ step, int32_t* __restrict__ ticket, OptHP h,
                  const UpdJob* __restrict__ jobs, int njobs, act_t* __restrict__ packed, float* __restrict__ tgt,
                  act_t* __restrict__ tgt_packed, int tfreq, int hier) {
  __shared__ __attribute__((aligned(16))) act_t tile[32 * 72];
  float lr_t = h.lr;
  if constexpr (OP == 3) {
    const float b1p = beta_pow[0], b2p = beta_pow[1];
    lr_t = h.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  }
  const bool sync = tgt != nullptr && step != nullptr && ((step[0] + 1) % tfreq) == 0;
  constexpr bool TWO = OP == 2 || OP == 3 || OP == 5 || OP == 6;
  const int t = threadIdx.x;
  for (int ji = blockIdx.x; ji < njobs; ji += gridDim.x) {
    const UpdJob jb = jobs[ji];
    float w[8], g[8], a[8], b[8];
    bool ok[8];
    if (jb.kind == 1) {                                   // elementwise chunk of up to 2048
      const int base = jb.src_off + t * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ok[j] = t * 8 + j < jb.K;
        const int i = base + j;
        w[j] = ok[j] ? W[i] : 0.f; g[j] = ok[j] ? G[i] : 0.f;
        a[j] = (OP != 0 && ok[j]) ? S0[i] : 0.f; b[j] = (TWO && ok[j]) ? S1[i] : 0.f;
      }
      upd8<OP>(w, g, a, b, base, h.reg_end, h, lr_t, ok);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (!ok[j]) continue;
        const int i = base + j;
        W[i] = w[j];
        if constexpr (OP != 0) S0[i] = a[j];
        if constexpr (TWO) S1[i] = b[j];
        if (sync) tgt[i] = w[j];
        if (jb.fwd_off >= 0) {                            // fp32 copy inside the packed buffer
          reinterpret_cast<float*>(packed + jb.fwd_off)[t * 8 + j] = w[j];
          if (sync) reinterpret_cast<float*>(tgt_packed + jb.fwd_off)[t * 8 + j] = w[j];
        }
      }
      continue;
    }
    // ---- tile: row r, 8 columns c8..c8+7
    const int r = t >> 3, c8 = (t & 7) * 8;
    const int k = jb.k0 + r, n = jb.n0 + c8;
    const int64_t e0 = (int64_t)jb.src_off + (int64_t)k * jb.N + n;
    const bool rowok = k < jb.K;
    const bool vec = rowok && n + 8 <= jb.N && (jb.N % 4) == 0;
    if (vec) {
      const float4* W4 = reinterpret_cast<const float4*>(W + e0);
      const float4* G4 = reinterpret_cast<const float4*>(G + e0);
      const float4 w0 = W4[0], w1 = W4[1], g0 = G4[0], g1 = G4[1];
      w[0] = w0.x; w[1] = w0.y; w[2] = w0.z; w[3] = w0.w; w[4] = w1.x; w[5] = w1.y; w[6] = w1.z; w[7] = w1.w;
      g[0] = g0.x; g[1] = g0.y; g[2] = g0.z; g[3] = g0.w; g[4] = g1.x; g[5] = g1.y; g[6] = g1.z; g[7] = g1.w;
      if constexpr (OP != 0) {
        const float4 a0 = reinterpret_cast<const float4*>(S0 + e0)[0], a1 = reinterpret_cast<const float4*>(S0 + e0)[1];
        a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w; a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
      }
      if constexpr (TWO) {
        const float4 b0 = reinterpret_cast<const float4*>(S1 + e0)[0], b1 = reinterpret_cast<const float4*>(S1 + e0)[1];
        b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ok[j] = true;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ok[j] = rowok && n + j < jb.N;
        const int64_t i = e0 + j;
        w[j] = ok[j] ? W[i] : 0.f; g[j] = ok[j] ? G[i] : 0.f;
        a[j] = (OP != 0 && ok[j]) ? S0[i] : 0.f; b[j] = (TWO && ok[j]) ? S1[i] : 0.f;
      }
    }
    upd8<OP>(w, g, a, b, (int)e0, h.reg_end, h, lr_t, ok);
    if (vec) {
      float4* W4 = reinterpret_cast<float4*>(W + e0);
      W4[0] = make_float4(w[0], w[1], w[2], w[3]); W4[1] = make_float4(w[4], w[5], w[6], w[7]);
      if (sync) {
        float4* T4 = reinterpret_cast<float4*>(tgt + e0);
        T4[0] = W4[0]; T4[1] = W4[1];
      }
      if constexpr (OP != 0) {
        float4* A4 = reinterpret_cast<float4*>(S0 + e0);
        A4[0] = make_float4(a[0], a[1], a[2], a[3]); A4[1] = make_float4(a[4], a[5], a[6], a[7]);
      }
      if constexpr (TWO) {
        float4* B4 = reinterpret_cast<float4*>(S1 + e0);
        B4[0] = make_float4(b[0], b[1], b[2], b[3]); B4[1] = make_float4(b[4], b[5], b[6], b[7]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (!ok[j]) continue;
        const int64_t i = e0 + j;
        W[i] = w[j];
        if constexpr (OP != 0) S0[i] = a[j];
        if constexpr (TWO) S1[i] = b[j];
        if (sync) tgt[i] = w[j];
      }
    }
    bfx8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (act_t)(ok[j] ? w[j] : 0.f);
    // dgrad fragments straight from the registers
    if (jb.dg_mode != 0 && rowok) {
      int kp, np;                                        // K' of the first of the 8 values, N'
      if (jb.dg_mode == 2) { kp = n; np = k; }           // dense: K' = out (n), N' = in (k)
      else { const int tap = k / jb.dg_cin, ci = k - tap * jb.dg_cin; kp = tap * jb.N + n; np = ci; }
      const int lane = ((kp & 31) >> 3) * 16 + (np & 15);
      const int64_t o = jb.dg_off + ((int64_t)((jb.dg_ks_off + (kp >> 5)) * jb.dg_N16 + jb.dg_nt_off + (np >> 4)) * 64 + lane) * 8;
      if (n < jb.N) {
        *reinterpret_cast<bfx8*>(packed + o) = v;
        if (sync) *reinterpret_cast<bfx8*>(tgt_packed + o) = v;
      }
    }
    // forward fragments through an LDS transpose of the bf16 tile
    *reinterpret_cast<bfx8*>(tile + r * 72 + c8) = v;
    __syncthreads();
    {
      const int nt = t >> 6, l = t & 63, nl = nt * 16 + (l & 15), kk = 8 * (l >> 4);
      if (jb.n0 + nt * 16 < jb.N) {
        bfx8 f;
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = tile[(kk + j) * 72 + nl];
        const int64_t o = jb.fwd_off + ((int64_t)((jb.fwd_ks_off + (jb.k0 >> 5)) * jb.fwd_N16 + jb.fwd_nt_off +
                                                  ((jb.n0 >> 4) + nt)) * 64 + l) * 8;
        *reinterpret_cast<bfx8*>(packed + o) = f;
        if (sync) *reinterpret_cast<bfx8*>(tgt_packed + o) = f;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    bool last;
    if (hier) {
      // two-level arrival ticket (one block per job: ~1k arrivals): blocks count into one
      // of 16 sub-tickets on their own 128-byte lines; each sub-ticket's last arriver
      // counts into the top ticket, whose last arriver is the grid's last block
      const int j = blockIdx.x & (kTicketSubs - 1);
      const int members = ((int)gridDim.x - j + kTicketSubs - 1) / kTicketSubs;
      int32_t* sub = ticket + kTicketStride * (1 + j);
      last = false;
      if (__hip_atomic_fetch_add(sub, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == members - 1) {
        __hip_atomic_store(sub, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int nsub = (int)gridDim.x < kTicketSubs ? (int)gridDim.x : kTicketSubs;
        last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsub - 1;
      }
    } else {
      last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
    }
    if (last) {
      if (step) step[0] += 1;
      if constexpr (OP == 3) {
        beta_pow[0] *= h.b1;
        beta_pow[1] *= h.b2;
      }
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// target <- tau * online + (1 - tau) * target, optionally only when step % freq == 0.
__global__ void __launch_bounds__(256)
target_update_kernel(float* __restrict__ dst, const float* __restrict__ src, float tau,
                     const int64_t* __restrict__ step, int freq, int n4, float* __restrict__ dst2,
                     const float* __restrict__ src2, int n4b) {
  if (step != nullptr && (step[0] % freq) != 0) return;
  if (dst2 != nullptr) {   // hard copy of a second buffer pair (packed bf16 weights)
    float4* D2 = reinterpret_cast<float4*>(dst2);
    const float4* S2 = reinterpret_cast<const float4*>(src2);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4b; i += gridDim.x * blockDim.x) D2[i] = S2[i];
  }
  float4* D = reinterpret_cast<float4*>(dst);
  const float4* S = reinterpret_cast<const float4*>(src);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    float4 s = S[i];
    if (tau >= 1.f) {
      D[i] = s;
    } else {
      float4 d = D[i];
      const float k = 1.f - tau;
      D[i] = make_float4(tau * s.x + k * d.x, tau * s.y + k * d.y, tau * s.z + k * d.z, tau * s.w + k * d.w);
    }
  }
}

__global__ void step_bump_kernel(int64_t* step) { step[0] += 1; }

}  // namespace dqn

using namespace dqn;

static int grid_for(int n4) {
  int g = (n4 + 255) / 256;
  return g < 1 ? 1 : (g > 2048 ? 2048 : g);
}

// The optimizer's arrival ticket is one atomic word: keep the grid at one
// block per CU (grid-stride) so the ticket sees <= 256 arrivals, not ~1.6k.
static int grid_for_ticket(int n4) {
  int g = (n4 + 255) / 256;
  return g < 1 ? 1 : (g > 256 ? 256 : g);
}

void launch_optimizer_step(int op, float* w, const float* g, float* s0, float* s1, float* beta_pow,
                           int64_t* step, int32_t* ticket, const float* hp9, float lr, float reg, int reg_end,
                           float grad_scale, int n, float* tgt, int tfreq, hipStream_t st) {
  OptHP h;
  h.lr = lr; h.reg = reg; h.grad_scale = grad_scale; h.reg_end = reg_end;
  h.momentum = hp9[0]; h.rho = hp9[1]; h.rms_mom = hp9[2]; h.rms_eps = hp9[3];
  h.b1 = hp9[4]; h.b2 = hp9[5]; h.adam_eps = hp9[6]; h.ad_rho = hp9[7]; h.ad_eps = hp9[8];
  const int n4 = n / 4;
  dim3 grid(grid_for_ticket(n4)), block(256);
  switch (op) {
    case 0: hipLaunchKernelGGL(optim_kernel<0>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 1: hipLaunchKernelGGL(optim_kernel<1>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 2: hipLaunchKernelGGL(optim_kernel<2>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 3: hipLaunchKernelGGL(optim_kernel<3>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 4: hipLaunchKernelGGL(optim_kernel<4>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 5: hipLaunchKernelGGL(optim_kernel<5>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 6: hipLaunchKernelGGL(optim_kernel<6>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    default: break;
  }
}

void launch_optim_pack(int op, float* w, const float* g, float* s0, float* s1, float* beta_pow, int64_t* step,
                       int32_t* ticket, const float* hp9, float lr, float reg, int reg_end, float grad_scale,
                       const void* jobs, int njobs, void* packed, float* tgt, void* tgt_packed, int tfreq,
                       int max_grid, hipStream_t st) {
  OptHP h;
  h.lr = lr; h.reg = reg; h.grad_scale = grad_scale; h.reg_end = reg_end;
  h.momentum = hp9[0]; h.rho = hp9[1]; h.rms_mom = hp9[2]; h.rms_eps = hp9[3];
  h.b1 = hp9[4]; h.b2 = hp9[5]; h.adam_eps = hp9[6]; h.ad_rho = hp9[7]; h.ad_eps = hp9[8];
  // max_grid <= 256: grid-stride over the jobs with a flat ticket (<= 256 arrivals);
  // larger: one block per job (up to max_grid) with the two-level ticket
  const int cap = max_grid > 256 ? max_grid : 256;
  const int grid = njobs < cap ? njobs : cap;
  const int hier = grid > 256 ? 1 : 0;
  const UpdJob* J = reinterpret_cast<const UpdJob*>(jobs);
  act_t* P = reinterpret_cast<act_t*>(packed);
  act_t* TP = reinterpret_cast<act_t*>(tgt_packed);
  const int tf = tfreq < 1 ? 1 : tfreq;
#define OPK(N) hipLaunchKernelGGL(optim_pack_kernel<N>, dim3(grid), dim3(256), 0, st, w, g, s0, s1, beta_pow, step, \
                                  ticket, h, J, njobs, P, tgt, TP, tf, hier)
  switch (op) {
    case 0: OPK(0); break; case 1: OPK(1); break; case 2: OPK(2); break; case 3: OPK(3); break;
    case 4: OPK(4); break; case 5: OPK(5); break; case 6: OPK(6); break;
    default: break;
  }
#undef OPK
}

int upd_job_ints() { return (int)(sizeof(UpdJob) / sizeof(int)); }

void launch_target_update(float* dst, const float* src, float tau, const int64_t* step, int freq, int n,
                          float* dst2, const float* src2, int n2, hipStream_t st) {
  const int n4 = n / 4;
  hipLaunchKernelGGL(target_update_kernel, dim3(grid_for(n4)), dim3(256), 0, st, dst, src, tau, step,
                     freq < 1 ? 1 : freq, n4, dst2, src2, n2 / 4);
}

void launch_step_bump(int64_t* step, hipStream_t st) {
  hipLaunchKernelGGL(step_bump_kernel, dim3(1), dim3(1), 0, st, step);
}
