// Rainbow pieces of the HIP executor: the C51 distributional head and the
// factorised-Gaussian noisy-layer parameter mix / gradient split.
//
// Reference: the reference has scalar heads only (/root/reference/src/network.py:401-409);
// C51 (Bellemare et al. 2017) and noisy nets (Fortunato et al. 2018) are the
// BASELINE.json config-5 extensions. Torch oracles: dist_dqn_amd/models/losses.py
// (c51_loss, categorical_projection) and models/torch_net.py (_dense with noise).
//
//   c51_head_kernel   logits [B][A*N] (+ dueling value [B][N]) on MFMA for up to
//                     3 instances, dueling combine per atom, softmax with one
//                     wave64 per (sample, action) row (lanes = atoms, N <= 64),
//                     Double-DQN action choice, categorical projection through
//                     LDS float atomics, cross-entropy loss / priorities, and the
//                     output-layer backward (dW, db, dWv, dbv, dH masked by ReLU).
//                     Acting mode: Q = sum_n p_n z_n -> q_out / fused actor step.
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

// logits of one instance -> lg [B][NO] (+ vl [B][NA] for dueling), bias added
DQN_DEV void c51_logits(const HeadArgs& a, int inst, float* lg, float* vl, int lane, int wave, int nwave,
                        int64_t* prof = nullptr) {
  const int B = a.B, NA = a.atoms, NO = a.A * NA, HID = a.HID, HH = a.dueling ? 2 * HID : HID;
  const int N16 = (NO + 15) / 16, N16v = (NA + 15) / 16, mtiles = (B + 15) / 16, K32 = HID / 32;
  const int ntask = mtiles * (N16 + (a.dueling ? N16v : 0));
  const bfx8* pw = reinterpret_cast<const bfx8*>(a.pw[inst]);
  const bfx8* pv = reinterpret_cast<const bfx8*>(a.pwv[inst]);
  const int kg = 8 * (lane >> 4);
  int pi = 0;
  for (int task = wave; task < ntask; task += nwave) {
    if (prof) prof[pi++] = (int64_t)__builtin_amdgcn_s_memtime();
    const int mt = task % mtiles, t2 = task / mtiles;
    const bool val = t2 >= N16;                              // dueling value-stream tile
    const int nt = val ? t2 - N16 : t2;
    const int b_row = mt * 16 + (lane & 15);
    const bool rok = b_row < B;
    const act_t* hrow = reinterpret_cast<const act_t*>(a.h[inst]) + (int64_t)(rok ? b_row : 0) * HH;
    const act_t* src = (a.dueling && !val) ? hrow + HID : hrow;  // [value | advantage] halves of h
    const bfx8* W = val ? pv : pw;
    const int n16 = val ? N16v : N16;
    const int col0 = nt * 16 + (lane & 15);
    const float bias_pre = val ? (col0 < NA ? a.bv[inst][col0] : 0.f) : (col0 < NO ? a.b[inst][col0] : 0.f);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < K32; ks += 8) {           // 8 k-steps of loads in flight per batch
      bfx8 af[8], bf[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool kok = ks + u < K32;
        af[u] = rok && kok ? *reinterpret_cast<const bfx8*>(src + (ks + u) * 32 + kg) : rz8();
        bf[u] = kok ? W[((ks + u) * n16 + nt) * 64 + lane] : rz8();
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = DQN_MFMA16_BUILTIN(af[u], bf[u], acc, 0, 0, 0);
    }
    const int col = nt * 16 + (lane & 15);
    const float bias = bias_pre;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = mt * 16 + 4 * (lane >> 4) + r;
      if (b >= B) continue;
      if (val) {
        if (col < NA) vl[b * NA + col] = acc[r] + bias;
      } else if (col < NO) {
        lg[b * NO + col] = acc[r] + bias;
      }
    }
  }
  if (prof) prof[pi++] = (int64_t)__builtin_amdgcn_s_memtime();
}

// logits of one instance from the precomputed igemm outputs (global fp32) into LDS
DQN_DEV void c51_load_logits(const HeadArgs& a, int inst, float* lg, float* vl, int tid, int nth) {
  const int B = a.B, NA = a.atoms, NO = a.A * NA;
  const float* src = a.lgi[inst];
  for (int t = tid; t < B * NO; t += nth) lg[t] = src[t];
  if (a.dueling) {
    const float* sv = a.vli[inst];
    for (int t = tid; t < B * NA; t += nth) vl[t] = sv[t];
  }
}

DQN_DEV float c51_z(const HeadArgs& a, int n) {
  return a.vmin + (a.vmax - a.vmin) * (float)n / (float)(a.atoms - 1);
}

// dueling combine per atom, then in-place softmax of every (b, a) row: SIXTEEN LANES PER
// ROW (one DPP row; atom n = l16 + 16 i, i < 4, so atoms <= 64), max / sum reductions on
// DPP row ops (no LDS crossbar). If logp != nullptr the log-probabilities of each
// sample's TAKEN action row are kept there ([B][NA]); if q != nullptr the expected value
// q[b][i] = sum_n p_n z_n is written too (action selection / acting).
DQN_DEV void c51_softmax(const HeadArgs& a, float* lg, const float* vl, float* logp, float* q, int tid, int nth,
                         int B) {
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
    const bool keep = logp != nullptr && i == a.act[b];
    const float ls = keep ? __logf(s) : 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = l16 + 16 * u;
      if (n < NA) {
        const float p = e[u] * inv;
        r[n] = p;
        qs += p * c51_z(a, n);
        if (keep) logp[b * NA + n] = x[u] - mx - ls;
      }
    }
    if (q != nullptr) {
      qs = row16_sum(qs);
      if (l16 == 0) q[row] = qs;
    }
  }
  __syncthreads();
}

DQN_DEV void c51_rows_softmax(const HeadArgs& a, float* pc, float* logp, int tid, int nth);

// Only ONE action row per sample matters for the target (a*) and online (taken action)
// distributions: combine (dueling: v + adv_i - mean_j adv_j) straight from the precomputed
// global logits into a compact [B][NA] LDS buffer and softmax those B rows (16 lanes per
// row) instead of staging and normalising all B*A rows. logp (optional): log-probabilities.
DQN_DEV void c51_rows(const HeadArgs& a, const float* src, const float* vsrc, const int32_t* rows, float* pc,
                      float* logp, int tid, int nth) {
  const int B = a.B, A = a.A, NA = a.atoms, NO = A * NA;
  for (int t = tid; t < B * NA; t += nth) {
    const int b = t / NA, n = t - b * NA;
    const float* col = src + b * NO + n;
    float x = col[rows[b] * NA];
    if (a.dueling) {
      float mean = 0.f;
      for (int i = 0; i < A; ++i) mean += col[i * NA];
      mean /= (float)A;
      const float v = vsrc[b * NA + n] - mean;
      x += v;
    }
    pc[t] = x;
  }
  __syncthreads();
  c51_rows_softmax(a, pc, logp, tid, nth);
}

// in-place softmax of the B compact rows pc[b][0..NA) (16 lanes per row)
DQN_DEV void c51_rows_softmax(const HeadArgs& a, float* pc, float* logp, int tid, int nth) {
  const int B = a.B, NA = a.atoms;
  const int l16 = tid & 15;
  for (int b = tid >> 4; b < B; b += nth >> 4) {               // uniform per 16-lane group
    float* r = pc + b * NA;
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
    const float ls = logp != nullptr ? __logf(s) : 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = l16 + 16 * u;
      if (n < NA) {
        r[n] = e[u] * inv;
        if (logp != nullptr) logp[b * NA + n] = x[u] - mx - ls;
      }
    }
  }
  __syncthreads();
}

// LDS plan of the training head (floats). Base: lg [B][NO], vl / mt / lp [B][NA],
// q [B][A], red [32], astar [B], actor scratch [E], pc [B][NA]. Staged (when it fits one CU's 160 KB): the
// target and online logits [B][NO] + [B][NA] each, and act / rew / gam / done / wts [B].
DQN_DEV_HOST_INLINE size_t c51_base_floats(const HeadArgs& a) {
  const size_t B = a.B, NA = a.atoms, NO = (size_t)a.A * NA;
  return B * NO + 4 * B * NA + B * a.A + 32 + B + (a.has_actor ? a.actor.E : 0);
}
DQN_DEV_HOST_INLINE size_t c51_stage_floats(const HeadArgs& a) {
  return 2 * ((size_t)a.B * a.A * a.atoms + (size_t)a.B * a.atoms) + 5 * (size_t)a.B;
}
DQN_DEV_HOST_INLINE bool c51_staged(const HeadArgs& a) {
  const bool dbl = a.h[2] != nullptr;
  return !a.infer && a.lgi[0] != nullptr && a.lgi[1] != nullptr && (!dbl || a.lgi[2] != nullptr) &&
         (c51_base_floats(a) + c51_stage_floats(a)) * sizeof(float) <= 160 * 1024;
}

// Every input phases 1-3 read, in ONE batch of global loads per thread instead of one
// dependent round trip per phase: the selection instance's logits into lg / vl, the target
// (Double DQN) and online logits into lgT / vlT / lgO / vlO, and the per-sample scalars into
// sc = [act | rew | gam | done | wts]. Fixed-size register batches from fixed base pointers
// (no pointer tables: those land in scratch); elements beyond a batch take a plain loop.
constexpr int kStageLg = 10, kStageV = 2;   // per-thread batch: B*NO <= 10 * 1024, B*NA <= 2 * 1024
template <int U>
DQN_DEV void stage_ld(const float* src, int n, int tid, int nth, float (&r)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = tid + u * nth;
    r[u] = src[t < n ? t : 0];                  // (t >= n: re-reads element 0, discarded)
  }
}
template <int U>
DQN_DEV void stage_st(float* dst, const float* src, int n, int tid, int nth, const float (&r)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = tid + u * nth;
    if (t < n) dst[t] = r[u];
  }
  for (int t = tid + U * nth; t < n; t += nth) dst[t] = src[t];
}
DQN_DEV void c51_stage(const HeadArgs& a, int ninst, float* lg, float* vl, float* lgT, float* vlT, float* lgO,
                       float* vlO, float* sc, int tid, int nth) {
  const int B = a.B, NA = a.atoms, NO = a.A * NA, NV = a.dueling ? B * NA : 0;
  const int sel = ninst == 3 ? 2 : 1;
  const bool dbl = ninst == 3;
  const float* any = a.lgi[0];                // valid base for empty segments
  const float* l0 = a.lgi[sel];
  const float* l1 = dbl ? a.lgi[1] : any;
  const float* l2 = a.lgi[0];
  const float* v0 = NV ? a.vli[sel] : any;
  const float* v1 = NV && dbl ? a.vli[1] : any;
  const float* v2 = NV ? a.vli[0] : any;
  const int n1 = dbl ? B * NO : 0, nv1 = dbl ? NV : 0;
  float r0[kStageLg], r1[kStageLg], r2[kStageLg], q0[kStageV], q1[kStageV], q2[kStageV];
  stage_ld(l0, B * NO, tid, nth, r0);
  stage_ld(l1, n1, tid, nth, r1);
  stage_ld(l2, B * NO, tid, nth, r2);
  stage_ld(v0, NV, tid, nth, q0);
  stage_ld(v1, nv1, tid, nth, q1);
  stage_ld(v2, NV, tid, nth, q2);
  const int sg = tid / B, sb = tid - sg * B;   // scalars: thread tid < 4B loads one
  const float* sp = sg == 0 ? reinterpret_cast<const float*>(a.act) : sg == 1 ? a.rew : sg == 2 ? a.gam : a.done;
  const float sv = sp[tid < 4 * B ? sb : 0];
  const float wv = a.wts != nullptr ? a.wts[tid < B ? tid : 0] : 1.f;
  stage_st(lg, l0, B * NO, tid, nth, r0);
  stage_st(lgT, l1, n1, tid, nth, r1);
  stage_st(lgO, l2, B * NO, tid, nth, r2);
  stage_st(vl, v0, NV, tid, nth, q0);
  stage_st(vlT, v1, nv1, tid, nth, q1);
  stage_st(vlO, v2, NV, tid, nth, q2);
  if (tid < 4 * B) sc[tid] = sv;             // (act bits copied as raw 32-bit words)
  if (tid < B) sc[4 * B + tid] = wv;
  for (int t = tid + nth; t < 5 * B; t += nth) {   // B > nth / 4: the rest of the scalars
    const int g = t / B, b = t - g * B;
    sc[t] = g == 0 ? __int_as_float(a.act[b]) : g == 1 ? a.rew[b] : g == 2 ? a.gam[b] : g == 3 ? a.done[b]
          : (a.wts != nullptr ? a.wts[b] : 1.f);
  }
}

// Fused acting (training launch, last block): the actors' E logits rows -> softmax ->
// expected Q -> eps-greedy / env step / replay append (+ PER insert), all in this block's LDS.
DQN_DEV void c51_act_block(const HeadArgs& a, float* sm) {
  const int E = a.act_E, NA = a.atoms, NO = a.A * NA;
  const int tid = threadIdx.x, nth = blockDim.x;
  const ActorPre apre = actor_prefetch(a.actor);           // loads overlap the logits copy
  float* lg = sm;                                          // [E][NO]
  float* vl = lg + E * NO;                                 // [E][NA]
  float* q = vl + E * NA;                                  // [E][A]
  for (int t = tid; t < E * NO; t += nth) lg[t] = a.act_lgi[t];
  if (a.dueling)
    for (int t = tid; t < E * NA; t += nth) vl[t] = a.act_vli[t];
  __syncthreads();
  c51_softmax(a, lg, vl, nullptr, q, tid, nth, E);
  actor_step_block(a.actor, q, lg, apre);                  // (the probabilities are dead after q)
}

__global__ void __launch_bounds__(1024) c51_head_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if (a.act_E > 0 && !a.infer && blockIdx.x == gridDim.x - 1) {
    c51_act_block(a, sm);
    return;
  }
  // (the learner's blocks: all but the fused acting block)
  const int nblk = (int)gridDim.x - (a.act_E > 0 && !a.infer ? 1 : 0);
  const int B = a.B, A = a.A, NA = a.atoms, NO = A * NA, HID = a.HID, HH = a.dueling ? 2 * HID : HID;
  float* lg = sm;                       // [B][NO] logits -> probabilities
  float* vl = lg + B * NO;              // [B][NA] dueling value logits
  float* mt = vl + B * NA;              // [B][NA] projected target distribution
  float* lp = mt + B * NA;              // [B][NA] log p of the taken action (online s)
  float* q = lp + B * NA;               // [B][A] expected Q (selection / acting)
  float* red = q + B * A;               // [32]
  int* astar = reinterpret_cast<int*>(red + 32);   // [B]
  int* sdone = astar + B;               // [E] fused actor scratch
  float* pc = reinterpret_cast<float*>(sdone + (a.has_actor ? a.actor.E : 0));   // [B][NA] one row per sample
  const bool staged = c51_staged(a);
  float* lgT = pc + B * NA;
  float* vlT = lgT + B * NO;
  float* lgO = vlT + B * NA;
  float* vlO = lgO + B * NO;
  float* sc = vlO + B * NA;             // [act | rew | gam | done | wts] x B
  const int32_t* sact = staged ? reinterpret_cast<const int32_t*>(sc) : a.act;
  const int tid = threadIdx.x, nth = blockDim.x;
  const int lane = tid & 63, wave = tid >> 6, nwave = nth >> 6;
  const int ninst = a.infer ? 1 : (a.h[2] != nullptr ? 3 : 2);
  int64_t* prof = (a.prof != nullptr && blockIdx.x == 0 && tid == 0) ? a.prof : nullptr;
#define C51_MARK(i) if (prof) prof[i] = (int64_t)__builtin_amdgcn_s_memtime()
  C51_MARK(0);
  if (a.zero_ptr != nullptr) {
    float4* z4 = reinterpret_cast<float4*>(a.zero_ptr);
    for (int t = blockIdx.x * nth + tid; t < a.zero_n / 4; t += nblk * nth) z4[t] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  auto logits = [&](int inst) {          // precomputed (igemm) or in-block MFMA logits
    if (a.lgi[inst] != nullptr) c51_load_logits(a, inst, lg, vl, tid, nth);
    else c51_logits(a, inst, lg, vl, lane, wave, nwave);
  };
  if (a.infer) {
    logits(0);
    __syncthreads();
    c51_softmax(a, lg, vl, nullptr, q, tid, nth, B);
    if (a.q_out != nullptr)
      for (int t = tid; t < B * A; t += nth) a.q_out[t] = q[t];
    if (a.has_actor) actor_step_block(a.actor, q, lg);       // (the probabilities are dead after q)
    return;
  }
  // ---- 1. action choice on s' (Double DQN: online net, else the target net)
  const int sel = ninst == 3 ? 2 : 1;
  if (staged) c51_stage(a, ninst, lg, vl, lgT, vlT, lgO, vlO, sc, tid, nth);
  else logits(sel);
  __syncthreads();
  C51_MARK(1);
  c51_softmax(a, lg, vl, nullptr, q, tid, nth, B);
  C51_MARK(2);
  for (int b = tid; b < B; b += nth) {
    int best = 0;
    float bv = q[b * A];
    for (int i = 1; i < A; ++i) if (q[b * A + i] > bv) { bv = q[b * A + i]; best = i; }
    astar[b] = best;
  }
  __syncthreads();
  C51_MARK(3);
  // ---- 2. target distribution of a* projected onto the support
  // pc[b] = target distribution of a*[b]
  if (sel == 1) {
    for (int t = tid; t < B * NA; t += nth) pc[t] = lg[(t / NA) * NO + astar[t / NA] * NA + t % NA];
  } else if (a.lgi[1] != nullptr) {
    if (staged) c51_rows(a, lgT, vlT, astar, pc, nullptr, tid, nth);
    else c51_rows(a, a.lgi[1], a.vli[1], astar, pc, nullptr, tid, nth);
  } else {
    logits(1);
    __syncthreads();
    c51_softmax(a, lg, vl, nullptr, nullptr, tid, nth, B);
    for (int t = tid; t < B * NA; t += nth) pc[t] = lg[(t / NA) * NO + astar[t / NA] * NA + t % NA];
  }
  for (int t = tid; t < B * NA; t += nth) mt[t] = 0.f;
  __syncthreads();
  {
    const float dz = (a.vmax - a.vmin) / (float)(NA - 1);
    for (int b = wave; b < B; b += nwave) {
      if (lane < NA) {
        const float p = pc[b * NA + lane];
        const float rw = staged ? sc[B + b] : a.rew[b], gm = staged ? sc[2 * B + b] : a.gam[b];
        const float dn = staged ? sc[3 * B + b] : a.done[b];
        float tz = rw + gm * (1.f - dn) * c51_z(a, lane);
        tz = fminf(fmaxf(tz, a.vmin), a.vmax);
        const float bj = (tz - a.vmin) / dz;
        const float lo = floorf(bj), hi = ceilf(bj);
        const int l = (int)lo, u = (int)hi;
        atomicAdd(&mt[b * NA + l], p * (hi - bj + (l == u ? 1.f : 0.f)));
        atomicAdd(&mt[b * NA + u], p * (bj - lo));
      }
    }
  }
  C51_MARK(4);
  // ---- 3. online distribution of (s, a): cross-entropy, d logits
  __syncthreads();                      // projection reads of pc done, its atomics complete
  C51_MARK(14);
  // pc[b] = online distribution of the taken action, lp its log
  if (a.lgi[0] != nullptr) {
    if (staged) c51_rows(a, lgO, vlO, sact, pc, lp, tid, nth);
    else c51_rows(a, a.lgi[0], a.vli[0], a.act, pc, lp, tid, nth);
  } else {
    logits(0);
    __syncthreads();
    c51_softmax(a, lg, vl, lp, nullptr, tid, nth, B);
    for (int t = tid; t < B * NA; t += nth) pc[t] = lg[(t / NA) * NO + a.act[t / NA] * NA + t % NA];
    __syncthreads();
  }
  C51_MARK(15);
  float contrib = 0.f;
  for (int b = wave; b < B; b += nwave) {
    const float ce = -wave_sum_dpp(lane < NA ? mt[b * NA + lane] * lp[b * NA + lane] : 0.f);
    const float w = staged ? sc[4 * B + b] : (a.wts != nullptr ? a.wts[b] : 1.f);
    if (lane < NA) {   // d(mean w*CE)/d logit of the taken action = w/B (p - m); reuse lp for it
      const float p = pc[b * NA + lane];
      lp[b * NA + lane] = w / (float)B * (p - mt[b * NA + lane]);
    }
    if (lane == 0) {
      contrib += w * ce;
      if (blockIdx.x == 0) a.prio[b] = ce;
    }
  }
  {
    const float s = wave_sum_dpp(contrib);
    if (lane == 0) red[wave] = s;
  }
  C51_MARK(16);
  __syncthreads();
  if (tid == 0 && blockIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < nwave; ++i) s += red[i];
    a.loss[0] = s / (float)B;
  }
  C51_MARK(5);
  // ---- 4. output-layer backward (online instance 0) on MFMA, tiles spread over every
  // wave of every block. dOut[b][j] (j = i*NA + n) = g[b][n] * ((i == act_b) - 1/A dueling)
  // goes to LDS (over the dead logits); g = lp; dV[b][n] = g[b][n].
  const float inva = a.dueling ? 1.f / (float)A : 0.f;
  float* dout = lg;
  for (int t = tid; t < B * NO; t += nth) {
    const int b = t / NO, j = t - b * NO, i = j / NA, n = j - i * NA;
    dout[t] = lp[b * NA + n] * ((i == sact[b] ? 1.f : 0.f) - inva);
  }
  __syncthreads();
  const int gw = blockIdx.x * nwave + wave, GW = nblk * nwave;
  const int kg = 8 * (lane >> 4), l16 = lane & 15;
  const act_t* h0 = reinterpret_cast<const act_t*>(a.h[0]);
  const int KB = (B + 31) / 32;                 // k-steps over the batch
  // (a) dW[k][j] = sum_b h[b][k] dOut[b][j]  (+ dWv with g): M = HID rows, N = outputs
  {
    const int MT = HID / 16, NT = (NO + 15) / 16, NTv = a.dueling ? (NA + 15) / 16 : 0;
    for (int task = gw; task < MT * (NT + NTv); task += GW) {
      const int mt = task % MT, t2 = task / MT;
      const bool val = t2 >= NT;
      const int nt = val ? t2 - NT : t2, ncol = val ? NA : NO;
      const act_t* hsrc = (a.dueling && !val) ? h0 + HID : h0;   // advantage half / value half
      const float* bsrc = val ? lp : dout;
      const int k = mt * 16 + l16, j = nt * 16 + l16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int kb = 0; kb < KB; ++kb) {
        bfx8 af, bf;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int b = kb * 32 + kg + u;
          af[u] = b < B ? hsrc[(int64_t)b * HH + k] : (act_t)0.f;
          bf[u] = (act_t)(b < B && j < ncol ? bsrc[b * ncol + j] * kLossScale : 0.f);
        }
        acc = DQN_MFMA16_BUILTIN(af, bf, acc, 0, 0, 0);
      }
      if (j < ncol) {
        float* dst = val ? a.dwv : a.dw;
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(int64_t)(mt * 16 + 4 * (lane >> 4) + r) * ncol + j] = acc[r] * kInvLossScale;
      }
    }
  }
  C51_MARK(6);
  // (b) dH[b][k] = (sum_j dOut[b][j] W[k][j]) * (h > 0); value half: sum_n g[b][n] Wv[k][n]
  {
    act_t* dh = reinterpret_cast<act_t*>(a.dh);
    const int MT = (B + 15) / 16, NT = HH / 16;
    for (int task = gw; task < MT * NT; task += GW) {
      const int mt = task % MT, nt = task / MT;
      const int kcol0 = nt * 16;
      const bool val = a.dueling && kcol0 < HID;
      const int kk = (a.dueling && !val ? kcol0 - HID : kcol0) + l16;   // row of W / Wv
      const int KD = val ? NA : NO;                                       // reduction length
      const float* Wrow = val ? a.wv[0] + (int64_t)kk * NA : a.w[0] + (int64_t)kk * NO;
      const float* asrc = val ? lp : dout;
      const int b = mt * 16 + l16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < (KD + 31) / 32; ++ks) {
        bfx8 af, bf;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int jj = ks * 32 + kg + u;
          af[u] = (act_t)(b < B && jj < KD ? asrc[b * KD + jj] * kLossScale : 0.f);   // dH leaves scaled
          bf[u] = (act_t)(jj < KD ? Wrow[jj] : 0.f);
        }
        acc = DQN_MFMA16_BUILTIN(af, bf, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int bb = mt * 16 + 4 * (lane >> 4) + r;
        if (bb < B) {
          const int64_t o = (int64_t)bb * HH + kcol0 + l16;
          dh[o] = (act_t)((float)h0[o] > 0.f ? acc[r] : 0.f);
        }
      }
    }
  }
  C51_MARK(7);
  // (c) bias gradients
  const int gt = blockIdx.x * nth + tid, gn = nblk * nth;
  for (int j = gt; j < NO; j += gn) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dout[b * NO + j];
    a.db[j] = s;
  }
  if (a.dueling)
    for (int n = gt; n < NA; n += gn) {
      float s = 0.f;
      for (int b = 0; b < B; ++b) s += lp[b * NA + n];
      a.dbv[n] = s;
    }
  C51_MARK(8);
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
  for (int q = threadIdx.x; 4 * q < total; q += blockDim.x) {
    const u32x4 r = philox(seed ^ 0x2545f4914f6cdd1dull, ctr, (uint32_t)q, 0x6e6f6973u);
    const uint32_t u[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float u1 = ((float)(u[2 * h] >> 8) + 1.f) * (1.0f / 16777216.0f);   // (0, 1]
      const float u2 = (float)(u[2 * h + 1] >> 8) * (1.0f / 16777216.0f);       // [0, 1)
      const float rad = sqrtf(-2.f * __logf(u1));
      float sn, cs;
      __sincosf(6.283185307179586f * u2, &sn, &cs);
      const float z[2] = {rad * cs, rad * sn};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int i = 4 * q + 2 * h + j;
        if (i < n) out0[i] = z[j];
        else if (i < total) out1[i - n] = z[j];
      }
    }
  }
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
  const size_t n = (c51_base_floats(a) + (c51_staged(a) ? c51_stage_floats(a) : 0)) * sizeof(float);
  // the fused actor's PER tree insert reuses the (dead) probabilities at the start of LDS
  return (a.has_actor || a.act_E > 0) && a.actor.tsum != nullptr && n < sizeof(SumtreeLds) ? sizeof(SumtreeLds) : n;
}

void launch_c51_head(const HeadArgs& a, hipStream_t st) {
  // training: phases 1-3 run redundantly in every block (L2-hot inputs); the output-layer
  // backward tiles spread over all 32 x 16 waves
  hipLaunchKernelGGL(c51_head_kernel, dim3(a.infer ? 1 : 32 + (a.act_E > 0 ? 1 : 0)), dim3(1024),
                     c51_head_lds_bytes(a), st, a);
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
