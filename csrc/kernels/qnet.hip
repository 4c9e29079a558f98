// Q-network layer kernels for gfx950 (CDNA4): every GEMM-shaped op on the
// bf16 MFMA (v_mfma_f32_16x16x32_bf16, fp32 accumulate), wave64 tiles.
//
// Reference layers (TF 0.x ops, /root/reference/src/network.py:389-424):
// conv2d + bias + relu (+ max_pool), matmul + bias (+ relu), and their
// autodiff backward. Here:
//   * pack_kernel      fp32 master weights (TF layouts) -> bf16 MFMA B-fragments
//                      ([K/32][N/16][64 lanes][8]) for the forward and for dgrad;
//   * igemm_kernel     implicit GEMM C[M][N] = A[M][K] B[K][N] with the A operand
//                      produced on the fly by a loader (conv im2col from NHWC u8/bf16,
//                      conv dgrad gather, dense rows) straight into registers and
//                      B fragments read as one 16-byte load per lane; epilogues fuse
//                      input scale + bias + ReLU (forward) or the ReLU mask (dgrad);
//                      optional split-K across the waves of a block (LDS reduce);
//   * wgrad_kernel     dW[K][N] = sum_m A[m][K]^T dZ[m][N] with both operands staged
//                      transposed in LDS (padded rows: conflict-free ds_read_b128),
//                      bias gradient fused, fp32 atomics only across M-chunks;
//   * head_loss_kernel output layer + dueling combine + TD loss + dQ + head backward
//                      (dW, db, dH masked by ReLU) in ONE workgroup.
#include "common.h"
#include "actor_dev.h"
#include "../include/dqn_nets_k.h"

namespace dqn {

typedef __attribute__((ext_vector_type(8))) act_t bfx8;

DQN_DEV bfx8 zero8() {
  bfx8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (act_t)0.f;
  return z;
}

DQN_DEV bfx8 u8x8_to_bf(uint32_t lo, uint32_t hi) {
  bfx8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (act_t)(float)((lo >> (8 * j)) & 0xffu);
    r[4 + j] = (act_t)(float)((hi >> (8 * j)) & 0xffu);
  }
  return r;
}

DQN_DEV f32x4 mfma16(const bfx8& a, const bfx8& b, const f32x4& c) {
  return DQN_MFMA16_BUILTIN(a, b, c, 0, 0, 0);
}

// ============================================================== weight packing
// dst2 (optional): the target network's packed copy, written too when step % freq == 0
// (the fused hard target sync: online was just copied to the target's fp32 master).
__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ src, act_t* __restrict__ dst,
                                                   const PackJob* __restrict__ jobs, act_t* __restrict__ dst2,
                                                   const int64_t* __restrict__ step, int freq) {
  const PackJob jb = jobs[blockIdx.y];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const bool sync = dst2 != nullptr && step != nullptr && (step[0] % freq) == 0;
  if (jb.mode == 3) {                           // contiguous fp32 copy (bias concatenation)
    if (t < jb.K) {
      const float x = src[jb.src_off + t];
      reinterpret_cast<float*>(dst + jb.dst_off)[t] = x;
      if (sync) reinterpret_cast<float*>(dst2 + jb.dst_off)[t] = x;
    }
    return;
  }
  const int K32 = (jb.K + 31) / 32, N16 = (jb.N + 15) / 16;
  if (t >= K32 * N16 * 64) return;
  const int l = t & 63, nt = (t >> 6) % N16, ks = (t >> 6) / N16;
  const int n = nt * 16 + (l & 15);
  bfx8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = ks * 32 + 8 * (l >> 4) + j;
    float x = 0.f;
    if (k < jb.K && n < jb.N) {
      if (jb.mode == 0) {                       // natural [K][N] (conv HWIO fwd, dense fwd)
        x = src[jb.src_off + (int64_t)k * jb.N + n];
      } else if (jb.mode == 1) {                // conv dgrad: k=(tap, co), n=ci  <- W[tap][ci][co]
        const int tap = k / jb.p2, co = k - tap * jb.p2;
        x = src[jb.src_off + ((int64_t)tap * jb.p1 + n) * jb.p2 + co];
      } else {                                  // dense transpose: k=o, n=i <- W[i][o] (OUT = p0)
        x = src[jb.src_off + (int64_t)n * jb.p0 + k];
      }
    }
    v[j] = (act_t)x;
  }
  const int64_t o = jb.dst_off + ((int64_t)((jb.ks_off + ks) * jb.dst_N16 + jb.nt_off + nt) * 64 + l) * 8;
  *reinterpret_cast<bfx8*>(dst + o) = v;
  if (sync) *reinterpret_cast<bfx8*>(dst2 + o) = v;
}

// ================================================================== A loaders
// Each loader is built per (instance, row m) and returns the 8 consecutive
// K-values [k0, k0+8) of row m as a bf16x8 MFMA A-fragment.
template <typename Tin, int CIN, int KH, int KW, int S>
struct ConvLoader {
  const Tin* base;
  int IH, IW, iy0, ix0;
  bool ok;
  DQN_DEV ConvLoader() {}
  DQN_DEV ConvLoader(const ConvArgs& a, int inst, int m) {
    const int ohw = a.OH * a.OW;
    ok = m < a.M;
    const int mm = ok ? m : 0;
    const int b = mm / ohw, r = mm - b * ohw, oy = r / a.OW, ox = r - oy * a.OW;
    IH = a.IH; IW = a.IW;
    iy0 = oy * S - a.pad_t;
    ix0 = ox * S - a.pad_l;
    base = reinterpret_cast<const Tin*>(a.in[inst]) + (int64_t)b * IH * IW * CIN;
  }
  DQN_DEV bfx8 frag(int k0) const {
    if (!ok) return zero8();
    const int kh = k0 / (KW * CIN), rem = k0 - kh * (KW * CIN), kw = rem / CIN, ci = rem - kw * CIN;
    const int iy = iy0 + kh, ix = ix0 + kw;
    if constexpr (sizeof(Tin) == 1) {
      static_assert(CIN == 4, "uint8 input path expects 4 stacked frames");
      // 8 bytes = pixels (ix, ix+1) x 4 frames
      uint32_t lo = 0, hi = 0;
      if (iy >= 0 && iy < IH) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(base + (int64_t)iy * IW * CIN);
        if (ix >= 0 && ix < IW) lo = row[ix];
        if (ix + 1 >= 0 && ix + 1 < IW) hi = row[ix + 1];
      }
      return u8x8_to_bf(lo, hi);
    } else {
      if (iy < 0 || iy >= IH || ix < 0 || ix >= IW) return zero8();
      return *reinterpret_cast<const bfx8*>(base + ((int64_t)iy * IW + ix) * CIN + ci);
    }
  }
};

// conv1 straight from the replay's frame ring: row m = (b, oy, ox), k = (kh, kw, c)
// with the 4 stacked frames of sample b given by a slot table slots[b][4]
// (replay state_idx rows / actor stacks). Fuses the frame-stack gather into
// the first layer: no materialised [B, 84, 84, 4] copy.
template <int KH, int KW, int S>
struct FrameLoader {
  const uint8_t* fb[4];
  int IH, IW, iy0, ix0;
  bool ok;
  DQN_DEV FrameLoader() {}
  DQN_DEV FrameLoader(const ConvArgs& a, int inst, int m) {
    const int ohw = a.OH * a.OW;
    ok = m < a.M;
    const int mm = ok ? m : 0;
    const int b = mm / ohw, r = mm - b * ohw, oy = r / a.OW, ox = r - oy * a.OW;
    IH = a.IH; IW = a.IW;
    iy0 = oy * S - a.pad_t;
    ix0 = ox * S - a.pad_l;
    const int4 sl = reinterpret_cast<const int4*>(a.in[inst])[b];
    const uint8_t* fr = reinterpret_cast<const uint8_t*>(a.frames);
    fb[0] = fr + (int64_t)sl.x * a.frame_hw;
    fb[1] = fr + (int64_t)sl.y * a.frame_hw;
    fb[2] = fr + (int64_t)sl.z * a.frame_hw;
    fb[3] = fr + (int64_t)sl.w * a.frame_hw;
  }
  DQN_DEV bfx8 frag(int k0) const {
    if (!ok) return zero8();
    const int kh = k0 / (KW * 4), kw = (k0 - kh * (KW * 4)) / 4;   // k0 % 8 == 0 -> kw even, c = 0
    const int iy = iy0 + kh, ix = ix0 + kw;
    bfx8 r = zero8();
    if (iy < 0 || iy >= IH) return r;
    const int off = iy * IW + ix;
    const bool in0 = ix >= 0 && ix < IW, in1 = ix + 1 >= 0 && ix + 1 < IW;
    if (in0 && in1 && ((off & 1) == 0)) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t v = *reinterpret_cast<const uint16_t*>(fb[c] + off);   // pixels ix, ix+1 of frame c
        r[c] = (act_t)(float)(v & 0xffu);
        r[4 + c] = (act_t)(float)(v >> 8);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (in0) r[c] = (act_t)(float)fb[c][off];
        if (in1) r[4 + c] = (act_t)(float)fb[c][off + 1];
      }
    }
    return r;
  }
};

// dgrad gather: row m = (b, iy, ix) of the conv INPUT, k = (kh, kw, co);
// A[m][k] = dZ[b][oy][ox][co] where iy + pad_t - kh = S*oy (else 0).
template <int COUT, int KH, int KW, int S>
struct DgradLoader {
  const act_t* base;
  int OH, OW, ty, tx;
  bool ok;
  DQN_DEV DgradLoader() {}
  DQN_DEV DgradLoader(const ConvArgs& a, int inst, int m) {
    const int ihw = a.IH * a.IW;
    ok = m < a.M;
    const int mm = ok ? m : 0;
    const int b = mm / ihw, r = mm - b * ihw, iy = r / a.IW, ix = r - iy * a.IW;
    OH = a.OH; OW = a.OW;
    ty = iy + a.pad_t;
    tx = ix + a.pad_l;
    base = reinterpret_cast<const act_t*>(a.in[inst]) + (int64_t)b * OH * OW * COUT;
  }
  DQN_DEV bfx8 frag(int k0) const {
    if (!ok) return zero8();
    const int tap = k0 / COUT, co = k0 - tap * COUT, kh = tap / KW, kw = tap - kh * KW;
    const int ny = ty - kh, nx = tx - kw;
    if (ny < 0 || nx < 0) return zero8();
    const int oy = ny / S, ox = nx / S;
    if (oy * S != ny || ox * S != nx || oy >= OH || ox >= OW) return zero8();
    return *reinterpret_cast<const bfx8*>(base + ((int64_t)oy * OW + ox) * COUT + co);
  }
};

struct DenseLoader {
  const act_t* row;
  bool ok;
  DQN_DEV DenseLoader() {}
  DQN_DEV DenseLoader(const ConvArgs& a, int inst, int m) {
    ok = m < a.M;
    // row stride: a.IW when given (a K-wide slice of wider rows, e.g. one half of the
    // dueling [value | advantage] hidden layer), else K
    row = reinterpret_cast<const act_t*>(a.in[inst]) + (int64_t)(ok ? m : 0) * (a.IW > 0 ? a.IW : a.K);
  }
  DQN_DEV bfx8 frag(int k0) const {
    if (!ok) return zero8();
    return *reinterpret_cast<const bfx8*>(row + k0);
  }
};

// ============================================================ implicit GEMM
// Block = WM x WN x KSPLIT waves (4 or 8); wave tile = (MT*16) x (NT*16).
// EPI: 0 = scale*acc + bias, ReLU, bf16 out; 1 = scale*acc + bias, fp32 out (no ReLU);
//      2 = acc * (mask > 0), bf16 out (ReLU backward through the layer input).
template <class LD, int MT, int NT, int WM, int WN, int KSPLIT, int EPI, int U = 4>
__global__ void __launch_bounds__(512) igemm_kernel(ConvArgs a) {
  static_assert(WM * WN * KSPLIT == 4 || WM * WN * KSPLIT == 8, "4 or 8 waves per block");
  __shared__ float red[KSPLIT > 1 ? WM * WN * (KSPLIT - 1) * MT * NT * 256 : 1];
  const int inst = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wk = wave % KSPLIT, wn = (wave / KSPLIT) % WN, wm = wave / (KSPLIT * WN);
  const int m_base = blockIdx.x * (WM * MT * 16) + wm * MT * 16;
  const int nt_base = blockIdx.y * (WN * NT) + wn * NT;
  const int K32 = (a.K + 31) / 32;
  const bfx8* __restrict__ Bp = reinterpret_cast<const bfx8*>(a.w[inst]);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // each lane owns row (lane & 15) of every m-tile and k-group (lane >> 4)
  LD ld[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) ld[i] = LD(a, inst, m_base + i * 16 + (lane & 15));
  const int kg = 8 * (lane >> 4);
  const int ks_lo = (K32 * wk) / KSPLIT, ks_hi = (K32 * (wk + 1)) / KSPLIT;
  // U k-steps per batch: all A/B fragment loads of the batch are issued before
  // its MFMAs, so U x (MT + NT) global loads are in flight per wave (the loop
  // is latency-bound at these sizes, not MFMA-bound). A partial last batch is
  // predicated (zero fragments) instead of falling back to one step at a time;
  // a U that covers the wave's whole K range pays the load latency once.
  for (int ks = ks_lo; ks < ks_hi; ks += U) {
    bfx8 af[U][MT], bf[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool kok = ks + u < ks_hi;
#pragma unroll
      for (int i = 0; i < MT; ++i) af[u][i] = kok ? ld[i].frag((ks + u) * 32 + kg) : zero8();
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[u][j] = kok ? Bp[((int64_t)(ks + u) * a.N16 + nt_base + j) * 64 + lane] : zero8();
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[u][i], bf[u][j], acc[i][j]);
  }
  if constexpr (KSPLIT > 1) {
    // waves wk > 0 hand partial tiles to wk == 0 through LDS
    const int slot = ((wm * WN + wn) * (KSPLIT - 1));
    if (wk > 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            red[(((slot + wk - 1) * MT + i) * NT + j) * 256 + r * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (wk != 0) return;
#pragma unroll
    for (int s = 0; s < KSPLIT - 1; ++s)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += red[(((slot + s) * MT + i) * NT + j) * 256 + r * 64 + lane];
  }
  // epilogue: C/D layout col = lane & 15, row = 4*(lane >> 4) + r
  const float scale = a.scale[inst];
  const float* __restrict__ bias = a.bias[inst];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = (nt_base + j) * 16 + (lane & 15);
    if (n >= a.N) continue;
    const float bv = (EPI == 2 || bias == nullptr) ? 0.f : bias[n];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m_base + i * 16 + 4 * (lane >> 4) + r;
        if (m >= a.M) continue;
        float v = acc[i][j][r];
        const int64_t o = (int64_t)m * a.ldo + n;
        if constexpr (EPI == 0) {
          v = fmaxf(v * scale + bv, 0.f);
          reinterpret_cast<act_t*>(a.out[inst])[o] = (act_t)v;
        } else if constexpr (EPI == 1) {
          reinterpret_cast<float*>(a.out[inst])[o] = v * scale + bv;
        } else {
          const float mk = (float)reinterpret_cast<const act_t*>(a.mask[inst])[o];
          reinterpret_cast<act_t*>(a.out[inst])[o] = (act_t)(mk > 0.f ? v : 0.f);
        }
      }
    }
  }
}

// ================================================================ weight grad
// dW[k][n] (+)= scale * sum_{m in chunk} A[m][k] * dZ[m][n];  db[n] (+)= sum_m dZ[m][n]
// grid: x = M-chunk (MC rows), y = K-range (KB), z = N-range (NB). ONE staging
// pass per block: all global loads of the chunk are issued first (register
// staging), then written TRANSPOSED to LDS ([k][m], [n][m], rows padded by 8
// elements) so each lane's 8 consecutive m are one ds_read_b128; then
// (KB/16)x(NB/16) output tiles x MC/32 MFMA k-steps. fp32 atomics only when
// more than one M-chunk contributes to a weight.
template <int MC, int KB, int NB>
struct WgradTile {
  static constexpr int LR = MC + 8;
  static constexpr size_t lds_bytes = (size_t)(KB + NB) * LR * sizeof(act_t);
};

// Body shared by the per-layer launch and the grouped launch (one block = one
// (M-chunk, K-range, N-range) tile; LDS passed in so a grouped kernel can carve
// every member's staging from one buffer).
template <class LD, int MC, int KB, int NB>
DQN_DEV void wgrad_block(const ConvArgs& a, const WgradArgs& g, int bx, int by, int bz, act_t* lds) {
  constexpr int LR = MC + 8;
  constexpr int TPR = 256 / MC;                  // threads per staged row
  constexpr int GA = KB / 8 / TPR, GZ = NB / 8 / TPR;
  constexpr int TILES = (KB / 16) * (NB / 16), PERW = TILES / 4, KSTEPS = MC / 32;
  static_assert(256 % MC == 0 && (KB / 8) % TPR == 0 && (NB / 8) % TPR == 0 && TILES % 4 == 0, "tiling");
  act_t* At = lds;
  act_t* Zt = lds + KB * LR;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m_lo = bx * MC, k_lo = by * KB, n_lo = bz * NB;
  {
    const int r = threadIdx.x % MC, p = threadIdx.x / MC;
    const int m = m_lo + r;
    const bool mok = m < a.M;
    const act_t* dz = reinterpret_cast<const act_t*>(g.dz) + (int64_t)(mok ? m : 0) * g.ldz + n_lo;
    LD ld(a, 0, m);
    bfx8 va[GA], vz[GZ];
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int k0 = k_lo + (p + i * TPR) * 8;
      va[i] = k0 < a.K ? ld.frag(k0) : zero8();
    }
#pragma unroll
    for (int i = 0; i < GZ; ++i) {
      const int c8 = (p + i * TPR) * 8;
      vz[i] = (mok && n_lo + c8 < g.N) ? *reinterpret_cast<const bfx8*>(dz + c8) : zero8();
    }
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int c8 = (p + i * TPR) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) At[(c8 + j) * LR + r] = va[i][j];
    }
#pragma unroll
    for (int i = 0; i < GZ; ++i) {
      const int c8 = (p + i * TPR) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) Zt[(c8 + j) * LR + r] = vz[i][j];
    }
  }
  __syncthreads();
  const bool atomic = g.atomic != 0;
  if (g.db != nullptr && by == 0) {
    for (int n = threadIdx.x; n < NB; n += 256) {
      float s = 0.f;
      const act_t* zr = Zt + n * LR;
#pragma unroll 8
      for (int r = 0; r < MC; ++r) s += (float)zr[r];
      const int nn = n_lo + n;
      if (nn < g.N) {
        float* pdb = nn < g.nsplit ? g.db + nn : g.db2 + (nn - g.nsplit);
        s *= kInvLossScale;
        if (atomic) atomicAdd(pdb, s); else *pdb = s;
      }
    }
  }
  const int kg = 8 * (lane >> 4), row = lane & 15;
  constexpr int NTt = NB / 16;
#pragma unroll
  for (int i = 0; i < PERW; ++i) {
    const int tile = wave + 4 * i;
    const int kt = tile / NTt, nt = tile - kt * NTt;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const bfx8 af = *reinterpret_cast<const bfx8*>(At + (kt * 16 + row) * LR + 32 * s + kg);
      const bfx8 bf = *reinterpret_cast<const bfx8*>(Zt + (nt * 16 + row) * LR + 32 * s + kg);
      acc = mfma16(af, bf, acc);
    }
    const int n = n_lo + nt * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k_lo + kt * 16 + 4 * (lane >> 4) + r;
      if (k < a.K && n < g.N) {
        float* p = n < g.nsplit ? g.dw + (int64_t)k * g.nsplit + n
                                : g.dw2 + (int64_t)k * (g.N - g.nsplit) + (n - g.nsplit);
        const float v = acc[r] * (g.scale * kInvLossScale);
        if (atomic) atomicAdd(p, v); else *p = v;
      }
    }
  }
}

template <class LD, int MC, int KB, int NB>
__global__ void __launch_bounds__(256) wgrad_kernel(ConvArgs a, WgradArgs g) {
  __shared__ __attribute__((aligned(16))) act_t lds[WgradTile<MC, KB, NB>::lds_bytes / sizeof(act_t)];
  wgrad_block<LD, MC, KB, NB>(a, g, blockIdx.x, blockIdx.y, blockIdx.z, lds);
}

// =========================================================== fused head + loss
// Instances of the last hidden layer H (bf16): h[0] = online(s), h[1] = target(s'),
// h[2] = online(s') (Double DQN). Plain: Q = H W + b. Dueling: H = [Hv | Ha],
// Q = (Hv wv + bv) + (Ha Wa + ba) - mean_a(Ha Wa + ba).
// Q tiles come from MFMA over packed head fragments (16 rows x 16 actions per
// wave task); the TD loss, dQ and the head backward (dW, db, dH masked by
// ReLU(H) > 0) follow in the same workgroup.
// head_body: one workgroup's share (blk of nblk) of the head. B / h0 / infer / actor /
// q_out / zeroing are parameters so the fused-acting block can run the acting path
// on the actors' hidden layer inside the learner's launch.
constexpr int kHeadPartFloats = 16 * 64 * 4;
constexpr int kHeadActorScratch = 64;          // actor LDS scratch after red[32] (E <= 64)
constexpr int kHeadMaxA = 32;                  // output biases staged in LDS up to this many actions
DQN_DEV void head_body(const HeadArgs& a, float* hsm, const int B, const void* h0, const bool infer,
                       const bool has_actor, float* q_out, const bool do_zero, const int blk, const int nblk) {
  const int A = a.A, HID = a.HID, HH = a.dueling ? 2 * HID : HID;
  float* part_lds = hsm;                    // [16 waves][64][4] split-K partial Q tiles
  float* q = hsm + kHeadPartFloats;         // [3][B][A]
  float* vv = q + 3 * B * A;                // [3][B] dueling value stream
  float* dq = vv + 3 * B;                   // [B][A]  dL/dQ (dueling: dL/dA)
  float* dv = dq + B * A;                   // [B]     dueling: dL/dV
  float* red = dv + B;                      // [32] (+ actor scratch)
  float* bl = red + 32 + kHeadActorScratch; // [3][A] output bias, [3] value bias (A <= kHeadMaxA)
  const int tid = threadIdx.x, nth = blockDim.x;
  const int lane = tid & 63, wave = tid >> 6, nwave = nth >> 6;
  const int ninst = infer ? 1 : (a.h[2] != nullptr ? 3 : 2);
  auto hptr = [&](int inst) { return inst == 0 && h0 != nullptr ? h0 : a.h[inst]; };
  // phase stamps (scripts/probe_head.py): learner block 0 -> prof[0..7], acting block -> prof[16..19]
  int64_t* prof = (a.prof != nullptr && tid == 0 && blk == 0) ? a.prof + (infer && has_actor ? 16 : 0) : nullptr;
#define HEAD_MARK(i) if (prof) prof[i] = (int64_t)__builtin_amdgcn_s_memtime()
  HEAD_MARK(0);
  ActorPre apre{};
  if (infer && has_actor) apre = actor_prefetch(a.actor);   // loads overlap the Q tiles
  float tr = 0.f, tg = 0.f, td = 0.f, tw = 1.f;              // this thread's sample (TD loss)
  int ta = 0;
  if (!infer && tid < B) {
    tr = a.rew[tid]; tg = a.gam[tid]; td = a.done[tid]; ta = a.act[tid];
    if (a.wts != nullptr) tw = a.wts[tid];
  }
  // Small operands of the later phases are loaded NOW, so their latency hides under the
  // Q-tile loads: the TD-loss inputs (registers) and the output biases (LDS). (The dW / dH
  // operands are NOT: their ~50 loads per thread would queue ahead of the Q-tile loads.)
  const bool bias_lds = A <= kHeadMaxA;
  if (bias_lds) {
    for (int t = tid; t < ninst * A; t += nth) bl[t] = a.b[t / A][t % A];
    if (a.dueling && tid < ninst) bl[3 * kHeadMaxA + tid] = a.bv[tid][0];
  }
  const int gt = blk * nth + tid, gn = nblk * nth;
  const act_t* hb0 = reinterpret_cast<const act_t*>(a.h[0]);
  const act_t* ha0 = a.dueling ? hb0 + HID : hb0;
  const float* W0 = a.w[0];
  // ---- 1. Q tiles on MFMA: task = (instance, 16-row tile, n-tile); the dueling value
  // stream is one extra n-tile. The K loop of every task is split over kspl waves (all
  // waves busy, one batch of loads in flight per wave); partial tiles meet in LDS.
  const int mtiles = (B + 15) / 16, K32 = HID / 32, ntl = a.N16 + (a.dueling ? 1 : 0);
  const int ntask = ninst * mtiles * ntl;
  int kspl = nwave / ntask;
  kspl = kspl < 1 ? 1 : (kspl > K32 ? K32 : kspl);
  const int kps = (K32 + kspl - 1) / kspl;                 // k-steps per wave part
  for (int wt = wave; wt < ntask * kspl; wt += nwave) {
    const int task = wt / kspl, part = wt - task * kspl;
    const int nt = task % ntl, im = task / ntl;
    const int inst = im / mtiles, mt = im - inst * mtiles;
    const int b_row = mt * 16 + (lane & 15);
    const bool rok = b_row < B;
    const act_t* hrow = reinterpret_cast<const act_t*>(hptr(inst)) + (int64_t)(rok ? b_row : 0) * HH;
    const act_t* ha = a.dueling ? hrow + HID : hrow;
    const bfx8* pw = reinterpret_cast<const bfx8*>(a.pw[inst]);
    const bfx8* pv = reinterpret_cast<const bfx8*>(a.pwv[inst]);
    const int kg = 8 * (lane >> 4);
    const bool val = nt == a.N16;
    const act_t* src = val ? hrow : ha;
    const int k_lo = part * kps, k_hi = min(K32, k_lo + kps);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int ks = k_lo; ks < k_hi; ks += 4) {            // 4 k-steps of loads in flight per batch
      bfx8 af[4], bf[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool kok = ks + u < k_hi;
        af[u] = rok && kok ? *reinterpret_cast<const bfx8*>(src + (ks + u) * 32 + kg) : zero8();
        bf[u] = !kok ? zero8() : val ? pv[(ks + u) * 64 + lane] : pw[((ks + u) * a.N16 + nt) * 64 + lane];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = mfma16(af[u], bf[u], acc);
    }
    if (kspl > 1) {
      *reinterpret_cast<f32x4*>(part_lds + (wt * 64 + lane) * 4) = acc;
      continue;
    }
    const int act = nt * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = mt * 16 + 4 * (lane >> 4) + r;
      if (val) {
        if ((lane & 15) == 0 && b < B) vv[inst * B + b] = acc[r] + a.bv[inst][0];
      } else if (b < B && act < A) {
        q[(inst * B + b) * A + act] = acc[r] + a.b[inst][act];
      }
    }
  }
  if (kspl > 1) {                                          // (the bias LDS is written before this barrier)                                          // sum the parts of every task
    __syncthreads();
    for (int t = tid; t < ntask * 64; t += nth) {
      const int task = t >> 6, ln = t & 63;
      const int nt = task % ntl, im = task / ntl;
      const int inst = im / mtiles, mt = im - inst * mtiles;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < kspl; ++p) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(part_lds + ((task * kspl + p) * 64 + ln) * 4);
        acc += v;
      }
      const bool val = nt == a.N16;
      const int act = nt * 16 + (ln & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = mt * 16 + 4 * (ln >> 4) + r;
        if (val) {
          if ((ln & 15) == 0 && b < B) vv[inst * B + b] = acc[r] + (bias_lds ? bl[3 * kHeadMaxA + inst] : a.bv[inst][0]);
        } else if (b < B && act < A) {
          q[(inst * B + b) * A + act] = acc[r] + (bias_lds ? bl[inst * A + act] : a.b[inst][act]);
        }
      }
    }
  }
  __syncthreads();
  HEAD_MARK(1);
  if (a.dueling) {
    for (int t = tid; t < ninst * B; t += nth) {
      float mean = 0.f;
      for (int i = 0; i < A; ++i) mean += q[t * A + i];
      mean /= (float)A;
      const float v = vv[t];
      for (int i = 0; i < A; ++i) q[t * A + i] += v - mean;
    }
    __syncthreads();
  }
  if (infer) {                              // acting: Q of instance 0 only
    if (q_out != nullptr)
      for (int t = tid; t < B * A; t += nth) q_out[t] = q[t];
    HEAD_MARK(2);
    if (has_actor) actor_step_block(a.actor, q, part_lds, apre);      // (split-K partials are dead)
    HEAD_MARK(3);
    return;
  }
  // ---- 2. TD loss (one thread per sample)
  float contrib = 0.f;
  if (tid < B) {
    const int b = tid;
    const float* sel = q + ((ninst == 3 ? 2 : 1) * B + b) * A;
    int best = 0;
    float bvv = sel[0];
    for (int i = 1; i < A; ++i) if (sel[i] > bvv) { bvv = sel[i]; best = i; }
    const float nxt = q[(B + b) * A + best];
    const float y = tr + tg * (1.f - td) * nxt;
    const int at = ta;
    const float d = q[b * A + at] - y;
    const float w = tw;
    float per, dper;
    if (a.huber) {
      const float ad = fabsf(d);
      per = ad <= a.delta ? 0.5f * d * d : a.delta * (ad - 0.5f * a.delta);
      dper = ad <= a.delta ? d : copysignf(a.delta, d);
    } else {
      per = d * d;
      dper = 2.f * d;
    }
    contrib = w * per;
    const float gsc = w * dper / (float)B;
    for (int i = 0; i < A; ++i) dq[b * A + i] = (i == at) ? gsc : 0.f;
    if (a.dueling) {
      // Q_i = V + A_i - mean(A): dV = sum_i dQ_i, dA_i = dQ_i - mean(dQ)
      dv[b] = gsc;
      for (int i = 0; i < A; ++i) dq[b * A + i] -= gsc / (float)A;
    }
    if (blk == 0) a.prio[b] = fabsf(d);
  }
  {
    const float s = wave_sum(contrib);
    if (lane == 0) red[wave] = s;
  }
  if (q_out != nullptr && blk == 0)
    for (int t = tid; t < B * A; t += nth) q_out[t] = q[t];
  __syncthreads();
  if (tid == 0 && blk == 0) {
    float s = 0.f;
    for (int i = 0; i < nwave; ++i) s += red[i];
    a.loss[0] = s / (float)B;
  }
  HEAD_MARK(2);
  // ---- 3. head backward (online instance 0 only), partitioned over the grid's
  // blocks (phases 1-2 above are recomputed by every block: cheap MFMA work);
  // k fastest across threads -> coalesced H reads
  act_t* dh = reinterpret_cast<act_t*>(a.dh);
  for (int t = gt; t < HID * A; t += gn) {              // dW[k][i] = sum_b Ha[b][k] dA[b][i]
    const int i = t / HID, k = t - i * HID;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += (float)ha0[(int64_t)b * HH + k] * dq[b * A + i];
    a.dw[k * A + i] = s;
  }
  for (int i = gt; i < A; i += gn) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dq[b * A + i];
    a.db[i] = s;
  }
  if (a.dueling) {
    for (int k = gt; k < HID; k += gn) {
      float s = 0.f;
      for (int b = 0; b < B; ++b) s += (float)hb0[(int64_t)b * HH + k] * dv[b];
      a.dwv[k] = s;
    }
    if (gt == 0) {
      float s = 0.f;
      for (int b = 0; b < B; ++b) s += dv[b];
      a.dbv[0] = s;
    }
  }
  HEAD_MARK(3);
  // dH[b][k] = (sum_i dA[b][i] W[k][i]) * (H > 0);   dueling value half: dV[b] * wv[k]
  const float* Wd = W0;                                 // output W [HID][A]
  const float* wvd = a.wv[0];
  for (int t = gt; t < B * HH; t += gn) {
    const int b = t / HH, k = t - b * HH;
    float s = 0.f;
    if (a.dueling && k < HID) {
      s = dv[b] * wvd[k];
    } else {
      const int kk = a.dueling ? k - HID : k;
      for (int i = 0; i < A; ++i) s += dq[b * A + i] * Wd[kk * A + i];
    }
    const float hval = (float)hb0[t];
    dh[t] = (act_t)(hval > 0.f ? s * kLossScale : 0.f);   // scaled: see dqn_act.h
  }
  // ---- 4. zero the gradient range the conv wgrads accumulate into (nothing in this
  //         kernel touches it; saves a fill launch). Last, so no barrier waits on it.
  if (do_zero && a.zero_ptr != nullptr) {
    float4* z4 = reinterpret_cast<float4*>(a.zero_ptr);
    for (int t = blk * nth + tid; t < a.zero_n / 4; t += nblk * nth) z4[t] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  HEAD_MARK(4);
#undef HEAD_MARK
}

__global__ void __launch_bounds__(1024) head_loss_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  // fused acting: the LAST workgroup runs the acting step on the actors' hidden layer
  // (online weights = instance 0), the others the learner's loss + head backward
  if (a.act_E > 0 && blockIdx.x == gridDim.x - 1) {
    head_body(a, hsm, a.act_E, a.act_h, true, true, nullptr, false, 0, 1);
    return;
  }
  head_body(a, hsm, a.B, nullptr, a.infer != 0, a.has_actor != 0, a.q_out, true, blockIdx.x,
            gridDim.x - (a.act_E > 0 ? 1 : 0));
}

}  // namespace dqn

using namespace dqn;

// ------------------------------------------------------------------ launchers
void launch_pack(const float* src, void* dst, const PackJob* jobs_dev, int njobs, int max_threads, void* dst2,
                 const int64_t* step, int freq, hipStream_t st) {
  dim3 grid((max_threads + 255) / 256, njobs);
  hipLaunchKernelGGL(pack_kernel, grid, dim3(256), 0, st, src, reinterpret_cast<act_t*>(dst), jobs_dev,
                     reinterpret_cast<act_t*>(dst2), step, freq < 1 ? 1 : freq);
}

#define IGEMM_LAUNCH_U(LD, MT, NT, WM, WN, KS, EPI, U)                                                \
  do {                                                                                                  \
    dim3 grid((a.M + WM * MT * 16 - 1) / (WM * MT * 16), (a.N + WN * NT * 16 - 1) / (WN * NT * 16), ninst); \
    hipLaunchKernelGGL((igemm_kernel<LD, MT, NT, WM, WN, KS, EPI, U>), grid, dim3(64 * WM * WN * KS), 0, st, a); \
  } while (0)
#define IGEMM_LAUNCH(LD, MT, NT, WM, WN, KS, EPI) IGEMM_LAUNCH_U(LD, MT, NT, WM, WN, KS, EPI, 4)

using NatC1 = ConvLoader<uint8_t, 4, 8, 8, 4>;
using NatC2 = ConvLoader<act_t, 32, 4, 4, 2>;
using NatC3 = ConvLoader<act_t, 64, 3, 3, 1>;
using NatD3 = DgradLoader<64, 3, 3, 1>;
using NatD2 = DgradLoader<64, 4, 4, 2>;
using NatF1 = FrameLoader<8, 8, 4>;

// layer kinds: see dqn_nets_k.h.  Tiles: (MT, NT, WM, WN, KSPLIT, EPI)
int launch_igemm(int kind, const ConvArgs& a, int ninst, hipStream_t st) {
  switch (kind) {
    // ---- forward, fused bias + ReLU, bf16 NHWC out
    case L_NAT_CONV1_FWD: IGEMM_LAUNCH(NatC1, 1, 2, 4, 1, 1, 0); return 0;       // K 256: 8 k-steps
    case L_NAT_CONV1_FRAMES: IGEMM_LAUNCH(NatF1, 1, 2, 4, 1, 1, 0); return 0;
    case L_NAT_CONV2_FWD: IGEMM_LAUNCH(NatC2, 1, 4, 2, 1, 2, 0); return 0;       // K 512: split-K 2
    case L_NAT_CONV3_FWD: IGEMM_LAUNCH(NatC3, 1, 4, 2, 1, 2, 0); return 0;       // K 576: split-K 2
    // K 3136 = 98 k-steps, split-K 8: one 13-step load batch per wave
    case L_DENSE_FWD_RELU: IGEMM_LAUNCH_U(DenseLoader, 2, 1, 1, 1, 8, 0, 13); return 0;
    case L_DENSE_FWD_F32: IGEMM_LAUNCH_U(DenseLoader, 2, 1, 1, 1, 8, 1, 13); return 0;
    // ---- backward data, ReLU mask of the layer input
    case L_DENSE_DGRAD: IGEMM_LAUNCH_U(DenseLoader, 2, 1, 1, 2, 2, 2, 8); return 0;   // K 512-1024
    case L_NAT_CONV3_DGRAD: IGEMM_LAUNCH_U(NatD3, 1, 4, 2, 1, 2, 2, 9); return 0;     // 18 k-steps
    case L_NAT_CONV2_DGRAD: IGEMM_LAUNCH_U(NatD2, 1, 2, 2, 1, 2, 2, 8); return 0;     // 32 k-steps
    default: return -1;
  }
}

#define WGRAD_LAUNCH(LD, MC, KB, NB)                                                                   \
  do {                                                                                                 \
    dim3 grid((a.M + MC - 1) / MC, (a.K + KB - 1) / KB, (g.N + NB - 1) / NB);                          \
    WgradArgs gg = g;                                                                                  \
    gg.atomic = grid.x > 1 ? 1 : 0;                                                                    \
    hipLaunchKernelGGL((wgrad_kernel<LD, MC, KB, NB>), grid, dim3(256), 0, st, a, gg);                 \
  } while (0)

int launch_wgrad(int kind, const ConvArgs& a, const WgradArgs& g, hipStream_t st) {
  switch (kind) {
    case L_NAT_CONV1_FWD: WGRAD_LAUNCH(NatC1, 128, 256, 32); return 0;   // 100 chunks (B=32)
    case L_NAT_CONV1_FRAMES: WGRAD_LAUNCH(NatF1, 128, 256, 32); return 0;
    case L_NAT_CONV2_FWD: WGRAD_LAUNCH(NatC2, 128, 128, 64); return 0;   // 21 x 4 blocks
    case L_NAT_CONV3_FWD: WGRAD_LAUNCH(NatC3, 128, 192, 64); return 0;   // 13 x 3 blocks
    case L_DENSE_FWD_RELU: WGRAD_LAUNCH(DenseLoader, 32, 64, 128); return 0;
    default: return -1;
  }
}

// ---- grouped weight gradients: every layer's wgrad in ONE launch (they are
// independent once the dgrad chain produced all dZ). Block ranges per member,
// longest member first; each block runs its member's wgrad_block.
namespace dqn {
template <class LD, int MC, int KB, int NB>
DQN_DEV void group_member(const ConvArgs& a, const WgradArgs& g, int b, int gx, int gy, act_t* lds) {
  const int bx = b % gx, r = b / gx, by = r % gy, bz = r / gy;
  wgrad_block<LD, MC, KB, NB>(a, g, bx, by, bz, lds);
}

__global__ void __launch_bounds__(256) wgrad_group_kernel(WgradGroup G) {
  extern __shared__ __attribute__((aligned(16))) act_t glds[];
  int b = blockIdx.x, i = 0;
  while (i < G.n - 1 && b >= G.nblk[i]) { b -= G.nblk[i]; ++i; }
  switch (G.kind[i]) {
    case L_NAT_CONV1_FWD: group_member<NatC1, 128, 256, 32>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;
    case L_NAT_CONV1_FRAMES: group_member<NatF1, 128, 256, 32>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;
    case L_NAT_CONV2_FWD: group_member<NatC2, 128, 128, 64>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;
    case L_NAT_CONV3_FWD: group_member<NatC3, 128, 192, 64>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;
    case L_DENSE_FWD_RELU: group_member<DenseLoader, 32, 64, 128>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;
    default: break;
  }
}
}  // namespace dqn

static bool wgrad_tiles(int kind, int& MC, int& KB, int& NB, size_t& lds) {
  switch (kind) {
    case L_NAT_CONV1_FWD: case L_NAT_CONV1_FRAMES: MC = 128; KB = 256; NB = 32; break;
    case L_NAT_CONV2_FWD: MC = 128; KB = 128; NB = 64; break;
    case L_NAT_CONV3_FWD: MC = 128; KB = 192; NB = 64; break;
    case L_DENSE_FWD_RELU: MC = 32; KB = 64; NB = 128; break;
    default: return false;
  }
  lds = (size_t)(KB + NB) * (MC + 8) * sizeof(act_t);
  return true;
}

int launch_wgrad_group(WgradGroup G, hipStream_t st) {
  int total = 0;
  size_t lds = 0;
  for (int i = 0; i < G.n; ++i) {
    int MC, KB, NB;
    size_t l;
    if (!wgrad_tiles(G.kind[i], MC, KB, NB, l)) return -1;
    G.gx[i] = (G.a[i].M + MC - 1) / MC;
    G.gy[i] = (G.a[i].K + KB - 1) / KB;
    const int gz = (G.g[i].N + NB - 1) / NB;
    G.nblk[i] = G.gx[i] * G.gy[i] * gz;
    G.g[i].atomic = G.gx[i] > 1 ? 1 : 0;
    total += G.nblk[i];
    lds = l > lds ? l : lds;
  }
  hipLaunchKernelGGL(wgrad_group_kernel, dim3(total), dim3(256), lds, st, G);
  return 0;
}

void launch_head_loss(const HeadArgs& a, hipStream_t st) {
  const size_t lds = (size_t)(kHeadPartFloats + 4 * a.B * a.A + 4 * a.B + 32 + kHeadActorScratch +
                              4 * kHeadMaxA) * sizeof(float);
  static size_t lds_set = 64 * 1024;          // dynamic LDS above 64 KB must be opted into
  if (lds > lds_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(head_loss_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    lds_set = lds;
  }
  // training: 8 blocks share the backward (+1 fused acting block); acting (infer): one block
  hipLaunchKernelGGL(head_loss_kernel, dim3(a.infer ? 1 : 8 + (a.act_E > 0 ? 1 : 0)), dim3(1024), lds, st, a);
}
