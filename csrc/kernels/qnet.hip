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
#include <stdio.h>
#include <stdlib.h>
#include "common.h"
#include "actor_dev.h"
#include "../include/dqn_nets_k.h"
#include "xgmi_dev.h"
#include "wgrad_dev.h"

namespace dqn {

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

// Write-through (agent-scope) store of one act_t of an MFMA C/D tile: 32-bit stores, 16-bit types
// pair with the adjacent column held by lane ^ 1 (both lanes of a pair are active together: same
// row, N even). For outputs another block of the same launch reads after a counter.
DQN_DEV void store_wt(act_t* p, act_t v, int lane) {
#if DQN_ACT_F32
  (void)lane;
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
#else
  const uint32_t mine = (uint32_t)__builtin_bit_cast(uint16_t, v);
  const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1, 64);
  if ((lane & 1) == 0)
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), mine | (other << 16), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// ============================================================ implicit GEMM
// Block = WM x WN x KSPLIT waves (4 or 8); wave tile = (MT*16) x (NT*16).
// EPI: 0 = scale*acc + bias, ReLU, bf16 out; 1 = scale*acc + bias, fp32 out (no ReLU);
//      2 = acc * (mask > 0), bf16 out (ReLU backward through the layer input).
// Body of one block (bx, by, bz) of a virtual (gx, gy, gz) GEMM grid: shared by igemm_kernel and
// the chained dgrad launch (dgrad_chain.hip). WT: the EPI 2 output leaves as write-through 32-bit
// stores (agent scope: another block of the same launch reads it after a counter).
// FZ: the factorised noisy forward of ConvArgs.fz_* (a second accumulator over the sigma fragments
// with the A fragments scaled by f(eps_in), staged in LDS; f(eps_out) joins in the epilogue).
// dblk / dnblk (>= 0 / > 0): this block's index / the block count for the side duties when the
// launch's grid is not the (gx, gy, gz) of this body (fc_fwd_fz_kernel)
constexpr int kFzMaxK = 4096;
template <class LD, int MT, int NT, int WM, int WN, int KSPLIT, int EPI, int U = 4, bool WT = false, bool FZ = false>
DQN_DEV void igemm_body(const ConvArgs& a, int bx, int by, int bz, int gx, int gy, int gz, int dblk = -1,
                        int dnblk = 0) {
  static_assert(WM * WN * KSPLIT == 4 || WM * WN * KSPLIT == 8, "4 or 8 waves per block");
  static_assert(!FZ || (EPI == 0 && WM * WN == 1), "factorised forward: dense forward tiles");
  __shared__ float red[KSPLIT > 1 ? (FZ ? 2 : 1) * WM * WN * (KSPLIT - 1) * MT * NT * 256 : 1];
  __shared__ float fin_s[FZ ? kFzMaxK : 1];
  const int inst = bz;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wk = wave % KSPLIT, wn = (wave / KSPLIT) % WN, wm = wave / (KSPLIT * WN);
  const int m_base = bx * (WM * MT * 16) + wm * MT * 16;
  const int nt_base = by * (WN * NT) + wn * NT;
  const int K32 = (a.K + 31) / 32;
  const bfx8* __restrict__ Bp = reinterpret_cast<const bfx8*>(a.w[inst]);

  f32x4 acc[MT][NT], acc2[FZ ? MT : 1][FZ ? NT : 1];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if constexpr (FZ) acc2[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  // FZ: the block's column half (its eps_in / eps_out segment; nsplit % 16 == 0, NT == 1)
  const int fzh = FZ && nt_base * 16 >= a.fz_nsplit ? 1 : 0;
  const bfx8* __restrict__ Bp2 = reinterpret_cast<const bfx8*>(FZ ? a.fz_w2 : nullptr);

  // each lane owns row (lane & 15) of every m-tile and k-group (lane >> 4)
  LD ld[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) ld[i] = LD(a, inst, m_base + i * 16 + (lane & 15));
  const int kg = 8 * (lane >> 4);
  const int ks_lo = (K32 * wk) / KSPLIT, ks_hi = (K32 * (wk + 1)) / KSPLIT;
  // EPI 2: the ReLU-mask operand of the epilogue is loaded NOW (clamped indices, no branch
  // per load) so its latency hides under the k-loop instead of serialising the epilogue
  float mk[EPI == 2 ? MT : 1][EPI == 2 ? NT : 1][4];
  if constexpr (EPI == 2) {
    if (wk == 0) {
      const act_t* __restrict__ msrc = reinterpret_cast<const act_t*>(a.mask[inst]);
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = min((nt_base + j) * 16 + (lane & 15), a.N - 1);
            const int m = min(m_base + i * 16 + 4 * (lane >> 4) + r, a.M - 1);
            mk[i][j][r] = (float)msrc[(int64_t)m * a.ldo + n];
          }
    }
  }
  // U k-steps per batch: all A/B fragment loads of the batch are issued before
  // its MFMAs, so U x (MT + NT) global loads are in flight per wave (the loop
  // is latency-bound at these sizes, not MFMA-bound). A partial last batch is
  // predicated (zero fragments) instead of falling back to one step at a time;
  // a U that covers the wave's whole K range pays the load latency once.
  for (int ks = ks_lo; ks < ks_hi; ks += U) {
    bfx8 af[U][MT], bf[U][NT], bf2[FZ ? U : 1][FZ ? NT : 1];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool kok = ks + u < ks_hi;
#pragma unroll
      for (int i = 0; i < MT; ++i) af[u][i] = kok ? ld[i].frag((ks + u) * 32 + kg) : zero8();
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int64_t bo = ((int64_t)(ks + u) * a.N16 + nt_base + j) * 64 + lane;
        bf[u][j] = kok ? Bp[bo] : zero8();
        if constexpr (FZ) bf2[u][j] = kok ? Bp2[bo] : zero8();
      }
    }
    if constexpr (FZ) {
      // f(eps_in) of the whole K into LDS while the fragments above are in flight (every wave
      // has exactly one first batch: the host checks K32 >= KSPLIT); [K, K32 * 32) = 0
      if (ks == ks_lo) {
        const float* ein = a.fz_noise + a.fz_ein[fzh];
        for (int k = (int)threadIdx.x; k < K32 * 32; k += (int)blockDim.x) {
          const float x = k < a.K ? ein[k] : 0.f;
          fin_s[k] = copysignf(sqrtf(fabsf(x)), x);
        }
        __syncthreads();
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float fv[8];
      if constexpr (FZ) {
        // (a batch step past the wave's range reads the first k-step: its A fragment is zero, and
        //  LDS past the staged K could hold NaN patterns)
        const int kf = (ks + u < ks_hi ? ks + u : ks_lo) * 32 + kg;
        const float4 f0 = *reinterpret_cast<const float4*>(fin_s + kf);
        const float4 f1 = *reinterpret_cast<const float4*>(fin_s + kf + 4);
        fv[0] = f0.x; fv[1] = f0.y; fv[2] = f0.z; fv[3] = f0.w; fv[4] = f1.x; fv[5] = f1.y; fv[6] = f1.z; fv[7] = f1.w;
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[u][i], bf[u][j], acc[i][j]);
        if constexpr (FZ) {
          bfx8 as;
#pragma unroll
          for (int q = 0; q < 8; ++q) as[q] = (act_t)((float)af[u][i][q] * fv[q]);
#pragma unroll
          for (int j = 0; j < NT; ++j) acc2[i][j] = mfma16(as, bf2[u][j], acc2[i][j]);
        }
      }
    }
  }
  // side-duty block index / count (GEMM blocks only)
  const int dn = dnblk > 0 ? dnblk : gx * gy * gz;
  const int db = dnblk > 0 ? dblk : (bz * gy + by) * gx + bx;
  // noise duty (every thread of the block, before the split-K waves retire)
  if (a.nz_out0 != nullptr) {
    const int nblk = dn, blk = db;
    const int nq = ((a.nz_out1 != nullptr ? 2 : 1) * a.nz_n + 3) / 4;
    const int nt = blockDim.x, tq = (int)threadIdx.x;
    const uint64_t seed = (uint64_t)a.nz_rng[0], ctr = (uint64_t)a.nz_rng[1];
    for (int q = blk * nt + tq; q < nq; q += nblk * nt) noise_normals4(a.nz_out0, a.nz_out1, a.nz_n, seed, ctr, q);
  }
  if constexpr (KSPLIT > 1) {
    // waves wk > 0 hand partial tiles to wk == 0 through LDS
    const int slot = ((wm * WN + wn) * (KSPLIT - 1));
    constexpr int kHalf = WM * WN * (KSPLIT - 1) * MT * NT * 256;     // (FZ: acc2 partials after acc's)
    if (wk > 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            red[(((slot + wk - 1) * MT + i) * NT + j) * 256 + r * 64 + lane] = acc[i][j][r];
            if constexpr (FZ) red[kHalf + (((slot + wk - 1) * MT + i) * NT + j) * 256 + r * 64 + lane] = acc2[i][j][r];
          }
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
          for (int r = 0; r < 4; ++r) {
            acc[i][j][r] += red[(((slot + s) * MT + i) * NT + j) * 256 + r * 64 + lane];
            if constexpr (FZ) acc2[i][j][r] += red[kHalf + (((slot + s) * MT + i) * NT + j) * 256 + r * 64 + lane];
          }
  }
  // side duties of the launch (ConvArgs aux): zero a gradient range (the conv weight gradients
  // accumulate into it with atomics later in the step) and sum the head's per-tile loss partials
  if (a.zero_ptr != nullptr) {
    const int nblk = dn, blk = db;
    float4* z4 = reinterpret_cast<float4*>(a.zero_ptr);
    for (int t = blk * 64 + lane; t < a.zero_n / 4; t += nblk * 64) z4[t] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (a.loss_parts != nullptr && db == 0) {
    const float v = lane < a.nparts ? a.loss_parts[lane] : 0.f;
    const float sl = wave_sum(v);
    if (lane == 0) a.loss_out[0] = sl * a.loss_mul;
  }
  // epilogue: C/D layout col = lane & 15, row = 4*(lane >> 4) + r
  const float scale = a.scale[inst];
  const float* __restrict__ bias = a.bias[inst];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = (nt_base + j) * 16 + (lane & 15);
    if (n >= a.N) continue;
    const float bv = (EPI == 2 || bias == nullptr) ? 0.f : bias[n];
    float fo = 0.f;                                                 // FZ: f(eps_out[n])
    if constexpr (FZ) {
      const float x = a.fz_noise[a.fz_eout[fzh] + n - (fzh ? a.fz_nsplit : 0)];
      fo = copysignf(sqrtf(fabsf(x)), x);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m_base + i * 16 + 4 * (lane >> 4) + r;
        if (m >= a.M) continue;
        float v = acc[i][j][r];
        if constexpr (FZ) v += fo * acc2[i][j][r];
        const int64_t o = (int64_t)m * a.ldo + n;
        if constexpr (EPI == 0) {
          v = fmaxf(v * scale + bv, 0.f);
          reinterpret_cast<act_t*>(a.out[inst])[o] = (act_t)v;
        } else if constexpr (EPI == 1) {
          reinterpret_cast<float*>(a.out[inst])[o] = v * scale + bv;
        } else if constexpr (!WT) {
          reinterpret_cast<act_t*>(a.out[inst])[o] = (act_t)(mk[i][j][r] > 0.f ? v : 0.f);
        } else {
          const act_t q = (act_t)(mk[i][j][r] > 0.f ? v : 0.f);
          store_wt(reinterpret_cast<act_t*>(a.out[inst]) + o, q, lane);
        }
      }
    }
  }
}

template <class LD, int MT, int NT, int WM, int WN, int KSPLIT, int EPI, int U = 4>
__global__ void __launch_bounds__(512) igemm_kernel(ConvArgs a) {
  if (a.gth != nullptr && (int)blockIdx.z == a.gth_z) {
    // side duty: the low-rank DP all-gather (its own grid.z slice; every block of it returns
    // here, uniformly, before any barrier of the GEMM body)
    const int gb = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    if (gb < a.gth_blocks) xgmi_gather_block(*reinterpret_cast<const XgmiGatherArgs*>(a.gth), gb, a.gth_blocks);
    return;
  }
  igemm_body<LD, MT, NT, WM, WN, KSPLIT, EPI, U>(a, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, gridDim.y,
                                                 gridDim.z - (a.gth != nullptr ? 1 : 0));
}

// Dense forward with a factorised noisy instance (ConvArgs.fz_*): grid (2, N/16, ninst). The
// factorised instance runs 16-row blocks (bx = row block: its blocks stream two B operands, so half
// the A rows keep their L2->CU bytes at the plain blocks'), every other instance the 32-row tiles
// of L_DENSE_FWD_RELU on bx == 0 (bx == 1 exits). Side duties over the active blocks.
template <int U>
__global__ void __launch_bounds__(512) fc_fwd_fz_kernel(ConvArgs a) {
  const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z, gy = gridDim.y, gz = gridDim.z;
  const int nact = gy * (gz + 1);
  if (bz == a.fz_inst) {
    igemm_body<DenseLoader, 1, 1, 1, 1, 8, 0, U, false, true>(a, bx, by, bz, 2, gy, gz, gy * (gz - 1) + by * 2 + bx,
                                                             nact);
  } else if (bx == 0) {
    igemm_body<DenseLoader, 2, 1, 1, 1, 8, 0, U>(a, 0, by, bz, 1, gy, gz, (bz - (bz > a.fz_inst ? 1 : 0)) * gy + by,
                                                 nact);
  }
}

// ===================================================== stride-2 dgrad by parity
// dX[b][iy][ix][ci] = sum_{kh,kw,co} dZ[b][(iy-kh)/2][(ix-kw)/2][co] W[kh][kw][ci][co] of a
// VALID stride-2 conv: only the taps with kh = iy mod 2 (+2), kw = ix mod 2 (+2) reach a given
// input pixel, so the implicit GEMM over all KH*KW taps (DgradLoader) multiplies 3 of every 4
// A fragments by zero. Here the input pixels are grouped by parity class (iy & 1, ix & 1): a
// class's rows share ONE 2x2 tap subset, K shrinks to (KH/2)(KW/2)*COUT (256 for Nature conv2,
// 8 k-steps instead of 32) and every fragment is a real one. Block = 16 rows of one class x all
// N (2 n-tiles) x the class's K in two halves (4 waves); the epilogue scatters the rows back
// to NHWC with the ReLU mask of the layer input.
template <int COUT, int KH, int KW>
DQN_DEV void dgrad_s2_body(const ConvArgs& a, int bx, int inst) {
  static_assert(KH % 2 == 0 && KW % 2 == 0 && COUT % 32 == 0, "2x2 tap classes, 32-deep k-steps");
  constexpr int CK = COUT / 32;                            // k-steps per tap
  constexpr int KSC = (KH / 2) * (KW / 2) * CK;            // the class's k-steps (8)
  constexpr int KHALF = KSC / 2;
  const int PH = a.IH / 2, PW = a.IW / 2, crow = PH * PW, cmt = (crow + 15) / 16;
  int blk = bx;
  const int mt = blk % cmt;
  blk /= cmt;
  const int cls = blk & 3, b = blk >> 2, cy = cls >> 1, cx = cls & 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nt = wave & 1, kh2 = wave >> 1;                // n-tile, k-half
  const int kg = 8 * (lane >> 4);
  const int r = mt * 16 + (lane & 15);                     // this lane's A row within the class
  const bool rok = r < crow;
  const int py = rok ? r / PW : 0, px = rok ? r - py * PW : 0;
  const act_t* dz = reinterpret_cast<const act_t*>(a.in[inst]) + (int64_t)b * a.OH * a.OW * COUT;
  const bfx8* __restrict__ Bp = reinterpret_cast<const bfx8*>(a.w[inst]);
  const act_t* __restrict__ msrc = reinterpret_cast<const act_t*>(a.mask[inst]);
  // epilogue mask operand first (its latency hides under the k-loop): rows 4 (lane >> 4) + i
  float mk[4];
  int64_t orow[4];
  const int n = nt * 16 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = mt * 16 + 4 * (lane >> 4) + i;
    const int q = rr < crow ? rr : 0, qy = q / PW, qx = q - qy * PW;
    orow[i] = rr < crow ? ((int64_t)(b * a.IH + 2 * qy + cy) * a.IW + 2 * qx + cx) : -1;
    mk[i] = kh2 == 0 && orow[i] >= 0 && n < a.N ? (float)msrc[orow[i] * a.ldo + n] : 0.f;
  }
  bfx8 af[KHALF], bf[KHALF];
#pragma unroll
  for (int u = 0; u < KHALF; ++u) {
    const int sidx = kh2 * KHALF + u, t = sidx / CK, h = sidx - t * CK;
    const int dh = t / (KW / 2), dw = t - dh * (KW / 2);
    const int kh = cy + 2 * dh, kw = cx + 2 * dw;
    const int oy = py - dh, ox = px - dw;
    const bool ok = rok && oy >= 0 && ox >= 0 && oy < a.OH && ox < a.OW;
    af[u] = ok ? *reinterpret_cast<const bfx8*>(dz + ((int64_t)oy * a.OW + ox) * COUT + h * 32 + kg) : zero8();
    const int ks = (kh * KW + kw) * CK + h;                // packed dgrad k-step of (tap, co-half)
    bf[u] = Bp[((int64_t)ks * a.N16 + nt) * 64 + lane];
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < KHALF; ++u) acc = mfma16(af[u], bf[u], acc);
  __shared__ f32x4 red[2][64];
  if (kh2 == 1) red[nt][lane] = acc;
  __syncthreads();
  if (kh2 == 1 || n >= a.N) return;
  acc += red[nt][lane];
  act_t* out = reinterpret_cast<act_t*>(a.out[inst]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (orow[i] >= 0) out[orow[i] * a.ldo + n] = (act_t)(mk[i] > 0.f ? acc[i] : 0.f);
}

template <int COUT, int KH, int KW>
__global__ void __launch_bounds__(256) dgrad_s2_kernel(ConvArgs a) {
  dgrad_s2_body<COUT, KH, KW>(a, blockIdx.x, blockIdx.z);
}

// ================================================================ weight grad
// dW[k][n] (+)= scale * sum_{m in chunk} A[m][k] * dZ[m][n];  db[n] (+)= sum_m dZ[m][n]
// grid: x = M-chunk (MC rows), y = K-range (KB), z = N-range (NB). ONE staging
// pass per block: all global loads of the chunk are issued first (register
// staging), then written TRANSPOSED to LDS ([k][m], [n][m], rows padded by 8
// elements) so each lane's 8 consecutive m are one ds_read_b128; then
// (KB/16)x(NB/16) output tiles x MC/32 MFMA k-steps. fp32 atomics only when
// more than one M-chunk contributes to a weight.
// Body shared by the per-layer launch and the grouped launch (one block = one
// (M-chunk, K-range, N-range) tile; LDS passed in so a grouped kernel can carve
// every member's staging from one buffer).
#if DQN_ACT_F32
template <class LD, int MC, int KB, int NB>
DQN_DEV void wgrad_block(const ConvArgs& a, const WgradArgs& g, int bx, int by, int bz, act_t* lds) {
  constexpr int LR = WgradTile<MC, KB, NB>::LR;
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
      va[i] = sel8(k0 < a.K, ld.frag(min(k0, a.K - 8)));          // (clamped: no branch per load)
    }
#pragma unroll
    for (int i = 0; i < GZ; ++i) {
      const int c8 = (p + i * TPR) * 8;
      const int cz = (n_lo + c8 < g.N ? n_lo + c8 : 0) - n_lo;     // masked groups read column 0
      vz[i] = sel8(mok && n_lo + c8 < g.N, *reinterpret_cast<const bfx8*>(dz + cz));
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

#else
template <class LD, int MC, int KB, int NB>
DQN_DEV void wgrad_block(const ConvArgs& a, const WgradArgs& g, int bx, int by, int bz, act_t* lds) {
  using Tl = WgradTile<MC, KB, NB>;
  constexpr int SA = Tl::SA, SZ = Tl::SZ;
  constexpr int TPR = 256 / MC;                  // threads per staged row
  constexpr int GA = KB / 8 / TPR, GZ = NB / 8 / TPR;
  constexpr int TILES = (KB / 16) * (NB / 16), PERW = TILES / 4, KSTEPS = MC / 32;
  static_assert(256 % MC == 0 && (KB / 8) % TPR == 0 && (NB / 8) % TPR == 0 && TILES % 4 == 0, "tiling");
  act_t* At = lds;                               // [MC][SA]
  act_t* Zt = lds + MC * SA;                     // [MC][SZ]
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
      va[i] = sel8(k0 < a.K, ld.frag(min(k0, a.K - 8)));          // (clamped: no branch per load)
    }
#pragma unroll
    for (int i = 0; i < GZ; ++i) {
      const int c8 = (p + i * TPR) * 8;
      const int cz = (n_lo + c8 < g.N ? n_lo + c8 : 0) - n_lo;     // masked groups read column 0
      vz[i] = sel8(mok && n_lo + c8 < g.N, *reinterpret_cast<const bfx8*>(dz + cz));
    }
#pragma unroll
    for (int i = 0; i < GA; ++i) *reinterpret_cast<bfx8*>(At + r * SA + (((p + i * TPR) * 8) ^ wsw(r))) = va[i];
#pragma unroll
    for (int i = 0; i < GZ; ++i) *reinterpret_cast<bfx8*>(Zt + r * SZ + (((p + i * TPR) * 8) ^ wsw(r))) = vz[i];
  }
  __syncthreads();
  const bool atomic = g.atomic != 0;
  if (g.db != nullptr && by == 0) {
    for (int n = threadIdx.x; n < NB; n += 256) {
      float s = 0.f;
#pragma unroll 8
      for (int r = 0; r < MC; ++r) s += (float)Zt[r * SZ + (n ^ wsw(r))];
      const int nn = n_lo + n;
      if (nn < g.N) {
        float* pdb = nn < g.nsplit ? g.db + nn : g.db2 + (nn - g.nsplit);
        s *= kInvLossScale;
        if (atomic) atomicAdd(pdb, s); else *pdb = s;
      }
    }
  }
  // operand lane map: k-group gq = lane >> 4 takes m rows {4 gq + q} (elements 0..3) and
  // {16 + 4 gq + q} (elements 4..7) of each 32-row k-step -- the same permutation of the
  // reduction index on both operands; one 32-lane half reads 8 consecutive rows per instruction
  const int gq = lane >> 4, rq = (lane >> 2) & 3, cp = 4 * (lane & 3);
  constexpr int NTt = NB / 16;
#pragma unroll
  for (int i = 0; i < PERW; ++i) {
    const int tile = wave + 4 * i;
    const int kt = tile / NTt, nt = tile - kt * NTt;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const act_t* pa = At + (4 * gq + rq) * SA + kt * 16 + (cp ^ wsw(4 * gq));
    const act_t* pz = Zt + (4 * gq + rq) * SZ + nt * 16 + (cp ^ wsw(4 * gq));
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const bfx8 af = join_tr(lds_tr16(pa + 32 * s * SA), lds_tr16(pa + (32 * s + 16) * SA));
      const bfx8 bf = join_tr(lds_tr16(pz + 32 * s * SZ), lds_tr16(pz + (32 * s + 16) * SZ));
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

// Deterministic grouped mode (no atomics): chunks bx .. bx + nch - 1 summed in registers in
// ascending order, then plain stores (the caller points dw / db at its partial slice)
template <class LD, int MC, int KB, int NB>
DQN_DEV void wgrad_block_det(const ConvArgs& a, const WgradArgs& g, int bx, int by, int bz, act_t* lds, int nch) {
  using Tl = WgradTile<MC, KB, NB>;
  constexpr int SA = Tl::SA, SZ = Tl::SZ;
  constexpr int TPR = 256 / MC;                  // threads per staged row
  constexpr int GA = KB / 8 / TPR, GZ = NB / 8 / TPR;
  constexpr int TILES = (KB / 16) * (NB / 16), PERW = TILES / 4, KSTEPS = MC / 32;
  static_assert(256 % MC == 0 && (KB / 8) % TPR == 0 && (NB / 8) % TPR == 0 && TILES % 4 == 0 && NB <= 256,
                "tiling");
  act_t* At = lds;                               // [MC][SA]
  act_t* Zt = lds + MC * SA;                     // [MC][SZ]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k_lo = by * KB, n_lo = bz * NB;
  const bool dob = g.db != nullptr && by == 0;
  // operand lane map: k-group gq = lane >> 4 takes m rows {4 gq + q} (elements 0..3) and
  // {16 + 4 gq + q} (elements 4..7) of each 32-row k-step -- the same permutation of the
  // reduction index on both operands; one 32-lane half reads 8 consecutive rows per instruction
  const int gq = lane >> 4, rq = (lane >> 2) & 3, cp = 4 * (lane & 3);
  constexpr int NTt = NB / 16;
  f32x4 acc[PERW];
#pragma unroll
  for (int i = 0; i < PERW; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbs = 0.f;
  for (int c = 0; c < nch; ++c) {
    const int r = threadIdx.x % MC, p = threadIdx.x / MC;
    const int m = (bx + c) * MC + r;
    const bool mok = m < a.M;
    const act_t* dz = reinterpret_cast<const act_t*>(g.dz) + (int64_t)(mok ? m : 0) * g.ldz + n_lo;
    LD ld(a, 0, m);
    bfx8 va[GA], vz[GZ];
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int k0 = k_lo + (p + i * TPR) * 8;
      va[i] = sel8(k0 < a.K, ld.frag(min(k0, a.K - 8)));          // (clamped: no branch per load)
    }
#pragma unroll
    for (int i = 0; i < GZ; ++i) {
      const int c8 = (p + i * TPR) * 8;
      const int cz = (n_lo + c8 < g.N ? n_lo + c8 : 0) - n_lo;     // masked groups read column 0
      vz[i] = sel8(mok && n_lo + c8 < g.N, *reinterpret_cast<const bfx8*>(dz + cz));
    }
    if (c > 0) __syncthreads();                  // the previous chunk's LDS reads are done
#pragma unroll
    for (int i = 0; i < GA; ++i) *reinterpret_cast<bfx8*>(At + r * SA + (((p + i * TPR) * 8) ^ wsw(r))) = va[i];
#pragma unroll
    for (int i = 0; i < GZ; ++i) *reinterpret_cast<bfx8*>(Zt + r * SZ + (((p + i * TPR) * 8) ^ wsw(r))) = vz[i];
    __syncthreads();
    if (dob && (int)threadIdx.x < NB) {
#pragma unroll 8
      for (int q = 0; q < MC; ++q) dbs += (float)Zt[q * SZ + ((int)threadIdx.x ^ wsw(q))];
    }
#pragma unroll
    for (int i = 0; i < PERW; ++i) {
      const int tile = wave + 4 * i;
      const int kt = tile / NTt, nt = tile - kt * NTt;
      const act_t* pa = At + (4 * gq + rq) * SA + kt * 16 + (cp ^ wsw(4 * gq));
      const act_t* pz = Zt + (4 * gq + rq) * SZ + nt * 16 + (cp ^ wsw(4 * gq));
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        const bfx8 af = join_tr(lds_tr16(pa + 32 * s * SA), lds_tr16(pa + (32 * s + 16) * SA));
        const bfx8 bf = join_tr(lds_tr16(pz + 32 * s * SZ), lds_tr16(pz + (32 * s + 16) * SZ));
        acc[i] = mfma16(af, bf, acc[i]);
      }
    }
  }
  const bool atomic = g.atomic != 0;
  if (dob && (int)threadIdx.x < NB) {
    const int nn = n_lo + threadIdx.x;
    if (nn < g.N) {
      float* pdb = nn < g.nsplit ? g.db + nn : g.db2 + (nn - g.nsplit);
      const float s = dbs * kInvLossScale;
      if (atomic) atomicAdd(pdb, s); else *pdb = s;
    }
  }
#pragma unroll
  for (int i = 0; i < PERW; ++i) {
    const int tile = wave + 4 * i;
    const int kt = tile / NTt, nt = tile - kt * NTt;
    const int n = n_lo + nt * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k_lo + kt * 16 + 4 * (lane >> 4) + q;
      if (k < a.K && n < g.N) {
        float* o = n < g.nsplit ? g.dw + (int64_t)k * g.nsplit + n
                                : g.dw2 + (int64_t)k * (g.N - g.nsplit) + (n - g.nsplit);
        const float v = acc[i][q] * (g.scale * kInvLossScale);
        if (atomic) atomicAdd(o, v); else *o = v;
      }
    }
  }
}
#endif


// Multi-chunk variant (the low-rank DP member, L_DENSE_WGRAD_LR): ONE block per weight tile sums
// g.mloop consecutive MC-row chunks in a fixed order, accumulators in registers, plain stores:
// bit-identical on every rank that runs it on the same all-gathered rows. Staged like the
// fp32 build's body ([k][m] / [n][m], m contiguous) for every element type; off the critical
// path (a graph branch beside the dgrad chain), so simplicity over staging speed. g.db_zero:
// store 0 into the bias gradient (ranks != 0: the caller's all-reduce then sums it once).
template <class LD, int MC, int KB, int NB>
DQN_DEV void wgrad_block_multi(const ConvArgs& a, const WgradArgs& g, int by, int bz, act_t* lds) {
  constexpr int LR = MC + 8;                     // [k][m] / [n][m] rows (every build: see WgradTile)
  constexpr int SA = KB + 16, SZ = NB + 16;      // 16-bit builds: row-major [m][k] / [m][n] (see WgradTile)
  constexpr int TPR = 256 / MC;
  constexpr int GA = KB / 8 / TPR, GZ = NB / 8 / TPR;
  constexpr int TILES = (KB / 16) * (NB / 16), PERW = TILES / 4, KSTEPS = MC / 32;
  static_assert(256 % MC == 0 && (KB / 8) % TPR == 0 && (NB / 8) % TPR == 0 && TILES % 4 == 0 && 256 % NB == 0,
                "tiling");
  act_t* At = lds;
  act_t* Zt = lds + (DQN_ACT_F32 ? KB * LR : MC * SA);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k_lo = by * KB, n_lo = bz * NB;
  const int kg = 8 * (lane >> 4), row = lane & 15;
  constexpr int NTt = NB / 16;
  const int nch = g.mloop > 1 ? g.mloop : 1;
  f32x4 accs[PERW];
#pragma unroll
  for (int i = 0; i < PERW; ++i) accs[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbs = 0.f;
  const int r = threadIdx.x % MC, p = threadIdx.x / MC;
  // chunk c's fragments into registers; the loads of up to kGrp chunks are issued in ONE batch
  // (one memory round trip per kGrp chunks instead of one per chunk)
  constexpr int kGrp = 4;
  auto load = [&](int c, bfx8* va, bfx8* vz) {
    const int m = c * MC + r;
    const bool mok = m < a.M;
    const act_t* dz = reinterpret_cast<const act_t*>(g.dz) + (int64_t)(mok ? m : 0) * g.ldz + n_lo;
    LD ld(a, 0, m);
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int k0 = k_lo + (p + i * TPR) * 8;
      va[i] = sel8(k0 < a.K, ld.frag(min(k0, a.K - 8)));
    }
#pragma unroll
    for (int i = 0; i < GZ; ++i) {
      const int c8 = (p + i * TPR) * 8;
      const int cz = (n_lo + c8 < g.N ? n_lo + c8 : 0) - n_lo;
      vz[i] = sel8(mok && n_lo + c8 < g.N, *reinterpret_cast<const bfx8*>(dz + cz));
    }
  };
  for (int c0 = 0; c0 < nch; c0 += kGrp) {
    bfx8 va[kGrp][GA], vz[kGrp][GZ];
#pragma unroll
    for (int u = 0; u < kGrp; ++u)
      if (c0 + u < nch) load(c0 + u, va[u], vz[u]);
#pragma unroll
    for (int u = 0; u < kGrp; ++u) {
    const int c = c0 + u;
    if (c >= nch) break;
    if (c > 0) __syncthreads();                    // the previous chunk's LDS reads are done
#if DQN_ACT_F32
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int c8 = (p + i * TPR) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) At[(c8 + j) * LR + r] = va[u][i][j];
    }
#pragma unroll
    for (int i = 0; i < GZ; ++i) {
      const int c8 = (p + i * TPR) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) Zt[(c8 + j) * LR + r] = vz[u][i][j];
    }
#else
    // one ds_write_b128 per fragment; the MFMA operands come back through transposed reads
#pragma unroll
    for (int i = 0; i < GA; ++i) *reinterpret_cast<bfx8*>(At + r * SA + (((p + i * TPR) * 8) ^ wsw(r))) = va[u][i];
#pragma unroll
    for (int i = 0; i < GZ; ++i) *reinterpret_cast<bfx8*>(Zt + r * SZ + (((p + i * TPR) * 8) ^ wsw(r))) = vz[u][i];
#endif
    __syncthreads();
#if DQN_ACT_F32
    if (g.db != nullptr && by == 0) {           // column tid % NB, rows tid / NB + k * (256 / NB)
      const act_t* zr = Zt + ((int)threadIdx.x % NB) * LR;
#pragma unroll 4
      for (int q = (int)threadIdx.x / NB; q < MC; q += 256 / NB) dbs += (float)zr[q];
    }
#pragma unroll
    for (int i = 0; i < PERW; ++i) {
      const int tile = wave + 4 * i;
      const int kt = tile / NTt, nt = tile - kt * NTt;
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        const bfx8 af = *reinterpret_cast<const bfx8*>(At + (kt * 16 + row) * LR + 32 * s + kg);
        const bfx8 bf = *reinterpret_cast<const bfx8*>(Zt + (nt * 16 + row) * LR + 32 * s + kg);
        accs[i] = mfma16(af, bf, accs[i]);
      }
    }
#else
    if (g.db != nullptr && by == 0) {           // column tid % NB, rows tid / NB + k * (256 / NB)
#pragma unroll 4
      for (int q = (int)threadIdx.x / NB; q < MC; q += 256 / NB) dbs += (float)Zt[q * SZ + (((int)threadIdx.x % NB) ^ wsw(q))];
    }
    // (the same reduction-index permutation on both operands as wgrad_block's 16-bit body)
    const int gq = lane >> 4, rq = (lane >> 2) & 3, cp = 4 * (lane & 3);
#pragma unroll
    for (int i = 0; i < PERW; ++i) {
      const int tile = wave + 4 * i;
      const int kt = tile / NTt, nt = tile - kt * NTt;
      const act_t* pa = At + (4 * gq + rq) * SA + kt * 16 + (cp ^ wsw(4 * gq));
      const act_t* pz = Zt + (4 * gq + rq) * SZ + nt * 16 + (cp ^ wsw(4 * gq));
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        const bfx8 af = join_tr(lds_tr16(pa + 32 * s * SA), lds_tr16(pa + (32 * s + 16) * SA));
        const bfx8 bf = join_tr(lds_tr16(pz + 32 * s * SZ), lds_tr16(pz + (32 * s + 16) * SZ));
        accs[i] = mfma16(af, bf, accs[i]);
      }
    }
#endif
    }
  }
  if (g.db != nullptr && by == 0) {
    // the 256 / NB row-group partials of each column, summed in a fixed order
    __syncthreads();                               // every chunk's LDS reads are done
    float* red = reinterpret_cast<float*>(lds);
    red[threadIdx.x] = dbs;
    __syncthreads();
    if ((int)threadIdx.x < NB) {
      float sum = 0.f;
      for (int q = 0; q < 256 / NB; ++q) sum += red[q * NB + threadIdx.x];
      const int nn = n_lo + threadIdx.x;
      if (nn < g.N) {
        float* pdb = nn < g.nsplit ? g.db + nn : g.db2 + (nn - g.nsplit);
        *pdb = g.db_zero ? 0.f : sum * kInvLossScale;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < PERW; ++i) {
    const int tile = wave + 4 * i;
    const int kt = tile / NTt, nt = tile - kt * NTt;
    const int n = n_lo + nt * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k_lo + kt * 16 + 4 * (lane >> 4) + q;
      if (k < a.K && n < g.N) {
        float* pw = n < g.nsplit ? g.dw + (int64_t)k * g.nsplit + n
                                 : g.dw2 + (int64_t)k * (g.N - g.nsplit) + (n - g.nsplit);
        *pw = accs[i][q] * (g.scale * kInvLossScale);
      }
    }
  }
}

template <class LD, int MC, int KB, int NB>
__global__ void __launch_bounds__(256) wgrad_multi_kernel(ConvArgs a, WgradArgs g) {
  __shared__ __attribute__((aligned(16))) act_t lds[DQN_ACT_F32 ? (KB + NB) * (MC + 8) : MC * (KB + NB + 32)];
  wgrad_block_multi<LD, MC, KB, NB>(a, g, blockIdx.y, blockIdx.z, lds);
}

template <class LD, int MC, int KB, int NB>
__global__ void __launch_bounds__(256) wgrad_kernel(ConvArgs a, WgradArgs g) {
  __shared__ __attribute__((aligned(16))) act_t lds[WgradTile<MC, KB, NB>::lds_bytes / sizeof(act_t)];
  wgrad_block<LD, MC, KB, NB>(a, g, blockIdx.x, blockIdx.y, blockIdx.z, lds);
}

// =========================================================== fused head + loss
// Scalar heads (plain or dueling; MSE or Huber TD loss): output layer + TD loss + dL/dQ.
// Parallel over samples: each LEARNER block owns a 16-sample tile, computes its rows of Q
// for every instance (online(s), target(s'), online(s') for Double DQN) on MFMA with the
// K loop split over 8 waves (every load of the block issued in ONE batch: h fragments,
// packed output-layer fragments, TD inputs, biases), then the TD loss, |TD| priorities,
// dL/dQ (published as dqv [B][A + 1] = dQ | dV for the fused fc dgrad, which carries the
// head backward) and its loss partial (summed by the fc dgrad launch). Fused acting: one
// ACTING block per env computes that env's 16-row Q tile with the online weights, then the
// env's eps-greedy decision, synthetic frame and replay append; the last acting block to
// arrive (ticket) advances the cursors / eps / rng (and inserts into the PER tree).
// INFER blocks (q_values) write their rows of Q.
constexpr int kHeadRows = 16, kHeadWaves = 8, kHeadThreads = 64 * kHeadWaves;
constexpr int kHeadKPW = 2;                     // k-steps per wave: HID <= 32 * kHeadWaves * kHeadKPW = 512
constexpr int kHeadMaxNt = 3;                   // n-tiles: A <= 32 (2) + the dueling value tile
constexpr int kHeadMaxW = 512 * 33;             // output layer staged for dH: HID * A (+ HID) floats
struct HeadSmem {
  float part[kHeadWaves][3][kHeadMaxNt][256];  // per-wave split-K partial tiles
  float q[3][kHeadRows][32];                   // Q rows of the block's tile
  float v[3][kHeadRows];                       // dueling value stream
  float dq[kHeadRows][33];                     // dL/dQ rows (| dV)
  float w[kHeadMaxW];                          // online output layer: W [HID][A] then w_v [HID]
  float red[kHeadWaves];
  SumtreeLds st;                               // acting: PER insert scratch
  int flag;
};

// Q[inst][r][*] (+ V) of rows r0..r0+15 for ninst instances into S.q / S.v. Instance i reads
// hidden layer hs[i] and packed weights pw[wi[i]] / pwv[wi[i]]; biases b[wi[i]], bv[wi[i]].
DQN_DEV void head_q_tile(const HeadArgs& a, HeadSmem& S, const void* h0, const void* h1, const void* h2,
                         int w0, int w1, int w2, const int ninst, const int r0, const int nrows,
                         bfx8 (*h0f)[2] = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int A = a.A, HID = a.HID, HH = a.dueling ? 2 * HID : HID, K32 = HID / 32;
  const int ntl = a.N16 + (a.dueling ? 1 : 0);
  const int kg = 8 * (lane >> 4);
  const int row = min(r0 + (lane & 15), r0 + nrows - 1);          // clamped: no branch per load
  const int ks0 = wave * kHeadKPW;
  // one batch: every A / B fragment of this wave (<= 3 inst x 2 k-steps x (2 A + 3 B))
  bfx8 af[3][kHeadKPW][2], bf[3][kHeadKPW][kHeadMaxNt];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int ii = i < ninst ? i : 0;
    const act_t* hr = reinterpret_cast<const act_t*>(ii == 0 ? h0 : ii == 1 ? h1 : h2) + (int64_t)row * HH;
    const int wi = ii == 0 ? w0 : ii == 1 ? w1 : w2;
    const bfx8* pw = reinterpret_cast<const bfx8*>(wi == 0 ? a.pw[0] : wi == 1 ? a.pw[1] : a.pw[2]);
    const bfx8* pv = reinterpret_cast<const bfx8*>(wi == 0 ? a.pwv[0] : wi == 1 ? a.pwv[1] : a.pwv[2]);
#pragma unroll
    for (int u = 0; u < kHeadKPW; ++u) {
      const int ks = min(ks0 + u, K32 - 1);
      af[i][u][0] = *reinterpret_cast<const bfx8*>(hr + (a.dueling ? HID : 0) + ks * 32 + kg);   // plain / adv
      af[i][u][1] = a.dueling ? *reinterpret_cast<const bfx8*>(hr + ks * 32 + kg) : zero8();     // value
#pragma unroll
      for (int t = 0; t < kHeadMaxNt; ++t) {
        const bool isv = a.dueling && t == a.N16;
        const int tt = min(t, a.N16 - 1);
        bf[i][u][t] = t >= ntl ? zero8() : isv ? pv[ks * 64 + lane] : pw[(ks * a.N16 + tt) * 64 + lane];
      }
    }
  }
  if (h0f != nullptr) {                        // instance 0's h fragments (the learner's dH mask)
#pragma unroll
    for (int u = 0; u < kHeadKPW; ++u) { h0f[u][0] = af[0][u][0]; h0f[u][1] = af[0][u][1]; }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (i >= ninst) break;
#pragma unroll
    for (int t = 0; t < kHeadMaxNt; ++t) {
      if (t >= ntl) break;
      const bool isv = a.dueling && t == a.N16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < kHeadKPW; ++u)
        if (ks0 + u < K32) acc = mfma16(af[i][u][isv ? 1 : 0], bf[i][u][t], acc);
      *reinterpret_cast<f32x4*>(&S.part[wave][i][t][lane * 4]) = acc;
    }
  }
  __syncthreads();
  // sum the 8 waves' partial tiles; C/D layout: col = lane & 15, row = 4 * (lane >> 4) + r
  for (int e = tid; e < ninst * ntl * 256; e += kHeadThreads) {
    const int i = e / (ntl * 256), rem = e - i * ntl * 256, t = rem >> 8, x = rem & 255;
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < kHeadWaves; ++w) sum += S.part[w][i][t][x];
    const int ln = x >> 2, r = 4 * (ln >> 4) + (x & 3), col = ln & 15;
    const int wi = i == 0 ? w0 : i == 1 ? w1 : w2;
    if (a.dueling && t == a.N16) {
      if (col == 0) S.v[i][r] = sum + (wi == 0 ? a.bv[0] : wi == 1 ? a.bv[1] : a.bv[2])[0];
    } else {
      const int c = t * 16 + col;
      if (c < A) S.q[i][r][c] = sum + (wi == 0 ? a.b[0] : wi == 1 ? a.b[1] : a.b[2])[c];
    }
  }
  __syncthreads();
  if (a.dueling) {
    for (int e = tid; e < ninst * kHeadRows; e += kHeadThreads) {
      const int i = e / kHeadRows, r = e - i * kHeadRows;
      float mean = 0.f;
      for (int c = 0; c < A; ++c) mean += S.q[i][r][c];
      mean /= (float)A;
      for (int c = 0; c < A; ++c) S.q[i][r][c] += S.v[i][r] - mean;
    }
    __syncthreads();
  }
}

// AT = the action count at compile time (the common Atari counts; 0 = runtime): the per-action
// loops (argmax, dH inner products, dQ rows) unroll, so their LDS reads are issued together
template <int AT>
__global__ void __launch_bounds__(kHeadThreads) head_loss_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) char head_smem[];
  HeadSmem& S = *reinterpret_cast<HeadSmem*>(head_smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int A = AT > 0 ? AT : a.A, A1 = A + 1;
  const int nlearn = a.infer ? 0 : (a.B + kHeadRows - 1) / kHeadRows;
  const bool acting = a.infer ? a.has_actor != 0 : (a.act_E > 0 && (int)blockIdx.x >= nlearn);
  int64_t* prof = (a.prof != nullptr && tid == 0 && (blockIdx.x == 0 || (acting && (int)blockIdx.x == nlearn)))
                      ? a.prof + (acting ? 16 : 0) : nullptr;
#define HEAD_MARK(i) if (prof) prof[i] = (int64_t)__builtin_amdgcn_s_memtime()
  HEAD_MARK(0);
  if (acting) {
    // ---- one env per block: its 16-row Q tile (online weights), then that env's step
    const int e = (int)blockIdx.x - nlearn;
    const ActorArgs& x = a.actor;
    const int E = x.E;
    const ActorPre pre = actor_prefetch(x);                      // overlaps the Q loads
    int32_t st_e[4] = {0, 0, 0, 0};                              // env e's frame stack (thread 0)
    if (tid == 0)
      for (int c = 0; c < 4; ++c) st_e[c] = x.stacks[(int64_t)e * x.K + min(c, x.K - 1)];
    // env e's frames first (rng-only), then its Q row, then decision / append / advance
    actor_env_frames(x, e, pre);
    const int r0 = (e / kHeadRows) * kHeadRows;
    const void* hh = a.infer ? a.h[0] : a.act_h;
    head_q_tile(a, S, hh, hh, hh, 0, 0, 0, 1, r0, min(kHeadRows, E - r0));
    HEAD_MARK(1);
    const float* qe = &S.q[0][e - r0][0];
    if (a.infer && a.q_out != nullptr && tid < A) a.q_out[(int64_t)e * A + tid] = qe[tid];
    __syncthreads();
    HEAD_MARK(2);
    actor_env_finish(x, qe, e, pre, st_e, &S.flag, S.st);
    HEAD_MARK(3);
    return;
  }
  const int r0 = (int)blockIdx.x * kHeadRows, nrows = min(kHeadRows, a.B - r0);
  if (a.infer) {                                               // q_values: rows of Q
    head_q_tile(a, S, a.h[0], a.h[0], a.h[0], 0, 0, 0, 1, r0, nrows);
    if (a.q_out != nullptr)
      for (int t = tid; t < nrows * A; t += kHeadThreads) a.q_out[(int64_t)r0 * A + t] = S.q[0][t / A][t % A];
    return;
  }
  // ---- learner tile: TD inputs and the online output layer (for dH) first: their loads join
  //      the Q tile's batch (clamped indices: unconditional loads)
  const int ninst = a.h[2] != nullptr ? 3 : 2;
  const int HID = a.HID, HH = a.dueling ? 2 * HID : HID;
  float tr = 0.f, tg = 0.f, td = 0.f, tw = 1.f;
  int ta = 0;
  if (tid < nrows) {
    const int b = r0 + tid;
    tr = a.rew[b]; tg = a.gam[b]; td = a.done[b]; ta = a.act[b];
    if (a.wts != nullptr) tw = a.wts[b];
  }
  const int nw = HID * A, nwt = nw + (a.dueling ? HID : 0);
  // (clamped indices, unconditional loads: a predicated load per iteration compiles to a branch
  //  + wait each; AT known: just enough iterations for HID <= 512)
  constexpr int kWIt = AT > 0 ? (512 * (AT + 1) + kHeadThreads - 1) / kHeadThreads : kHeadMaxW / kHeadThreads;
  float wr[kWIt];
#pragma unroll
  for (int i = 0; i < kWIt; ++i) {
    const int t = min(tid + kHeadThreads * i, nwt - 1);
    wr[i] = t < nw ? a.w[0][t] : a.wv[0][t - nw];
  }
  bfx8 h0f[kHeadKPW][2];
  head_q_tile(a, S, a.h[0], a.h[1], a.h[2], 0, 1, 2, ninst, r0, nrows, h0f);
#pragma unroll
  for (int i = 0; i < kWIt; ++i)
    if (tid + kHeadThreads * i < nwt) S.w[tid + kHeadThreads * i] = wr[i];
  HEAD_MARK(1);
  float contrib = 0.f;
  if (tid < nrows) {
    const int b = r0 + tid;
    const float* sel = &S.q[ninst == 3 ? 2 : 1][tid][0];
    int best = 0;
    float bvv = sel[0];
#pragma unroll
    for (int i = 1; i < (AT > 0 ? AT : 32); ++i)
      if ((AT > 0 || i < A) && sel[i] > bvv) { bvv = sel[i]; best = i; }
    const float nxt = S.q[1][tid][best];
    const float y = tr + tg * (1.f - td) * nxt;
    const float d = S.q[0][tid][ta] - y;
    float per, dper;
    if (a.huber) {
      const float ad = fabsf(d);
      per = ad <= a.delta ? 0.5f * d * d : a.delta * (ad - 0.5f * a.delta);
      dper = ad <= a.delta ? d : copysignf(a.delta, d);
    } else {
      per = d * d;
      dper = 2.f * d;
    }
    contrib = tw * per;
    const float gsc = tw * dper / (float)a.B;
    // Q_i = V + A_i - mean(A): dV = sum_i dQ_i, dA_i = dQ_i - mean(dQ)
    const float sub = a.dueling ? gsc / (float)A : 0.f;
#pragma unroll
    for (int i = 0; i < (AT > 0 ? AT : 32); ++i)
      if (AT > 0 || i < A) S.dq[tid][i] = ((i == ta) ? gsc : 0.f) - sub;
    S.dq[tid][A] = a.dueling ? gsc : 0.f;
    a.prio[b] = fabsf(d);
  }
  if (wave == 0) {
    const float sum = wave_sum(contrib);
    if (lane == 0) a.loss_parts[blockIdx.x] = sum;           // summed by the fc dgrad launch
  }
  __syncthreads();
  // dQ (| dV) as act_t [B][64] (plain / adv in columns 0..31, value in 32; zero padding): the dZ
  // operand of the output layer's weight-gradient members of the grouped wgrad launch (+ Q rows)
  for (int t = tid; t < nrows * 64; t += kHeadThreads) {
    const int r = t >> 6, c = t & 63;
    const float g = c < A ? S.dq[r][c] : (c == 32 && a.dueling ? S.dq[r][A] : 0.f);
    reinterpret_cast<act_t*>(a.dq16)[(int64_t)(r0 + r) * 64 + c] = (act_t)(g * kLossScale);
  }
  if (a.q_out != nullptr)
    for (int t = tid; t < nrows * A; t += kHeadThreads) a.q_out[(int64_t)r0 * A + t] = S.q[0][t / A][t % A];
  HEAD_MARK(2);
  // ---- dH[row][k] = (sum_i dQ[row][i] W[k][i]) * (h > 0) (dueling: value units dV wv[k]), from
  //      the online h fragments this wave already holds: row lane & 15, units ks * 32 + kg + j
  {
    const int rr = lane & 15, row = r0 + rr;
    const int kg = 8 * (lane >> 4);
    act_t* dh = reinterpret_cast<act_t*>(a.dh);
    const float* g = S.dq[rr];
#pragma unroll
    for (int u = 0; u < kHeadKPW; ++u) {
      const int ks = wave * kHeadKPW + u;
      if (ks >= HID / 32) break;
      const int k0 = ks * 32 + kg;
      bfx8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float* w = S.w + (k0 + j) * A;
        float sj = 0.f;
        if constexpr (AT > 0) {
#pragma unroll
          for (int i = 0; i < AT; ++i) sj += g[i] * w[i];
        } else {
          for (int i = 0; i < A; ++i) sj += g[i] * w[i];
        }
        o[j] = (act_t)((float)h0f[u][0][j] > 0.f ? sj * kLossScale : 0.f);     // scaled: see dqn_act.h
      }
      if (row < a.B) *reinterpret_cast<bfx8*>(dh + (int64_t)row * HH + (a.dueling ? HID : 0) + k0) = o;
      if (a.dueling) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          o[j] = (act_t)((float)h0f[u][1][j] > 0.f ? g[A] * S.w[nw + k0 + j] * kLossScale : 0.f);
        if (row < a.B) *reinterpret_cast<bfx8*>(dh + (int64_t)row * HH + k0) = o;
      }
    }
  }
  HEAD_MARK(3);
#undef HEAD_MARK
}

}  // namespace dqn

using namespace dqn;

// ================================================================ dgrad chain
// (ChainArgs, dqn_nets_k.h) The three dgrad GEMMs of the Nature backward in one launch: a stage
// waits for its own inputs only (row group / sample counters), so the launch boundaries between
// them -- drain + ramp, ~2-3 us each -- become overlap. Producers' outputs are write-through
// full lines, and a consumer reads a line only after its counter says every writer finished, so
// its L2 cannot hold an older copy of it (L2 is invalidated at kernel start).
// counters: one per 128-byte line (kChainStride ints), so the pollers of one counter never share
// a line with another counter's arrivals
constexpr int kChainStride = 32;

DQN_DEV void chain_arrive(int32_t* c, int n) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // this wave's write-through stores done
  __syncthreads();
  if (threadIdx.x < n)
    __hip_atomic_fetch_add(c + threadIdx.x * kChainStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

DQN_DEV void chain_wait(const int32_t* c, int want, int32_t* err) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      __builtin_amdgcn_s_sleep(8);                             // (~0.2 us: light on the counter's line)
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {    // 1 s: flag it, never hang
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) dgrad_chain_kernel(ChainArgs c) {
  int b = blockIdx.x;
  int32_t* c0 = c.cnt;                                      // stage-0 row groups
  int32_t* c1 = c.cnt + c.gx0 * kChainStride;               // stage-1 samples
  int32_t* err = c1 + c.B * kChainStride;
  if (b < c.n0) {
    const int bx = b % c.gx0, by = b / c.gx0;
    igemm_body<DenseLoader, 1, 1, 1, 1, 4, 2, DQN_ACT_F32 ? 2 : 4, true>(c.a[0], bx, by, 0, c.gx0, c.gy0, 1);
    chain_arrive(c0 + bx * kChainStride, 1);
    return;
  }
  b -= c.n0;
  if (b < c.n1) {
    const int m0 = b * 16, m1 = min(m0 + 15, c.a[1].M - 1);
    const int s0 = m0 / c.rows1, s1 = m1 / c.rows1;
    chain_wait(c0 + (s0 / 16) * kChainStride, c.gy0, err);
    if (s1 / 16 != s0 / 16) chain_wait(c0 + (s1 / 16) * kChainStride, c.gy0, err);
    igemm_body<DgradLoader<64, 3, 3, 1>, 1, 2, 1, 2, 2, 2, 9, true>(c.a[1], b, 0, 0, c.n1, 1, 1);
    if (c.n2 > 0) chain_arrive(c1 + s0 * kChainStride, s1 - s0 + 1);
    return;
  }
  b -= c.n1;
  const ConvArgs& a2 = c.a[2];
  const int cmt = ((a2.IH / 2) * (a2.IW / 2) + 15) / 16;
  const int s = (b / cmt) >> 2;                                  // dgrad_s2_body's block order
  const int need = (s * c.rows1 + c.rows1 - 1) / 16 - (s * c.rows1) / 16 + 1;
  chain_wait(c1 + s * kChainStride, need, err);
  dgrad_s2_body<64, 4, 4>(a2, b, 0);
}

// ------------------------------------------------------------------ launchers
void launch_pack(const float* src, void* dst, const PackJob* jobs_dev, int njobs, int max_threads, void* dst2,
                 const int64_t* step, int freq, hipStream_t st) {
  dim3 grid((max_threads + 255) / 256, njobs);
  hipLaunchKernelGGL(pack_kernel, grid, dim3(256), 0, st, src, reinterpret_cast<act_t*>(dst), jobs_dev,
                     reinterpret_cast<act_t*>(dst2), step, freq < 1 ? 1 : freq);
}

// fp32 build: fragments take twice the VGPRs, so each load batch holds half the k-steps
constexpr int kLoadBatch(int u) { return DQN_ACT_F32 ? (u + 1) / 2 : u; }
#define IGEMM_LAUNCH_U(LD, MT, NT, WM, WN, KS, EPI, U)                                                \
  do {                                                                                                  \
    dim3 grid((a.M + WM * MT * 16 - 1) / (WM * MT * 16), (a.N + WN * NT * 16 - 1) / (WN * NT * 16),             \
              ninst + (a.gth != nullptr ? 1 : 0));                                                                \
    if (a.gth != nullptr && (a.gth_z != ninst || (int)(grid.x * grid.y) < a.gth_blocks)) return -2;                \
    hipLaunchKernelGGL((igemm_kernel<LD, MT, NT, WM, WN, KS, EPI, kLoadBatch(U)>), grid, dim3(64 * WM * WN * KS), 0, st, a); \
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
    // K 3136 = 98 k-steps, split-K 8: one 13-step load batch per wave; 16-row blocks so the
    // B=32 step spreads over 2x the CUs (each block's L2->CU bytes are the bound, not MFMA)
    case L_DENSE_FWD_RELU:
      if (a.fz_w2 != nullptr) {     // factorised noisy instance (host-checked: M <= 32, N % 16 == 0)
        if (a.gth != nullptr || a.M > 32 || a.fz_inst < 0 || a.fz_inst >= ninst) return -2;
        hipLaunchKernelGGL((fc_fwd_fz_kernel<kLoadBatch(13)>), dim3(2, a.N16, ninst), dim3(512), 0, st, a);
        return 0;
      }
      // 32-row blocks once 16-row blocks would exceed one per CU (Rainbow's 2 x 64 x 3 = 384:
      // +0.5-1.3%, profiles/r4_fc_fwd_tiles_ab.txt; at <= 256 blocks, e.g. the unfolded flagship's
      // 192, the 16-row blocks measured 4% faster in round 3)
      if (((a.M + 15) / 16) * ((a.N + 15) / 16) * ninst > 256) { IGEMM_LAUNCH_U(DenseLoader, 2, 1, 1, 1, 8, 0, 13); return 0; }
      IGEMM_LAUNCH_U(DenseLoader, 1, 1, 1, 1, 8, 0, 13); return 0;
    case L_DENSE_FWD_F32: IGEMM_LAUNCH_U(DenseLoader, 2, 1, 1, 1, 8, 1, 13); return 0;
    // ---- backward data, ReLU mask of the layer input
    // K 512-1024: 16 x 16 blocks, split-K 4 (2x the blocks of 16 x 32 split-K 2; A/B interleaved on one
    // box: flagship +0.2-0.3%, dd +0.7-2.0%, Rainbow +0.7-1.1%, profiles/r4_fc_dgrad_tiles_ab.txt). The
    // dgrad chain's fc stage uses the same tiling (bit-identical to this launch).
    case L_DENSE_DGRAD: IGEMM_LAUNCH_U(DenseLoader, 1, 1, 1, 1, 4, 2, 4); return 0;
    case L_NAT_CONV3_DGRAD: IGEMM_LAUNCH_U(NatD3, 1, 2, 1, 2, 2, 2, 9); return 0;     // 18 k-steps, 16 x 64 blocks
    case L_NAT_CONV2_DGRAD:
      // parity-class dgrad (8 k-steps of real taps instead of 32 with 3/4 zeros); the generic
      // igemm path for shapes the class kernel does not cover
      if (a.N16 == 2 && a.IH % 2 == 0 && a.IW % 2 == 0 && a.pad_t == 0 && a.pad_l == 0 && a.zero_ptr == nullptr &&
          a.nz_out0 == nullptr && a.loss_parts == nullptr && 2 * a.OH + 2 == a.IH && 2 * a.OW + 2 == a.IW) {
        const int cmt = ((a.IH / 2) * (a.IW / 2) + 15) / 16, B = a.M / (a.IH * a.IW);
        hipLaunchKernelGGL((dgrad_s2_kernel<64, 4, 4>), dim3(B * 4 * cmt, 1, ninst), dim3(256), 0, st, a);
        return 0;
      }
      IGEMM_LAUNCH_U(NatD2, 1, 2, 2, 1, 2, 2, 8); return 0;     // 32 k-steps
    default: return -1;
  }
}

int launch_dgrad_chain(const ConvArgs& a0, const ConvArgs& a1, const ConvArgs& a2, int32_t* cnt, int B,
                       hipStream_t st) {
  // stage 0: dense dgrad, 16-row x 64-column tiles (full 128-byte lines of dz3 per block row)
  // stage 1: conv3 dgrad (64 input channels = one 128-byte line per row)
  // stage 2: conv2 dgrad by parity classes (the conditions of launch_igemm's D2 fast path)
  // (a2.out == nullptr: two stages -- the conv2 dgrad stays its own launch, where its 52-VGPR blocks
  //  run 8 per SIMD instead of the chain's 3)
  const bool s2 = a2.out[0] != nullptr;
  if (cnt == nullptr || B < 1 || B > 1024 || a0.M != B || a0.N % 64 != 0 || a1.N != 64 || a1.M % B != 0 ||
      a1.in[0] != a0.out[0] || a1.zero_ptr != nullptr || a1.loss_parts != nullptr || a0.gth != nullptr)
    return -1;
  if (s2 && (a2.N16 != 2 || a2.IH % 2 != 0 || a2.IW % 2 != 0 || a2.pad_t != 0 || a2.pad_l != 0 ||
             2 * a2.OH + 2 != a2.IH || 2 * a2.OW + 2 != a2.IW || a2.M != B * a2.IH * a2.IW ||
             a2.in[0] != a1.out[0] || a2.zero_ptr != nullptr || a2.loss_parts != nullptr))
    return -1;
  ChainArgs c{};
  c.a[0] = a0; c.a[1] = a1; c.a[2] = a2;
  c.gx0 = (B + 15) / 16;
  c.gy0 = a0.N / 16;
  c.n0 = c.gx0 * c.gy0;
  c.n1 = (a1.M + 15) / 16;
  c.rows1 = a1.M / B;
  c.n2 = s2 ? B * 4 * (((a2.IH / 2) * (a2.IW / 2) + 15) / 16) : 0;
  c.B = B;
  c.cnt = cnt;
  hipLaunchKernelGGL(dgrad_chain_kernel, dim3(c.n0 + c.n1 + c.n2), dim3(256), 0, st, c);
  return 0;
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
    case L_HEAD_WGRAD: WGRAD_LAUNCH(DenseLoader, 32, 64, 64); return 0;
    case L_DENSE_WGRAD_LR: {                     // ONE block per weight tile over all g.mloop 64-row chunks
      if (g.mloop < 1 || 64 * g.mloop < a.M) return -1;
      // tiles per block: 32 x 64 (784 blocks for Nature's fc; measured 11.0 vs 11.7 us for 64 x 128
      // at W = 8 alone, round 2)
      dim3 grid(1, (a.K + 31) / 32, (g.N + 63) / 64);
      hipLaunchKernelGGL((wgrad_multi_kernel<DenseLoader, 64, 32, 64>), grid, dim3(256), 0, st, a, g);
      return 0;
    }
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
#if DQN_ACT_F32
  wgrad_block<LD, MC, KB, NB>(a, g, bx, by, bz, lds);
#else
  constexpr bool kPart = MC == 128 && !std::is_same<LD, DenseLoader>::value;
  constexpr bool kMulti = kPart;
  if constexpr (kMulti) {
    if (g.part == nullptr && g.mloop > 1) {
      // chunk group bx: mloop consecutive M-chunks summed in registers, ONE set of fp32 atomics
      // per group (the atomic bytes of the member / mloop: they run at the memory side, ~1.3 TB/s
      // chip-wide, the grouped launch's floor with one set per chunk)
      const int nch = (a.M + MC - 1) / MC, c0 = bx * g.mloop;
      wgrad_block_det<LD, MC, KB, NB>(a, g, c0, by, bz, lds, min(nch, c0 + g.mloop) - c0);
      return;
    }
  }
  if (!kPart || g.part == nullptr) {
    wgrad_block<LD, MC, KB, NB>(a, g, bx, by, bz, lds);
    return;
  }
  // deterministic: chunk group bx -> its partial slice ([K][N] weights, then [N] bias), as the
  // member's own dW / db with no split (plain stores)
  WgradArgs gp = g;
  const int nch = (a.M + MC - 1) / MC, c0 = bx * g.mloop;
  gp.dw = g.part + (int64_t)bx * g.pstride;
  gp.db = gp.dw + (int64_t)a.K * g.N;
  gp.nsplit = g.N;
  gp.atomic = 0;
  if constexpr (kPart) wgrad_block_det<LD, MC, KB, NB>(a, gp, c0, by, bz, lds, min(nch, c0 + g.mloop) - c0);
#endif
}

// conv members' M-chunk: 128 rows (kind as is: the fp32 build, whose 256-row staging would not
// fit twice per CU, and the deterministic partial members) or 256 rows (kind | kGrpMC256: 80 KB,
// 2 blocks / CU, half the blocks and atomic partials: the 16-bit builds)
constexpr int kGrpMC256 = 0x40;
#define GRP_CONV_CASES(OFF, MC)                                                                                    \
  case L_NAT_CONV1_FWD + OFF: group_member<NatC1, MC, 64, 32>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;    \
  case L_NAT_CONV1_FRAMES + OFF: group_member<NatF1, MC, 64, 32>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break; \
  case L_NAT_CONV2_FWD + OFF: group_member<NatC2, MC, 64, 64>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;    \
  case L_NAT_CONV3_FWD + OFF: group_member<NatC3, MC, 64, 64>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;
// (<= 128 VGPRs: 4 waves / SIMD, the 4 blocks / CU the conv members' LDS allows)
// (fp32 build: 3 waves / EU -- at 4 the 128-VGPR cap spilled 20 B / lane to scratch)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DQN_ACT_F32 ? 3 : 4))) wgrad_group_kernel(WgradGroup Gv) {
  extern __shared__ __attribute__((aligned(16))) act_t glds[];
  // members are read straight from the kernel-argument segment (the group is the only, offset-0
  // argument): indexing the by-value parameter with the runtime member index otherwise lets the
  // compiler copy all ~2.7 KB of it to scratch once the members' bodies grow
  (void)Gv;
  const WgradGroup& G = *(const WgradGroup*)__builtin_amdgcn_kernarg_segment_ptr();
  int b = blockIdx.x, i = 0;
  while (i < G.n - 1 && b >= G.nblk[i]) { b -= G.nblk[i]; ++i; }
  switch (G.kind[i]) {
    GRP_CONV_CASES(0, 128)
    GRP_CONV_CASES(kGrpMC256, 256)
    case L_DENSE_FWD_RELU: group_member<DenseLoader, 32, 64, 128>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;
    case L_HEAD_WGRAD: group_member<DenseLoader, 32, 64, 64>(G.a[i], G.g[i], b, G.gx[i], G.gy[i], glds); break;
    default: break;
  }
}
#undef GRP_CONV_CASES
}  // namespace dqn

static bool wgrad_tiles(int kind, int& MC, int& KB, int& NB, size_t& lds) {
  switch (kind) {
    case L_NAT_CONV1_FWD: case L_NAT_CONV1_FRAMES: MC = 128; KB = 64; NB = 32; break;
    case L_NAT_CONV2_FWD: MC = 128; KB = 64; NB = 64; break;
    case L_NAT_CONV3_FWD: MC = 128; KB = 64; NB = 64; break;
    case L_NAT_CONV1_FWD + kGrpMC256: case L_NAT_CONV1_FRAMES + kGrpMC256: MC = 256; KB = 64; NB = 32; break;
    case L_NAT_CONV2_FWD + kGrpMC256: MC = 256; KB = 64; NB = 64; break;
    case L_NAT_CONV3_FWD + kGrpMC256: MC = 256; KB = 64; NB = 64; break;
    case L_DENSE_FWD_RELU: MC = 32; KB = 64; NB = 128; break;
    case L_HEAD_WGRAD: MC = 32; KB = 64; NB = 64; break;
    default: return false;
  }
#if DQN_ACT_F32
  lds = (size_t)(KB + NB) * (MC + kF32Pad) * sizeof(act_t);   // WgradTile<...>::lds_bytes
#else
  lds = (size_t)MC * (KB + 16 + NB + 16) * sizeof(act_t);      // WgradTile<...>::lds_bytes
#endif
  return true;
}

int launch_wgrad_group(WgradGroup G, hipStream_t st) {
  int total = 0;
  size_t lds = 0;
  // conv M-chunk: 256 rows (half the blocks and half the fp32 atomic bytes of 128-row chunks;
  // measured round 3, alternating on one box: flagship 13.87k vs 13.60k SGD steps/s, Rainbow
  // 7.88k vs 7.77k, profiles/r3_wgrad_mc.md) in the 16-bit builds; 128 in the fp32 build (its
  // 256-row staging is 135 KB of LDS: one block per CU).
  const bool mc256 = !DQN_ACT_F32;
  for (int i = 0; i < G.n; ++i) {
    if (G.g[i].part != nullptr) continue;       // (partial members: 128-row chunks, see below)
    if (mc256 && G.kind[i] >= L_NAT_CONV1_FWD && G.kind[i] <= L_NAT_CONV3_FWD) G.kind[i] += kGrpMC256;
    else if (mc256 && G.kind[i] == L_NAT_CONV1_FRAMES) G.kind[i] += kGrpMC256;
  }
  for (int i = 0; i < G.n; ++i) {
    int MC, KB, NB;
    size_t l;
    if (!wgrad_tiles(G.kind[i], MC, KB, NB, l)) return -1;
    if (l > 160 * 1024) return -2;
    G.gx[i] = (G.a[i].M + MC - 1) / MC;
    if (G.g[i].part != nullptr) {               // chunk groups of mloop chunks, one partial each
      if (DQN_ACT_F32 || MC != 128 || G.g[i].mloop < 1 || G.g[i].pstride < G.a[i].K * G.g[i].N + G.g[i].N) return -3;
      G.gx[i] = (G.gx[i] + G.g[i].mloop - 1) / G.g[i].mloop;
    } else {
      G.g[i].mloop = 1;                          // (one M-chunk per block, fp32 atomics across chunks)
    }
    G.gy[i] = (G.a[i].K + KB - 1) / KB;
    const int gz = (G.g[i].N + NB - 1) / NB;
    G.nblk[i] = G.gx[i] * G.gy[i] * gz;
    G.g[i].atomic = G.gx[i] > 1 && G.g[i].part == nullptr ? 1 : 0;
    total += G.nblk[i];
    lds = l > lds ? l : lds;
  }
  hipLaunchKernelGGL(wgrad_group_kernel, dim3(total), dim3(256), lds, st, G);
  return 0;
}

int wgrad_fused_plan(WgradGroup& G, int conv_chunks) {
  int total = 0;
  G.slots_member = -1;
  for (int i = 0; i < G.n; ++i) {
    int MC, KB, NB;
    if (!fused_wgrad_tiles(G.kind[i], MC, KB, NB) || G.g[i].part != nullptr) return -1;
    if (G.kind[i] == L_NAT_CONV1_FRAMES) G.slots_member = i;
    const int nch = (G.a[i].M + MC - 1) / MC;
    const int per = G.kind[i] == L_HEAD_WGRAD ? 1 : conv_chunks;
    G.g[i].mloop = per;
    G.gx[i] = (nch + per - 1) / per;
    G.gy[i] = (G.a[i].K + KB - 1) / KB;
    G.nblk[i] = G.gx[i] * G.gy[i] * ((G.g[i].N + NB - 1) / NB);
    G.g[i].atomic = G.gx[i] > 1 ? 1 : 0;
    total += G.nblk[i];
  }
  return total;
}

void launch_head_loss(const HeadArgs& a, hipStream_t st) {
  static bool lds_set = false;                // dynamic LDS above 64 KB must be opted into
  if (!lds_set) {
    const void* fns[] = {reinterpret_cast<const void*>(head_loss_kernel<0>), reinterpret_cast<const void*>(head_loss_kernel<2>),
                         reinterpret_cast<const void*>(head_loss_kernel<3>), reinterpret_cast<const void*>(head_loss_kernel<4>),
                         reinterpret_cast<const void*>(head_loss_kernel<6>), reinterpret_cast<const void*>(head_loss_kernel<9>),
                         reinterpret_cast<const void*>(head_loss_kernel<18>)};
    for (const void* f : fns)
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(HeadSmem));
    lds_set = true;
  }
  const int tiles = (a.B + kHeadRows - 1) / kHeadRows;
  int grid;
  if (a.infer) grid = a.has_actor ? a.actor.E : tiles;        // acting launch: one block per env
  else grid = tiles + (a.act_E > 0 ? a.act_E : 0);            // learner tiles (+ fused acting blocks)
#define HEAD(AT) hipLaunchKernelGGL(head_loss_kernel<AT>, dim3(grid), dim3(kHeadThreads), sizeof(HeadSmem), st, a)
  switch (a.A) {                   // the Atari action counts (and CartPole's 2) at compile time
    case 2: HEAD(2); break;
    case 3: HEAD(3); break;
    case 4: HEAD(4); break;
    case 6: HEAD(6); break;
    case 9: HEAD(9); break;
    case 18: HEAD(18); break;
    default: HEAD(0); break;
  }
#undef HEAD
}

