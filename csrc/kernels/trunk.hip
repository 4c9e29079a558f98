// Fused Nature-CNN trunk: conv1 -> conv2 -> conv3 (+bias, ReLU) for ONE sample
// per workgroup, with the intermediate activations kept in LDS.
//
// Reference: three tf.nn.conv2d + bias + relu ops, each a separate kernel with
// its activations round-tripping through memory (/root/reference/src/network.py:389-399
// for the reference's SAME/max-pool variant; Nature geometry here: VALID
// 8x8/4 -> 4x4/2 -> 3x3/1, 84x84x4 -> 20x20x32 -> 9x9x64 -> 7x7x64).
//
// Per block (8 waves, one (sample, instance) pair):
//   stage 1  conv1: 400 x 32 x 256 implicit GEMM, A gathered straight from the
//            replay frame ring through the sample's 4 frame slots (or from a
//            NHWC uint8 stack), B = packed bf16 MFMA fragments (L2-resident);
//            result (bias, input scale, ReLU) -> LDS act1 [400][40]
//   stage 2  conv2: 81 x 64 x 512, A = im2col reads of act1 from LDS (16 B per
//            lane) -> LDS act2 [81][72]
//   stage 3  conv3: 49 x 64 x 576, A from act2 -> global x3 (the fc input)
// x1 / x2 are also written to global (the backward's ReLU masks / wgrad inputs).
// Everything is v_mfma_f32_16x16x32_bf16 with fp32 accumulation.
#include "common.h"
#include "../include/dqn_nets_k.h"

namespace dqn {

typedef __attribute__((ext_vector_type(8))) __bf16 bfx8;

namespace trunk {
constexpr int IH = 84, IW = 84, HW = IH * IW;
constexpr int O1 = 20, N1 = 32, K1 = 256, R1 = O1 * O1;       // conv1: 8x8/4
constexpr int O2 = 9, N2 = 64, K2 = 512, R2 = O2 * O2;        // conv2: 4x4/2
constexpr int O3 = 7, N3 = 64, K3 = 576, R3 = O3 * O3;        // conv3: 3x3/1
constexpr int L1 = N1 + 8, L2 = N2 + 8;                       // padded LDS rows (elements)
}  // namespace trunk

DQN_DEV bfx8 tz8() {
  bfx8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
  return z;
}

DQN_DEV f32x4 tmfma(const bfx8& a, const bfx8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// conv1 A fragment for output pixel p (row of the GEMM), k0 = 8-aligned K index
// (kh, kw..kw+1, 4 frames). fb[c] = base of frame c of this sample (slot path)
// or nullptr with `nhwc` = the sample's [84][84][4] stack.
DQN_DEV bfx8 conv1_frag(const uint8_t* const* fb, const uint8_t* nhwc, int p, int k0) {
  using namespace trunk;
  if (p >= R1) return tz8();
  const int oy = p / O1, ox = p - oy * O1;
  const int kh = k0 >> 5, kw = (k0 & 31) >> 2;
  const int off = (oy * 4 + kh) * IW + ox * 4 + kw;     // pixel ix (even), ix + 1
  bfx8 r;
  if (nhwc != nullptr) {
    const uint2 v = *reinterpret_cast<const uint2*>(nhwc + (int64_t)off * 4);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      r[c] = (__bf16)(float)((v.x >> (8 * c)) & 0xffu);
      r[4 + c] = (__bf16)(float)((v.y >> (8 * c)) & 0xffu);
    }
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t v = *reinterpret_cast<const uint16_t*>(fb[c] + off);
      r[c] = (__bf16)(float)(v & 0xffu);
      r[4 + c] = (__bf16)(float)(v >> 8);
    }
  }
  return r;
}

__global__ void __launch_bounds__(512) trunk_fwd_kernel(TrunkArgs a) {
  using namespace trunk;
  __shared__ __attribute__((aligned(16))) __bf16 act1[R1 * L1];
  __shared__ __attribute__((aligned(16))) __bf16 act2[R2 * L2];
  const int b = blockIdx.x, inst = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = lane & 15, kg = 8 * (lane >> 4);
  const float scale = a.scale;

  // ---------------------------------------------------------------- conv1
  const uint8_t* fb[4] = {nullptr, nullptr, nullptr, nullptr};
  const uint8_t* nhwc = nullptr;
  if (a.slots[inst] != nullptr) {
    const int4 sl = reinterpret_cast<const int4*>(a.slots[inst])[b];
    fb[0] = a.frames + (int64_t)sl.x * HW;
    fb[1] = a.frames + (int64_t)sl.y * HW;
    fb[2] = a.frames + (int64_t)sl.z * HW;
    fb[3] = a.frames + (int64_t)sl.w * HW;
  } else {
    nhwc = a.states[inst] + (int64_t)b * HW * 4;
  }
  {
    const bfx8* W1 = reinterpret_cast<const bfx8*>(a.w1[inst]);
    const float* bias = a.b1[inst];
    constexpr int MT = (R1 + 15) / 16;               // 25 m-tiles x 2 n-tiles (whole N per task)
    for (int mt = wave; mt < MT; mt += 8) {
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      const int p = mt * 16 + row;
#pragma unroll
      for (int kb = 0; kb < K1 / 32; kb += 4) {
        bfx8 af[4], b0[4], b1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          af[u] = conv1_frag(fb, nhwc, p, (kb + u) * 32 + kg);
          b0[u] = W1[((kb + u) * 2 + 0) * 64 + lane];
          b1[u] = W1[((kb + u) * 2 + 1) * 64 + lane];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc0 = tmfma(af[u], b0[u], acc0);
          acc1 = tmfma(af[u], b1[u], acc1);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + 4 * (lane >> 4) + r;
        if (m < R1) {
          act1[m * L1 + row] = (__bf16)fmaxf(acc0[r] * scale + bias[row], 0.f);
          act1[m * L1 + 16 + row] = (__bf16)fmaxf(acc1[r] * scale + bias[16 + row], 0.f);
        }
      }
    }
  }
  __syncthreads();
  // x1 -> global (backward masks / conv2 wgrad input), 16 B per thread
  if (a.x1[inst] != nullptr) {
    __bf16* x1 = a.x1[inst] + (int64_t)b * R1 * N1;
    for (int t = threadIdx.x; t < R1 * N1 / 8; t += 512) {
      const int m = t / (N1 / 8), c8 = (t - m * (N1 / 8)) * 8;
      *reinterpret_cast<bfx8*>(x1 + m * N1 + c8) = *reinterpret_cast<const bfx8*>(act1 + m * L1 + c8);
    }
  }
  // ---------------------------------------------------------------- conv2
  {
    const bfx8* W2 = reinterpret_cast<const bfx8*>(a.w2[inst]);
    const float* bias = a.b2[inst];
    constexpr int MT = (R2 + 15) / 16;               // 6 m-tiles x 2 n-tile pairs = 12 tasks
    for (int task = wave; task < MT * 2; task += 8) {
      const int mt = task >> 1, np = task & 1;
      const int p = mt * 16 + row;
      const bool ok = p < R2;
      const int oy = ok ? p / O2 : 0, ox = ok ? p - oy * O2 : 0;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll 1
      for (int kb = 0; kb < K2 / 32; kb += 4) {
        bfx8 af[4], b0[4], b1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k0 = (kb + u) * 32 + kg;             // k = (kh*4 + kw)*32 + ci
          const int tap = k0 >> 5, ci = k0 & 31, kh = tap >> 2, kw = tap & 3;
          af[u] = ok ? *reinterpret_cast<const bfx8*>(act1 + ((oy * 2 + kh) * O1 + ox * 2 + kw) * L1 + ci) : tz8();
          b0[u] = W2[((kb + u) * 4 + np * 2 + 0) * 64 + lane];
          b1[u] = W2[((kb + u) * 4 + np * 2 + 1) * 64 + lane];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc0 = tmfma(af[u], b0[u], acc0);
          acc1 = tmfma(af[u], b1[u], acc1);
        }
      }
      const int n0 = np * 32 + row, n1 = np * 32 + 16 + row;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + 4 * (lane >> 4) + r;
        if (m < R2) {
          act2[m * L2 + n0] = (__bf16)fmaxf(acc0[r] + bias[n0], 0.f);
          act2[m * L2 + n1] = (__bf16)fmaxf(acc1[r] + bias[n1], 0.f);
        }
      }
    }
  }
  __syncthreads();
  if (a.x2[inst] != nullptr) {
    __bf16* x2 = a.x2[inst] + (int64_t)b * R2 * N2;
    for (int t = threadIdx.x; t < R2 * N2 / 8; t += 512) {
      const int m = t / (N2 / 8), c8 = (t - m * (N2 / 8)) * 8;
      *reinterpret_cast<bfx8*>(x2 + m * N2 + c8) = *reinterpret_cast<const bfx8*>(act2 + m * L2 + c8);
    }
  }
  // ---------------------------------------------------------------- conv3
  {
    const bfx8* W3 = reinterpret_cast<const bfx8*>(a.w3[inst]);
    const float* bias = a.b3[inst];
    __bf16* x3 = a.x3[inst] + (int64_t)b * R3 * N3;
    const int mt = wave >> 1, np = wave & 1;           // 4 m-tiles x 2 n-tile pairs = 8 tasks
    const int p = mt * 16 + row;
    const bool ok = p < R3;
    const int oy = ok ? p / O3 : 0, ox = ok ? p - oy * O3 : 0;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll 1
    for (int kb = 0; kb < K3 / 32; kb += 6) {           // 18 k-steps = 3 batches of 6
      bfx8 af[6], b0[6], b1[6];
#pragma unroll
      for (int u = 0; u < 6; ++u) {
        const int k0 = (kb + u) * 32 + kg;               // k = (kh*3 + kw)*64 + ci
        const int tap = k0 >> 6, ci = k0 & 63, kh = tap / 3, kw = tap - kh * 3;
        af[u] = ok ? *reinterpret_cast<const bfx8*>(act2 + ((oy + kh) * O2 + ox + kw) * L2 + ci) : tz8();
        b0[u] = W3[((kb + u) * 4 + np * 2 + 0) * 64 + lane];
        b1[u] = W3[((kb + u) * 4 + np * 2 + 1) * 64 + lane];
      }
#pragma unroll
      for (int u = 0; u < 6; ++u) {
        acc0 = tmfma(af[u], b0[u], acc0);
        acc1 = tmfma(af[u], b1[u], acc1);
      }
    }
    const int n0 = np * 32 + row, n1 = np * 32 + 16 + row;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mt * 16 + 4 * (lane >> 4) + r;
      if (m < R3) {
        x3[m * N3 + n0] = (__bf16)fmaxf(acc0[r] + bias[n0], 0.f);
        x3[m * N3 + n1] = (__bf16)fmaxf(acc1[r] + bias[n1], 0.f);
      }
    }
  }
}

}  // namespace dqn

using namespace dqn;

void launch_trunk_fwd(const TrunkArgs& a, int B, int ninst, hipStream_t st) {
  hipLaunchKernelGGL(trunk_fwd_kernel, dim3(B, ninst), dim3(512), 0, st, a);
}
