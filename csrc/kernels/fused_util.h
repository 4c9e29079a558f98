// Shared device helpers of the per-sample fused network kernels (trunk.hip: Nature
// trunk; cnn.hip: the reference SAME + max-pool network): bf16 fragments, the
// transposed-MFMA epilogue packing, uint8 frame -> bf16 NHWC LDS staging and the
// LDS k-split partial-sum exchange.
#pragma once
#include "common.h"

namespace dqn {

typedef __attribute__((ext_vector_type(8))) act_t bfx8;

DQN_DEV bfx8 tz8() {
  bfx8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (act_t)0.f;
  return z;
}

DQN_DEV f32x4 f4(const float4& v) { return f32x4{v.x, v.y, v.z, v.w}; }

// ReLU + 4 floats -> 4 packed act_t (8 bytes; 16 in the fp32 build): pk4_t
#if DQN_ACT_F32
typedef float4 pk4_t;
DQN_DEV pk4_t pack4(const f32x4& v) {
  return make_float4(fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f));
}
#else
typedef uint2 pk4_t;
DQN_DEV pk4_t pack4(const f32x4& v) {
  const act_t a = (act_t)fmaxf(v[0], 0.f), b = (act_t)fmaxf(v[1], 0.f);
  const act_t c = (act_t)fmaxf(v[2], 0.f), d = (act_t)fmaxf(v[3], 0.f);
  return make_uint2((uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16),
                    (uint32_t)__builtin_bit_cast(uint16_t, c) | ((uint32_t)__builtin_bit_cast(uint16_t, d) << 16));
}
#endif

// 8 consecutive input-image elements (in_t, LDS) as an MFMA fragment
DQN_DEV bfx8 ld_in8(const in_t* p) {
#if DQN_ACT_F32
  typedef __attribute__((ext_vector_type(8))) in_t in8;
  const in8 v = *reinterpret_cast<const in8*>(p);
  bfx8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (float)v[j];
  return r;
#else
  return *reinterpret_cast<const bfx8*>(p);
#endif
}

DQN_DEV f32x4 tmfma(const bfx8& a, const bfx8& b, const f32x4& c) {
  return DQN_MFMA16_BUILTIN(a, b, c, 0, 0, 0);
}

// 4 pixels x 4 channels (one uint32 per channel plane, or one uint4 NHWC word
// group) -> 4 NHWC bf16 pixels (32 B) in LDS.
DQN_DEV uint32_t bfpair(uint32_t a, uint32_t b) {   // two integers 0..255 -> packed in_t (exact)
  const in_t x = (in_t)(float)a, y = (in_t)(float)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

DQN_DEV void planes_to_lds(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, in_t* dst) {
  uint32_t o[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int sh = 8 * i;
    o[2 * i] = bfpair((c0 >> sh) & 0xffu, (c1 >> sh) & 0xffu);
    o[2 * i + 1] = bfpair((c2 >> sh) & 0xffu, (c3 >> sh) & 0xffu);
  }
  reinterpret_cast<uint4*>(dst)[0] = make_uint4(o[0], o[1], o[2], o[3]);
  reinterpret_cast<uint4*>(dst)[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

#if DQN_ACT_F32
// fp32 build, layers whose input is exact in bf16 (conv1: the uint8 frames): the fp32 weight fragment
// as three bf16 fragments whose sum is exactly the fp32 value (8 + 8 + 8 significand bits), so three
// bf16 MFMAs (16x16x32) give products that are exact in fp32 and fp32 accumulation -- the fp32
// convolution up to summation order -- instead of eight fp32 MFMAs (16x16x4) per 32-deep k-step.
typedef __attribute__((ext_vector_type(8))) __bf16 b16x8;
DQN_DEV void split3_bf16(const bfx8& v, b16x8& h, b16x8& m, b16x8& l) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 hj = (__bf16)v[j];
    const float r1 = v[j] - (float)hj;
    const __bf16 mj = (__bf16)r1;
    h[j] = hj;
    m[j] = mj;
    l[j] = (__bf16)(r1 - (float)mj);
  }
}
DQN_DEV f32x4 mfma3_bf16(const b16x8& h, const b16x8& m, const b16x8& l, const b16x8& x, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(l, x, c, 0, 0, 0);      // (small terms first)
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(m, x, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(h, x, c, 0, 0, 0);
}
#endif

// K-split partial-sum exchange: waves of k-half 1 park their fp32 accumulators
// in LDS, waves of k-half 0 add them after the barrier.
DQN_DEV void park(float* red, int slot, int lane, const f32x4& acc) {
  reinterpret_cast<f32x4*>(red)[slot * 64 + lane] = acc;
}
DQN_DEV f32x4 unpark(const float* red, int slot, int lane, f32x4 acc) {
  const f32x4 o = reinterpret_cast<const f32x4*>(red)[slot * 64 + lane];
  return acc + o;
}

}  // namespace dqn
