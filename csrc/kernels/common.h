// Shared device helpers for the gfx950 (CDNA4) kernels of dist_dqn_amd.
// Wave64 everywhere: lane = threadIdx.x & 63, reductions over 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include "../include/dqn_act.h"

#define DQN_DEV __device__ __forceinline__
#define DQN_DEV_HOST_INLINE __host__ __device__ inline

// Device-side bounds checks of the debug build (DQN_DEBUG=1 python setup.py build_ext):
// a failing check traps the kernel with file:line; compiled out of the release build.
#ifdef DQN_DEBUG
#include <cassert>
#define DQN_ASSERT(c) assert(c)
#else
#define DQN_ASSERT(c) ((void)0)
#endif

namespace dqn {

constexpr int kWave = 64;

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 { uint32_t x, y, z, w; };

DQN_DEV u32x4 philox(uint64_t key64, uint64_t ctr_hi, uint32_t ctr_lo0, uint32_t ctr_lo1) {
  uint32_t k0 = (uint32_t)key64, k1 = (uint32_t)(key64 >> 32);
  uint32_t c0 = ctr_lo0, c1 = ctr_lo1, c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

DQN_DEV float u01(uint32_t x) {  // [0, 1)
  return (float)(x >> 8) * (1.0f / 16777216.0f);
}

// Standard normals of the noisy-net stream: Box-Muller over Philox4x32-10 keyed by `seed`
// at counter `ctr`; call index q yields elements 4q .. 4q+3 of [out0[0, n) | out1[0, n)].
// (noise_normal_kernel and the fc dgrad launch's noise duty draw the same values.)
DQN_DEV void noise_normals4(float* out0, float* out1, int n, uint64_t seed, uint64_t ctr, int q) {
  const int total = out1 != nullptr ? 2 * n : n;
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

// ----------------------------------------------------------------- reductions
DQN_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DQN_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Reductions over the 16 lanes of one DPP row (lanes 16r..16r+15), result in every lane:
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror. VALU-only
// (no LDS crossbar, unlike __shfl_xor); all 16 lanes of the row must be active.
template <int CTRL>
DQN_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
DQN_DEV float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}
DQN_DEV float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return v;
}

// 4x4 transpose inside each lane quad (DPP quad_perm [1,0,3,2] then [2,3,0,1]): lane p of a
// quad holds row p of a 4x4 block on entry and column p on exit. VALU-only, all lanes active.
DQN_DEV void quad_transpose4(float (&v)[4]) {
  const int p = __lane_id() & 3;
  const bool odd = (p & 1) != 0, hi = (p & 2) != 0;
  float t0 = odd ? v[0] : v[1], t1 = odd ? v[2] : v[3];
  t0 = dpp_f<0xB1>(t0);
  t1 = dpp_f<0xB1>(t1);
  if (odd) { v[0] = t0; v[2] = t1; } else { v[1] = t0; v[3] = t1; }
  t0 = hi ? v[0] : v[2];
  t1 = hi ? v[1] : v[3];
  t0 = dpp_f<0x4E>(t0);
  t1 = dpp_f<0x4E>(t1);
  if (hi) { v[0] = t0; v[1] = t1; } else { v[2] = t0; v[3] = t1; }
}

// Whole-wave sum: DPP row sums, then the 4 row totals via readlane (uniform result).
DQN_DEV float wave_sum_dpp(float v) {
  v = row16_sum(v);
  const int iv = __float_as_int(v);
  return (__int_as_float(__builtin_amdgcn_readlane(iv, 0)) + __int_as_float(__builtin_amdgcn_readlane(iv, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(iv, 32)) + __int_as_float(__builtin_amdgcn_readlane(iv, 48)));
}

DQN_DEV float wave_max_dpp(float v) {
  v = row16_max(v);
  const int iv = __float_as_int(v);
  return fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(iv, 0)), __int_as_float(__builtin_amdgcn_readlane(iv, 16))),
               fmaxf(__int_as_float(__builtin_amdgcn_readlane(iv, 32)), __int_as_float(__builtin_amdgcn_readlane(iv, 48))));
}

// -------------------------------------------------------------------- bf16
DQN_DEV uint16_t f2bf(float f) {  // round-to-nearest-even (NaN kept by the cast path)
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}
DQN_DEV float bf2f(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x4 = __attribute__((ext_vector_type(4))) float;

#if DQN_ACT_F32
// fp32 build: one 32-deep k-step of the 16-bit builds' fragment layout as 8 16x16x4 fp32
// MFMAs (lane group g supplies k = 8g + j to the j-th; see dqn_act.h)
typedef __attribute__((ext_vector_type(8))) float f32x8_frag;
DQN_DEV f32x4 mfma_f32_k32(const f32x8_frag& a, const f32x8_frag& b, f32x4 c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], c, 0, 0, 0);
  return c;
}
#endif
using f32x16 = __attribute__((ext_vector_type(16))) float;
typedef __attribute__((ext_vector_type(8))) act_t bfx8;     // one MFMA operand (8 act_t per lane)

#if !DQN_ACT_F32
// 16-bit builds: MFMA operands of a row-major LDS tile through transposed reads.
// lds_tr16: 4 rows x 16 columns of 16-bit elements, column-major into the lanes of each
// 16-lane group (lane 4q + p addresses row q, columns 4p..4p+3; lane i receives column i,
// row q in element q); join_tr: two of them (rows r and r + 16) as one 8-element operand.
typedef short s16x4 __attribute__((ext_vector_type(4)));
DQN_DEV s16x4 lds_tr16(const act_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(reinterpret_cast<uintptr_t>(p)));
}
DQN_DEV bfx8 join_tr(s16x4 lo, s16x4 hi) {
  union { s16x4 h[2]; bfx8 v; } u;
  u.h[0] = lo;
  u.h[1] = hi;
  return u.v;
}
#endif

}  // namespace dqn
