// Element type of the MFMA network kernels' activations, activation gradients and
// packed weight fragments (fp32 accumulation and fp32 master weights/gradients always).
//   default build (_C):      bf16  -> v_mfma_f32_16x16x32_bf16
//   -DDQN_F16 build (_C_f16): fp16  -> v_mfma_f32_16x16x32_f16  (BASELINE config 5's fp16
//                             path; same MFMA rate on CDNA4, 3 more mantissa bits, 5 fewer
//                             exponent bits -> a static loss scale keeps the backward's
//                             activation gradients out of the fp16 subnormal range)
#pragma once
#ifdef DQN_F16
typedef _Float16 act_t;
#define DQN_ACT_F16 1
#define DQN_MFMA16_BUILTIN __builtin_amdgcn_mfma_f32_16x16x32_f16
#else
typedef __bf16 act_t;
#define DQN_ACT_F16 0
#define DQN_MFMA16_BUILTIN __builtin_amdgcn_mfma_f32_16x16x32_bf16
#endif

namespace dqn {
// dL/dH leaves the fp32 head scaled by kLossScale; every weight-gradient kernel
// multiplies its fp32 result by kInvLossScale, so the flat gradient is unscaled.
constexpr float kLossScale = DQN_ACT_F16 ? 1024.f : 1.f;
constexpr float kInvLossScale = 1.f / kLossScale;
}  // namespace dqn
