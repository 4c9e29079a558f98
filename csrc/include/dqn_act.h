// Element type of the MFMA network kernels' activations, activation gradients and
// packed weight fragments (fp32 accumulation and fp32 master weights/gradients always).
//   default build (_C):      bf16  -> v_mfma_f32_16x16x32_bf16
//   -DDQN_F16 build (_C_f16): fp16  -> v_mfma_f32_16x16x32_f16  (BASELINE config 5's fp16
//                             path; same MFMA rate on CDNA4, 3 more mantissa bits, 5 fewer
//                             exponent bits -> a static loss scale keeps the backward's
//                             activation gradients out of the fp16 subnormal range)
//   -DDQN_F32 build (_C_f32): fp32  -> v_mfma_f32_16x16x4_f32, 8 per 32-deep k-step (the
//                             reference's fp32 training precision, --dtype=fp32). The
//                             fragment layouts stay those of the 16-bit builds: a lane's 8
//                             consecutive k values feed 8 MFMAs whose 4 lane groups cover
//                             k = {8g + j}, so the 8 sums are the full 32-deep dot product.
// in_t: element type of the uint8 input images staged in LDS by the fused trunks: bf16 in
// every build (integers 0..255 are exact in bf16), which keeps the fp32 build's LDS plan.
#pragma once
#if defined(DQN_F32)
typedef float act_t;
#define DQN_ACT_F16 0
#define DQN_ACT_F32 1
#define DQN_MFMA16_BUILTIN(a, b, c, x, y, z) ::dqn::mfma_f32_k32((a), (b), (c))
#elif defined(DQN_F16)
typedef _Float16 act_t;
#define DQN_ACT_F16 1
#define DQN_ACT_F32 0
#define DQN_MFMA16_BUILTIN __builtin_amdgcn_mfma_f32_16x16x32_f16
#else
typedef __bf16 act_t;
#define DQN_ACT_F16 0
#define DQN_ACT_F32 0
#define DQN_MFMA16_BUILTIN __builtin_amdgcn_mfma_f32_16x16x32_bf16
#endif
#if DQN_ACT_F16
typedef _Float16 in_t;
#else
typedef __bf16 in_t;
#endif

namespace dqn {
// dL/dH leaves the fp32 head scaled by kLossScale; every weight-gradient kernel
// multiplies its fp32 result by kInvLossScale, so the flat gradient is unscaled.
constexpr float kLossScale = DQN_ACT_F16 ? 1024.f : 1.f;
constexpr float kInvLossScale = 1.f / kLossScale;
}  // namespace dqn
