#include "hip/hip_runtime.h"
// Batched RGB->gray + bilinear resize on the GPU (for device-resident envs).
// Bit-exact with the cv2-compatible fixed-point oracle in
// dist_dqn_amd/utils/image.py (reference call: /root/reference/src/utils.py:39-45).
#include "common.h"
#include "../include/dqn_kernels.h"

namespace dqn {

DQN_DEV void axis_coef(int d, int src, int dst, int& s, int& c0) {
  const double scale = (double)src / (double)dst;
  float f = (float)((d + 0.5) * scale - 0.5);
  int si = (int)floorf(f);
  f -= (float)si;
  if (si < 0) { si = 0; f = 0.f; }
  if (si >= src - 1) { si = src - 1; f = 0.f; }
  s = si;
  c0 = (int)rintf((1.f - f) * 2048.f);
}

DQN_DEV int gray_at(const uint8_t* img, int Ws, int y, int x) {
  const uint8_t* p = img + ((int64_t)y * Ws + x) * 3;
  return (4899 * (int)p[0] + 9617 * (int)p[1] + 1868 * (int)p[2] + (1 << 13)) >> 14;
}

__global__ void preprocess_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int N, int Hs,
                                  int Ws, int H, int W) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * H * W) return;
  const int n = t / (H * W), r = t - n * H * W, y = r / W, x = r - y * W;
  int sx, cx0, sy, cy0;
  axis_coef(x, Ws, W, sx, cx0);
  axis_coef(y, Hs, H, sy, cy0);
  const int sx1 = min(sx + 1, Ws - 1), sy1 = min(sy + 1, Hs - 1);
  const uint8_t* img = in + (int64_t)n * Hs * Ws * 3;
  const int h0 = gray_at(img, Ws, sy, sx) * cx0 + gray_at(img, Ws, sy, sx1) * (2048 - cx0);
  const int h1 = gray_at(img, Ws, sy1, sx) * cx0 + gray_at(img, Ws, sy1, sx1) * (2048 - cx0);
  const long long v = ((long long)h0 * cy0 + (long long)h1 * (2048 - cy0) + (1 << 21)) >> 22;
  out[t] = (uint8_t)min(max(v, 0ll), 255ll);
}

}  // namespace dqn

using namespace dqn;

void launch_preprocess_batch(const uint8_t* in, uint8_t* out, int N, int Hs, int Ws, int H, int W, hipStream_t st) {
  const int total = N * H * W;
  hipLaunchKernelGGL(preprocess_kernel, dim3((total + 255) / 256), dim3(256), 0, st, in, out, N, Hs, Ws, H, W);
}
