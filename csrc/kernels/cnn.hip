// The reference Q-network `cnn` (/root/reference/src/network.py:317-424): three
// [conv SAME -> +bias -> ReLU -> max-pool 2x2/2 SAME] blocks, 84x84x4 ->
// 21x21x32 -> 11x11x32 -> 6x6x64 -> 3x3x64 -> 3x3x64 -> 2x2x64 = 256 features.
// Per-sample fused kernels (one workgroup = one sample), MFMA bf16 / fp32 acc:
//
//   cnn_fwd_kernel  stage the uint8 stack (frame-ring slots or NHWC) into LDS as a
//                   zero-PADDED bf16 88x88x4 image (SAME padding costs no bounds
//                   checks), conv1 -> a1 (LDS), pool1 -> padded p1 (LDS), conv2 ->
//                   a2, pool2 -> padded p2, conv3 (k-split over 2 wave groups) -> a3,
//                   pool3 -> the 256 fc inputs. Online(s) keeps a1/p1/a2/p2/a3 in
//                   global memory for the backward; other instances write x3 only.
//   cnn_bwd_kernel  from dp3 (fc dgrad, already masked by the pooled ReLU output):
//                   pool3 backward (argmax recomputed, first max in row-major order
//                   like the oracle's max_pool2d) + ReLU mask -> dz3, conv3 dgrad
//                   (MFMA, packed dgrad fragments), pool2 backward -> dz2, conv2
//                   dgrad, pool1 backward -> dz1. dz1/dz2/dz3 feed the grouped
//                   weight-gradient launch (qnet.hip) with padded conv loaders.
#include "common.h"
#include "fused_util.h"
#include "../include/dqn_nets_k.h"

namespace dqn {
namespace cnn {
constexpr int IH = 84, HW = IH * IH, XP = 2, XW = IH + 2 * XP;   // padded input 88 x 88
constexpr int O1 = 21, R1 = O1 * O1, N1 = 32, K1 = 256, L1 = N1 + 8;
constexpr int Q1 = 11, P1W = Q1 + 3, LP1 = N1 + 8;                 // conv2 SAME pad: top/left 1, bottom/right 2
constexpr int O2 = 6, R2 = O2 * O2, N2 = 64, K2 = 512, L2 = N2 + 8;
constexpr int Q2 = 3, P2W = Q2 + 2, LP2 = N2 + 8;                  // conv3 SAME pad 1
constexpr int O3 = 3, R3 = O3 * O3, N3 = 64, K3 = 576, L3 = N3 + 8;
constexpr int Q3 = 2;                                               // pool3 (SAME, pad bottom/right 1)
// LDS carve-up of the (dead after conv1) padded-input region, in act_t elements
constexpr int OFF_P1 = 0, OFF_A2 = OFF_P1 + P1W * P1W * LP1, OFF_P2 = OFF_A2 + R2 * L2,
              OFF_A3 = OFF_P2 + P2W * P2W * LP2, OFF_RED = OFF_A3 + R3 * L3;
static_assert((OFF_RED * sizeof(act_t)) % 16 == 0 &&
              OFF_RED * sizeof(act_t) + 4096 <= XW * XW * 4 * sizeof(in_t), "fwd LDS carve-up");
}  // namespace cnn

DQN_DEV bfx8 max8(bfx8 a, const bfx8& b) {
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = (float)b[j] > (float)a[j] ? b[j] : a[j];
  return a;
}

__global__ void __launch_bounds__(512) cnn_fwd_kernel(CnnFwdArgs a) {
  using namespace cnn;
  __shared__ __attribute__((aligned(16))) in_t xin[XW * XW * 4];
  __shared__ __attribute__((aligned(16))) act_t a1[R1 * L1];
  act_t* const xa = reinterpret_cast<act_t*>(xin);
  act_t* p1p = xa + OFF_P1;
  act_t* a2 = xa + OFF_A2;
  act_t* p2p = xa + OFF_P2;
  act_t* a3 = xa + OFF_A3;
  float* red = reinterpret_cast<float*>(xa + OFF_RED);
  const int b = blockIdx.x, inst = blockIdx.y;
  if (a.M[inst] > 0 && b >= a.M[inst]) return;          // (fused actor instance: E < B samples)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // probe stamps: 0 start, 1 input staged, 2 conv1, 3 pool1, 4 conv2, 5 pool2, 6 conv3, 7 end
  int64_t* prof = (a.prof != nullptr && tid == 0) ? a.prof + 8 * ((int64_t)inst * gridDim.x + b) : nullptr;
#define CNN_MARK(i) if (prof) prof[i] = (int64_t)__builtin_amdgcn_s_memrealtime()
  CNN_MARK(0);
  const int l16 = lane & 15, kg = 8 * (lane >> 4), cq = 4 * (lane >> 4);
  const bool keep = inst == 0 && a.a1 != nullptr;

  // ---- input loads first (4 pixels x 4 channels per task), then weights / biases
  constexpr int NT = HW / 4;
  uint32_t in[4][4];
  const bool slot_path = a.slots[inst] != nullptr;
  if (slot_path) {
    const int4 sl = reinterpret_cast<const int4*>(a.slots[inst])[b];
    const uint32_t* f0 = reinterpret_cast<const uint32_t*>(a.frames + (int64_t)sl.x * HW);
    const uint32_t* f1 = reinterpret_cast<const uint32_t*>(a.frames + (int64_t)sl.y * HW);
    const uint32_t* f2 = reinterpret_cast<const uint32_t*>(a.frames + (int64_t)sl.z * HW);
    const uint32_t* f3 = reinterpret_cast<const uint32_t*>(a.frames + (int64_t)sl.w * HW);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = tid + 512 * j;
      if (t < NT) { in[j][0] = f0[t]; in[j][1] = f1[t]; in[j][2] = f2[t]; in[j][3] = f3[t]; }
    }
  } else {
    const uint4* src = reinterpret_cast<const uint4*>(a.states[inst] + (int64_t)b * HW * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = tid + 512 * j;
      if (t < NT) { const uint4 v = src[t]; in[j][0] = v.x; in[j][1] = v.y; in[j][2] = v.z; in[j][3] = v.w; }
    }
  }
  const int nq = wave & 3, hi = wave >> 2;
  // conv2 / conv3 fragments: issued before pool1 / pool2 (their latency partly overlaps those
  // stages). Issuing them with the input loads instead delayed the input staging by ~1.2 us and the
  // whole forward by ~0.3 us (scripts/probe_cnn.py, round 6), so kept per stage.
  constexpr bool kEarlyW = false;
  bfx8 w2r[K2 / 32], w3r[K3 / 64];
  auto load_w2 = [&]() {
    const bfx8* W2 = reinterpret_cast<const bfx8*>(a.w2[inst]);
#pragma unroll
    for (int ks = 0; ks < K2 / 32; ++ks) w2r[ks] = W2[(ks * 4 + nq) * 64 + lane];
  };
  auto load_w3 = [&]() {
    const bfx8* W3 = reinterpret_cast<const bfx8*>(a.w3[inst]);
#pragma unroll
    for (int j = 0; j < K3 / 64; ++j) w3r[j] = W3[((hi * (K3 / 64) + j) * 4 + nq) * 64 + lane];
  };
  if constexpr (kEarlyW) {
    load_w2();
    load_w3();
  }
  bfx8 w1r[2][K1 / 32];
  {
    const bfx8* W1 = reinterpret_cast<const bfx8*>(a.w1[inst]);
#pragma unroll
    for (int ks = 0; ks < K1 / 32; ++ks) {
      w1r[0][ks] = W1[(ks * 2 + 0) * 64 + lane];
      w1r[1][ks] = W1[(ks * 2 + 1) * 64 + lane];
    }
  }
  const float4 bias1a = *reinterpret_cast<const float4*>(a.b1[inst] + cq);
  const float4 bias1b = *reinterpret_cast<const float4*>(a.b1[inst] + 16 + cq);
  const float4 bias2 = *reinterpret_cast<const float4*>(a.b2[inst] + nq * 16 + cq);
  const float4 bias3 = *reinterpret_cast<const float4*>(a.b3[inst] + nq * 16 + cq);

  // ---- zero-padded bf16 NHWC image: interior from the loads, 2-pixel zero border
  for (int t = tid; t < 4 * XW + 4 * IH; t += 512) {       // 688 border pixels
    int y, x;
    if (t < 4 * XW) { const int r = t / XW; y = r < 2 ? r : r + IH; x = t - r * XW; }
    else { const int u = t - 4 * XW, r = u / 4, c = u - r * 4; y = r + XP; x = c < 2 ? c : c + IH; }
    *reinterpret_cast<uint2*>(xin + (y * XW + x) * 4) = make_uint2(0u, 0u);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int t = tid + 512 * j;
    if (t >= NT) continue;
    const int y = (4 * t) / IH, x = 4 * t - y * IH;          // 4 consecutive pixels of one row
    in_t* dst = xin + ((y + XP) * XW + x + XP) * 4;
    if (slot_path) {
      planes_to_lds(in[j][0], in[j][1], in[j][2], in[j][3], dst);
    } else {
      uint32_t c[4];
#pragma unroll
      for (int ch = 0; ch < 4; ++ch)
        c[ch] = ((in[j][0] >> 8 * ch) & 0xffu) | (((in[j][1] >> 8 * ch) & 0xffu) << 8) |
                (((in[j][2] >> 8 * ch) & 0xffu) << 16) | (((in[j][3] >> 8 * ch) & 0xffu) << 24);
      planes_to_lds(c[0], c[1], c[2], c[3], dst);
    }
  }
  __syncthreads();
  CNN_MARK(1);

  // ---- conv1 (8x8/4 SAME) -> a1 = ReLU(scale*acc + b); both n-tiles per wave
#if DQN_ACT_F32
  // fp32 build: the uint8 input is exact in bf16, so each fp32 weight fragment runs as three bf16
  // fragments (split3_bf16, fused_util.h): 3 bf16 MFMAs instead of 8 fp32 ones per k-step. A wave's
  // m-tiles (4) share each split, made once per k-step.
  {
    const float scale = a.scale;
    const int kw = kg >> 2;
    act_t* ga1 = keep ? a.a1 + (int64_t)b * R1 * N1 : nullptr;
    constexpr int NMT = (R1 + 15) / 16, MTW = (NMT + 7) / 8;
    f32x4 c0[MTW], c1[MTW];
    int off[MTW];
    bool okm[MTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      const int mt = wave + 8 * i, p = mt * 16 + l16;
      okm[i] = mt < NMT && p < R1;
      const int q = okm[i] ? p : 0, oy = q / O1, ox = q - oy * O1;
      off[i] = ((oy * 4) * XW + ox * 4 + kw) * 4;
      c0[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      c1[i] = c0[i];
    }
#pragma unroll
    for (int ks = 0; ks < K1 / 32; ++ks) {
      b16x8 h0, m0, l0, h1, m1, l1;
      split3_bf16(w1r[0][ks], h0, m0, l0);
      split3_bf16(w1r[1][ks], h1, m1, l1);
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        if (wave + 8 * i >= NMT) continue;                  // (wave-uniform)
        b16x8 x;
        if (okm[i]) {
          x = *reinterpret_cast<const b16x8*>(xin + off[i] + ks * XW * 4);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = (__bf16)0.f;
        }
        c0[i] = mfma3_bf16(h0, m0, l0, x, c0[i]);
        c1[i] = mfma3_bf16(h1, m1, l1, x, c1[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      if (!okm[i]) continue;
      const int p = (wave + 8 * i) * 16 + l16;
      const pk4_t v0 = pack4(c0[i] * scale + f4(bias1a)), v1 = pack4(c1[i] * scale + f4(bias1b));
      *reinterpret_cast<pk4_t*>(a1 + p * L1 + cq) = v0;
      *reinterpret_cast<pk4_t*>(a1 + p * L1 + 16 + cq) = v1;
      if (ga1 != nullptr) {
        *reinterpret_cast<pk4_t*>(ga1 + p * N1 + cq) = v0;
        *reinterpret_cast<pk4_t*>(ga1 + p * N1 + 16 + cq) = v1;
      }
    }
  }
#else
  {
    const float scale = a.scale;
    const int kw = kg >> 2;
    act_t* ga1 = keep ? a.a1 + (int64_t)b * R1 * N1 : nullptr;
    for (int mt = wave; mt < (R1 + 15) / 16; mt += 8) {
      const int p = mt * 16 + l16;
      const bool ok = p < R1;
      const int oy = ok ? p / O1 : 0, ox = ok ? p - oy * O1 : 0;
      const in_t* base = xin + ((oy * 4) * XW + ox * 4 + kw) * 4;
      bfx8 fa[K1 / 32];
#pragma unroll
      for (int ks = 0; ks < K1 / 32; ++ks) fa[ks] = ok ? ld_in8(base + ks * XW * 4) : tz8();
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
      for (int ks = 0; ks < K1 / 32; ++ks) {
        c0 = tmfma(w1r[0][ks], fa[ks], c0);
        c1 = tmfma(w1r[1][ks], fa[ks], c1);
      }
      if (ok) {
        const pk4_t v0 = pack4(c0 * scale + f4(bias1a)), v1 = pack4(c1 * scale + f4(bias1b));
        *reinterpret_cast<pk4_t*>(a1 + p * L1 + cq) = v0;
        *reinterpret_cast<pk4_t*>(a1 + p * L1 + 16 + cq) = v1;
        if (ga1 != nullptr) {
          *reinterpret_cast<pk4_t*>(ga1 + p * N1 + cq) = v0;
          *reinterpret_cast<pk4_t*>(ga1 + p * N1 + 16 + cq) = v1;
        }
      }
    }
  }
#endif
  CNN_MARK(2);
  if constexpr (!kEarlyW) load_w2();
  __syncthreads();

  // ---- pool1 (SAME 21 -> 11, bottom/right window cut) -> padded p1 (zero border)
  for (int t = tid; t < Q1 * Q1 * 4; t += 512) {
    const int pix = t >> 2, c8 = (t & 3) * 8, py = pix / Q1, px = pix - py * Q1;
    bfx8 m = *reinterpret_cast<const bfx8*>(a1 + ((2 * py) * O1 + 2 * px) * L1 + c8);
    if (2 * px + 1 < O1) m = max8(m, *reinterpret_cast<const bfx8*>(a1 + ((2 * py) * O1 + 2 * px + 1) * L1 + c8));
    if (2 * py + 1 < O1) {
      m = max8(m, *reinterpret_cast<const bfx8*>(a1 + ((2 * py + 1) * O1 + 2 * px) * L1 + c8));
      if (2 * px + 1 < O1) m = max8(m, *reinterpret_cast<const bfx8*>(a1 + ((2 * py + 1) * O1 + 2 * px + 1) * L1 + c8));
    }
    *reinterpret_cast<bfx8*>(p1p + ((py + 1) * P1W + px + 1) * LP1 + c8) = m;
    if (keep) *reinterpret_cast<bfx8*>(a.p1 + (int64_t)b * Q1 * Q1 * N1 + pix * N1 + c8) = m;
  }
  for (int t = tid; t < (P1W * P1W - Q1 * Q1) * 4; t += 512) {   // 75 border pixels x 4
    const int bp = t >> 2, c8 = (t & 3) * 8;
    int y, x;
    if (bp < 3 * P1W) { const int r = bp / P1W; y = r == 0 ? 0 : Q1 + r; x = bp - r * P1W; }
    else { const int u = bp - 3 * P1W, r = u / 3, c = u - r * 3; y = r + 1; x = c == 0 ? 0 : Q1 + c; }
    *reinterpret_cast<bfx8*>(p1p + (y * P1W + x) * LP1 + c8) = tz8();
  }
  __syncthreads();
  CNN_MARK(3);

  // ---- conv2 (4x4/2 SAME) -> a2: wave = n-tile (wave & 3), m-tiles {wave>>2, +2}
  {
    act_t* ga2 = keep ? a.a2 + (int64_t)b * R2 * N2 : nullptr;
    for (int mt = hi; mt < (R2 + 15) / 16; mt += 2) {
      const int p = mt * 16 + l16;
      const bool ok = p < R2;
      const int oy = ok ? p / O2 : 0, ox = ok ? p - oy * O2 : 0;
      const act_t* base = p1p + ((oy * 2) * P1W + ox * 2) * LP1 + kg;
      bfx8 fa[K2 / 32];
#pragma unroll
      for (int ks = 0; ks < K2 / 32; ++ks)                 // k = (kh*4 + kw)*32 + ci
        fa[ks] = ok ? *reinterpret_cast<const bfx8*>(base + ((ks >> 2) * P1W + (ks & 3)) * LP1) : tz8();
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < K2 / 32; ++ks) c = tmfma(w2r[ks], fa[ks], c);
      if (ok) {
        const pk4_t v = pack4(c + f4(bias2));
        *reinterpret_cast<pk4_t*>(a2 + p * L2 + nq * 16 + cq) = v;
        if (ga2 != nullptr) *reinterpret_cast<pk4_t*>(ga2 + p * N2 + nq * 16 + cq) = v;
      }
    }
  }
  CNN_MARK(4);
  if constexpr (!kEarlyW) load_w3();
  __syncthreads();

  // ---- pool2 (6 -> 3) -> padded p2
  for (int t = tid; t < Q2 * Q2 * 8; t += 512) {
    const int pix = t >> 3, c8 = (t & 7) * 8, py = pix / Q2, px = pix - py * Q2;
    const act_t* r0 = a2 + ((2 * py) * O2 + 2 * px) * L2 + c8;
    bfx8 m = max8(*reinterpret_cast<const bfx8*>(r0), *reinterpret_cast<const bfx8*>(r0 + L2));
    m = max8(m, *reinterpret_cast<const bfx8*>(r0 + O2 * L2));
    m = max8(m, *reinterpret_cast<const bfx8*>(r0 + O2 * L2 + L2));
    *reinterpret_cast<bfx8*>(p2p + ((py + 1) * P2W + px + 1) * LP2 + c8) = m;
    if (keep) *reinterpret_cast<bfx8*>(a.p2 + (int64_t)b * Q2 * Q2 * N2 + pix * N2 + c8) = m;
  }
  for (int t = tid; t < (P2W * P2W - Q2 * Q2) * 8; t += 512) {   // 16 border pixels x 8
    const int bp = t >> 3, c8 = (t & 7) * 8;
    int y, x;
    if (bp < 2 * P2W) { const int r = bp / P2W; y = r == 0 ? 0 : P2W - 1; x = bp - r * P2W; }
    else { const int u = bp - 2 * P2W, r = u / 2; y = r + 1; x = (u & 1) ? P2W - 1 : 0; }
    *reinterpret_cast<bfx8*>(p2p + (y * P2W + x) * LP2 + c8) = tz8();
  }
  __syncthreads();
  CNN_MARK(5);

  // ---- conv3 (3x3/1 SAME) -> a3: wave = (n-tile, k-half), partials exchanged in LDS
  {
    const int p = l16;
    const bool ok = p < R3;
    const int oy = ok ? p / O3 : 0, ox = ok ? p - oy * O3 : 0;
    const act_t* base = p2p + (oy * P2W + ox) * LP2 + kg;
    bfx8 fa[K3 / 64];
#pragma unroll
    for (int j = 0; j < K3 / 64; ++j) {                    // k = (kh*3 + kw)*64 + ci
      const int ks = hi * (K3 / 64) + j, tap = ks >> 1, kh = tap / 3, kw = tap - kh * 3;
      fa[j] = ok ? *reinterpret_cast<const bfx8*>(base + (kh * P2W + kw) * LP2 + (ks & 1) * 32) : tz8();
    }
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < K3 / 64; ++j) c = tmfma(w3r[j], fa[j], c);
    if (hi == 1) park(red, nq, lane, c);
    __syncthreads();
    if (hi == 0) {
      c = unpark(red, nq, lane, c);
      if (ok) {
        CNN_MARK(6);
        const pk4_t v = pack4(c + f4(bias3));
        *reinterpret_cast<pk4_t*>(a3 + p * L3 + nq * 16 + cq) = v;
        if (keep) *reinterpret_cast<pk4_t*>(a.a3 + (int64_t)b * R3 * N3 + p * N3 + nq * 16 + cq) = v;
      }
    }
  }
  __syncthreads();

  // ---- pool3 (SAME 3 -> 2, windows {0,1} and {2}) -> the 256 fc inputs (HWC order)
  if (tid < Q3 * Q3 * 8) {
    const int pix = tid >> 3, c8 = (tid & 7) * 8, py = pix / Q3, px = pix - py * Q3;
    bfx8 m = *reinterpret_cast<const bfx8*>(a3 + ((2 * py) * O3 + 2 * px) * L3 + c8);
    if (2 * px + 1 < O3) m = max8(m, *reinterpret_cast<const bfx8*>(a3 + ((2 * py) * O3 + 2 * px + 1) * L3 + c8));
    if (2 * py + 1 < O3) {
      m = max8(m, *reinterpret_cast<const bfx8*>(a3 + ((2 * py + 1) * O3 + 2 * px) * L3 + c8));
      if (2 * px + 1 < O3) m = max8(m, *reinterpret_cast<const bfx8*>(a3 + ((2 * py + 1) * O3 + 2 * px + 1) * L3 + c8));
    }
    *reinterpret_cast<bfx8*>(a.x3[inst] + (int64_t)b * Q3 * Q3 * N3 + pix * N3 + c8) = m;
  }
  CNN_MARK(7);
}

// ======================================================================= backward
// Window-major pool backward (one thread = one 2x2/2 window x 8 channels): the window's valid cells of
// the pre-pool map `act` (LDS, L elements per pixel) are read once, the first max in row-major order
// over the valid cells (the oracle's max_pool2d routing) per channel gets d = dp[window][c] where that
// maximum is > 0 (ReLU), every other cell 0. (Round 5 ran one thread per pre-pool element, each
// re-reading its whole window: pool1's backward alone took ~10 us of the launch, scripts/probe_cnn.py.)
// out[dy * 2 + dx]: the cells' 8 values; valid[]: the cell is inside the map.
template <int OH, int OW, int L>
DQN_DEV void pool_bwd8(const act_t* act, const float* dpw, int py, int px, int c8, bfx8* out, bool* valid) {
  bfx8 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int y = 2 * py + (i >> 1), x = 2 * px + (i & 1);
    valid[i] = y < OH && x < OW;
    v[i] = valid[i] ? *reinterpret_cast<const bfx8*>(act + (y * OW + x) * L + c8) : tz8();
  }
  const float4 d0 = *reinterpret_cast<const float4*>(dpw + c8), d1 = *reinterpret_cast<const float4*>(dpw + c8 + 4);
  const float d[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float best = -INFINITY;
    int bi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float f = (float)v[i][j];
      if (valid[i] && f > best) { best = f; bi = i; }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i][j] = (act_t)((i == bi && best > 0.f) ? d[j] : 0.f);
  }
}

__global__ void __launch_bounds__(512) cnn_bwd_kernel(CnnBwdArgs a) {
  using namespace cnn;
  __shared__ __attribute__((aligned(16))) act_t a1s[R1 * N1];
  __shared__ __attribute__((aligned(16))) act_t a2s[R2 * N2];
  __shared__ __attribute__((aligned(16))) act_t a3s[R3 * N3];
  __shared__ __attribute__((aligned(16))) act_t dz3s[R3 * L3];
  __shared__ __attribute__((aligned(16))) act_t dz2s[R2 * L2];
  __shared__ __attribute__((aligned(16))) float dp3s[Q3 * Q3 * N3];
  __shared__ __attribute__((aligned(16))) float dp2[Q2 * Q2 * N2];
  __shared__ __attribute__((aligned(16))) float dp1[Q1 * Q1 * N1];
  __shared__ __attribute__((aligned(16))) float red[4 * 256];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, kg = 8 * (lane >> 4);
  // two or four workgroups per sample (gridDim.y): all run the cheap stages up to dz2 (part 0 writes
  // dz3 / dz2), then each takes its share of the conv2 dgrad m-tiles and their pool1 windows -- one
  // workgroup per sample held the 32-sample backward on 32 CUs, the conv2 dgrad MFMA-bound there
  // in the fp32 build (16 of its 30 us, scripts/probe_cnn.py). Four parts: ref fp32 9.1k -> 10.6k,
  // bf16 17.4k -> 18.6k SGD steps/s (KernelTuning.cnn_bwd_parts)
  const int part = blockIdx.y, nparts = gridDim.y;
  // probe stamps: 0 start, 1 loads, 2 pool3, 3 conv3 dgrad, 4 pool2, 5 conv2 dgrad, 6 a1 staged, 7 end
  int64_t* prof = (a.prof != nullptr && tid == 0 && part == 0) ? a.prof + 8 * (int64_t)b : nullptr;
  CNN_MARK(0);
  const act_t* ga1 = a.a1 + (int64_t)b * R1 * N1;
  const act_t* ga2 = a.a2 + (int64_t)b * R2 * N2;
  const act_t* ga3 = a.a3 + (int64_t)b * R3 * N3;
  // every global load of the kernel that does not depend on its own results, issued up front in one
  // batch: a1 (needed only by the last stage: held in registers until then, so the first stages wait
  // for a2 / a3 / dp3 alone), the conv3 dgrad fragments of this wave, the first conv2 dgrad batch
  // (issued after conv3 below). Round 5 issued them stage by stage: the conv2 dgrad alone waited on
  // 8 dependent L2 round trips per wave (23.7 us for the launch, profiles/r6_kernel_stats_ref_bf16_v1.md).
  constexpr int NA1 = (R1 * N1 / 8 + 511) / 512;
  bfx8 a1r[NA1];
#pragma unroll
  for (int j = 0; j < NA1; ++j) {
    const int t = tid + 512 * j;
    a1r[j] = t < R1 * N1 / 8 ? reinterpret_cast<const bfx8*>(ga1)[t] : tz8();
  }
  const int nq3 = wave & 3, hi3 = wave >> 2;
  bfx8 w3r[K3 / 64];
  {
    const bfx8* W = reinterpret_cast<const bfx8*>(a.w3d);
#pragma unroll
    for (int j = 0; j < K3 / 64; ++j) w3r[j] = W[((hi3 * (K3 / 64) + j) * 4 + nq3) * 64 + lane];
  }
  for (int t = tid; t < R2 * N2 / 8; t += 512)
    reinterpret_cast<bfx8*>(a2s)[t] = reinterpret_cast<const bfx8*>(ga2)[t];
  if (tid < R3 * N3 / 8) reinterpret_cast<bfx8*>(a3s)[tid] = reinterpret_cast<const bfx8*>(ga3)[tid];
  if (tid < Q3 * Q3 * N3) dp3s[tid] = (float)a.dp3[(int64_t)b * Q3 * Q3 * N3 + tid];
  __syncthreads();
  CNN_MARK(1);

  // ---- pool3 backward + ReLU mask -> dz3 (LDS + global): window-major, 8 channels per thread
  if (tid < Q3 * Q3 * (N3 / 8)) {
    const int w = tid / (N3 / 8), c8 = (tid - w * (N3 / 8)) * 8, py = w / Q3, px = w - py * Q3;
    bfx8 o[4];
    bool ok[4];
    pool_bwd8<O3, O3, N3>(a3s, dp3s + w * N3, py, px, c8, o, ok);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!ok[i]) continue;
      const int p = (2 * py + (i >> 1)) * O3 + 2 * px + (i & 1);
      *reinterpret_cast<bfx8*>(dz3s + p * L3 + c8) = o[i];
      if (part == 0) *reinterpret_cast<bfx8*>(a.dz3 + (int64_t)b * R3 * N3 + p * N3 + c8) = o[i];
    }
  }
  __syncthreads();
  CNN_MARK(2);

  // ---- conv3 dgrad -> dp2 [9][64]: A gathers dz3 (SAME pad 1, stride 1), B = packed dgrad (w3r)
  {
    const int m = l16;
    const int iy = m / O3, ix = m - iy * O3;
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < K3 / 64; ++j) {
      const int ks = hi3 * (K3 / 64) + j, tap = ks >> 1, kh = tap / 3, kw = tap - kh * 3;
      const int oy = iy + 1 - kh, ox = ix + 1 - kw, co = (ks & 1) * 32 + kg;
      const bool ok = m < R3 && oy >= 0 && oy < O3 && ox >= 0 && ox < O3;
      const bfx8 af = ok ? *reinterpret_cast<const bfx8*>(dz3s + (oy * O3 + ox) * L3 + co) : tz8();
      c = tmfma(af, w3r[j], c);
    }
    if (hi3 == 1) park(red, nq3, lane, c);
    __syncthreads();
    if (hi3 == 0) {
      c = unpark(red, nq3, lane, c);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mm = 4 * (lane >> 4) + r;
        if (mm < R3) dp2[mm * N2 + nq3 * 16 + l16] = c[r];
      }
    }
  }
  // conv2 dgrad operands: wave w owns n-tile nt = w & 1 of the m-tiles w >> 1 and (w >> 1) + 4 -- the
  // two tasks share their B fragments, loaded once per 8-deep batch, the next batch in flight (16-bit
  // builds: double-buffered) while this one's MFMAs run; batch 0 issued now, under pool2's work
  const bfx8* W2 = reinterpret_cast<const bfx8*>(a.w2d);
  // (one part: m-tiles w >> 1 and (w >> 1) + 4 per wave; two parts: m-tile 4 part + (w >> 1) only;
  //  four parts: m-tile 2 part + ((w >> 1) & 1), the K range halved over w >> 2, partials met in LDS)
  const int nt2 = wave & 1;
  const int mtA = nparts == 4 ? 2 * part + ((wave >> 1) & 1) : (wave >> 1) + 4 * part;
  const int kh2 = nparts == 4 ? wave >> 2 : 0;
  const int q0 = 2 * kh2, q1 = nparts == 4 ? q0 + 2 : 4;   // this wave's 8-deep k-step batches
  const bool twom = nparts == 1;
  constexpr int NB2 = DQN_ACT_F32 ? 1 : 2;                 // B batches in registers
  bfx8 bf[NB2][8];
#pragma unroll
  for (int u = 0; u < 8; ++u) bf[0][u] = W2[((8 * q0 + u) * 2 + nt2) * 64 + lane];
  __syncthreads();
  CNN_MARK(3);

  // ---- pool2 backward + mask -> dz2 (window-major)
  if (tid < Q2 * Q2 * (N2 / 8)) {
    const int w = tid / (N2 / 8), c8 = (tid - w * (N2 / 8)) * 8, py = w / Q2, px = w - py * Q2;
    bfx8 o[4];
    bool ok[4];
    pool_bwd8<O2, O2, N2>(a2s, dp2 + w * N2, py, px, c8, o, ok);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!ok[i]) continue;
      const int p = (2 * py + (i >> 1)) * O2 + 2 * px + (i & 1);
      *reinterpret_cast<bfx8*>(dz2s + p * L2 + c8) = o[i];
      if (part == 0) *reinterpret_cast<bfx8*>(a.dz2 + (int64_t)b * R2 * N2 + p * N2 + c8) = o[i];
    }
  }
  __syncthreads();
  CNN_MARK(4);

  // ---- conv2 dgrad -> dp1 [121][32]: 8 m-tiles x 2 n-tiles, K = 16 taps x 64 (32 k-steps)
  {
    f32x4 cA = {0.f, 0.f, 0.f, 0.f}, cB = cA;
    const int mA = mtA * 16 + l16, mB = (mtA + 4) * 16 + l16;
    const int iyA = mA / Q1, ixA = mA - iyA * Q1, iyB = mB / Q1, ixB = mB - iyB * Q1;
    auto gather = [&](int m, int iy, int ix, int ks) -> bfx8 {
      const int tap = ks >> 1, kh = tap >> 2, kw = tap & 3, co = (ks & 1) * 32 + kg;
      const int ny = iy + 1 - kh, nx = ix + 1 - kw;              // SAME pad_t = pad_l = 1, stride 2
      const bool ok = m < Q1 * Q1 && ny >= 0 && nx >= 0 && !(ny & 1) && !(nx & 1) && (ny >> 1) < O2 &&
                      (nx >> 1) < O2;
      return ok ? *reinterpret_cast<const bfx8*>(dz2s + ((ny >> 1) * O2 + (nx >> 1)) * L2 + co) : tz8();
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) {                           // 4 batches of 8 k-steps
      if (q < q0 || q >= q1) continue;
      const int cur = NB2 == 2 ? (q & 1) : 0;
      if (NB2 == 1 && q > q0) {
#pragma unroll
        for (int u = 0; u < 8; ++u) bf[0][u] = W2[((8 * q + u) * 2 + nt2) * 64 + lane];
      }
      if (NB2 == 2 && q + 1 < q1) {
#pragma unroll
        for (int u = 0; u < 8; ++u) bf[(q + 1) & (NB2 - 1)][u] = W2[((8 * (q + 1) + u) * 2 + nt2) * 64 + lane];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int ks = 8 * q + u;
        cA = tmfma(gather(mA, iyA, ixA, ks), bf[cur][u], cA);
        if (twom) cB = tmfma(gather(mB, iyB, ixB, ks), bf[cur][u], cB);
      }
    }
    if (nparts == 4) {                                      // the two K halves of each task
      if (kh2 == 1) park(red, wave & 3, lane, cA);
      __syncthreads();
      if (kh2 == 0) cA = unpark(red, wave & 3, lane, cA);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ma = mtA * 16 + 4 * (lane >> 4) + r, mb = (mtA + 4) * 16 + 4 * (lane >> 4) + r;
      if (kh2 == 0 && ma < Q1 * Q1) dp1[ma * N1 + nt2 * 16 + l16] = cA[r];
      if (twom && mb < Q1 * Q1) dp1[mb * N1 + nt2 * 16 + l16] = cB[r];
    }
  }
  CNN_MARK(5);
  // a1 into LDS for the last stage (its loads were issued at the kernel start)
#pragma unroll
  for (int j = 0; j < NA1; ++j) {
    const int t = tid + 512 * j;
    if (t < R1 * N1 / 8) reinterpret_cast<bfx8*>(a1s)[t] = a1r[j];
  }
  __syncthreads();
  CNN_MARK(6);

  // ---- pool1 backward + mask -> dz1 (global only: the conv1 wgrad input)
  act_t* gdz1 = a.dz1 + (int64_t)b * R1 * N1;
  // (this part's windows: the dp1 rows its conv2 dgrad m-tiles made -- 128 / nparts per part)
  const int w_lo = (128 / nparts) * part, w_hi = min(Q1 * Q1, w_lo + 128 / nparts);
  for (int t = tid + w_lo * (N1 / 8); t < w_hi * (N1 / 8); t += 512) {      // (window-major, one round)
    const int w = t / (N1 / 8), c8 = (t - w * (N1 / 8)) * 8, py = w / Q1, px = w - py * Q1;
    bfx8 o[4];
    bool ok[4];
    pool_bwd8<O1, O1, N1>(a1s, dp1 + w * N1, py, px, c8, o, ok);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!ok[i]) continue;
      const int p = (2 * py + (i >> 1)) * O1 + 2 * px + (i & 1);
      *reinterpret_cast<bfx8*>(gdz1 + p * N1 + c8) = o[i];
    }
  }
  CNN_MARK(7);
#undef CNN_MARK
}

}  // namespace dqn

using namespace dqn;

void launch_cnn_fwd(const CnnFwdArgs& a, int B, int ninst, hipStream_t st) {
  hipLaunchKernelGGL(cnn_fwd_kernel, dim3(B, ninst), dim3(512), 0, st, a);
}

void launch_cnn_bwd(const CnnBwdArgs& a, int B, int parts, hipStream_t st) {
  hipLaunchKernelGGL(cnn_bwd_kernel, dim3(B, (parts == 2 || parts == 4) ? parts : 1), dim3(512), 0, st, a);
}
