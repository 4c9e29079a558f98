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
// Everything is v_mfma_f32_16x16x32_bf16 with fp32 accumulation. The conv2 / conv3 m-tiles take
// their pixels in the order of trunk_perm.h (scripts/gen_trunk_perm.py), chosen so the im2col
// ds_read_b128 of a tile hits distinct LDS banks (row-major tiles: 1.8x / 2.5x the read cycles).
#include <stdlib.h>
#include "common.h"
#include "fused_util.h"
#include "sample_dev.h"
#include "trunk_perm.h"
#include "../include/dqn_nets_k.h"

namespace dqn {

namespace trunk {
constexpr int IH = 84, IW = 84, HW = IH * IW;
constexpr int O1 = 20, N1 = 32, K1 = 256, R1 = O1 * O1;       // conv1: 8x8/4
constexpr int O2 = 9, N2 = 64, K2 = 512, R2 = O2 * O2;        // conv2: 4x4/2
constexpr int O3 = 7, N3 = 64, K3 = 576, R3 = O3 * O3;        // conv3: 3x3/1
constexpr int L1 = N1 + 8, L2 = N2 + 8;                       // padded LDS rows (elements)
// Row split (gridDim.z == 2): part 0 computes conv3 rows 0-3, part 1 rows 4-6, each from its
// own receptive field (conv2 rows 0-5 / 4-8, conv1 rows 0-13 / 8-19, input rows 0-59 / 32-83),
// so one sample runs on two CUs (the learner's ~100 workgroups leave most of the 256 CUs idle;
// the halo costs ~30% extra conv1 work per sample, not latency). Row starts / counts per part:
constexpr int kIn0[2] = {0, 32}, kInN[2] = {60, 52};
constexpr int kC10[2] = {0, 8}, kC1N[2] = {14, 12}, kC1Own[2] = {0, 10}, kC1OwnE[2] = {10, 20};
constexpr int kC20[2] = {0, 4}, kC2N[2] = {6, 5}, kC2Own[2] = {0, 5}, kC2OwnE[2] = {5, 9};
constexpr int kC30[2] = {0, 4}, kC3N[2] = {4, 3};
constexpr int kInMax = 60, kC1Max = 14, kC2Max = 6;
}  // namespace trunk

__global__ void __launch_bounds__(512) trunk_fwd_kernel(TrunkArgs a) {
  using namespace trunk;
  const int part = blockIdx.z, split = gridDim.z;               // split 1: whole image
  const int in0 = split > 1 ? kIn0[part] : 0, inN = split > 1 ? kInN[part] : IH;
  const int c10 = split > 1 ? kC10[part] : 0, c1n = split > 1 ? kC1N[part] : O1;
  const int c1o = split > 1 ? kC1Own[part] - c10 : 0, c1e = split > 1 ? kC1OwnE[part] - c10 : O1;
  const int c20 = split > 1 ? kC20[part] : 0, c2n = split > 1 ? kC2N[part] : O2;
  const int c2o = split > 1 ? kC2Own[part] - c20 : 0, c2e = split > 1 ? kC2OwnE[part] - c20 : O2;
  const int c30 = split > 1 ? kC30[part] : 0, c3n = split > 1 ? kC3N[part] : O3;
  // xin: the sample's input rows as bf16 NHWC [rows*84][4] (converted once); dead after conv1,
  // so act2 and the conv3 K-split partials live in the same bytes afterwards. Sized for the
  // whole image (split 1); a part uses the first kInMax rows.
  __shared__ __attribute__((aligned(16))) in_t xin[HW * 4];
  __shared__ __attribute__((aligned(16))) act_t act1[R1 * L1];
  // conv1's packed weights, loaded ONCE per block and handed to every wave through LDS (every
  // wave needs all of them: direct per-wave loads moved 8 x 16 KB over the CU's ~30 B/clk L2 path)
  __shared__ __attribute__((aligned(16))) bfx8 wl1[(K1 / 32) * 2 * 64];
  act_t* act2 = reinterpret_cast<act_t*>(xin);
  constexpr size_t kRedOff = (R2 * L2 * sizeof(act_t) + 255) / 256 * 256;   // conv3 k-half partials after act2
  float* red = reinterpret_cast<float*>(reinterpret_cast<char*>(xin) + kRedOff);
  static_assert(kRedOff + 4 * 4 * 1024 <= sizeof(xin), "act2 + partials fit xin");
  static_assert(kRedOff + 4 * 6 * 1024 <= sizeof(xin), "act2 + conv2 partials fit xin");
  static_assert(sizeof(SampleLds) <= sizeof(xin), "sampler scratch fits xin");
  const int b = blockIdx.x, inst = blockIdx.y;
  if (a.M[inst] > 0 && b >= a.M[inst]) return;          // (fused actor instance: E < B samples)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kg = 8 * (lane >> 4);
  int64_t* prof = a.prof != nullptr && tid == 0 && part == 0 ? a.prof + ((int64_t)inst * gridDim.x + b) * 16 : nullptr;
#define TRUNK_MARK(i) if (prof) prof[i] = (int64_t)__builtin_amdgcn_s_memtime()
  TRUNK_MARK(0);

  // ---------------------------------------------------------------- fused sampling
  // (the sampler launch folded in: xin is dead until the frames land, so it holds the
  // sampler's LDS scratch; every sampled workgroup draws the same batch)
  const bool sampled = a.smp.size != nullptr && inst < a.smp.ninst;
  int4 sl_s = make_int4(0, 0, 0, 0);
  if (sampled) {
    SampleLds& sls = *reinterpret_cast<SampleLds*>(xin);
    const uint32_t n = (uint32_t)max(a.smp.size[0], 1);
    const uint64_t seed = (uint64_t)a.smp.rng[0], ctr = (uint64_t)a.smp.rng[1];
    draw_distinct(seed, ctr, n, a.smp.B, sls);
    const int32_t tr = sls.cand[b];
    __syncthreads();                                    // every lane has its index before xin is reused
    DQN_ASSERT(tr >= 0 && (uint32_t)tr < n);
    const int4 st = reinterpret_cast<const int4*>(a.smp.state_idx)[tr];
    const int32_t nx = a.smp.next_idx[tr];
    sl_s = inst == 0 ? st : make_int4(st.y, st.z, st.w, nx);
    if (tid == 0) {
      if (inst == 0 && part == 0) write_sample_slots(a.smp, b, tr, st, nx);
      // relaxed ticket (as optim.hip): every workgroup read the counter before its add
      const int t = __hip_atomic_fetch_add(a.smp.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == a.smp.B * a.smp.ninst * split - 1) {
        a.smp.rng[1] = (int64_t)(ctr + 1);
        __hip_atomic_store(a.smp.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }

  // ---------------------------------------------------------------- input loads (first)
  // inN*21 tasks of 4 pixels (rows in0 .. in0+inN-1); a thread owns tasks tid + 512 j (j < 4)
  constexpr int NT = HW / 4;
  const int nt_in = inN * (IW / 4), t_in0 = in0 * (IW / 4);
  uint32_t in[4][4];
  const bool slot_path = sampled || a.slots[inst] != nullptr;
  if (slot_path) {
    // (component-wise select: a select between the register int4 and a loaded one put the
    // sampled slots in scratch memory)
    int4 sl = sl_s;
    if (!sampled) {
      const int4 v = reinterpret_cast<const int4*>(a.slots[inst])[b];
      sl.x = v.x; sl.y = v.y; sl.z = v.z; sl.w = v.w;
    }
    const uint32_t* f0 = reinterpret_cast<const uint32_t*>(a.frames + (int64_t)sl.x * HW) + t_in0;
    const uint32_t* f1 = reinterpret_cast<const uint32_t*>(a.frames + (int64_t)sl.y * HW) + t_in0;
    const uint32_t* f2 = reinterpret_cast<const uint32_t*>(a.frames + (int64_t)sl.z * HW) + t_in0;
    const uint32_t* f3 = reinterpret_cast<const uint32_t*>(a.frames + (int64_t)sl.w * HW) + t_in0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = tid + 512 * j;
      if (t < nt_in) { in[j][0] = f0[t]; in[j][1] = f1[t]; in[j][2] = f2[t]; in[j][3] = f3[t]; }
    }
  } else {
    const uint4* src = reinterpret_cast<const uint4*>(a.states[inst] + (int64_t)b * HW * 4) + t_in0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = tid + 512 * j;
      if (t < nt_in) { const uint4 v = src[t]; in[j][0] = v.x; in[j][1] = v.y; in[j][2] = v.z; in[j][3] = v.w; }
    }
  }
  static_assert(NT <= 4 * 512, "4 tasks per thread cover the image");

  // Weight fragments (L2-resident packed bf16), each read from L2 by ONE wave of the block
  // (the CU's L2 path, ~30 B/clk, is this kernel's bound; the input image is 28 KB):
  //   conv1 - every wave both n-tiles, all K: the block loads the 16 KB once (2 fragments per
  //           thread) and every wave takes its registers from LDS (wl1)
  //   conv2 - wave owns n-tile (wave & 3) and k-half (wave >> 2), all m-tiles; the k-halves'
  //           partial sums meet in LDS
  //   conv3 - wave owns n-tile (wave & 3) and k-half (wave >> 2); loaded after conv1
  //           into the registers conv1 no longer needs.
  const int nq = wave & 3, hi = wave >> 2;
  // this lane's tile-row pixels of conv2 / conv3 (-1: padding row), loaded with the inputs
  const int pv = split > 1 ? 1 + part : 0;
  int p2r[(R2 + 15) / 16], p3r[(R3 + 15) / 16];
#pragma unroll
  for (int mt = 0; mt < (R2 + 15) / 16; ++mt) p2r[mt] = kTrunkP2[pv][mt * 16 + row];
#pragma unroll
  for (int mt = 0; mt < (R3 + 15) / 16; ++mt) p3r[mt] = kTrunkP3[pv][mt * 16 + row];
#if !DQN_ACT_F32
  bfx8 w1r[2][K1 / 32];
#endif
  bfx8 w2r[K2 / 64];
  const bfx8* W3 = reinterpret_cast<const bfx8*>(a.w3[inst]);
  bfx8 w1s[2];
  {
    const bfx8* W1 = reinterpret_cast<const bfx8*>(a.w1[inst]);
    const bfx8* W2 = reinterpret_cast<const bfx8*>(a.w2[inst]);
    w1s[0] = W1[tid];
    w1s[1] = W1[tid + 512];
#if !DQN_ACT_F32
#pragma unroll
    for (int j = 0; j < K2 / 64; ++j) w2r[j] = W2[((hi * (K2 / 64) + j) * 4 + nq) * 64 + lane];
#endif
  }
  static_assert((K1 / 32) * 2 * 64 == 2 * 512, "two conv1 fragments per thread");
  // The MFMAs below run transposed (weights as the A operand): lane l then holds 4
  // consecutive output channels 4*(l>>4)..+3 of pixel (l & 15) -> one 8-byte store.
  const int cq = 4 * (lane >> 4);
  const float4 bias1a = *reinterpret_cast<const float4*>(a.b1[inst] + cq);
  const float4 bias1b = *reinterpret_cast<const float4*>(a.b1[inst] + 16 + cq);
  const float4 bias2 = *reinterpret_cast<const float4*>(a.b2[inst] + nq * 16 + cq);
  const float4 bias3 = *reinterpret_cast<const float4*>(a.b3[inst] + nq * 16 + cq);

  // ---------------------------------------------------------------- u8 -> bf16 NHWC in LDS
  if (slot_path) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = tid + 512 * j;
      if (t < nt_in) planes_to_lds(in[j][0], in[j][1], in[j][2], in[j][3], xin + 16 * t);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = tid + 512 * j;
      if (t < nt_in) {   // NHWC word q = pixel 4t+q's 4 channels: transpose to planes then convert
        uint32_t c[4];
#pragma unroll
        for (int ch = 0; ch < 4; ++ch)
          c[ch] = ((in[j][0] >> 8 * ch) & 0xffu) | (((in[j][1] >> 8 * ch) & 0xffu) << 8) |
                  (((in[j][2] >> 8 * ch) & 0xffu) << 16) | (((in[j][3] >> 8 * ch) & 0xffu) << 24);
        planes_to_lds(c[0], c[1], c[2], c[3], xin + 16 * t);
      }
    }
  }
#if DQN_ACT_F32
  // fp32 fragments are 32 B per lane: stored as two 16-byte planes (lane-contiguous), so a wave's
  // b128 reads of one plane are conflict-free (lane-interleaved 32-byte entries put lanes l and l + 8
  // of a 16-lane read phase on the same banks: 2-way conflicts on every weight read of conv1)
  {
    float4* wp = reinterpret_cast<float4*>(wl1);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = tid + 512 * h, f = e >> 6, l = e & 63;
      wp[(2 * f) * 64 + l] = make_float4(w1s[h][0], w1s[h][1], w1s[h][2], w1s[h][3]);
      wp[(2 * f + 1) * 64 + l] = make_float4(w1s[h][4], w1s[h][5], w1s[h][6], w1s[h][7]);
    }
  }
#else
  wl1[tid] = w1s[0];
  wl1[tid + 512] = w1s[1];
#endif
  __syncthreads();
#if !DQN_ACT_F32
#pragma unroll
  for (int ks = 0; ks < K1 / 32; ++ks) {
    w1r[0][ks] = wl1[(ks * 2 + 0) * 64 + lane];
    w1r[1][ks] = wl1[(ks * 2 + 1) * 64 + lane];
  }
#endif
  TRUNK_MARK(1);

  // ---------------------------------------------------------------- conv1 -> act1 (+x1)
  // Every wave computes both n-tiles of its m-tiles (one LDS read per A fragment). Positions
  // are local to the part (row 0 = conv1 row c10; its input row 0 = image row 4 * c10 = in0).
  {
    const float scale = a.scale;
    const int kw = kg >> 2;                               // 0, 2, 4, 6: pixel pair of this lane
    const int np1 = c1n * O1;
    act_t* x1 = a.x1[inst] != nullptr ? a.x1[inst] + (int64_t)b * R1 * N1 + c10 * O1 * N1 : nullptr;
    auto load1 = [&](bfx8* f, int mt) {
      const int p = min(mt * 16 + row, np1 - 1), oy = p / O1, ox = p - oy * O1;   // (tail rows clamped)
      const in_t* base = xin + ((oy * 4) * IW + ox * 4 + kw) * 4;
#pragma unroll
      for (int ks = 0; ks < K1 / 32; ++ks) f[ks] = ld_in8(base + ks * IW * 4);
    };
    const int MT = (np1 + 15) / 16;                       // 25 m-tiles whole, 18 / 15 per part
#if DQN_ACT_F32
    // fp32 build: the frames are exact in bf16, so each fp32 weight fragment (LDS) runs as three bf16
    // fragments (split3_bf16, fused_util.h): 3 bf16 MFMAs per k-step instead of 8 fp32 ones. k-step
    // outer, the wave's m-tiles inner: one split per k-step and n-tile, shared by the m-tiles.
    constexpr int MTW = (R1 / 16 + 7) / 8;
    f32x4 c0[MTW], c1[MTW];
    const in_t* base[MTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      const int p = min((wave + 8 * i) * 16 + row, np1 - 1), oy = p / O1, ox = p - oy * O1;   // (tail clamped)
      base[i] = xin + ((oy * 4) * IW + ox * 4 + kw) * 4;
      c0[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      c1[i] = c0[i];
    }
    // (the fp32 weight fragments, 32 B per lane each, stay in LDS and are read per k-step: held in
    //  registers -- 128 VGPRs -- they pushed the kernel past 256 VGPRs into scratch spills)
    const float4* wp = reinterpret_cast<const float4*>(wl1);
    auto wfrag = [&](int f) {
      const float4 lo = wp[(2 * f) * 64 + lane], hi4 = wp[(2 * f + 1) * 64 + lane];
      bfx8 v;
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi4.x; v[5] = hi4.y; v[6] = hi4.z; v[7] = hi4.w;
      return v;
    };
#pragma unroll
    for (int ks = 0; ks < K1 / 32; ++ks) {              // k = (kh*8 + kw)*4 + c, kh = ks
      b16x8 h0, m0, l0, h1, m1, l1;
      split3_bf16(wfrag(ks * 2 + 0), h0, m0, l0);
      split3_bf16(wfrag(ks * 2 + 1), h1, m1, l1);
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        if (wave + 8 * i >= MT) continue;                 // wave-uniform
        const b16x8 x = *reinterpret_cast<const b16x8*>(base[i] + ks * IW * 4);
        c0[i] = mfma3_bf16(h0, m0, l0, x, c0[i]);
        c1[i] = mfma3_bf16(h1, m1, l1, x, c1[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      const int mt = wave + 8 * i;
      if (mt >= MT) break;                                // wave-uniform
      const int p = mt * 16 + row;
      if (p < np1) {
        const pk4_t v0 = pack4(c0[i] * scale + f4(bias1a)), v1 = pack4(c1[i] * scale + f4(bias1b));
        *reinterpret_cast<pk4_t*>(act1 + p * L1 + cq) = v0;
        *reinterpret_cast<pk4_t*>(act1 + p * L1 + 16 + cq) = v1;
        const int oy = p / O1;
        if (x1 != nullptr && oy >= c1o && oy < c1e) {   // conv2 wgrad input + ReLU mask (owned rows)
          *reinterpret_cast<pk4_t*>(x1 + p * N1 + cq) = v0;
          *reinterpret_cast<pk4_t*>(x1 + p * N1 + 16 + cq) = v1;
        }
      }
    }
#else
#pragma unroll
    for (int i = 0; i < (R1 / 16 + 7) / 8; ++i) {
      const int mt = wave + 8 * i;
      if (mt >= MT) break;                                // wave-uniform
      bfx8 fa[K1 / 32];                                   // (single-buffered: VGPR budget)
      load1(fa, mt);
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
      for (int ks = 0; ks < K1 / 32; ++ks) {              // k = (kh*8 + kw)*4 + c, kh = ks
        c0 = tmfma(w1r[0][ks], fa[ks], c0);
        c1 = tmfma(w1r[1][ks], fa[ks], c1);
      }
      const int p = mt * 16 + row;
      if (p < np1) {
        const pk4_t v0 = pack4(c0 * scale + f4(bias1a)), v1 = pack4(c1 * scale + f4(bias1b));
        *reinterpret_cast<pk4_t*>(act1 + p * L1 + cq) = v0;
        *reinterpret_cast<pk4_t*>(act1 + p * L1 + 16 + cq) = v1;
        const int oy = p / O1;
        if (x1 != nullptr && oy >= c1o && oy < c1e) {   // conv2 wgrad input + ReLU mask (owned rows)
          *reinterpret_cast<pk4_t*>(x1 + p * N1 + cq) = v0;
          *reinterpret_cast<pk4_t*>(x1 + p * N1 + 16 + cq) = v1;
        }
      }
    }
#endif
  }
  // conv3 fragments into the registers conv1 released (latency hidden by conv2)
  bfx8 w3r[K3 / 64];
#if DQN_ACT_F32
  // fp32 build (2x the fragment registers): conv2's weights now, conv3's after conv2's MFMAs
  {
    const bfx8* W2 = reinterpret_cast<const bfx8*>(a.w2[inst]);
#pragma unroll
    for (int j = 0; j < K2 / 64; ++j) w2r[j] = W2[((hi * (K2 / 64) + j) * 4 + nq) * 64 + lane];
  }
#else
#pragma unroll
  for (int j = 0; j < K3 / 64; ++j) w3r[j] = W3[((hi * (K3 / 64) + j) * 4 + nq) * 64 + lane];
#endif
  __syncthreads();
  TRUNK_MARK(2);
  // ---------------------------------------------------------------- conv2 -> act2 (+x2)
  {
    constexpr int KH = K2 / 64;                           // 8 k-steps (taps) per k-half
    constexpr int MTX = (R2 + 15) / 16;                   // 6 m-tiles whole (4 / 3 per part)
    const int np2 = c2n * O2, MT = (np2 + 15) / 16;
    float* red2 = red;                                    // xin is dead: k-half partials after act2
    auto load2 = [&](bfx8* f, int mt) {
      const int p = p2r[mt];
      const bool ok = p >= 0;
      const int oy = ok ? p / O2 : 0, ox = ok ? p - oy * O2 : 0;
      const act_t* base = act1 + ((oy * 2) * O1 + ox * 2) * L1 + kg;
#pragma unroll
      for (int j = 0; j < KH; ++j) {                      // k = (kh*4 + kw)*32 + ci, tap = 8 hi + j
        const int tap = hi * KH + j, kh = tap >> 2, kw = tap & 3;
        f[j] = ok ? *reinterpret_cast<const bfx8*>(base + (kh * O1 + kw) * L1) : tz8();
      }
    };
    f32x4 acc2[MTX];
#if DQN_ACT_F32
    // fp32 build: one operand buffer (the double buffer is 128 VGPRs of fp32 fragments); the LDS
    // latency it hid is small against the 64 fp32 MFMAs of an m-tile
    bfx8 fa1[KH];
#pragma unroll
    for (int mt = 0; mt < MTX; ++mt) {
      if (mt >= MT) break;                                // block-uniform
      load2(fa1, mt);
      acc2[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < KH; ++j) acc2[mt] = tmfma(w2r[j], fa1[j], acc2[mt]);
    }
#pragma unroll
    for (int j = 0; j < K3 / 64; ++j) w3r[j] = W3[((hi * (K3 / 64) + j) * 4 + nq) * 64 + lane];
#else
    bfx8 fa[2][KH];
    load2(fa[0], 0);
#pragma unroll
    for (int mt = 0; mt < MTX; ++mt) {
      if (mt >= MT) break;                                // block-uniform
      if (mt + 1 < MT) load2(fa[(mt + 1) & 1], mt + 1);
      __builtin_amdgcn_sched_barrier(0);
      acc2[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < KH; ++j) acc2[mt] = tmfma(w2r[j], fa[mt & 1][j], acc2[mt]);
      __builtin_amdgcn_sched_barrier(0);
    }
#endif
    if (hi == 1) {
#pragma unroll
      for (int mt = 0; mt < MTX; ++mt)
        if (mt < MT) park(red2, nq * MTX + mt, lane, acc2[mt]);
    }
    __syncthreads();
    if (hi == 0) {
      act_t* x2 = a.x2[inst] != nullptr ? a.x2[inst] + (int64_t)b * R2 * N2 + c20 * O2 * N2 : nullptr;
#pragma unroll
      for (int mt = 0; mt < MTX; ++mt) {
        if (mt >= MT) break;
        const f32x4 c = unpark(red2, nq * MTX + mt, lane, acc2[mt]);
        const int p = p2r[mt];
        if (p >= 0) {
          const pk4_t v = pack4(c + f4(bias2));
          *reinterpret_cast<pk4_t*>(act2 + p * L2 + nq * 16 + cq) = v;
          const int oy = p / O2;
          if (x2 != nullptr && oy >= c2o && oy < c2e) *reinterpret_cast<pk4_t*>(x2 + p * N2 + nq * 16 + cq) = v;
        }
      }
    }
  }
  __syncthreads();
  TRUNK_MARK(6);
  // ---------------------------------------------------------------- conv3 -> x3 (global)
  {
    constexpr int MT = (R3 + 15) / 16;                    // 4 m-tiles whole (2 per part)
    constexpr int KJ = K3 / 64;                           // 9 k-steps per k-half
    const int np3 = c3n * O3, mtn = (np3 + 15) / 16;
    auto load3 = [&](bfx8* f, int mt) {
      const int p = p3r[mt];
      const bool ok = p >= 0;
      const int oy = ok ? p / O3 : 0, ox = ok ? p - oy * O3 : 0;
      const act_t* base = act2 + (oy * O2 + ox) * L2 + kg;
#pragma unroll
      for (int j = 0; j < KJ; ++j) {                      // k = (kh*3 + kw)*64 + ci
        const int ks = hi * KJ + j, tap = ks >> 1, kh = tap / 3, kw = tap - kh * 3;
        f[j] = ok ? *reinterpret_cast<const bfx8*>(base + (kh * O2 + kw) * L2 + (ks & 1) * 32) : tz8();
      }
    };
    f32x4 acc[MT];
#if DQN_ACT_F32
    bfx8 fa1[KJ];                                         // (fp32: single-buffered, as conv2)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      if (mt >= mtn) break;                               // block-uniform
      load3(fa1, mt);
      acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < KJ; ++j) acc[mt] = tmfma(w3r[j], fa1[j], acc[mt]);
    }
#else
    bfx8 fa[2][KJ];
    load3(fa[0], 0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      if (mt >= mtn) break;                               // block-uniform
      if (mt + 1 < mtn) load3(fa[(mt + 1) & 1], mt + 1);
      __builtin_amdgcn_sched_barrier(0);
      acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < KJ; ++j) acc[mt] = tmfma(w3r[j], fa[mt & 1][j], acc[mt]);
      __builtin_amdgcn_sched_barrier(0);
    }
#endif
    TRUNK_MARK(8);
    // k-half exchange: hi waves park fp32 partials in the (dead) input region
    if (hi == 1) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        if (mt < mtn) park(red, nq * MT + mt, lane, acc[mt]);
    }
    __syncthreads();
    TRUNK_MARK(9);
    if (hi == 0) {
      act_t* x3 = a.x3[inst] + (int64_t)b * R3 * N3 + c30 * O3 * N3;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if (mt >= mtn) break;
        const f32x4 v = unpark(red, nq * MT + mt, lane, acc[mt]);
        const int p = p3r[mt];
        if (p >= 0) *reinterpret_cast<pk4_t*>(x3 + p * N3 + nq * 16 + cq) = pack4(v + f4(bias3));
      }
    }
  }
  TRUNK_MARK(10);
#undef TRUNK_MARK
}

}  // namespace dqn

using namespace dqn;

void launch_trunk_fwd(const TrunkArgs& a, int B, int ninst, hipStream_t st) {
  // row split whenever the per-sample grid leaves CUs idle (the learner's 3-4 x 32 samples)
  const int split = B * ninst <= 192 ? 2 : 1;
  hipLaunchKernelGGL(trunk_fwd_kernel, dim3(B, ninst, split), dim3(512), 0, st, a);
}
