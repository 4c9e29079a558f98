// Weight-gradient building blocks shared by the layer kernels (qnet.hip) and the fused
// optimizer launch (optim.hip): the implicit-GEMM A loaders (conv im2col from NHWC u8 / act_t,
// conv1 straight from the replay frame ring, conv dgrad gather, dense rows), the row-major LDS
// staging of a weight-gradient chunk and, for the optimizer's fused "wgrad + update" launch, an
// NTH-thread tile that sums several M-chunks in registers.
//
// Reference: the autodiff weight gradients of the TF conv2d / matmul ops
// (/root/reference/src/network.py:389-409, minimize at :198-202).
#pragma once
#include "common.h"
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

// ================================================================== A loaders
// Each loader is built per (instance, row m) and returns the 8 consecutive
// K-values [k0, k0+8) of row m as a bf16x8 MFMA A-fragment.
// (Round 2 measured branch-free loaders -- clamped addresses + selects -- slower on the flagship
// step, 82.7 -> 88.0 us: the strided dgrad then loads the 3 of 4 invalid taps the early returns
// skip. The early-return loaders stay.)
DQN_DEV bfx8 sel8(bool keep, const bfx8& v) {
  bfx8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = keep ? v[j] : (act_t)0.f;
  return r;
}

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
      uint32_t lo = 0, hi = 0;                 // 8 bytes = pixels (ix, ix+1) x 4 frames
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
  // fetch / conv: frag split at the u8 -> act_t conversion, so a caller can issue several chunks'
  // loads before it first touches their data (the fused weight-gradient tiles)
  struct RawU8 { uint32_t lo, hi; };
  using Raw = typename std::conditional<sizeof(Tin) == 1, RawU8, bfx8>::type;
  DQN_DEV Raw fetch(int k0) const {
    if constexpr (sizeof(Tin) == 1) {
      Raw v{0u, 0u};
      if (!ok) return v;
      const int kh = k0 / (KW * CIN), kw = (k0 - kh * (KW * CIN)) / CIN;
      const int iy = iy0 + kh, ix = ix0 + kw;
      if (iy >= 0 && iy < IH) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(base + (int64_t)iy * IW * CIN);
        if (ix >= 0 && ix < IW) v.lo = row[ix];
        if (ix + 1 >= 0 && ix + 1 < IW) v.hi = row[ix + 1];
      }
      return v;
    } else {
      return frag(k0);
    }
  }
  DQN_DEV static bfx8 conv(const Raw& v) {
    if constexpr (sizeof(Tin) == 1) return u8x8_to_bf(v.lo, v.hi); else return v;
  }
};

// conv1 straight from the replay's frame ring: row m = (b, oy, ox), k = (kh, kw, c)
// with the 4 stacked frames of sample b given by a slot table slots[b][4]
// (replay state_idx rows / actor stacks). Fuses the frame-stack gather into
// the first layer: no materialised [B, 84, 84, 4] copy. A k-group of 8 is the pixel
// pair (ix, ix+1) x 4 frames with ix even (S, pad_l and IW even: Nature VALID and the
// reference's SAME geometry), so the pair is one aligned 16-bit load per frame and is
// either wholly inside or wholly outside the image.
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
  // fetch / conv (see ConvLoader): frame c's pixel pair (ix, ix + 1) as the 16 bits of v[c]
  struct Raw { uint32_t v[4]; };
  DQN_DEV Raw fetch(int k0) const {
    Raw w{{0u, 0u, 0u, 0u}};
    if (!ok) return w;
    const int kh = k0 / (KW * 4), kw = (k0 - kh * (KW * 4)) / 4;
    const int iy = iy0 + kh, ix = ix0 + kw;
    if (iy < 0 || iy >= IH) return w;
    const int off = iy * IW + ix;
    const bool in0 = ix >= 0 && ix < IW, in1 = ix + 1 >= 0 && ix + 1 < IW;
    if (in0 && in1 && ((off & 1) == 0)) {
#pragma unroll
      for (int c = 0; c < 4; ++c) w.v[c] = *reinterpret_cast<const uint16_t*>(fb[c] + off);
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        w.v[c] = (in0 ? (uint32_t)fb[c][off] : 0u) | (in1 ? (uint32_t)fb[c][off + 1] << 8 : 0u);
    }
    return w;
  }
  DQN_DEV static bfx8 conv(const Raw& w) {
    bfx8 r;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      r[c] = (act_t)(float)(w.v[c] & 0xffu);
      r[4 + c] = (act_t)(float)(w.v[c] >> 8);
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
    if (oy * S != ny || ox * S != nx || oy >= OH || ox >= OW) return zero8();   // (invalid taps: no load)
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
  using Raw = bfx8;
  DQN_DEV Raw fetch(int k0) const { return frag(k0); }
  DQN_DEV static bfx8 conv(const Raw& v) { return v; }
};

#if DQN_ACT_F32
// fp32 build: the chunk is staged TRANSPOSED ([k][m] and [n][m], m contiguous) so a lane's 8
// consecutive m values are two ds_read_b128. Rows of MC + 4 floats: a 16-lane read phase (rows
// 0..15 of one k / n group) then starts on 16 distinct 4-bank groups (MC + 8 put rows r and r + 8
// on the same banks: ~36 % bank conflicts in the fp32 grouped wgrad, profiles/r6_pmc_dqn_fp32.md).
constexpr int kF32Pad = 4;
// fused-tile staging swizzle: row kr (a k or n index) of the transposed chunk stores m at column
// m ^ fsw(kr) -- a multiple of 4 below 32, so 4-aligned m groups stay contiguous (float4 reads) and m
// stays inside its 32-aligned half
DQN_DEV int fsw(int kr) { return 4 * ((kr >> 3) & 7); }
template <int MC, int KB, int NB>
struct WgradTile {
  static constexpr int LR = MC + kF32Pad;
  static constexpr size_t lds_bytes = (size_t)(KB + NB) * LR * sizeof(act_t);
};
#else
// 16-bit builds: the chunk is staged ROW-major ([m][k] and [m][n], one ds_write_b128 per
// loaded 8-element fragment) and the MFMA operands (8 m values of one k / n column per lane)
// come from ds_read_b64_tr_b16 transposed reads. Row strides of X + 16 elements put the 8
// rows one 32-lane half reads (32 B each) on disjoint 8-bank ranges (stride / 4 B = 8 * odd
// banks for X = 32, 64, 128): conflict-free reads.
template <int MC, int KB, int NB>
struct WgradTile {
  static constexpr int SA = KB + 16, SZ = NB + 16;
  static constexpr size_t lds_bytes = (size_t)MC * (SA + SZ) * sizeof(act_t);
};
// (operands through lds_tr16 / join_tr transposed reads: common.h)
// Staging swizzle: the 16-byte slots of rows 4..7 mod 8 are swapped in pairs (element offset ^ 8).
// The ds_write_b128 of 8 consecutive rows (8-lane groups, banks mod 32) then hits distinct banks
// (row strides of 24 / 40 / 72 dwords otherwise put rows r and r + 4 on the same banks), and a
// transposed read still covers the same 32-byte half-row: its banks are unchanged.
DQN_DEV int wsw(int row) { return ((row >> 2) & 1) << 3; }
#endif


// ------------------------------------------------------------- fused-launch tile
// One weight-gradient tile (K-range by, N-range bz) over chunk group bx = nper consecutive
// MC-row chunks of M, run by NTH threads: the chunks are summed in registers (chunk c + 1's
// operands are loaded while chunk c's MFMAs run), then ONE set of fp32 atomics per group (plain
// stores when g.atomic == 0: one group covers M). Staging as the 16-bit wgrad_block: row-major
// [m][k] / [m][n] tiles with the slot swizzle, operands through transposed LDS reads. LDS:
// WgradTile<MC, KB, NB>::lds_bytes. Every thread of the block calls it (2 barriers per chunk).
// (fp32 build: the chunk staged transposed, WgradTile's fp32 layout; when NB / 8 < the threads per
//  row -- conv1's 32 columns with 64-row chunks -- only the first NB / 8 thread groups load dZ)
template <class LD, int MC, int KB, int NB, int NTH, int PF = 2>
DQN_DEV void wgrad_tile(const ConvArgs& a, const WgradArgs& g, int bx, int by, int bz, int nper, act_t* lds,
                        int64_t* ph = nullptr) {
  // ph (probe launches): s_memrealtime at tile start | each chunk staged | each chunk's MFMAs done |
  // results issued (thread 0; the caller stamps the drain)
#define WG_MARK(i) if (ph != nullptr && threadIdx.x == 0 && (i) < 7) ph[i] = (int64_t)__builtin_amdgcn_s_memrealtime()
  WG_MARK(0);
  using Tl = WgradTile<MC, KB, NB>;
  constexpr int NW = NTH / 64, TPR = NTH / MC;
  constexpr int GA = KB / 8 / TPR;
  constexpr bool ZPART = NB / 8 < TPR;           // (fewer dZ fragments per row than threads per row)
  constexpr int GZ = ZPART ? 1 : NB / 8 / TPR;
  constexpr int TILES = (KB / 16) * (NB / 16), PERW = TILES / NW, KSTEPS = MC / 32;
  static_assert(NTH % MC == 0 && GA >= 1 && GA * TPR * 8 == KB && (ZPART || GZ * TPR * 8 == NB) &&
                TILES % NW == 0 && NB <= NTH, "fused wgrad tiling");
#if DQN_ACT_F32
  constexpr int LR = Tl::LR;
  act_t* At = lds;                               // [KB][LR]: A transposed, m contiguous
  act_t* Zt = lds + KB * LR;                     // [NB][LR]
#else
  constexpr int SA = Tl::SA, SZ = Tl::SZ;
  act_t* At = lds;                               // [MC][SA]
  act_t* Zt = lds + MC * SA;                     // [MC][SZ]
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k_lo = by * KB, n_lo = bz * NB;
  const int nchunks = (a.M + MC - 1) / MC, c0 = bx * nper;
  const int nch = min(nchunks, c0 + nper) - c0;
  const bool dob = g.db != nullptr && by == 0;
  // thread -> (row r, piece p): the TPR threads of a row adjacent, so a wave's 16-byte loads cover
  // whole 64-byte runs of 16 rows (row-major NHWC / dZ rows) instead of 16 bytes of 64 rows each: 4x
  // fewer cache-line requests through the CU's address unit per load instruction (fused launch
  // 22.7 -> 21.3 us, bf16). fp32: the transposed staging then swizzles m by k (fsw below).
  // 16-bit builds: the 4 rows of one 16-lane ds_write_b128 pass are rows {0,2,4,6} / {1,3,5,7} (+8) of
  // the wave's 16: at 160-byte row strides rows 0 and 3 share banks (2-way conflicts, 22 % of the
  // launch's LDS cycles, profiles/r6_pmc_final_dqn.md); rows 0, 2, 4, 6 start on disjoint 16-bank windows
#if DQN_ACT_F32
  const int r = tid / TPR, p = tid % TPR;
#else
  static_assert(TPR != 4 || MC % 16 == 0, "row interleave: 16-row waves");
  const int q16 = (tid & 63) / TPR, pass = q16 >> 2;
  const int r = TPR == 4 ? (tid >> 6) * 16 + (pass >> 1) * 8 + (q16 & 3) * 2 + (pass & 1) : tid / TPR;
  const int p = tid % TPR;
#endif
  // two chunk slots in registers: both chunks' loads are issued before either is converted / staged
  // (the u8 conv1 loaders convert inside frag(), and the frame loader's addresses depend on a
  // slot-table load: chunk by chunk, the tile paid ~4 dependent round trips for its 2 chunks)
  using Raw = typename LD::Raw;
  Raw ra0[GA], ra1[GA], ra2[GA];
  bfx8 vz0[GZ], vz1[GZ], vz2[GZ];
  auto fetch_z = [&](int c, bfx8* vz) {
    const int m = (c0 + c) * MC + r;
    const bool mok = m < a.M;
    const act_t* dz = reinterpret_cast<const act_t*>(g.dz) + (int64_t)(mok ? m : 0) * g.ldz + n_lo;
#pragma unroll
    for (int i = 0; i < GZ; ++i) {
      const int c8 = (p + i * TPR) * 8;
      const bool zok = (!ZPART || c8 < NB) && n_lo + c8 < g.N;
      const int cz = (zok ? n_lo + c8 : 0) - n_lo;                  // masked groups read column 0
      vz[i] = sel8(mok && zok, *reinterpret_cast<const bfx8*>(dz + cz));
    }
  };
  auto fetch_a = [&](const LD& ld, Raw* ra) {
#pragma unroll
    for (int i = 0; i < GA; ++i) ra[i] = ld.fetch(min(k_lo + (p + i * TPR) * 8, a.K - 8));   // (clamped)
  };
  auto stage = [&](int c, const Raw* ra, const bfx8* vz) {
    if (c > 0) __syncthreads();                  // the previous chunk's LDS reads are done
#if DQN_ACT_F32
    // (row c8 + j of the transposed tile holds m = r at column r ^ fsw(c8): the 8 piece-lanes of a
    //  row m write 8 k rows 8 * LR words apart -- 2 bank groups -- at distinct columns)
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int c8 = (p + i * TPR) * 8, k0 = k_lo + c8;
      const bfx8 v = sel8(k0 < a.K, LD::conv(ra[i]));
#pragma unroll
      for (int j = 0; j < 8; ++j) At[(c8 + j) * LR + (r ^ fsw(c8))] = v[j];
    }
#pragma unroll
    for (int i = 0; i < GZ; ++i) {
      const int c8 = (p + i * TPR) * 8;
      if (!ZPART || c8 < NB) {
#pragma unroll
        for (int j = 0; j < 8; ++j) Zt[(c8 + j) * LR + (r ^ fsw(c8))] = vz[i][j];
      }
    }
#else
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int k0 = k_lo + (p + i * TPR) * 8;
      *reinterpret_cast<bfx8*>(At + r * SA + (((p + i * TPR) * 8) ^ wsw(r))) = sel8(k0 < a.K, LD::conv(ra[i]));
    }
#pragma unroll
    for (int i = 0; i < GZ; ++i) *reinterpret_cast<bfx8*>(Zt + r * SZ + (((p + i * TPR) * 8) ^ wsw(r))) = vz[i];
#endif
    __syncthreads();
  };
  const int gq = lane >> 4, rq = (lane >> 2) & 3, cp = 4 * (lane & 3);
  constexpr int NTt = NB / 16;
  f32x4 acc[PERW];
#pragma unroll
  for (int i = 0; i < PERW; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbs = 0.f;
  auto compute = [&]() {
#if DQN_ACT_F32
    if (dob && tid < NB) {
      const act_t* zr = Zt + tid * LR;
      const int zs = fsw(tid);
#pragma unroll 8
      for (int q = 0; q < MC; ++q) dbs += (float)zr[q ^ zs];        // (m order)
    }
    const int kg = 8 * (lane >> 4), row = lane & 15;
    // 8 consecutive m of one k / n row: two 4-float groups, each contiguous under the swizzle
    auto rd8 = [&](const act_t* base, int kr, int m0) {
      const act_t* rp = base + kr * LR;
      const int sw = fsw(kr);
      const float4 lo = *reinterpret_cast<const float4*>(rp + (m0 ^ sw));
      const float4 hi = *reinterpret_cast<const float4*>(rp + ((m0 + 4) ^ sw));
      bfx8 v;
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      return v;
    };
#pragma unroll
    for (int i = 0; i < PERW; ++i) {
      const int tile = wave + NW * i;
      const int kt = tile / NTt, nt = tile - kt * NTt;
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        const bfx8 af = rd8(At, kt * 16 + row, 32 * s + kg);
        const bfx8 bf = rd8(Zt, nt * 16 + row, 32 * s + kg);
        acc[i] = mfma16(af, bf, acc[i]);
      }
    }
#else
    if (dob && tid < NB) {
#pragma unroll 8
      for (int q = 0; q < MC; ++q) dbs += (float)Zt[q * SZ + (tid ^ wsw(q))];
    }
#pragma unroll
    for (int i = 0; i < PERW; ++i) {
      const int tile = wave + NW * i;
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
#endif
  };
  {
    // loaders of the first PF chunks first (the frame loader's slot-table loads), then the dZ rows, then
    // the A fragments: waiting for chunk 0's data leaves the later chunks' loads in flight
    // (PF = 1: the A/B baseline -- chunk c + 1's loads issued after chunk c is staged; PF = 3: a
    //  three-chunk tile waits on ONE memory round trip instead of two)
    const LD l0(a, 0, c0 * MC + r);
    fetch_z(0, vz0);
    if (PF >= 2 && nch > 1) fetch_z(1, vz1);
    if (PF >= 3 && nch > 2) fetch_z(2, vz2);
    if constexpr (PF >= 2) {
      const LD l1(a, 0, (c0 + 1) * MC + r);
      fetch_a(l0, ra0);
      if (nch > 1) fetch_a(l1, ra1);
      if constexpr (PF >= 3) {
        const LD l2(a, 0, (c0 + 2) * MC + r);
        if (nch > 2) fetch_a(l2, ra2);
      }
    } else {
      fetch_a(l0, ra0);
    }
  }
  // chunk j's data lives in slot j % PF (PF = 1: slots j & 1, refilled one chunk ahead); a slot is
  // refilled PF chunks ahead right after it is staged
  auto refill = [&](int j, Raw* ra, bfx8* vz) {
    if (j < nch) {
      const LD l(a, 0, (c0 + j) * MC + r);
      fetch_z(j, vz);
      fetch_a(l, ra);
    }
  };
  if constexpr (PF >= 3) {
    for (int c = 0; c < nch; c += 3) {
      stage(c, ra0, vz0);
      WG_MARK(1 + 2 * c);
      refill(c + 3, ra0, vz0);
      compute();
      WG_MARK(2 + 2 * c);
      if (c + 1 < nch) {
        stage(c + 1, ra1, vz1);
        WG_MARK(3 + 2 * c);
        refill(c + 4, ra1, vz1);
        compute();
        WG_MARK(4 + 2 * c);
      }
      if (c + 2 < nch) {
        stage(c + 2, ra2, vz2);
        refill(c + 5, ra2, vz2);
        compute();
      }
    }
  } else {
    for (int c = 0; c < nch; c += 2) {
      stage(c, ra0, vz0);
      WG_MARK(1 + 2 * c);
      if constexpr (PF >= 2) refill(c + 2, ra0, vz0); else refill(c + 1, ra1, vz1);
      compute();
      WG_MARK(2 + 2 * c);
      if (c + 1 < nch) {
        stage(c + 1, ra1, vz1);
        WG_MARK(3 + 2 * c);
        if constexpr (PF >= 2) refill(c + 3, ra1, vz1); else refill(c + 2, ra0, vz0);
        compute();
        WG_MARK(4 + 2 * c);
      }
    }
  }
  const bool atomic = g.atomic != 0;
  if (dob && tid < NB) {
    const int nn = n_lo + tid;
    if (nn < g.N) {
      float* pdb = nn < g.nsplit ? g.db + nn : g.db2 + (nn - g.nsplit);
      const float s = dbs * kInvLossScale;
      // (plain results are written through to memory: a consumer in the same launch reads them)
      if (atomic) atomicAdd(pdb, s); else __hip_atomic_store(pdb, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#pragma unroll
  for (int i = 0; i < PERW; ++i) {
    const int tile = wave + NW * i;
    const int kt = tile / NTt, nt = tile - kt * NTt;
    const int n = n_lo + nt * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k_lo + kt * 16 + 4 * (lane >> 4) + q;
      if (k < a.K && n < g.N) {
        float* o = n < g.nsplit ? g.dw + (int64_t)k * g.nsplit + n
                                : g.dw2 + (int64_t)k * (g.N - g.nsplit) + (n - g.nsplit);
        const float v = acc[i][q] * (g.scale * kInvLossScale);
        if (atomic) atomicAdd(o, v); else __hip_atomic_store(o, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (ph != nullptr && threadIdx.x == 0) ph[6] = (int64_t)__builtin_amdgcn_s_memrealtime();
#undef WG_MARK
}

// The fused launch's tiles per member kind (NTH = 512 threads, 128-row chunks -- 64 in the fp32
// build, whose staging is twice the bytes --, <= 40 KB of LDS: the optimizer blocks beside them keep
// 4 blocks / CU). Returns false for a kind the fused launch does not run.
constexpr int kFusedWgMC = DQN_ACT_F32 ? 64 : 128;
#ifndef DQN_WG_PREFETCH
#define DQN_WG_PREFETCH 2
#endif
constexpr int kWgPrefetch = DQN_WG_PREFETCH;
DQN_DEV_HOST_INLINE bool fused_wgrad_tiles(int kind, int& MC, int& KB, int& NB) {
  switch (kind) {
    case L_NAT_CONV1_FWD: case L_NAT_CONV1_FRAMES: MC = kFusedWgMC; KB = 64; NB = 32; return true;
    case L_NAT_CONV2_FWD: case L_NAT_CONV3_FWD: MC = kFusedWgMC; KB = 64; NB = 64; return true;
    case L_HEAD_WGRAD: MC = 64; KB = 64; NB = 64; return true;
    default: return false;
  }
}

using FwC1 = ConvLoader<uint8_t, 4, 8, 8, 4>;
using FwC2 = ConvLoader<act_t, 32, 4, 4, 2>;
using FwC3 = ConvLoader<act_t, 64, 3, 3, 1>;
using FwF1 = FrameLoader<8, 8, 4>;

// Block b of the fused launch's weight-gradient range: find its member (block ranges in member
// order, longest first) and run the member's tile. G lives in device memory (built once per
// workspace by the host planner, wgrad_fused_plan). Returns member * 256 + K-range.
template <int NTH>
DQN_DEV int fused_wgrad_block(const WgradGroup& G, int b, act_t* lds, int64_t* ph = nullptr) {
  int i = 0;
  while (i < G.n - 1 && b >= G.nblk[i]) { b -= G.nblk[i]; ++i; }
  const int gx = G.gx[i], gy = G.gy[i];
  const int bx = b % gx, rr = b / gx, by = rr % gy, bz = rr / gy;
  const ConvArgs& a = G.a[i];
  const WgradArgs& g = G.g[i];
// (two chunks' loads up front: the fused launch 23.5 -> 23.0 us alone, scripts/probe_split.py,
//  gpurun_out/r5ab; the one-ahead order stays as wgrad_tile<..., 1>. kWgPrefetch chunks up front:
//  DQN_WG_PREFETCH at build time, default 2)
#define WG_TILE(LD, MC_, KB_, NB_) wgrad_tile<LD, MC_, KB_, NB_, NTH, kWgPrefetch>(a, g, bx, by, bz, g.mloop, lds, ph)
  switch (G.kind[i]) {
    case L_NAT_CONV1_FWD: WG_TILE(FwC1, kFusedWgMC, 64, 32); break;
    case L_NAT_CONV1_FRAMES: WG_TILE(FwF1, kFusedWgMC, 64, 32); break;
    case L_NAT_CONV2_FWD: WG_TILE(FwC2, kFusedWgMC, 64, 64); break;
    case L_NAT_CONV3_FWD: WG_TILE(FwC3, kFusedWgMC, 64, 64); break;
    case L_HEAD_WGRAD: WG_TILE(DenseLoader, 64, 64, 64); break;
    default: break;
  }
#undef WG_TILE
  return i * 256 + by;                           // (member, K-range) of the tile
}

}  // namespace dqn
