// Fused multi-tensor optimizer + weight packing kernel (optim_pack_kernel) and its launch
// descriptor. Included by optim.hip (launchers) and by the optim_ops_*.hip translation units,
// which instantiate it per optimizer (DQN_OPTIM_DEFINE_OPS) so the build compiles them in parallel.
//
// Reference: tf.train.{GradientDescent,Momentum,RMSProp,Adam,Adagrad,Adadelta,Ftrl}
// Optimizer.minimize() colocated with the variables on the parameter server
// (/root/reference/src/network.py:159-203) -- one ApplyX op per variable plus the separate L2
// term in the loss (network.py:151-152,311,407).
#pragma once
#include <stdlib.h>
#include <type_traits>
#include "common.h"
#include "sample_dev.h"
#include "sumtree_dev.h"
#include "wgrad_dev.h"
#include "xgmi_dev.h"
#include "../include/dqn_kernels.h"

namespace dqn {

struct OptHP {
  float lr, reg, grad_scale;
  float momentum, rho, rms_mom, rms_eps, b1, b2, adam_eps, ad_rho, ad_eps;
  int reg_end;
  // noisy nets, factorised target fc (UpdJob.eff bit 1): the target's packed fc weights hold mu
  // fragments and this buffer (the packed layout) its sigma fragments, written only when they change
  // (a sync step, or a mix-only call on the target); the target forward mixes the noise in itself
  void* tsg;
  // 1: update only, no packed fragments / fp32 copies written (the async-PS server, which never
  // runs the network: it re-packs once when serving ends)
  int no_pack;
  // probe launches only (DQN_OPT_PROF=1, nullptr otherwise): [0, 16) s_memtime phase stamps of
  // blocks 0 and 1, then per block [start, ready, end] s_memrealtime (100 MHz) for blocks < kTlBlocks
  // (ready: a dependent job's wait is over / the sampler's draw is done)
  int64_t* prof;
};
constexpr int kProfPhases = 16, kTlBlocks = 4096, kTilePhBlocks = 512;
// (two fc jobs per block of a WG launch would halve its 785 fc blocks -- they reach the CUs over
//  ~4 us, behind the weight-gradient tiles -- but a second inlined job raised the launch from 97
//  to 168 VGPRs, 3 waves / SIMD; measured round 4, not kept)   // (+ [8] tile phases per wgrad block)

// Contraction is pinned off in the update math so every kernel that inlines it
// (optim_kernel's float4 loop, optim_pack_kernel's tiles) rounds identically:
// with fp-contract=fast the backend fuses differently per call site.
DQN_DEV float opt_grad(float g, float w, bool reg, const OptHP& h) {
#pragma clang fp contract(off)
  float x = g * h.grad_scale;
  if (reg) x += h.reg * w;
  return x;
}

template <int OP>
DQN_DEV void update_one(float& w, float g, float& s0, float& s1, const OptHP& h, float lr_t) {
#pragma clang fp contract(off)
  if constexpr (OP == 0) {            // sgd
    w -= h.lr * g;
  } else if constexpr (OP == 1) {     // momentum (non-Nesterov)
    s0 = h.momentum * s0 + g;
    w -= h.lr * s0;
  } else if constexpr (OP == 2) {     // rmsprop: ms (init 1), mom
    s0 = h.rho * s0 + (1.f - h.rho) * g * g;
    s1 = h.rms_mom * s1 + h.lr * g / sqrtf(s0 + h.rms_eps);
    w -= s1;
  } else if constexpr (OP == 7) {     // rmsprop with momentum 0 (the TF / reference default):
    s0 = h.rho * s0 + (1.f - h.rho) * g * g;   // mom = 0 * mom + u == u exactly, so mom is
    s1 = h.lr * g / sqrtf(s0 + h.rms_eps);     // written (checkpoint slot) but never read
    w -= s1;
  } else if constexpr (OP == 3) {     // adam (TF epsilon-hat form)
    s0 = h.b1 * s0 + (1.f - h.b1) * g;
    s1 = h.b2 * s1 + (1.f - h.b2) * g * g;
    w -= lr_t * s0 / (sqrtf(s1) + h.adam_eps);
  } else if constexpr (OP == 4) {     // adagrad (accumulator init 0.1)
    s0 += g * g;
    w -= h.lr * g / sqrtf(s0);
  } else if constexpr (OP == 5) {     // adadelta
    s0 = h.ad_rho * s0 + (1.f - h.ad_rho) * g * g;
    const float upd = sqrtf(s1 + h.ad_eps) / sqrtf(s0 + h.ad_eps) * g;
    s1 = h.ad_rho * s1 + (1.f - h.ad_rho) * upd * upd;
    w -= h.lr * upd;
  } else {                            // ftrl (lr_power -0.5, l1 = l2 = 0)
    const float na = s0 + g * g;
    s1 += g - (sqrtf(na) - sqrtf(s0)) / h.lr * w;
    const float quad = sqrtf(na) / h.lr;
    w = fabsf(s1) > 0.f ? -s1 / quad : 0.f;
    s0 = na;
  }
}

// ------------------------------------------------------------- update + pack
// The optimizer step fused with the executor's weight packing: a 512-thread workgroup
// owns a 32 (k) x 64 (n) tile of a weight matrix (TF layout [K][N]), each thread 4
// consecutive n of one row (one float4 per operand: few VGPRs, high occupancy). It
// updates the tile in registers, writes fp32 weights + slots back, and emits the tile's
// bf16 MFMA fragments straight away:
//   * forward fragments ([K/32][N/16][64][8]: 8 consecutive k per lane): a wave owns an
//     8 (k) x 32 (n) sub-tile with lane = 8 * col-group + row, so the 4 lanes of a quad hold
//     4 consecutive rows x the same 4 columns; one 4x4 DPP transpose per quad leaves each
//     lane 4 consecutive k of one column = half of a fragment slot, stored directly (no LDS
//     round trip, no barrier; the LDS transpose it replaces ran at ~40% bank conflicts);
//   * dgrad fragments (dense transpose, or conv (tap, co) x ci) directly from the
//     thread's registers: its 4 consecutive K' ARE 4 consecutive n of one row (half
//     of one lane's 8-value slot).
// Elementwise items (biases, ...) carry an optional fp32 copy into the packed
// buffer (the concatenated fc bias). Same ticket as optim_kernel; the hard target
// sync writes the target's fp32 master and packed fragments under the predicate.
typedef __attribute__((ext_vector_type(4))) act_t bfx4;

constexpr int kTicketSubs = 16, kTicketStride = 32;    // sharded arrival counters: int32 words, 128 B apart
constexpr int kPackThreads = 512;
// ticket[kSlotFlag] != 0: momentum-0 RMSProp also stores its `mom` slot this step. That slot
// (mom = 0 * mom + update) is never read by the update, only saved under its TF name, so the
// hot path skips its 4 bytes / parameter and the checkpoint manager raises the flag for the
// step before a save (optim.py Optimizer.request_slots).
constexpr int kSlotFlag = 1;
// ticket[kErrFlag] != 0: an optim_pack launch's end-of-launch wait gave up (lost arrival; never
// expected -- the learner's periodic check reads it)
constexpr int kErrFlag = 2;

// Fused fc weight gradient (FcFuse): a 32 (k) x 64 (n) update tile's dW = X^T dH over M rows,
// 32-row chunks staged ROW-major in LDS (strides + 16 elements: conflict-free transposed reads,
// as the grouped wgrad), wave w owning the 16 x 16 sub-tile (k: w >> 2, n: w & 3) as dW^T =
// dH^T X on one v_mfma_f32_16x16x32 per chunk (lane: one k, 4 consecutive n), then through
// an fp32 LDS tile into the update's own thread map (row r, 4 consecutive n).
// (fp32 build: the same 32-row chunks staged row-major, each MFMA operand lane reading its 8 rows of
//  one column with strided 4-byte reads: row strides of 34 / 66 floats put a read's 4 lane groups
//  (rows 8 g + j) 16 banks apart -- conflict-free)
constexpr int kFcSX = DQN_ACT_F32 ? 32 + 2 : 32 + 16, kFcSH = DQN_ACT_F32 ? 64 + 2 : 64 + 16, kFcRS = 64 + 4;
constexpr int kFcStage = 32 * (kFcSX + kFcSH) * (int)sizeof(act_t);
constexpr int kFcLds = kFcStage > 32 * kFcRS * 4 ? kFcStage : 32 * kFcRS * 4;   // staging, fp32 dW tile, 4 x 512 fp32
static_assert(4 * 512 * 4 <= kFcLds, "fc LDS plan");

// dynamic LDS of a WG launch: the largest fused weight-gradient tile and the FcFuse staging
constexpr int kFusedWgLds = (int)WgradTile<kFusedWgMC, 64, 64>::lds_bytes > kFcLds ? (int)WgradTile<kFusedWgMC, 64, 64>::lds_bytes
                                                                                    : kFcLds;
static_assert(kFusedWgLds <= 40 * 1024, "WG launch LDS: 4 blocks / CU");
static_assert((int)WgradTile<64, 64, 64>::lds_bytes <= kFusedWgLds && (int)WgradTile<kFusedWgMC, 64, 32>::lds_bytes <= kFusedWgLds,
              "every fused tile fits");

struct UpdJob {
  int kind;                      // 0 = tile, 1 = elementwise chunk
  int src_off, K, N, k0, n0;     // tile: tensor offset / shape / origin; elem: offset, count (K)
  int fwd_off, fwd_N16, fwd_nt_off, fwd_ks_off;   // forward fragments (elem: fp32 copy offset or -1)
  int dg_mode, dg_off, dg_N16, dg_nt_off, dg_ks_off, dg_cin;   // dgrad: 0 none, 1 conv, 2 dense
  // noisy nets (factorised Gaussian): the sigma tensor is updated in the same thread as mu
  // and the packed / eff values are mu + sigma * f(noise[ein + k]) f(noise[eout + n])
  // (ein < 0: f = 1, biases; elem chunks: eout already offset to the chunk start)
  int sig_off, ein_off, eout_off;
  int eff;                       // bit 0: also store the effective fp32 value at eff[src index];
                                 // bit 1: factorised target tile (OptHP.tsg), no per-step target mix
  // fc weight tile / fc bias chunk whose gradient the launch forms from FcFuse rows: the
  // tensor's first column in dH (-1: read the flat gradient)
  int fc_col;
  // WG launches: the gradient is produced by weight-gradient member `dep` of this launch (-1:
  // final at launch start); the block waits for that member's done counter first
  int dep;
  // gradient = sum of part_n partial slices (the grouped conv wgrad's deterministic chunk-group
  // sums, qnet.hip): element d of the tensor at part[part_off + p * part_stride + d], p ascending
  int part_off, part_n, part_stride;
};

DQN_DEV float fnz(float x) { return copysignf(sqrtf(fabsf(x)), x); }

template <int OP>
DQN_DEV void upd4(float* w, const float* g, float* a, float* b, int64_t k0flat, int reg_end, const OptHP& h,
                  float lr_t, const bool* ok) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!ok[j]) continue;
    update_one<OP>(w[j], opt_grad(g[j], w[j], k0flat + j < reg_end, h), a[j], b[j], h, lr_t);
  }
}

// MODE bits: kModeNoisy (noisy jobs in the work list), kModeTmix (+ the target's mix + pack),
// kModePer (the sampler block runs the prioritized sum-tree path). Paths a mode excludes are
// not instantiated: their registers would cost the plain nets occupancy. Mode 0: 5 waves / SIMD
// (at 8 it spilled 120 B / lane to scratch: 16.1 -> 12.8 us alone, scripts/probe_optim.py,
// gpurun_out/r5ae); the fc-only mode stays at 8 (its 52 B spill measured 2.5 % faster than 6 waves).
// kModeFc: some jobs form their gradient from FcFuse rows (16-bit builds).
// kModeWg (16-bit builds): the launch also computes the grouped weight gradients. Grid: [the lead
// block: sampler + closer] [the WgradGroup's tiles (device memory, wgrad_dev.h)] [the jobs whose
// gradient is final at launch start: the fc layers, from FcFuse rows]. Each tile, once its fp32
// atomics have completed, adds to its (member, K-range) counter (and, K-range 0, the member's bias
// counter); the tile whose add completes a count acquires (agent scope) and runs the optimizer
// jobs of those rows itself (WgradGroup dep ranges of the job table, past the block-assigned
// jobs). Nothing waits while holding a CU slot, except the sampler block: it writes the next
// minibatch's frame-slot tables only after the member reading the current ones (conv1 from the
// frame ring) is done -- the lowest block id, so every producer it waits for is already resident.
// LDS: one dynamic buffer (<= 40 KB: 4 blocks / CU, as the plain update).
// kModeWg: the weight-gradient tiles beside the update items need ~165 VGPRs: 3 waves / SIMD (at the
// 8-blocks-per-CU bound of the plain update they spilled to scratch: 4.5x slower tiles, measured).
// kModeFew: a launch of few work blocks (the second launch of a split update): 4 waves / SIMD
// (128 VGPRs: no spills in the item body, occupancy is moot) and a returning arrival ticket per
// block -- the last block to arrive closes the launch, nobody polls.
// kModeDp (with kModeWg, data parallelism): the dependent jobs sum their gradient slots over every rank
// inside the launch (DpExchange, dqn_kernels.h): no all-reduce launch between backward and update.
constexpr int kModeNoisy = 1, kModeTmix = 2, kModePer = 4, kModeFc = 8, kModeWg = 16, kModeFew = 32, kModeDp = 64;

// A static LDS buffer only in the instantiations that use one (ALLOC; TAG keeps two buffers of one
// size apart): the WG launches must carry no static LDS (see smem below).
template <bool ALLOC, size_t N, int TAG>
struct OptShm {
  DQN_DEV static unsigned char* get() {
    __shared__ __attribute__((aligned(16))) unsigned char b[N];
    return b;
  }
};
template <size_t N, int TAG>
struct OptShm<false, N, TAG> {
  DQN_DEV static unsigned char* get() { return nullptr; }
};
template <int OP, int MODE>
__global__ void __launch_bounds__(kPackThreads, (MODE & kModeDp) ? 4 : (MODE & kModeWg) ? (kWgPrefetch >= 3 ? 4 : 3) : (MODE & kModeFew) ? 4 : (MODE & ~kModeFc) == 0 ? (DQN_ACT_F32 ? 4 : (MODE & kModeFc) ? 8 : 5) : (((MODE & (kModeTmix | kModeNoisy)) || !(OP == -1 || OP == 0 || OP == 3 || OP == 7)) ? 1 : 6))
optim_pack_kernel(float* __restrict__ W, const float* __restrict__ G, float* __restrict__ S0, float* __restrict__ S1,
                  float* __restrict__ beta_pow, int64_t* __restrict__ step, int32_t* __restrict__ ticket, OptHP h,
                  const UpdJob* __restrict__ jobs, int njobs, act_t* __restrict__ packed, float* __restrict__ tgt,
                  act_t* __restrict__ tgt_packed, int tfreq, const float* __restrict__ noise,
                  float* __restrict__ eff, const float* __restrict__ gnoise, float* __restrict__ noise_dst,
                  int noise_n, TrunkSample smp, PerStep per, const float* __restrict__ tnoise,
                  float* __restrict__ teff, act_t* __restrict__ tpk, int64_t* __restrict__ noise_rng, FcFuse ff,
                  const float* __restrict__ part, const WgradGroup* __restrict__ wg, int wg_blocks, DpLaunch dp) {
  // OP < 0: no optimizer update, only (noisy mix +) pack of W into `packed` / `eff`.
  // gnoise (noisy nets): the sample the forward used; sigma's gradient is then derived here,
  // dL/dsigma = dL/dW_eff * f(gnoise_in) f(gnoise_out) from the mu-slot gradient (identical
  // noise on every DP rank makes that exact for the all-reduced sum), instead of being read.
  // noise_dst: the grid's last block copies noise[0, noise_n) there (next sample -> current).
  // smp.size != nullptr: the grid's extra block (block 0) draws the NEXT step's uniform minibatch
  // (sample_dev.h) while the others update: the replay is quiet during this launch, and
  // the sampler leaves the next step's critical path.
  // tnoise (noisy nets, update calls): also mix + pack the TARGET under its next noise
  // sample into teff / tpk (the target's eff / packed buffers): no separate target mix launch.
  constexpr bool UPD = OP >= 0;
  constexpr bool TMIX = (MODE & kModeTmix) != 0, NZOK = (MODE & kModeNoisy) != 0, PEROK = (MODE & kModePer) != 0;
  constexpr bool FC = (MODE & kModeFc) != 0 && OP >= 0;
  constexpr bool WG = (MODE & kModeWg) != 0 && OP >= 0;
  constexpr bool FEW = (MODE & kModeFew) != 0 && OP >= 0;
  constexpr bool DP = WG && (MODE & kModeDp) != 0;
  // (TMIX is a template flag: the target-mix registers cost the plain nets occupancy)
  const bool tmix = TMIX && UPD && tnoise != nullptr && tgt != nullptr;
  // LDS: the sampler block's scratch (the update items exchange through DPP); WG launches carve
  // everything (weight-gradient staging, FcFuse staging) from the dynamic buffer instead
  constexpr size_t kSmpLds = sizeof(SampleLds) > sizeof(SumtreeLds) ? sizeof(SampleLds) : sizeof(SumtreeLds);
  extern __shared__ __attribute__((aligned(16))) unsigned char opt_dyn[];
  // (WG: no static LDS at all -- with even a few static bytes the 40 KB dynamic buffer became
  //  41.5 KB per block, 3 blocks per CU instead of 4, and the fc jobs queued behind the tiles;
  //  the lead block's sampler uses the dynamic buffer, which no tile of it needs)
  unsigned char* smem = WG ? opt_dyn : OptShm<!WG, kSmpLds, 0>::get();
  int64_t* tl = (h.prof != nullptr && threadIdx.x == 0 && blockIdx.x < kTlBlocks) ? h.prof + kProfPhases + 3 * blockIdx.x
                                                                                    : nullptr;
  if (tl) { tl[0] = (int64_t)__builtin_amdgcn_s_memrealtime(); tl[1] = 0; tl[2] = 0; }
  int32_t* cnt = ticket + kTicketStride;        // end-of-launch arrival counters (see the closing step)
  // ---- a weight-gradient tile, counted on its (member, K-range) when done (the last tile of a
  //      range ran that range's jobs serially: ~4 of them, 8-15 us each, measured; the jobs
  //      now wait in blocks of their own at the end of the grid and run in parallel)
  auto wg_tile_run = [&](int b) {
    int64_t* ph = (h.prof != nullptr && b < kTilePhBlocks) ? h.prof + kProfPhases + 3 * kTlBlocks + 8 * b : nullptr;
    const int mb = fused_wgrad_block<kPackThreads>(*wg, b, reinterpret_cast<act_t*>(opt_dyn), ph);
    const int m = mb >> 8, by = mb & 255;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's atomics / write-through stores done
    if (ph != nullptr && threadIdx.x == 0) ph[7] = (int64_t)__builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (threadIdx.x == 0) {
      if (tl) { tl[1] = m; tl[2] = (int64_t)__builtin_amdgcn_s_memrealtime(); }
      // count the tile on its (member, K-range) and -- K-range 0 -- the member's bias range; the
      // jobs of a range wait for its count in their own blocks (end of the grid), in parallel
      __hip_atomic_fetch_add(wg->done + kTicketStride * (kMaxWgradMembers + m * kWgSlots + by), 1,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (by == 0)
        __hip_atomic_fetch_add(wg->done + kTicketStride * (kMaxWgradMembers + m * kWgSlots + kWgSlots - 1), 1,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // (member-level count: the sampler waits for the frame-slot reader)
      __hip_atomic_fetch_add(wg->done + kTicketStride * m, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  if constexpr (WG && !FEW) {
    // tiles first, ahead of the launch-start reads below (the step / rng / slot-flag words): every
    // scalar load there is waited for in order (s_waitcnt lgkmcnt(0)), ~3 us of dependent round
    // trips before a tile issued its first operand load (probe_split timeline: tile blocks ran
    // 9.0 us of which 5.6 us inside the tile)
    // (block roles of the WG grid: the lead block, the tiles [1, 1 + wg_blocks), then the job blocks;
    //  round 5 measured the fc jobs interleaved with the tiles: 14.8k -> 13.6k SGD steps/s, removed)
    const int tb = (int)blockIdx.x - 1;
    if (tb >= 0 && tb < wg_blocks) {
      wg_tile_run(tb);
      __syncthreads();
      if (threadIdx.x == 0)                     // the end-of-launch arrival (see the closing step)
        __hip_atomic_fetch_add(cnt + kTicketStride * (blockIdx.x & (kTicketSubs - 1)), 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
  // block 0 leads (the sampler when the launch draws the next minibatch; always in WG launches,
  // whose block 0 then only closes the launch)
  const bool smp_on = smp.size != nullptr || per.sum != nullptr;
  const bool extra = smp_on || WG;
  const int wg0 = WG ? wg_blocks : 0;
  // the sampler is block 0: dispatched first, so its serial chain overlaps the whole update
  const bool sampler = smp_on && blockIdx.x == 0;
  const int nwork = (int)gridDim.x - (extra ? 1 : 0) - wg0;
  // block roles after the lead block. WG: the weight-gradient tiles [0, wg_blocks) (they returned at
  // the top of the kernel), then the job table, one job per block (DP: the dependent jobs
  // [dp.first, dp.first + dp.n) run in dp.blocks blocks)
  const int wid = WG ? ((int)blockIdx.x - 1 < wg_blocks ? -1 : (int)blockIdx.x - 1 - wg_blocks)
                     : (int)blockIdx.x - (extra ? 1 : 0) - wg0;      // work index of an update block
  float lr_t = h.lr;
  // the step words, read once at launch start: block 0's closing step writes their successors from
  // these registers (a load -> store round trip there sat on the launch's critical path); nothing
  // else writes them during the launch
  // ... read in ONE batch of unconditional scalar loads (null pointers swapped for a valid word whose
  // value is then ignored): loaded one by one behind their null checks, each cost a pointer load, a
  // wait, the value load and another wait -- several round trips before a job issued its first load
  const int64_t* step_p = step != nullptr ? step : reinterpret_cast<const int64_t*>(ticket);
  const int64_t* rng_p = noise_rng != nullptr ? noise_rng + 1 : step_p;
  const int64_t step_raw = step_p[0], rng_raw = rng_p[0];
  const int32_t flag_raw = ticket[kSlotFlag];
  float b1p = 1.f, b2p = 1.f;
  if constexpr (OP == 3) {
    b1p = beta_pow[0];
    b2p = beta_pow[1];
    lr_t = h.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  }
  const int64_t step_now = UPD && step != nullptr ? step_raw : 0;
  const int64_t rng_now = UPD && noise_rng != nullptr ? rng_raw : 0;         // (FEW: any block may close)
  const bool sync = UPD && tgt != nullptr && step != nullptr && ((step_now + 1) % tfreq) == 0;
  const bool psync = sync && tgt_packed != nullptr;
  constexpr bool TWO = OP == 2 || OP == 3 || OP == 5 || OP == 6 || OP == 7;   // second slot written
  const bool wtwo = OP != 7 || flag_raw != 0;                                  // (momentum-0 RMSProp: flagged)
  constexpr bool TWO_LD = TWO && OP != 7;                                      // ... and read
  constexpr bool ONE = UPD && OP != 0;
  int t = threadIdx.x;            // (DP job loop: re-derived per job, see there)
  int64_t* prof = (h.prof != nullptr && t == 0 && blockIdx.x < 2) ? h.prof + 8 * blockIdx.x : nullptr;
#define OPT_MARK(i) if (prof) prof[i] = (int64_t)__builtin_amdgcn_s_memtime()
  OPT_MARK(0);
  // WG: thread 0 polls member m's done counter (bounded: a lost arrival flags the error word
  // instead of hanging), then acquires; the caller's barrier releases the block's other waves
  auto wg_wait = [&](int m) {
    if (m < 0 || threadIdx.x != 0) return;
    const int32_t* dc = wg->done + kTicketStride * m;
    const int want = wg->nblk[m];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(dc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {   // 1 s: flag, do not hang
        ticket[kErrFlag] = 1;
        break;
      }
    }
    // (no acquire fence: the waiter reads nothing the member wrote -- it only must not overwrite
    //  the slot tables before the member's reads completed, which its count follows)
    if (tl) tl[1] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  if (PEROK && sampler && per.sum != nullptr) {
    // prioritized: this step's priorities into the tree (one wave), then the next step's
    // stratified sample from the updated tree (beta of the NEXT global_step)
    const int64_t step0 = per.step[0];                  // read before this block's ticket add
    const uint64_t seed = (uint64_t)per.rng[0], ctr = (uint64_t)per.rng[1];
    SumtreeLds& L = *reinterpret_cast<SumtreeLds*>(smem);
    int ins_first = 0;
    if (per.ins_n > 0) ins_first = (int)((per.ins_cursor[0] - per.ins_n + per.ins_cap) % per.ins_cap);
    sumtree_update_wave(per.sum, per.mn, per.maxp, per.upd_idx, per.upd_td, per.alpha, per.eps, 0, per.B, per.P,
                        per.levels, L, 0, 1, per.ins_n, ins_first, per.ins_cap);
    if constexpr (WG) wg_wait(wg->slots_member);        // (the current slot tables' reader is done)
    __syncthreads();                                    // tree writes visible to every lane of the block
    if ((int)threadIdx.x < per.B) {
      const float beta = fminf(1.f, per.beta0 + (1.f - per.beta0) * (float)(step0 + 1) / per.beta_steps);
      per_sample_lane(per.sum, per.mn, seed, ctr, per.size[0], threadIdx.x, per.B, per.P, beta, per.idx_out,
                      per.w_out, per.so);
    }
    __syncthreads();
    if (threadIdx.x == 0) per.rng[1] = (int64_t)(ctr + 1);
  } else if (sampler) {
    SampleLds& sls = *reinterpret_cast<SampleLds*>(smem);
    const uint32_t n = (uint32_t)max(smp.size[0], 1);
    const uint64_t seed = (uint64_t)smp.rng[0], ctr = (uint64_t)smp.rng[1];
    const int32_t v = draw_distinct(seed, ctr, n, smp.B, sls);
    if constexpr (WG) {
      wg_wait(wg->slots_member);                        // (the current slot tables' reader is done)
      __syncthreads();
    }
    if ((int)threadIdx.x < smp.B) {
      DQN_ASSERT(v >= 0 && (uint32_t)v < n);
      write_sample_slots(smp, threadIdx.x, v, reinterpret_cast<const int4*>(smp.state_idx)[v], smp.next_idx[v]);
    }
    if (threadIdx.x == 0) smp.rng[1] = (int64_t)(ctr + 1);   // every lane read it before the barriers
    if (tl) tl[1] = (int64_t)__builtin_amdgcn_s_memrealtime();
  }
  OPT_MARK(1);
  unsigned char* fcl = WG ? opt_dyn : OptShm<!WG, FC ? kFcLds : 16, 1>::get();
  // dW of this thread's 4 values (tile row k, columns n..n+3 of the item map) from the FcFuse rows
  // this thread's 8-element piece of fc operand rows m0 .. m0 + 31 of the item's 32 (k) x 64 (n)
  // tile: t < 128 a piece of an x row, 128 <= t < 384 one of a dh row
  auto fc_load = [&](const UpdJob& jb, int m0) {
    const bool lx = t < 128, lh = t >= 128 && t < 384;
    const int lr = lx ? (t >> 2) : ((t - 128) >> 3);
    const int lc = lx ? 8 * (t & 3) : 8 * ((t - 128) & 7);
    const act_t* X = reinterpret_cast<const act_t*>(ff.x);
    const act_t* H = reinterpret_cast<const act_t*>(ff.dh);
    const int m = m0 + lr;
    bfx8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (act_t)0.f;
    // (32-bit element offsets off the uniform bases: no per-thread 64-bit address kept live)
    if (m < ff.M) {
      if (lx && jb.k0 + lc < jb.K)
        v = *reinterpret_cast<const bfx8*>(X + (uint32_t)(m * ff.ldx + jb.k0 + lc));
      else if (lh && jb.n0 + lc < jb.N)
        v = *reinterpret_cast<const bfx8*>(H + (uint32_t)(m * ff.ldh + jb.fc_col + jb.n0 + lc));
    }
    return v;
  };
  // dW of this thread's 4 values (tile row k, columns n..n+3 of the item map) from the FcFuse rows;
  // v0: this thread's piece of the first 32-row chunk, loaded with the item's HBM batch
  auto fc_tile_grad = [&](const UpdJob& jb, float* g, bfx8 v0) {
    act_t* Xs = reinterpret_cast<act_t*>(fcl);           // [32][kFcSX]: x[m][k0 .. k0 + 32)
    act_t* Hs = Xs + 32 * kFcSX;                         // [32][kFcSH]: dh[m][col + n0 .. + 64)
    float* R = reinterpret_cast<float*>(fcl);            // [32][kFcRS] fp32 dW tile (after the MFMAs)
    const int wv = t >> 6, lane = t & 63;
    const int kt = wv >> 2, nt = wv & 3;
    const bool lx = t < 128, lh = t >= 128 && t < 384;
    const int lr = lx ? (t >> 2) : ((t - 128) >> 3);
    const int lc = lx ? 8 * (t & 3) : 8 * ((t - 128) & 7);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#if !DQN_ACT_F32
    const int gq = lane >> 4, rq = (lane >> 2) & 3, cp = 4 * (lane & 3);
    const act_t* ph = Hs + (4 * gq + rq) * kFcSH + nt * 16 + cp;
    const act_t* px = Xs + (4 * gq + rq) * kFcSX + kt * 16 + cp;
#endif
    for (int m0 = 0; m0 < ff.M; m0 += 32) {
      const bfx8 v = m0 == 0 ? v0 : fc_load(jb, m0);
      __syncthreads();                 // previous chunk's operand reads / previous item's R reads done
#if DQN_ACT_F32
      // (8-byte stores: the padded row strides keep even float offsets; 8 scalar stores per row piece
      //  put the fp32 launch's LDS bank conflicts at 31 %, profiles/r6_pmc_final_ref_fp32.md)
      {
        float* dst = lx ? Xs + lr * kFcSX + lc : Hs + lr * kFcSH + lc;
        if (lx || lh) {
#pragma unroll
          for (int j = 0; j < 8; j += 2) *reinterpret_cast<float2*>(dst + j) = make_float2(v[j], v[j + 1]);
        }
      }
      __syncthreads();
      // A = dh^T (rows n), B = x (columns k): lane (row = lane & 15, g = lane >> 4) holds chunk rows
      // 8 g .. 8 g + 7 of its column (the fp32 k32 operand layout, dqn_act.h)
      bfx8 af, bfm;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        af[j] = Hs[(8 * (lane >> 4) + j) * kFcSH + nt * 16 + (lane & 15)];
        bfm[j] = Xs[(8 * (lane >> 4) + j) * kFcSX + kt * 16 + (lane & 15)];
      }
      acc = DQN_MFMA16_BUILTIN(af, bfm, acc, 0, 0, 0);
#else
      if (lx) *reinterpret_cast<bfx8*>(Xs + lr * kFcSX + lc) = v;
      else if (lh) *reinterpret_cast<bfx8*>(Hs + lr * kFcSH + lc) = v;
      __syncthreads();
      // A = dh^T (rows n), B = x (columns k); the same row permutation on both operands
      acc = DQN_MFMA16_BUILTIN(join_tr(lds_tr16(ph), lds_tr16(ph + 16 * kFcSH)),
                               join_tr(lds_tr16(px), lds_tr16(px + 16 * kFcSX)), acc, 0, 0, 0);
#endif
    }
    __syncthreads();                   // operand reads done before R overwrites the staging
    // acc[r] = dW[k = kt * 16 + (lane & 15)][n = nt * 16 + 4 * (lane >> 4) + r]
    *reinterpret_cast<float4*>(R + (kt * 16 + (lane & 15)) * kFcRS + nt * 16 + 4 * (lane >> 4)) =
        make_float4(acc[0] * kInvLossScale, acc[1] * kInvLossScale, acc[2] * kInvLossScale, acc[3] * kInvLossScale);
    __syncthreads();
    const int r = (wv >> 1) * 8 + (lane & 7), c4 = (wv & 1) * 32 + (lane >> 3) * 4;
    const float4 gv = *reinterpret_cast<const float4*>(R + r * kFcRS + c4);
    g[0] = gv.x; g[1] = gv.y; g[2] = gv.z; g[3] = gv.w;
  };
  // fc bias chunk (<= 512 values, thread t < 128 owns n = 4t..4t+3): sum_m dh[m][col + n] over 4
  // row phases, combined in a fixed order
  auto fc_bias_grad = [&](const UpdJob& jb, float* g) {
    float* R = reinterpret_cast<float*>(fcl);            // [4][512]
    const act_t* H = reinterpret_cast<const act_t*>(ff.dh);
    const int cg = t & 127, ph = t >> 7, c = 4 * cg;
    float sm[4] = {0.f, 0.f, 0.f, 0.f};
    if (c < jb.K) {
#pragma unroll 4
      for (int m = ph; m < ff.M; m += 4) {
        const bfx4 v = *reinterpret_cast<const bfx4*>(H + (uint32_t)(m * ff.ldh + jb.fc_col + c));
#pragma unroll
        for (int j = 0; j < 4; ++j) sm[j] += (float)v[j];
      }
    }
    __syncthreads();                   // previous item's LDS reads done
    *reinterpret_cast<float4*>(R + ph * 512 + c) = make_float4(sm[0], sm[1], sm[2], sm[3]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = (4 * t + j) & 511;
      g[j] = ((R[i] + R[512 + i]) + (R[1024 + i] + R[1536 + i])) * kInvLossScale;
    }
  };
  // One job item = a 32x64 tile (or a 2048-element chunk) updated by 4 consecutive elements per
  // thread. The body is instantiated per (AL = 16-byte aligned float4 rows, NZ = noisy) so that
  // every global load of the item (mu / sigma / grad / slots / target / noise factors) is an
  // UNCONDITIONAL load issued in one batch: out-of-range threads read the job's first element
  // (clamped address) and discard it. (Per-thread predicated loads put a branch and a full
  // vmcnt wait between loads and serialise the item on memory latency.)
  bool gsc1 = false;             // WG dependent job: its gradient is read with sc1 loads
  // ---- DP: the cross-rank sum of dependent job `dslot`'s gradient slot (xgmi_dev.h dpx_sum: push to
  // every peer's inbox, flag, wait, sum in rank order -- bit-identical on every rank)
  int dslot = -1;
  float gdp[4] = {0.f, 0.f, 0.f, 0.f};
  // (live: this thread holds an element of the job -- the others neither push nor read: a 32 x 64
  //  tile of the output layer holds 32 x A values, e.g. 6 of 64 columns)
  auto dp_sum = [&](float* g, bool live) {
    if constexpr (DP) {
      const float4 acc = dpx_sum(*dp.x, dslot, t, make_float4(g[0], g[1], g[2], g[3]), live);
      g[0] = acc.x; g[1] = acc.y; g[2] = acc.z; g[3] = acc.w;
    } else {
      (void)g;
      (void)live;
    }
  };
  // dependent job jb's summed gradient into gdp (this thread's 4 values in the item's thread map),
  // before the item issues its own loads: nothing else is live across the exchange's waits
  auto dp_grad = [&](const UpdJob& jb) {
    int64_t d0;
    bool ok[4];
    if (jb.kind == 1) {
      d0 = 4 * t;
#pragma unroll
      for (int j = 0; j < 4; ++j) ok[j] = 4 * t + j < jb.K;
    } else {
      const int wv = t >> 6, l = t & 63;
      const int k = jb.k0 + (wv >> 1) * 8 + (l & 7), n = jb.n0 + (wv & 1) * 32 + (l >> 3) * 4;
      d0 = (int64_t)k * jb.N + n;
#pragma unroll
      for (int j = 0; j < 4; ++j) ok[j] = k < jb.K && n + j < jb.N;
    }
    // (sc1: produced by this launch's tiles, see dep_wait; out-of-range lanes read element 0)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G + jb.src_off), (short)0,
                                                                        0x7ffffff0, 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      gdp[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4 * (ok[j] ? d0 + j : 0)), 0, 16));
    dp_sum(gdp, ok[0] || ok[1] || ok[2] || ok[3]);
  };
  auto item = [&](const UpdJob& jb, auto al_c, auto nz_c, auto dg_c) {
    // DG: dL/dsigma is derived from the mu-slot gradient (gnoise given), not read
    constexpr bool AL = decltype(al_c)::value, NZ = decltype(nz_c)::value, DG = decltype(dg_c)::value;
    const bool elem = jb.kind == 1;
    float g[4];
    const bool fcj = FC && jb.fc_col >= 0;
    bool ok[4];
    int k, n;                      // row (tile) and column / element index within the tensor
    bool rowok;
    int64_t e0;
    if (elem) {                    // chunk of up to 2048 elements: 4 per thread
      k = 0;
      n = 4 * t;
      rowok = true;
      e0 = (int64_t)jb.src_off + n;
#pragma unroll
      for (int j = 0; j < 4; ++j) ok[j] = n + j < jb.K;
    } else {                       // tile: row r, columns c4..c4+3 (wave: 8 rows x 32 columns)
      const int wv = t >> 6, l = t & 63;
      const int r = (wv >> 1) * 8 + (l & 7), c4 = (wv & 1) * 32 + (l >> 3) * 4;
      k = jb.k0 + r;
      n = jb.n0 + c4;
      rowok = k < jb.K;
      e0 = (int64_t)jb.src_off + (int64_t)k * jb.N + n;
#pragma unroll
      for (int j = 0; j < 4; ++j) ok[j] = rowok && n + j < jb.N;
    }
    const int64_t d0 = e0 - jb.src_off;                  // offset within the tensor
    // clamped element indices: AL -> all 4 in range or none (one float4), else per element
    int64_t ix[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) ix[j] = (AL ? ok[0] : ok[j]) ? d0 + j : 0;
    auto ld = [&](const float* base, int64_t off, float* v) {
      if constexpr (AL) {
        const float4 x = *reinterpret_cast<const float4*>(base + off + ix[0]);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = base[off + ix[j]];
      }
    };
    // sc1 (L1-bypassing) loads of bytes other workgroups of this launch produced: 16 B per lane through
    // a buffer descriptor where the 4 values are contiguous (one buffer_load_dwordx4 ... sc1), else 4 B each
    auto sc1_ld = [&](const float* base, int64_t off, float* v) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0,
                                                                          0x7ffffff0, 0x00020000);
      if constexpr (AL) {
        typedef unsigned int u32x4_ __attribute__((ext_vector_type(4)));
        const float4 x = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(4 * (off + ix[0])), 0, 16));
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4 * (off + ix[j])), 0, 16));
      }
    };
    auto st = [&](float* base, int64_t off, const float* v) {
      if constexpr (AL) {
        if (ok[0]) {
          f32x4* p = reinterpret_cast<f32x4*>(base + off + d0);
          const f32x4 x = {v[0], v[1], v[2], v[3]};
          *p = x;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (ok[j]) base[off + d0 + j] = v[j];
      }
    };
    const int64_t mo = jb.src_off, so = NZ ? jb.sig_off : jb.src_off;
    // factorised target tile: the target's mu / sigma fragments only change at a sync (or in a
    // mix-only call on the target itself), so no per-step target loads / mix / pack for it
    const bool tfj = NZ && !elem && (jb.eff & 2) != 0 && h.tsg != nullptr;
    const bool tmj = tmix && !tfj;
    float w[4], a[4], b[4], ws[4], gs[4], as[4], bs[4], tw[4], tws[4], e[4], te[4];
    // ---- every load of the item, issued before any math
    ld(W, mo, w);
    if constexpr (ONE) ld(S0, mo, a);
    if constexpr (TWO_LD) ld(S1, mo, b);
    if constexpr (NZ) {
      ld(W, so, ws);
      if constexpr (UPD) {
        if constexpr (!DG) {
          if (gsc1) {
            sc1_ld(G, so, gs);
          } else {
            ld(G, so, gs);
          }
        }
        if constexpr (ONE) ld(S0, so, as);
        if constexpr (TWO_LD) ld(S1, so, bs);
      }
    }
    // the target's mu / sigma in the same batch (one memory round trip per item: the extra
    // VGPRs keep the same 2 blocks / CU, the block is 8 waves and the budget 128 VGPRs)
    if (tmj) {
      ld(tgt, mo, tw);
      if constexpr (NZ) ld(tgt, so, tws);
    }
    // the fc tile's first 32 operand rows (L2 / MALL) join the batch: fc_tile_grad then waits on
    // one round trip instead of issuing its own after the batch has drained
    bfx8 fx0;
    if constexpr (FC && UPD) {
      if (fcj && !elem) fx0 = fc_load(jb, 0);
    }
    // factorised-noise factors (loaded with the item's batch, before the fc gradient: a separate
    // round trip after it cost Rainbow's items ~1 us each): f(eps_in[k]) (1 for biases / chunks) and f(eps_out[n + j])
    float nin = 1.f, nout[4] = {1.f, 1.f, 1.f, 1.f}, gin = 1.f, gout[4] = {1.f, 1.f, 1.f, 1.f};
    float tin = 1.f, tout[4] = {1.f, 1.f, 1.f, 1.f};     // (tmix: the target's next sample)
    const bool hin = NZ && !elem && jb.ein_off >= 0;
    const int ki = NZ ? jb.ein_off + (hin && rowok ? k : 0) : 0;     // clamped: always in range
    if constexpr (NZ) {
      const float* gn = DG ? gnoise : noise;             // (DG: the sample the forward used)
      const float ni = noise[hin ? ki : 0], gi = DG ? gn[hin ? ki : 0] : 1.f;
      float no[4], go[4], to[4] = {1.f, 1.f, 1.f, 1.f}, ti = 1.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int oi = jb.eout_off + (ok[j] ? n + j : 0);
        no[j] = noise[oi]; go[j] = DG ? gn[oi] : 1.f;
        if (tmj) to[j] = tnoise[oi];
      }
      if (tmj) ti = tnoise[hin ? ki : 0];
      if (hin) { nin = fnz(ni); gin = fnz(gi); }
#pragma unroll
      for (int j = 0; j < 4; ++j) { nout[j] = fnz(no[j]); gout[j] = fnz(go[j]); }
      if (tmj) {
        if (hin) tin = fnz(ti);
#pragma unroll
        for (int j = 0; j < 4; ++j) tout[j] = fnz(to[j]);
      }
    }
    if constexpr (UPD) {
      // fused fc weight / bias gradient (block-uniform), formed while the item's HBM loads
      // above are in flight (its X / dH rows are L2-resident)
      if constexpr (FC) {
        if (fcj) {
          OPT_MARK(5);
          if (elem) fc_bias_grad(jb, g); else fc_tile_grad(jb, g, fx0);
          OPT_MARK(6);
        }
      }
      if (part != nullptr && jb.part_n > 0) {
        // fixed-order sum of the chunk-group partials (block-uniform branch), 4 loads in flight
        float pv[4];
        ld(part, jb.part_off, g);
#pragma unroll 4
        for (int p = 1; p < jb.part_n; ++p) {
          ld(part, jb.part_off + (int64_t)p * jb.part_stride, pv);
#pragma unroll
          for (int j = 0; j < 4; ++j) g[j] += pv[j];
        }
      } else if (!fcj) {
        if (gsc1) {                                       // produced in this launch (see the dep wait)
          if constexpr (DP) {
            if (dslot >= 0) {                             // block-uniform: the sum over every rank, formed
#pragma unroll                                            // before the item's loads (dp_grad)
              for (int j = 0; j < 4; ++j) g[j] = gdp[j];
            } else {
              sc1_ld(G, mo, g);
            }
          } else {
            sc1_ld(G, mo, g);
          }
        } else {
          ld(G, mo, g);
        }
      }
    }
    // ---- update
    if constexpr (UPD) {
      if constexpr (NZ && DG) {                           // dL/dsigma from the mu-slot gradient
#pragma unroll
        for (int j = 0; j < 4; ++j) gs[j] = ok[j] ? g[j] * gin * gout[j] : 0.f;
      }
      upd4<OP>(w, g, a, b, e0, h.reg_end, h, lr_t, ok);
      st(W, mo, w);
      if constexpr (ONE) st(S0, mo, a);
      if constexpr (TWO) if (wtwo) st(S1, mo, b);
      if (sync) st(tgt, mo, w);
      if constexpr (NZ) {
        upd4<OP>(ws, gs, as, bs, so + d0, h.reg_end, h, lr_t, ok);
        st(W, so, ws);
        if constexpr (ONE) st(S0, so, as);
        if constexpr (TWO) if (wtwo) st(S1, so, bs);
        if (sync) st(tgt, so, ws);
      }
    }
    // ---- effective values (noisy: mu + sigma f(eps_in) f(eps_out)) of this net and, tmix,
    //      of the TARGET under its own next noise sample
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      e[j] = w[j];
      if constexpr (NZ) e[j] = (tfj && !UPD) ? w[j] : w[j] + ws[j] * nin * nout[j];   // (mix-only on a
    }                                                     //  factorised target: mu fragments)
    if (tmj) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float mu = sync ? w[j] : tw[j];
        te[j] = mu;
        if constexpr (NZ) te[j] = mu + (sync ? ws[j] : tws[j]) * tin * tout[j];
      }
      if (jb.eff & 1) st(teff, mo, te);
    }
    if (jb.eff & 1) st(eff, mo, e);
    if (elem) {
      if (jb.fwd_off >= 0 && !h.no_pack) {                // fp32 copy inside the packed buffer
        float* pf = reinterpret_cast<float*>(packed + jb.fwd_off) + n;
        float* tf = psync ? reinterpret_cast<float*>(tgt_packed + jb.fwd_off) + n : nullptr;
        float* mf = tmix ? reinterpret_cast<float*>(tpk + jb.fwd_off) + n : nullptr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!ok[j]) continue;
          pf[j] = e[j];
          if (tf) tf[j] = e[j];
          if (mf) mf[j] = te[j];
        }
      }
      return;                      // uniform per block: no barrier below is skipped unevenly
    }
    // bf16 fragments of this tile into dst (+ dst2): dgrad straight from the registers (4
    // consecutive K' of one lane's slot), forward after a 4x4 transpose inside each lane quad
    auto emit = [&](const float* ev, act_t* dst, act_t* dst2, bool dgrad) {
      float x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = ok[j] ? ev[j] : 0.f;
      if (dgrad && jb.dg_mode != 0 && rowok && n < jb.N) {
        bfx4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (act_t)x[j];
        int kp, np;                                        // K' of the first of the 4 values, N'
        if (jb.dg_mode == 2) { kp = n; np = k; }           // dense: K' = out (n), N' = in (k)
        else { const int tap = k / jb.dg_cin, ci = k - tap * jb.dg_cin; kp = tap * jb.N + n; np = ci; }
        const int lane = ((kp & 31) >> 3) * 16 + (np & 15);
        const int64_t o = jb.dg_off +
                          ((int64_t)((jb.dg_ks_off + (kp >> 5)) * jb.dg_N16 + jb.dg_nt_off + (np >> 4)) * 64 + lane) * 8 +
                          (kp & 7);
        *reinterpret_cast<bfx4*>(dst + o) = v;
        if (dst2) *reinterpret_cast<bfx4*>(dst2 + o) = v;
      }
      quad_transpose4(x);          // lane: column (n - q) + q, rows 4 * half .. + 3 of its quad
      const int l = t & 63, q = l & 3, half = (l >> 2) & 1, rg = (t >> 6) >> 1;
      const int col = n + q;       // n: this lane's first column before the transpose (quad-uniform)
      if ((col & ~15) < jb.N) {    // n-tile exists (columns past N inside it are zeros)
        bfx4 f;
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = (act_t)x[j];
        const int64_t o = jb.fwd_off + ((int64_t)((jb.fwd_ks_off + (jb.k0 >> 5)) * jb.fwd_N16 + jb.fwd_nt_off +
                                                  (col >> 4)) * 64 + rg * 16 + (col & 15)) * 8 + half * 4;
        *reinterpret_cast<bfx4*>(dst + o) = f;
        if (dst2) *reinterpret_cast<bfx4*>(dst2 + o) = f;
      }
    };
    OPT_MARK(7);
    if (!h.no_pack) emit(e, packed, psync ? tgt_packed : nullptr, true);
    if (tmj) emit(te, tpk, nullptr, false);               // (the target runs forward only)
    if constexpr (NZ) {
      if (tfj) {
        act_t* sg = reinterpret_cast<act_t*>(h.tsg);
        if constexpr (UPD) {
          if (tmix && sync) {                             // the target just became this mu / sigma
            emit(w, tpk, nullptr, false);
            emit(ws, sg, nullptr, false);
          }
        } else {
          emit(ws, sg, nullptr, false);                   // (mix-only: `packed` got the mu fragments)
        }
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  auto run = [&](int ji) {
    const UpdJob jb = jobs[ji];
    const bool nz = NZOK && jb.sig_off >= 0;
    // float4 rows: 16-byte aligned tensor (and sigma) offsets and a row / chunk length % 4 == 0
    const bool al = ((jb.src_off | (nz ? jb.sig_off : 0)) & 3) == 0 && ((jb.kind == 1 ? jb.K : jb.N) & 3) == 0;
    if (!nz) {
      if (al) item(jb, T_{}, F_{}, F_{}); else item(jb, F_{}, F_{}, F_{});
    } else if constexpr (NZOK) {
      if (gnoise != nullptr) {
        if (al) item(jb, T_{}, T_{}, T_{}); else item(jb, F_{}, T_{}, T_{});
      } else {
        if (al) item(jb, T_{}, T_{}, F_{}); else item(jb, F_{}, T_{}, F_{});
      }
    }
  };
  if constexpr (WG) {
    // (the tile blocks ran wg_tile_run at the top of the kernel and returned)
  }
  // a job whose gradient a weight-gradient range of this launch produces (its blocks come after every
  // tile in the grid, so the tiles are resident or done: the wait ends)
  auto dep_wait = [&](int d) {
    if constexpr (WG) {
      if (threadIdx.x == 0) {
        const int m = d / kWgSlots;
        const int want = wg->nblk[m] / wg->gy[m];        // tiles per K-range
        const int32_t* c = wg->done + kTicketStride * (kMaxWgradMembers + d);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
          __builtin_amdgcn_s_sleep(2);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {   // 1 s: flag, do not hang
            ticket[kErrFlag] = 1;
            break;
          }
        }
        // (no acquire fence: the item reads this gradient with agent-scope sc1 loads, and the
        //  tiles produced it by memory-side atomics / sc1 stores; the fence's L1 invalidate cost
        //  ~1.7 us on the launch's critical path)
      }
      __syncthreads();
      gsc1 = true;
    }
  };
  if constexpr (FC) {
    // one job per block (the launcher sizes the grid for it): no job loop, so no per-thread loop
    // invariants are hoisted and kept live across the fc barriers
    if constexpr (DP) {
      // job-table positions: [0, first) one job per block, [first, first + blocks) the dependent-job
      // blocks (each runs jobs first + b, first + b + blocks, ... in order: every rank's block b
      // waits on the same slots in the same order), then the rest of the table one per block
      // (one call site of the item: a second one cost ~50 VGPRs)
      const bool dblk = wid >= dp.first && wid < dp.first + dp.blocks;
      const int j0 = wid < dp.first || dblk ? wid : wid - dp.blocks + dp.n;
      const int j1 = dblk ? dp.first + dp.n : j0 + 1, js = dblk ? dp.blocks : 1;
      for (int ji = j0; wid >= 0 && ji < j1 && ji < njobs; ji += js) {
        // (t opaque per job: the item's thread-map values are recomputed instead of hoisted out of the
        //  loop and kept live across it -- +17 VGPRs and scratch spills otherwise)
        asm volatile("" : "+v"(t));
        const int d = jobs[ji].dep;
        if (d >= 0) dep_wait(d);
        if (dblk) {
          DQN_ASSERT(d >= 0 && ji - dp.first < dp.x->slots);
          dslot = ji - dp.first;
          dp_grad(jobs[ji]);
        }
        run(ji);
        if (dblk) __syncthreads();                        // (the next job's exchange reuses the slots)
      }
    } else if (wid >= 0 && wid < njobs) {
      if constexpr (WG) {
        const int d = jobs[wid].dep;
        if (d >= 0) dep_wait(d);
      }
      run(wid);
    }
  } else {
    for (int ji = wid < 0 ? njobs : wid; ji < njobs; ji += nwork) run(ji);
  }
  OPT_MARK(2);
  if (!UPD) return;
  // ---- end-of-launch bookkeeping (global_step, Adam beta powers, noise counter / copy) once
  //      every block has consumed the old values. Block 0 (the sampler block, or the first work
  //      block) does it: every other block makes ONE no-return arrival add on one of 16 counters
  //      (blockIdx & 15, own 128-byte lines) and exits at once -- no returned atomic keeps its CU
  //      slot (measured: a returning ticket per block cost Rainbow's 1714-block launch ~5 us) --
  //      while lanes 0..15 of block 0 poll the counters. Nothing waits on block 0, so the wait
  //      always ends (bounded anyway: a lost arrival flags ticket[kErrFlag] instead of hanging).
  if constexpr (FEW) {
    // every wave of this block consumed the old step / beta powers / noise in its item: one
    // returning add per block; the last arriver closes (counter 0 back to zero for the next launch)
    __shared__ int last_blk;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int k = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_blk = k == (int)gridDim.x - 1;
      if (last_blk) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_blk) return;
  } else if (blockIdx.x != 0) {
    __syncthreads();                                      // every wave of the block is past its reads
    if (tl) tl[2] = (int64_t)__builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(cnt + kTicketStride * (blockIdx.x & (kTicketSubs - 1)), 1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (!FEW && threadIdx.x < kTicketSubs) {
    const int j = threadIdx.x;
    const int want = ((int)gridDim.x - j + kTicketSubs - 1) / kTicketSubs - (j == 0 ? 1 : 0);
    int32_t* c = cnt + kTicketStride * j;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      __builtin_amdgcn_s_sleep(4);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) {   // 5 s (>> any launch): flag, do not hang
        ticket[kErrFlag] = 1;
        break;
      }
    }
    // consume exactly this launch's arrivals (not a reset to 0): after a timeout the late arrivals
    // cancel the deficit instead of counting toward -- and closing early -- the next launch
    __hip_atomic_fetch_add(c, -want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  OPT_MARK(3);
  if constexpr (WG) {            // every block has arrived: the sampler / range waits are over
    for (int t = threadIdx.x; t < kMaxWgradMembers + wg->n * kWgSlots; t += blockDim.x)
      if (t < wg->n || t >= kMaxWgradMembers)
        __hip_atomic_store(wg->done + kTicketStride * t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) {
    if (step) step[0] = step_now + 1;
    if constexpr (OP == 3) {
      beta_pow[0] = b1p * h.b1;
      beta_pow[1] = b2p * h.b2;
    }
    if (noise_rng != nullptr) noise_rng[1] = rng_now + 1;   // (the drawing launch completed before this one)
  }
  // every other block consumed gnoise before its arrival add: block 0 may overwrite it now --
  // float4 pieces, every load of a round issued before its stores (a load -> store chain per
  // element cost Rainbow's launch ~6.5 us at its end: 15.6k cycles for ~8.7k floats)
  if (noise_dst != nullptr) {
    const bool al16 = ((reinterpret_cast<uintptr_t>(noise) | reinterpret_cast<uintptr_t>(noise_dst)) & 15) == 0;
    const int n4 = al16 ? noise_n >> 2 : 0, tid = (int)threadIdx.x, nt = (int)blockDim.x;
    const float4* s4 = reinterpret_cast<const float4*>(noise);
    float4* d4 = reinterpret_cast<float4*>(noise_dst);
    constexpr int kU = 8;
    for (int base = 0; base < n4; base += kU * nt) {
      float4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) v[u] = s4[min(base + u * nt + tid, n4 - 1)];     // (clamped: no branch)
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (base + u * nt + tid < n4) d4[base + u * nt + tid] = v[u];
    }
    for (int i = 4 * n4 + tid; i < noise_n; i += nt) noise_dst[i] = noise[i];
  }
  OPT_MARK(4);
  if (tl) tl[2] = (int64_t)__builtin_amdgcn_s_memrealtime();
#undef OPT_MARK
}


// All arguments of one optim_pack_kernel launch (the launcher in optim.hip fills it; the
// per-optimizer instantiations live in optim_ops_*.hip so the build compiles them in parallel).
struct OptPackLaunch {
  int grid; size_t dyn; hipStream_t st;
  int mode; bool few;
  float* w; const float* g; float* s0; float* s1; float* beta_pow; int64_t* step; int32_t* ticket; OptHP h;
  const UpdJob* jobs; int njobs; act_t* packed; float* tgt; act_t* tgt_packed; int tfreq;
  const float* noise; float* eff; const float* gnoise; float* noise_dst; int noise_n;
  TrunkSample smp; PerStep per; const float* tnoise; float* teff; act_t* tpk; int64_t* noise_rng; FcFuse ff;
  const float* part; const WgradGroup* wg; int wg_blocks; DpLaunch dp;
};

template <int N>
void optim_pack_op(const OptPackLaunch& L);

#ifdef DQN_OPTIM_DEFINE_OPS
template <int N>
void optim_pack_op(const OptPackLaunch& L) {
#define OPM(M) hipLaunchKernelGGL((optim_pack_kernel<N, M>), dim3(L.grid), dim3(kPackThreads), L.dyn, L.st, L.w, L.g, \
                                  L.s0, L.s1, L.beta_pow, L.step, L.ticket, L.h, L.jobs, L.njobs, L.packed, L.tgt, \
                                  L.tgt_packed, L.tfreq, L.noise, L.eff, L.gnoise, L.noise_dst, L.noise_n, L.smp, L.per, \
                                  L.tnoise, L.teff, L.tpk, L.noise_rng, L.ff, L.part, L.wg, L.wg_blocks, \
                                  L.dp)
  if constexpr (N < 0) {
    OPM(kModeNoisy);                                    // mix + pack only (noisy nets)
  } else {
#if DQN_ACT_F32
    switch (L.mode) {
      case 0: OPM(0); break; case 1: OPM(1); break; case 3: OPM(3); break;
      case 4: OPM(4); break; case 5: OPM(5); break; case 7: OPM(7); break;
      // the fused fc weight gradient / weight-gradient + update / DP exchange modes (round 6: the
      // fp32 build's FcFuse and fused tiles)
      case 8: OPM(8); break; case 9: OPM(9); break; case 11: OPM(11); break;
      case 12: OPM(12); break; case 13: OPM(13); break; case 15: OPM(15); break;
      case 24: OPM(24); break; case 25: OPM(25); break; case 27: OPM(27); break;
      case 28: OPM(28); break; case 29: OPM(29); break; case 31: OPM(31); break;
      case 88: OPM(88); break; case 89: OPM(89); break; case 91: OPM(91); break;
      case 92: OPM(92); break; case 93: OPM(93); break; case 95: OPM(95); break;
      default: break;
    }
#else
    constexpr bool kFew = N == 0 || N == 3 || N == 7;   // (the common optimizers' few-block variants)
    if (kFew && L.few) {
      if constexpr (kFew) {
        switch (L.mode) {
          case 0: OPM(32); break; case 1: OPM(33); break; case 3: OPM(35); break;
          case 4: OPM(36); break; case 5: OPM(37); break; default: OPM(39); break;
        }
      }
    } else {
      switch (L.mode) {
        case 0: OPM(0); break; case 1: OPM(1); break; case 3: OPM(3); break;
        case 4: OPM(4); break; case 5: OPM(5); break; case 7: OPM(7); break;
        case 8: OPM(8); break; case 9: OPM(9); break; case 11: OPM(11); break;
        case 12: OPM(12); break; case 13: OPM(13); break; case 15: OPM(15); break;
        case 24: OPM(24); break; case 25: OPM(25); break; case 27: OPM(27); break;
        case 28: OPM(28); break; case 29: OPM(29); break; case 31: OPM(31); break;
        // data parallelism: the WG modes with the in-launch gradient exchange
        case 88: OPM(88); break; case 89: OPM(89); break; case 91: OPM(91); break;
        case 92: OPM(92); break; case 93: OPM(93); break; case 95: OPM(95); break;
        default: break;
      }
    }
#endif
  }
#undef OPM
}
#endif

}  // namespace dqn
