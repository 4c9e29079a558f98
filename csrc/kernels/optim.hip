// Fused multi-tensor optimizer over the flat parameter buffer (TF-0.x exact).
//
// Reference: tf.train.{GradientDescent,Momentum,RMSProp,Adam,Adagrad,Adadelta,Ftrl}
// Optimizer.minimize() colocated with the variables on the parameter server
// (/root/reference/src/network.py:159-203) — one ApplyX op per variable plus
// the separate L2 term in the loss (network.py:151-152,311,407).
//
// Here: ONE launch for all parameters; float4 vector loads; per element
//   g = grad * grad_scale (+ reg * w for flat[:reg_end])   -- 1/world DP averaging folded in
// then the TF update rule. Adam's beta powers (TF non-slot variables) are
// read by every block and advanced by the LAST block to finish (arrival
// ticket), together with global_step, so no extra launch is needed.
#include "optim_pack.h"

namespace dqn {

template <int OP>
__global__ void __launch_bounds__(256)
optim_kernel(float* __restrict__ w, const float* __restrict__ grad, float* __restrict__ s0,
             float* __restrict__ s1, float* __restrict__ beta_pow, int64_t* __restrict__ step,
             int32_t* __restrict__ ticket, OptHP h, int n4, float* __restrict__ tgt, int tfreq) {
  float lr_t = h.lr;
  // fused hard target sync: this update makes global_step s+1; the reference copies
  // target <- online after the train step when (s+1) % target_update_freq == 0
  const bool sync = tgt != nullptr && step != nullptr && ((step[0] + 1) % tfreq) == 0;
  const bool wmom = OP != 7 || ticket[1] != 0;     // (see kSlotFlag)
  float4* T = reinterpret_cast<float4*>(tgt);
  if constexpr (OP == 3) {
    const float b1p = beta_pow[0], b2p = beta_pow[1];
    lr_t = h.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  }
  float4* W = reinterpret_cast<float4*>(w);
  const float4* G = reinterpret_cast<const float4*>(grad);
  float4* S0 = reinterpret_cast<float4*>(s0);
  float4* S1 = reinterpret_cast<float4*>(s1);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    float4 wv = W[i], gv = G[i];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if constexpr (OP != 0) a = S0[i];
    if constexpr (OP == 2 || OP == 3 || OP == 5 || OP == 6) b = S1[i];      // (OP 7: mom never read)
    const bool reg = (i * 4) < h.reg_end;       // reg_end is a multiple of 64
    float ww[4] = {wv.x, wv.y, wv.z, wv.w}, gg[4] = {gv.x, gv.y, gv.z, gv.w};
    float aa[4] = {a.x, a.y, a.z, a.w}, bb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      update_one<OP>(ww[j], opt_grad(gg[j], ww[j], reg, h), aa[j], bb[j], h, lr_t);
    }
    const float4 nw = make_float4(ww[0], ww[1], ww[2], ww[3]);
    W[i] = nw;
    if (sync) T[i] = nw;
    if constexpr (OP != 0) S0[i] = make_float4(aa[0], aa[1], aa[2], aa[3]);
    if constexpr (OP == 2 || OP == 3 || OP == 5 || OP == 6 || OP == 7)
      if (wmom) S1[i] = make_float4(bb[0], bb[1], bb[2], bb[3]);
  }
  // last block advances global_step and (Adam) the beta powers. Every block
  // read beta_pow above, before its ticket add, so the update cannot race.
  if (threadIdx.x == 0) {
    // relaxed: the last arriver only WRITES beta_pow/step; every block's read of
    // beta_pow completed (value consumed in the loop) before its ticket add.
    // (An acq_rel agent atomic here costs an L2 writeback + invalidate per block.)
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (int)gridDim.x - 1) {
      if (step) step[0] += 1;
      if constexpr (OP == 3) {
        beta_pow[0] *= h.b1;
        beta_pow[1] *= h.b2;
      }
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}


// target <- tau * online + (1 - tau) * target, optionally only when step % freq == 0.
__global__ void __launch_bounds__(256)
target_update_kernel(float* __restrict__ dst, const float* __restrict__ src, float tau,
                     const int64_t* __restrict__ step, int freq, int n4, float* __restrict__ dst2,
                     const float* __restrict__ src2, int n4b) {
  if (step != nullptr && (step[0] % freq) != 0) return;
  if (dst2 != nullptr) {   // hard copy of a second buffer pair (packed bf16 weights)
    float4* D2 = reinterpret_cast<float4*>(dst2);
    const float4* S2 = reinterpret_cast<const float4*>(src2);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4b; i += gridDim.x * blockDim.x) D2[i] = S2[i];
  }
  float4* D = reinterpret_cast<float4*>(dst);
  const float4* S = reinterpret_cast<const float4*>(src);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    float4 s = S[i];
    if (tau >= 1.f) {
      D[i] = s;
    } else {
      float4 d = D[i];
      const float k = 1.f - tau;
      D[i] = make_float4(tau * s.x + k * d.x, tau * s.y + k * d.y, tau * s.z + k * d.z, tau * s.w + k * d.w);
    }
  }
}

__global__ void step_bump_kernel(int64_t* step) { step[0] += 1; }

}  // namespace dqn

using namespace dqn;

// The probe buffer of DQN_OPT_PROF=1 runs (scripts/probe_optim.py, probe_split.py): allocated at the
// first launch (eager, before any capture); nullptr otherwise.
static int64_t* optim_prof_buffer() {
  static int64_t* buf = nullptr;
  static const bool on = getenv("DQN_OPT_PROF") != nullptr && atoi(getenv("DQN_OPT_PROF")) != 0;
  if (on && buf == nullptr &&
      hipMalloc(&buf, (kProfPhases + 3 * (size_t)kTlBlocks + 8 * (size_t)kTilePhBlocks) * sizeof(int64_t)) != hipSuccess)
    buf = nullptr;
  return buf;
}

static int grid_for(int n4) {
  int g = (n4 + 255) / 256;
  return g < 1 ? 1 : (g > 2048 ? 2048 : g);
}

// The optimizer's arrival ticket is one atomic word: keep the grid at one
// block per CU (grid-stride) so the ticket sees <= 256 arrivals, not ~1.6k.
static int grid_for_ticket(int n4) {
  int g = (n4 + 255) / 256;
  return g < 1 ? 1 : (g > 256 ? 256 : g);
}

void launch_optimizer_step(int op, float* w, const float* g, float* s0, float* s1, float* beta_pow,
                           int64_t* step, int32_t* ticket, const float* hp9, float lr, float reg, int reg_end,
                           float grad_scale, int n, float* tgt, int tfreq, hipStream_t st) {
  OptHP h{};
  h.lr = lr; h.reg = reg; h.grad_scale = grad_scale; h.reg_end = reg_end;
  h.momentum = hp9[0]; h.rho = hp9[1]; h.rms_mom = hp9[2]; h.rms_eps = hp9[3];
  h.b1 = hp9[4]; h.b2 = hp9[5]; h.adam_eps = hp9[6]; h.ad_rho = hp9[7]; h.ad_eps = hp9[8];
  h.prof = nullptr;
  const int n4 = n / 4;
  dim3 grid(grid_for_ticket(n4)), block(256);
  switch (op) {
    case 0: hipLaunchKernelGGL(optim_kernel<0>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 1: hipLaunchKernelGGL(optim_kernel<1>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 2: hipLaunchKernelGGL(optim_kernel<2>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 3: hipLaunchKernelGGL(optim_kernel<3>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 4: hipLaunchKernelGGL(optim_kernel<4>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 5: hipLaunchKernelGGL(optim_kernel<5>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 6: hipLaunchKernelGGL(optim_kernel<6>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    case 7: hipLaunchKernelGGL(optim_kernel<7>, grid, block, 0, st, w, g, s0, s1, beta_pow, step, ticket, h, n4, tgt, tfreq < 1 ? 1 : tfreq); break;
    default: break;
  }
}

void launch_optim_pack(int op, float* w, const float* g, float* s0, float* s1, float* beta_pow, int64_t* step,
                       int32_t* ticket, const float* hp9, float lr, float reg, int reg_end, float grad_scale,
                       const void* jobs, int njobs, void* packed, float* tgt, void* tgt_packed, int tfreq,
                       int max_grid, const float* noise, float* eff, const float* gnoise, float* noise_dst,
                       int noise_n, const TrunkSample* smp, const PerStep* per, const float* tnoise, float* teff,
                       void* tpk, int64_t* noise_rng, const FcFuse* fc, const float* part, const void* wg,
                       int wg_blocks, const void* dp, void* tsg, int no_pack, hipStream_t st) {
  OptPackLaunch L{};
  OptHP& h = L.h;
  h.lr = lr; h.reg = reg; h.grad_scale = grad_scale; h.reg_end = reg_end;
  h.momentum = hp9[0]; h.rho = hp9[1]; h.rms_mom = hp9[2]; h.rms_eps = hp9[3];
  h.b1 = hp9[4]; h.b2 = hp9[5]; h.adam_eps = hp9[6]; h.ad_rho = hp9[7]; h.ad_eps = hp9[8];
  h.prof = optim_prof_buffer();
  h.tsg = tsg;
  h.no_pack = no_pack;
  // one block per job up to max_grid (grid-stride beyond it); block 0 (+1 sampler block when the
  // launch draws the next minibatch) closes the launch once every other block has arrived
  const FcFuse ff = (fc != nullptr && optim_fc_fuse()) ? *fc : FcFuse{nullptr, nullptr, 0, 0, 0};
  // (the FC modes run exactly one job per block)
  const int cap = ff.x != nullptr ? (njobs > 256 ? njobs : 256) : (max_grid > 256 ? max_grid : 256);
  L.smp = smp != nullptr ? *smp : TrunkSample{};
  L.per = per != nullptr ? *per : PerStep{};
  // WG: the launch also computes the grouped weight gradients (tiles after the lead block)
  const bool wgm = wg != nullptr && ff.x != nullptr && op >= 0;
  if (wg != nullptr && !wgm) return;      // (binding checks: a WG launch needs FcFuse rows and an update)
  // DP (WG under data parallelism): the dependent jobs run in dp->blocks blocks
  const DpLaunch dpl = (wgm && dp != nullptr) ? *reinterpret_cast<const DpLaunch*>(dp) : DpLaunch{nullptr, 0, 0, 0};
  if (dp != nullptr && (dpl.x == nullptr || dpl.blocks < 1 || dpl.blocks > dpl.n || dpl.first < 0 ||
                        dpl.first + dpl.n > njobs || dpl.n > kDpxMaxSlots))
    return;                               // (binding checks)
  const int nblk_jobs = dpl.x != nullptr ? njobs - dpl.n + dpl.blocks : njobs;
  // + the lead block (sampler / closer) + the weight-gradient tiles
  L.grid = (nblk_jobs < cap ? nblk_jobs : cap) + (L.smp.size != nullptr || L.per.sum != nullptr || wgm ? 1 : 0) +
           (wgm ? wg_blocks : 0);
  // (a noisy net always passes its noise sample; plain nets pass none)
  L.mode = (noise != nullptr ? kModeNoisy : 0) | (tnoise != nullptr ? kModeTmix : 0) |
           (L.per.sum != nullptr ? kModePer : 0) | (ff.x != nullptr && op >= 0 ? kModeFc : 0) | (wgm ? kModeWg : 0) |
           (dpl.x != nullptr ? kModeDp : 0);
  // few work blocks (16-bit builds, the common optimizers): no spills, returning-ticket close
  L.few = !DQN_ACT_F32 && !wgm && ff.x == nullptr && njobs <= 256 && (op == 0 || op == 3 || op == 7);
  L.dyn = wgm ? (size_t)kFusedWgLds : 0;
  L.st = st;
  L.w = w; L.g = g; L.s0 = s0; L.s1 = s1; L.beta_pow = beta_pow; L.step = step; L.ticket = ticket;
  L.jobs = reinterpret_cast<const UpdJob*>(jobs); L.njobs = njobs;
  L.packed = reinterpret_cast<act_t*>(packed); L.tgt = tgt; L.tgt_packed = reinterpret_cast<act_t*>(tgt_packed);
  L.tfreq = tfreq < 1 ? 1 : tfreq;
  L.noise = noise; L.eff = eff; L.gnoise = gnoise; L.noise_dst = noise_dst; L.noise_n = noise_n;
  L.tnoise = tnoise; L.teff = teff; L.tpk = reinterpret_cast<act_t*>(tpk); L.noise_rng = noise_rng; L.ff = ff;
  L.part = part; L.wg = reinterpret_cast<const WgradGroup*>(wg); L.wg_blocks = wgm ? wg_blocks : 0;
  L.dp = dpl;
  switch (op) {
    case -1: optim_pack_op<-1>(L); break;
    case 0: optim_pack_op<0>(L); break;
    case 1: optim_pack_op<1>(L); break;
    case 2: optim_pack_op<2>(L); break;
    case 3: optim_pack_op<3>(L); break;
    case 4: optim_pack_op<4>(L); break;
    case 5: optim_pack_op<5>(L); break;
    case 6: optim_pack_op<6>(L); break;
    case 7: optim_pack_op<7>(L); break;
    default: break;
  }
}

int upd_job_ints() { return (int)(sizeof(UpdJob) / sizeof(int)); }
void optim_prof_read(int64_t* out16) {
  int64_t* b = optim_prof_buffer();
  if (b != nullptr) (void)hipMemcpy(out16, b, kProfPhases * sizeof(int64_t), hipMemcpyDeviceToHost);
}
int optim_tile_phases_read(int64_t* out, int nblocks) {
  int64_t* b = optim_prof_buffer();
  nblocks = b == nullptr ? 0 : (nblocks < kTilePhBlocks ? nblocks : kTilePhBlocks);
  if (nblocks > 0)
    (void)hipMemcpy(out, b + kProfPhases + 3 * kTlBlocks, 8 * (size_t)nblocks * sizeof(int64_t), hipMemcpyDeviceToHost);
  return nblocks;
}
int optim_timeline_read(int64_t* out, int nblocks) {
  int64_t* b = optim_prof_buffer();
  nblocks = b == nullptr ? 0 : (nblocks < kTlBlocks ? nblocks : kTlBlocks);
  if (nblocks > 0)
    (void)hipMemcpy(out, b + kProfPhases, 3 * (size_t)nblocks * sizeof(int64_t), hipMemcpyDeviceToHost);
  return nblocks;
}
int optim_fc_fuse() { return 1; }   // (every build since round 6: the fp32 FcFuse / fused tiles)

void launch_target_update(float* dst, const float* src, float tau, const int64_t* step, int freq, int n,
                          float* dst2, const float* src2, int n2, hipStream_t st) {
  const int n4 = n / 4;
  hipLaunchKernelGGL(target_update_kernel, dim3(grid_for(n4)), dim3(256), 0, st, dst, src, tau, step,
                     freq < 1 ? 1 : freq, n4, dst2, src2, n2 / 4);
}

void launch_step_bump(int64_t* step, hipStream_t st) {
  hipLaunchKernelGGL(step_bump_kernel, dim3(1), dim3(1), 0, st, step);
}
