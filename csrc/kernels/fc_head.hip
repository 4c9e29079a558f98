// Fused fc forward + scalar head ("head fold") for gfx950: ONE launch computes the hidden layer
// h = ReLU(x3 W_fc + b) of every instance AND the output layer, dueling combine, TD loss, dQ and
// the head backward dH -- the work of igemm_kernel<Dense, ..., EPI 0> + head_loss_kernel, whose
// launch boundary and h re-read it removes.
//
// Block = one 16-row x 16-column tile of h for one instance (8 waves: split-K over the 3136-deep
// K, LDS reduce; the igemm fc tiling). Its epilogue stores the bf16 h tile and immediately folds
// it into the output layer: partial Q[r][a] = sum_{16 cols} h[r][c] W2[c][a] (dueling: value tiles
// into column A), one write-through store per value into the tile's own slot of
// [instance][row][32][tile] (the tail sums the slots in tile order: bit-reproducible). Each
// block then arrives on its row group's counter once its write-through h stores and atomics have
// completed (s_waitcnt; no L2 write-back fence); the LAST arriver of a group (acquire) owns that
// group's tail:
//   learner group  Q = acc + b (+ V - mean A), double / plain DQN target, TD error, Huber / MSE,
//                  PER priorities, the per-group loss partial, dQ (act_t rows, the output-layer
//                  weight-gradient dZ) and dH = (dQ W2^T) * (h > 0) over the group's h rows (written
//                  by the other blocks of this launch as write-through stores, read after the acquire);
//   actor group    (fused acting: the actors' states are one more instance, online weights) the
//                  actors' Q rows -> eps-greedy decision + replay append per env, the actor-state
//                  advance, the PER insert; the env frames were written by the group's first E
//                  blocks right after they arrived (they depend on the rng state only).
// The tail resets the counter it used: the next launch starts clean (every slot it reads is
// rewritten by every launch).
// Reference semantics: output layer + TD loss + its gradient, /root/reference/src/network.py:
// 389-424 (layers), src/dqn.py (loss, double DQN); dueling: Wang et al..
#include "common.h"
#include "actor_dev.h"
#include "wgrad_dev.h"
#include "../include/dqn_nets_k.h"

namespace dqn {

constexpr int kFoldThreads = 512;
constexpr int kFoldMaxA = 18;                  // Atari's full action set
constexpr int kFoldMaxHid = 512;
// k-steps per load batch (fp32: twice the VGPRs each). kFoldU1: one block per CU (the whole K slice of a
// wave in one batch); kFoldU2: two blocks per CU (<= 128 VGPRs), for grids above the CU count -- the
// dueling net's 2 x 64 x 3 = 384 blocks, which otherwise lost the spin mode (all blocks resident)
constexpr int kFoldU1 = DQN_ACT_F32 ? 7 : 13, kFoldU2 = DQN_ACT_F32 ? 4 : 8;

struct FoldLds {
  float red[7 * 256];                          // split-K partial tiles of waves 1..7
  float ht[16][17];                            // the tile's h (bf16-rounded, as stored)
  act_t hv[16][16];                            // the tile's h as stored
  float w2t[16 * kFoldMaxA];                   // the tile's rows of the output layer (fold)
  float w2[kFoldMaxHid * kFoldMaxA + kFoldMaxHid];   // tail: online output layer (+ value column)
  float q[3][17][33];                          // tail: Q rows per instance (+ the bias row)
  float dq[16][33];                            // tail: dQ rows (| dV at A)
  int32_t pst[16][4];                          // actor tail: the envs' frame stacks
  int flag;
  int timed_out;                               // dH-tile block: the dQ wait expired
};

template <int AT, int kFoldU>
__global__ void __launch_bounds__(kFoldThreads, kFoldU == kFoldU2 ? 4 : 2) fc_head_kernel(ConvArgs a, HeadArgs h, FoldArgs f) {
  __shared__ __attribute__((aligned(16))) FoldLds S;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int inst = blockIdx.z;
  // phase stamps (probe): 0 start, 1 h tile reduced, 2 fold issued, 3 arrived, 4 tail Q loaded,
  // 5 TD done, 6 tail end
  int64_t* prof = (f.prof != nullptr && tid == 0)
                      ? f.prof + 8 * (((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x)
                      : nullptr;
#define FOLD_MARK(i) if (prof) prof[i] = (int64_t)__builtin_amdgcn_s_memrealtime()
  FOLD_MARK(0);
  if (f.zero_ptr != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0)
    for (int t = threadIdx.x; t < f.zero_n / 4; t += blockDim.x)
      reinterpret_cast<float4*>(f.zero_ptr)[t] = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool actor_inst = h.act_E > 0 && inst == f.nlearn;
  if (actor_inst && blockIdx.x > 0) return;     // the actors' E <= 16 rows: row group 0 only
  const int A = AT > 0 ? AT : h.A, A1 = A + 1;
  const int HID = h.HID, HH = h.dueling ? 2 * HID : HID;
  const int m_base = blockIdx.x * 16, nt = blockIdx.y;
  const int Mi = actor_inst ? h.act_E : a.M;   // valid rows of this instance
  const bool dh_tile = f.spin && !actor_inst && inst == 0;   // this block writes its own dH tile
  // ---- h tile operands: the first k batch is issued BEFORE the loads below (output-layer rows,
  //      biases, TD inputs, epoch / actor words): the LDS staging of those waits for its data, and
  //      with the fragments issued after it the block paid two round trips before its first MFMA
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  DenseLoader ld(a, inst, m_base + (lane & 15));
  const bfx8* __restrict__ Bp = reinterpret_cast<const bfx8*>(a.w[inst]);
  const int K32 = (a.K + 31) / 32, kg = 8 * (lane >> 4);
  const int ks_lo = (K32 * wave) / 8, ks_hi = (K32 * (wave + 1)) / 8;
  bfx8 af[kFoldU], bf[kFoldU];
  auto load_batch = [&](int ks) {
#pragma unroll
    for (int u = 0; u < kFoldU; ++u) {
      const bool kok = ks + u < ks_hi;
      af[u] = kok ? ld.frag((ks + u) * 32 + kg) : zero8();
      bf[u] = kok ? Bp[((int64_t)(ks + u) * a.N16 + nt) * 64 + lane] : zero8();
    }
  };
  load_batch(ks_lo);
  int e0 = 0;                                   // the group's dQ epoch before this launch's tail
  if (dh_tile) e0 = __hip_atomic_load(f.dq_epoch + blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool frames_duty = actor_inst && nt < h.act_E;
  // the frame duty's rng / cursor words (before the arrival: the tail advances them); scalars,
  // not an ActorPre (whose per-thread stack array put 88 bytes per lane in scratch)
  int64_t pf0 = 0, pseed = 0, pctr = 0;
  if (frames_duty) {
    pf0 = h.actor.cursor[1];
    pseed = h.actor.rng[0];
    pctr = h.actor.rng[1];
  }
  // the tile's 16 rows of the output layer (advantage / plain [16][A], or the 16 value weights),
  // staged now: their loads complete under the k-loop instead of after it
  const int wi = actor_inst ? 0 : inst;        // output-layer weights of the instance
  const bool vtile = h.dueling && nt * 16 < HID;
  const int k0 = h.dueling && !vtile ? nt * 16 - HID : nt * 16;
  if (tid < (vtile ? 16 : 16 * A)) S.w2t[tid] = vtile ? h.wv[wi][k0 + tid] : h.w[wi][(int64_t)k0 * A + tid];
  // what the group's tail reads besides the other blocks' results, loaded now by every block (any
  // block may turn out to be the last arriver): the output-layer biases of the group's instances
  // and the TD inputs of its rows
  float pb = 0.f;                               // bias of (instance tid / 32, column tid % 32)
  {
    const int ni_ = actor_inst ? 1 : f.nlearn, i = tid >> 5, c = tid & 31;
    if (i < ni_) {
      const int bw = actor_inst ? 0 : i;
      pb = c < A ? h.b[bw][c] : (c == A && h.dueling ? h.bv[bw][0] : 0.f);
    }
  }
  float tr = 0.f, tg = 0.f, tdn = 0.f, tw = 1.f;
  int ta = 0;
  if (!actor_inst && tid < 16 && m_base + tid < a.M) {
    const int b = m_base + tid;
    tr = h.rew[b]; tg = h.gam[b]; tdn = h.done[b]; ta = h.act[b];
    if (h.wts != nullptr) tw = h.wts[b];
  }

  // ---- h tile: split-K over 8 waves (igemm_kernel's Dense 1x1x1x1x8 tiling); batch 1 is in flight
  for (int ks = ks_lo; ks < ks_hi; ks += kFoldU) {
    if (ks != ks_lo) load_batch(ks);
#pragma unroll
    for (int u = 0; u < kFoldU; ++u) acc = mfma16(af[u], bf[u], acc);
  }
  if (wave > 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) S.red[(wave - 1) * 256 + r * 64 + lane] = acc[r];
  }
  __syncthreads();
  FOLD_MARK(1);
  if (wave == 0) {
#pragma unroll
    for (int s = 0; s < 7; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += S.red[s * 256 + r * 64 + lane];
    // epilogue: C/D layout col = lane & 15, row = 4 * (lane >> 4) + r
    const int col = lane & 15, n = nt * 16 + col;
    const float scale = a.scale[inst], bv = a.bias[inst][n];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * (lane >> 4) + r, m = m_base + row;
      const act_t v = (act_t)fmaxf(acc[r] * scale + bv, 0.f);
      S.hv[row][col] = v;
      S.ht[row][col] = m < Mi ? (float)v : 0.f;
    }
  }
  __syncthreads();
  // the h tile leaves as write-through 32-bit stores (agent scope, relaxed): the group's tail
  // reads it from another CU / XCD after the counter, with no L2 write-back fence on this side
  {
    constexpr int kPer = 4 / (int)sizeof(act_t);             // act_t per 32-bit word
    constexpr int kWords = 16 * 16 / kPer;
    if (tid < kWords) {
      const int row = tid / (16 / kPer), c0 = (tid - row * (16 / kPer)) * kPer, m = m_base + row;
      if (m < a.M) {
        uint32_t wv;
        __builtin_memcpy(&wv, &S.hv[row][c0], 4);
        uint32_t* dst = reinterpret_cast<uint32_t*>(reinterpret_cast<act_t*>(a.out[inst]) + (int64_t)m * a.ldo +
                                                    nt * 16 + c0);
        __hip_atomic_store(dst, wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  // ---- fold: partial output layer of this tile (value tiles: the first HID units, dueling)
  {
    if (tid < 16 * A1) {
      const int row = tid / A1, c = tid - row * A1;
      const bool mine = vtile ? c == A : c < A;
      if (mine && m_base + row < Mi) {
        float s = 0.f;
        if (vtile) {
#pragma unroll
          for (int j = 0; j < 16; ++j) s += S.ht[row][j] * S.w2t[j];
        } else {
#pragma unroll
          for (int j = 0; j < 16; ++j) s += S.ht[row][j] * S.w2t[j * A + c];
        }
        // this tile's partial, a write-through store into its own slot: the tail sums the slots
        // in a fixed order (bit-reproducible, no fp32 atomics)
        __hip_atomic_store(f.qacc + (((int64_t)inst * f.Mpad + m_base + row) * 32 + c) * gridDim.y + nt, s,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  // ---- arrival: this block's write-through h stores and Q atomics are complete (no L2 write-
  //      back fence: a buffer_wbl2 per wave of every block measured ~40 us for the launch), count;
  //      the last arriver goes on
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  FOLD_MARK(2);
  const int grp = actor_inst ? f.ngroups : (int)blockIdx.x;
  if (tid == 0) {
    const int target = actor_inst ? (int)gridDim.y : f.nlearn * (int)gridDim.y;
    const int old = __hip_atomic_fetch_add(f.cnt + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    S.flag = old == target - 1 ? 1 : 0;
    FOLD_MARK(3);
  }
  __syncthreads();
  if (frames_duty) {                                         // env nt's new frame(s): rng only
    ActorPre pre{};
    pre.f0 = pf0;
    pre.seed = (uint64_t)pseed;
    pre.ctr = (uint64_t)pctr;
    actor_env_frames(h.actor, nt, pre);
  }
  // dH tile of this block from the group's dQ rows: (dQ W2^T)[rows][the tile's 16 units] * (h > 0)
  auto dh_from = [&](const float (*dq)[33]) {
    if (tid < 256) {
      const int r = tid >> 4, j = tid & 15;
      if (r < min(16, a.M - m_base)) {
        float sacc;
        if (vtile) {
          sacc = dq[r][A] * S.w2t[j];
        } else {
          sacc = 0.f;
          if constexpr (AT > 0) {
#pragma unroll
            for (int i = 0; i < AT; ++i) sacc += dq[r][i] * S.w2t[j * AT + i];
          } else {
            for (int i = 0; i < A; ++i) sacc += dq[r][i] * S.w2t[j * A + i];
          }
        }
        reinterpret_cast<act_t*>(h.dh)[(int64_t)(m_base + r) * HH + nt * 16 + j] =
            (act_t)((float)S.hv[r][j] > 0.f ? sacc * kLossScale : 0.f);
      }
    }
  };
  if (!S.flag) {
    if (!dh_tile) return;
    // wait for the group's tail to publish dQ (every block of the launch is resident: spin mode)
    // (no acquire fence here: an L2 invalidation per waiting block costs the next launches their
    //  cached weights; the dQ rows are read with agent-scope loads, coherent like the stores)
    if (tid == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      S.timed_out = 0;
      while (__hip_atomic_load(f.dq_epoch + blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == e0) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {      // 1 s: never hang, never
          S.timed_out = 1;                                                 // train on stale dQ
          if (f.err != nullptr)
            __hip_atomic_store(f.err, 0x1000000 | (int)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    // timed out (flagged: the learner's device check raises): the tile is written as ZEROS -- the
    // group then adds nothing to this step's gradient, instead of the previous step's stale dH
    const int nr = S.timed_out ? 0 : min(16, a.M - m_base);
    for (int t = tid; t < 16 * A1; t += kFoldThreads) {
      const int r = t / A1, c = t - r * A1;
      S.dq[r][c] = r < nr ? __hip_atomic_load(f.dqg + (int64_t)(m_base + r) * 32 + c, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT)
                          : 0.f;
    }
    __syncthreads();
    dh_from(S.dq);
    return;
  }
  if (tid == 0) {
    // acquire, then plain loads of the partial-Q slots (and, not spin, the other blocks' h rows).
    // (round 5 measured sc1 slot loads without the fence 0.3-0.6 us slower, gpurun_out/r5v: removed)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(f.cnt + grp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();

  // ---- tail: every load it needs is issued at once -- the online h rows (dH mask, registers),
  //      the online output layer (LDS) and the group's partial-Q slots -- then Q, biases, dueling
  const int ni = actor_inst ? 1 : f.nlearn;
  const int i0 = actor_inst ? f.nlearn : 0;
  const int nrows = min(16, Mi - m_base);
  const int nch = HH / 8;                        // 8-unit chunks per h row
  constexpr int kHc = 2 * kFoldMaxHid * 16 / 8 / kFoldThreads;   // chunks per thread (<= 4)
  const act_t* h0 = reinterpret_cast<const act_t*>(h.h[0]);
  bfx8 hvr[kHc];
  if (!actor_inst && !f.spin) {
#pragma unroll
    for (int u = 0; u < kHc; ++u) {
      const int t = tid + u * kFoldThreads, r = t / nch;
      hvr[u] = r < nrows ? *reinterpret_cast<const bfx8*>(h0 + (int64_t)(m_base + r) * HH + (t - r * nch) * 8)
                         : zero8();
    }
    for (int t = tid; t < HID * A; t += kFoldThreads) S.w2[t] = h.w[0][t];
    if (h.dueling)
      for (int t = tid; t < HID; t += kFoldThreads) S.w2[HID * A + t] = h.wv[0][t];
  }
  {
    // Q rows: every (instance, row, column) sums its tiles' partial slots in tile order (dueling:
    // advantage columns over the advantage tiles, the value column over the value tiles), + bias
    const int NT = (int)gridDim.y, half = h.dueling ? NT / 2 : 0;
    if (tid < ni * 32) S.q[tid >> 5][16][tid & 31] = pb;          // (row 16: the bias row)
    for (int t = tid; t < ni * 16 * A1; t += kFoldThreads) {
      const int i = t / (16 * A1), rem = t - i * 16 * A1, r = rem / A1, c = rem - r * A1;
      float v = 0.f;
      if (r < nrows && (c < A || h.dueling)) {
        const int pb0 = 4 * (int)((((int64_t)(i0 + i) * f.Mpad + m_base + r) * 32 + c) * NT);   // byte offset
        const int lo = h.dueling ? (c < A ? half : 0) : 0, hi = h.dueling ? (c < A ? NT : half) : NT;
        const float* p = f.qacc + pb0 / 4;         // (summed in tile order)
        for (int u = lo; u < hi; u += 4) {
          const float4 x = *reinterpret_cast<const float4*>(p + u);
          v += x.x;
          v += x.y;
          v += x.z;
          v += x.w;
        }
      }
      S.q[i][r][c] = v;
    }
  }
  FOLD_MARK(4);
  __syncthreads();
  if (tid < ni * 16) {
    const int i = tid >> 4, r = tid & 15;
    float* q = S.q[i][r];
    const float* bq = S.q[i][16];
    for (int c = 0; c < A; ++c) q[c] += bq[c];
    if (h.dueling) {
      const float v = q[A] + bq[A];
      float mean = 0.f;
      for (int c = 0; c < A; ++c) mean += q[c];
      mean /= (float)A;
      for (int c = 0; c < A; ++c) q[c] += v - mean;
    }
  }
  __syncthreads();

  if (actor_inst) {
    // ---- fused acting: decision + replay append per env, state advance, PER insert
    const ActorArgs& x = h.actor;
    const ActorPre p = actor_prefetch(x);
    // (env e's stack through LDS: a pointer into the private ActorPre::st would put it in scratch)
    if (tid < x.E)
      for (int c2 = 0; c2 < 4; ++c2) S.pst[tid][c2] = p.st[c2];
    for (int e = tid; e < x.E; e += kFoldThreads) {
      int fs, rs;
      actor_env_step(x, S.q[0][e], e, p.t0, p.f0, p.eps0, p.eps_min, p.decay, p.seed, p.ctr, fs, rs, S.pst[e]);
    }
    if (tid == 0) actor_advance(x, p.t0, p.f0, p.size0, p.eps0, p.eps_min, p.decay, p.ctr, p.frames_done);
    if (x.tsum != nullptr)
      sumtree_update_wave(x.tsum, x.tmin, x.tmaxp, nullptr, nullptr, 0.f, 0.f, 1, x.E, x.tP, x.tlevels,
                          *reinterpret_cast<SumtreeLds*>(S.w2), (int)(p.t0 % x.C), x.C);
    return;
  }

  // ---- learner: TD target, loss, dQ, priorities (thread per row)
  float contrib = 0.f;
  if (tid < nrows) {
    const int b = m_base + tid;
    const float td = tdn;
    const float* sel = S.q[f.nlearn == 3 ? 2 : 1][tid];
    int best = 0;
    float bvv = sel[0];
#pragma unroll
    for (int i = 1; i < (AT > 0 ? AT : 32); ++i)
      if ((AT > 0 || i < A) && sel[i] > bvv) { bvv = sel[i]; best = i; }
    const float nxt = S.q[1][tid][best];
    const float y = tr + tg * (1.f - td) * nxt;
    const float d = S.q[0][tid][ta] - y;
    float per, dper;
    if (h.huber) {
      const float ad = fabsf(d);
      per = ad <= h.delta ? 0.5f * d * d : h.delta * (ad - 0.5f * h.delta);
      dper = ad <= h.delta ? d : copysignf(h.delta, d);
    } else {
      per = d * d;
      dper = 2.f * d;
    }
    contrib = tw * per;
    const float gsc = tw * dper / (float)h.B;
    // Q_i = V + A_i - mean(A): dV = sum_i dQ_i, dA_i = dQ_i - mean(dQ)
    const float sub = h.dueling ? gsc / (float)A : 0.f;
    for (int i = 0; i < A; ++i) S.dq[tid][i] = ((i == ta) ? gsc : 0.f) - sub;
    S.dq[tid][A] = h.dueling ? gsc : 0.f;
    h.prio[b] = fabsf(d);
  }
  if (wave == 0) {
    const float sum = wave_sum(contrib);
    if (lane == 0) h.loss_parts[blockIdx.x] = sum;       // summed by the fc dgrad launch
  }
  FOLD_MARK(5);
  __syncthreads();
  if (f.spin && !f.dbg_no_publish) {
    // publish the group's dQ rows (write-through), then its epoch: the online blocks waiting on it
    // write their dH tiles (this block too, when it is one of them)
    const int g = (int)blockIdx.x;
    for (int t = tid; t < nrows * A1; t += kFoldThreads) {
      const int r = t / A1, c = t - r * A1;
      __hip_atomic_store(f.dqg + (int64_t)(m_base + r) * 32 + c, S.dq[r][c], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int e = __hip_atomic_load(f.dq_epoch + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(f.dq_epoch + g, e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (dh_tile) dh_from(S.dq);
  }
  for (int t = tid; t < nrows * 64; t += kFoldThreads) {
    const int r = t >> 6, c = t & 63;
    const float g = c < A ? S.dq[r][c] : (c == 32 && h.dueling ? S.dq[r][A] : 0.f);
    reinterpret_cast<act_t*>(h.dq16)[(int64_t)(m_base + r) * 64 + c] = (act_t)(g * kLossScale);
  }
  if (h.q_out != nullptr)
    for (int t = tid; t < nrows * A; t += kFoldThreads) h.q_out[(int64_t)m_base * A + t] = S.q[0][t / A][t % A];
  // ---- dH[row][k] = (sum_i dQ[row][i] W[k][i]) * (h > 0) (dueling: value units dV wv[k]) over the
  //      group's online h rows (8 units per thread)
  act_t* dh = reinterpret_cast<act_t*>(h.dh);
  if (!f.spin) {
#pragma unroll
  for (int u = 0; u < kHc; ++u) {
    const int t = tid + u * kFoldThreads;
    if (t >= nrows * nch) break;
    const int r = t / nch, k0 = (t - r * nch) * 8;
    const int64_t o = (int64_t)(m_base + r) * HH + k0;
    const bfx8 hv = hvr[u];
    const float* g = S.dq[r];
    bfx8 out;
    if (h.dueling && k0 < HID) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        out[j] = (act_t)((float)hv[j] > 0.f ? g[A] * S.w2[HID * A + k0 + j] * kLossScale : 0.f);
    } else {
      const int kk = h.dueling ? k0 - HID : k0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float* w = S.w2 + (kk + j) * A;
        float s = 0.f;
        if constexpr (AT > 0) {
#pragma unroll
          for (int i = 0; i < AT; ++i) s += g[i] * w[i];
        } else {
          for (int i = 0; i < A; ++i) s += g[i] * w[i];
        }
        out[j] = (act_t)((float)hv[j] > 0.f ? s * kLossScale : 0.f);
      }
    }
    *reinterpret_cast<bfx8*>(dh + o) = out;
  }
  }
  if (prof) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FOLD_MARK(6);
  }
#undef FOLD_MARK
}

}  // namespace dqn

using namespace dqn;

int launch_fc_head(const ConvArgs& a, const HeadArgs& h, const FoldArgs& f, hipStream_t st) {
  const int ninst = f.nlearn + (h.act_E > 0 ? 1 : 0);
  if (h.A > kFoldMaxA || h.HID > kFoldMaxHid || h.act_E > 16 || a.N % 128 != 0 ||
      a.N != (h.dueling ? 2 * h.HID : h.HID) || f.ngroups != (a.M + 15) / 16 || f.Mpad < 16 * f.ngroups ||
      (f.nlearn != 2 && f.nlearn != 3) || ninst > kMaxInst)
    return -1;
  const dim3 grid((a.M + 15) / 16, a.N / 16, ninst);
  // spin mode needs every block resident at once: one per CU with the one-batch k-loop, two per CU
  // (LDS 58 KB, <= 128 VGPRs) with the two-batch variant; beyond that the tails write the whole dH
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const int nblk = (int)(grid.x * grid.y * grid.z);
  const bool two = f.two_per_cu && nblk > cus && nblk <= 2 * cus;
  if (f.spin && nblk > (two ? 2 * cus : cus)) {
    FoldArgs g = f;
    g.spin = 0;
    return launch_fc_head(a, h, g, st);
  }
  if (f.spin && (f.dqg == nullptr || f.dq_epoch == nullptr)) return -1;
#define FOLD(AT)                                                                                             \
  do {                                                                                                      \
    if (two) hipLaunchKernelGGL((fc_head_kernel<AT, kFoldU2>), grid, dim3(kFoldThreads), 0, st, a, h, f);   \
    else hipLaunchKernelGGL((fc_head_kernel<AT, kFoldU1>), grid, dim3(kFoldThreads), 0, st, a, h, f);       \
  } while (0)
  switch (h.A) {
    case 2: FOLD(2); break;
    case 3: FOLD(3); break;
    case 4: FOLD(4); break;
    case 6: FOLD(6); break;
    case 9: FOLD(9); break;
    case 18: FOLD(18); break;
    default: FOLD(0); break;
  }
#undef FOLD
  return 0;
}
