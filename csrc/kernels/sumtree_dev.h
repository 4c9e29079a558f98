// Prioritized-replay sum-tree device code shared by the standalone kernels (sumtree.hip)
// and the optimizer launch's extra block (optim.hip: priority update of this step's batch
// + the next step's prioritized sample, off the critical path).
// Tree layout: f32[2P], root at 1, leaf i at P + i (see replay/sumtree.py).
#pragma once
#include "common.h"
#include "../include/dqn_kernels.h"

namespace dqn {

constexpr int kMaxLevels = 30;

struct SumtreeLds {                 // LDS scratch of the one-wave update
  uint64_t keys[64], sk[64];
  float sv[64];
};

// B <= 64 (the Atari minibatch): ONE wave (wave 0 of the block; the other waves only meet
// the barriers) and no level barriers. Lanes are ranked by (leaf, batch position) through
// LDS, duplicates collapse onto the last batch position (last-writer-wins, as in the
// level-synchronous kernel). Every sibling value the climb needs is loaded up front in one
// batch of independent loads; a sibling that is itself on an updated path is the adjacent
// active lane in sorted order and comes over a lane shuffle instead. Then each level is
// pure ALU + shuffles; stores are fire-and-forget. Every thread of the block must call it.
DQN_DEV void sumtree_update_wave(float* __restrict__ sum, float* __restrict__ mn, float* __restrict__ maxp,
                                 const int32_t* __restrict__ idx, const float* __restrict__ td, float alpha,
                                 float eps, int use_max, int n, int P, int levels, SumtreeLds& L, int first = 0,
                                 int cap = 1, int n_ins = 0, int ins_first = 0, int ins_cap = 1) {
  // idx == nullptr: the n consecutive ring slots (first + lane) % cap.
  // n_ins > 0: lanes [0, n_ins) first insert the ring slots (ins_first + lane) % ins_cap at the
  // running max priority (new transitions), then lanes [n_ins, n_ins + n) are the n entries
  // above -- one climb, same result as the insertion followed by the update (a later batch
  // position wins a shared leaf; the inserted lanes' p = max_p leaves the running max alone).
  const int lane = threadIdx.x;
  const bool w0 = threadIdx.x < 64;
  const bool ins = lane < n_ins;
  const int j = lane - n_ins;
  const bool valid = lane < n_ins + n;
  DQN_ASSERT(n_ins + n <= 64);
  const float mp = maxp[0];
  float p = 0.f;
  if (valid) p = (ins || use_max) ? mp : powf(fabsf(td[j]) + eps, alpha);
  if (w0) {
    if (!use_max) {
      const float m = wave_max(valid ? p : 0.f);
      if (lane == 0) maxp[0] = fmaxf(mp, m);
    }
    // unique keys (the lane breaks ties); padding lanes sort last with leaf field 0xffffffff
    uint32_t li = 0;
    if (ins) li = (uint32_t)((ins_first + lane) % ins_cap);
    else if (valid) li = idx != nullptr ? (uint32_t)idx[j] : (uint32_t)((first + j) % cap);
    L.keys[lane] = ((uint64_t)(valid ? li : 0xffffffffu) << 6) | (uint64_t)lane;
  }
  __syncthreads();
  if (w0) {
    const uint64_t key = L.keys[lane];
    int rank = 0;
    for (int j = 0; j < 64; ++j) rank += L.keys[j] < key ? 1 : 0;
    L.sk[rank] = key;
    L.sv[rank] = p;
  }
  __syncthreads();
  if (w0) {                              // (the other waves only met the barriers)
    const uint64_t k = L.sk[lane];
    const float v0 = L.sv[lane];
    const bool ok = (k >> 6) != 0xffffffffull;
    const int leaf = ok ? (int)(k >> 6) : 0;
    DQN_ASSERT(!ok || leaf < P);
    // last lane of each equal-leaf run = the latest batch position: it owns the leaf
    const uint64_t kn = lane < 63 ? L.sk[lane + 1] : ~0ull;
    bool act = ok && (lane == 63 || (kn >> 6) != (k >> 6));
    int c = P + leaf;
    const int c0 = c;
    float vs = v0, vm = v0;
    if (act) {
      sum[c] = vs;
      mn[c] = vm;
    }
    // siblings are loaded kSibBatch levels at a time (one batch of independent loads per
    // chunk: kMaxLevels registers x2 would cost every block of the host launch occupancy).
    // A sibling that another lane writes during the climb is taken from that lane's shuffle,
    // so a load that raced with its store is never used.
    constexpr int kSibBatch = 10;
    for (int l0 = 0; l0 < kMaxLevels; l0 += kSibBatch) {
      if (l0 >= levels) break;                                  // uniform
      float sib_s[kSibBatch], sib_m[kSibBatch];
  #pragma unroll
      for (int u = 0; u < kSibBatch; ++u) {
        const int l = l0 + u;
        if (l < levels && act) {
          const int sb = (c0 >> l) ^ 1;
          sib_s[u] = sum[sb];
          sib_m[u] = mn[sb];
        } else {
          sib_s[u] = 0.f;
          sib_m[u] = INFINITY;
        }
      }
  #pragma unroll
      for (int u = 0; u < kSibBatch; ++u) {
        const int l = l0 + u;
        if (l >= levels) break;                                 // uniform
        const uint64_t am = __ballot(act);
        // nearest active lanes below / above
        const uint64_t below = am & ((1ull << lane) - 1ull);
        const uint64_t above = lane < 63 ? am & ~((2ull << lane) - 1ull) : 0ull;
        const int lo = below ? 63 - __clzll((long long)below) : lane;
        const int hi = above ? __ffsll((long long)above) - 1 : lane;
        const int nlo = __shfl(c, lo, 64), nhi = __shfl(c, hi, 64);
        const float slo = __shfl(vs, lo, 64), shi = __shfl(vs, hi, 64);
        const float mlo = __shfl(vm, lo, 64), mhi = __shfl(vm, hi, 64);
        const bool right = c & 1;
        const int sib = c ^ 1;
        float os = sib_s[u], om = sib_m[u];
        bool sib_act = false;
        if (right && below && nlo == sib) { os = slo; om = mlo; sib_act = true; }
        if (!right && above && nhi == sib) { os = shi; om = mhi; sib_act = true; }
        const float ps = right ? os + vs : vs + os;
        const float pm = fminf(vm, om);
        // the left sibling of an active pair carries on; the right one retires
        if (right && sib_act) act = false;
        c >>= 1;
        vs = ps;
        vm = pm;
        if (act) {
          sum[c] = vs;
          mn[c] = vm;
        }
      }
    }
  }
}

// Stratified proportional sample of lane i < B: leaf index and max-normalised IS weight
// w = (N p)^-beta / (N p_min)^-beta (+ the per-sample outputs when so.st_slots is set).
DQN_DEV int per_sample_lane(const float* __restrict__ sum, const float* __restrict__ mn, uint64_t seed,
                            uint64_t ctr, int nsize, int i, int B, int P, float beta, int32_t* __restrict__ idx_out,
                            float* __restrict__ w_out, const SampleOut& so) {
  const float total = sum[1];
  u32x4 r = philox(seed ^ 0x5bd1e995ull, ctr, (uint32_t)i, 0x7u);
  float u = ((float)i + u01(r.x)) * (total / (float)B);
  // descent kPerDepth levels per memory round trip: every (left, right) child pair of the
  // kPerDepth-deep subtree under `node` (2^kPerDepth - 1 pairs, one 8-byte load each: the two
  // children are adjacent) is loaded in one batch, then the walk through it is ALU + selects.
  // 20 levels (P = 2^20) take 5 dependent loads instead of 20 (~1 us each from the MALL: the
  // prioritized sampler block was the longest block of Rainbow's optimizer launch). Same
  // decisions as one level at a time, so the same leaves.
  constexpr int kPerDepth = 4, kPairs = (1 << kPerDepth) - 1;
  int node = 1, depth = 0;
  const int L = 31 - __clz(P);                      // log2(P): P is a power of two
  const float2* __restrict__ pairs = reinterpret_cast<const float2*>(sum);   // pairs[n] = (sum[2n], sum[2n+1])
  while (node < P) {
    const int d = min(kPerDepth, L - depth);          // (uniform: every lane descends in step)
    float2 v[kPairs];
#pragma unroll
    for (int r = 0; r < kPerDepth; ++r)
#pragma unroll
      for (int j = 0; j < (1 << r); ++j)
        v[(1 << r) - 1 + j] = r < d ? pairs[(node << r) + j] : make_float2(0.f, 0.f);
    int cur = node;
#pragma unroll
    for (int r = 0; r < kPerDepth; ++r) {
      if (r >= d) break;
      const int j = cur - (node << r);
      float2 c = v[(1 << r) - 1];
#pragma unroll
      for (int q = 1; q < (1 << r); ++q)
        if (j == q) c = v[(1 << r) - 1 + q];
      const bool right = (u >= c.x) && (c.y > 0.f);
      u = right ? u - c.x : u;
      cur = 2 * cur + (right ? 1 : 0);
    }
    node = cur;
    depth += d;
  }
  const int n = max(nsize, 1);
  int leaf = min(node - P, n - 1);
  DQN_ASSERT(leaf >= 0 && node >= P && node < 2 * P);
  idx_out[i] = leaf;
  const float p = sum[P + leaf] / total;
  const float pmin = mn[1] / total;
  w_out[i] = powf((float)n * p, -beta) / powf((float)n * pmin, -beta);
  if (so.st_slots != nullptr) {
    so.a_out[i] = so.actions[leaf];
    so.r_out[i] = so.rewards[leaf];
    so.d_out[i] = so.dones[leaf];
    so.g_out[i] = so.gammas[leaf];
    const int K = so.K;
    for (int c = 0; c < K; ++c) {
      const int v = so.state_idx[(int64_t)leaf * K + c];
      so.st_slots[i * K + c] = v;
      if (c > 0) so.nx_slots[i * K + c - 1] = v;
    }
    so.nx_slots[i * K + K - 1] = so.next_idx[leaf];
  }
  return leaf;
}

}  // namespace dqn
