// Peer-to-peer signalling over xGMI shared by the all-reduce / all-gather kernels
// (xgmi_ar.hip) and the fc dgrad launch's gather side duty (qnet.hip): system-scope release
// stores into the peers' signal words, bounded acquire polls of one's own.
#pragma once
#include "common.h"
#include "../include/dqn_kernels.h"

namespace dqn {

constexpr uint64_t kXgmiTimeoutTicks = 1000000000ull;   // 10 s at 100 MHz

DQN_DEV uint32_t load_acq(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
DQN_DEV void store_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// publish this block's writes, then raise flag `val` for block b in every peer's signal words
DQN_DEV void signal_all(const XgmiArgs& a, int b, uint32_t val) {
  __threadfence_system();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world) store_rel(a.sig[t] + a.rank * kXgmiMaxBlocks + b, val);
}

// Which wait of which call timed out (the error word's first report wins; err[1..3] then hold the
// expected flag value, the value last seen and the call's per-block counter):
//   err[0] = 1 << 31 | phase << 24 | peer << 16 | block
// (kXgmiPhaseDpx: the in-launch gradient exchange of the fused update, optim_pack.h; block = job slot)
constexpr int kXgmiPhaseReduceScatter = 1, kXgmiPhaseAllGather = 2, kXgmiPhaseGather = 3, kXgmiPhaseDpx = 4;

// wait until every peer raised flag >= val for block b; false on timeout
DQN_DEV bool wait_all(const XgmiArgs& a, int b, uint32_t val, int phase) {
  const int t = threadIdx.x;
  __shared__ int timed_out;
  if (t == 0) timed_out = 0;
  __syncthreads();
  if (t < a.world) {
    const uint32_t* f = a.sig[a.rank] + t * kXgmiMaxBlocks + b;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t seen;
    while ((int32_t)((seen = load_acq(f)) - val) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kXgmiTimeoutTicks) {
        const int code = (int)(0x80000000u | ((uint32_t)phase << 24) | ((uint32_t)t << 16) | (uint32_t)b);
        if (atomicCAS(a.err, 0, code) == 0) {
          a.err[1] = (int)val;
          a.err[2] = (int)seen;
          a.err[3] = (int)a.seq[b];
        }
        timed_out = 1;
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");    // system-scope acquire for every thread
  return timed_out == 0;
}


// All-gather of two segments (one signal per call): A  my segments -> my staging, signal
// "A done" (k + 1); C  every PEER's chunk b -> out[s] + q * bytes[s] from its staging, my own chunk
// straight from my segments (no round trip through the uncached staging; W = 1: no staging, no
// signal at all). Block b of every rank handles chunk b of the concatenated payload, so it waits
// only for block b of its peers. Staging alternates parity per call: a rank writes parity p again
// at call k + 2 only after every peer signalled A of call k + 1, i.e. finished reading call k.
DQN_DEV void xgmi_gather_block(const XgmiGatherArgs& g, int b, int G) {
  const XgmiArgs& a = g.x;
  const int t = threadIdx.x, NT = blockDim.x;
  const int W = a.world, r = a.rank;
  const uint32_t k = a.seq[b];
  const long par = (long)(k & 1u);
  auto stage = [&](int q) -> uint4* { return reinterpret_cast<uint4*>(reinterpret_cast<char*>(a.data[q]) + par * a.cap); };
  const long v0 = g.bytes[0] / 16, v1 = g.bytes[1] / 16, nv = v0 + v1;
  const long per = (nv + G - 1) / G;
  const long lo = per * b < nv ? per * b : nv;
  const long hi = per * (b + 1) < nv ? per * (b + 1) : nv;
  DQN_ASSERT(16 * nv <= a.cap && b < kXgmiMaxBlocks);
  const uint4* s0 = reinterpret_cast<const uint4*>(g.src[0]);
  const uint4* s1 = reinterpret_cast<const uint4*>(g.src[1]);
  uint4* o0 = reinterpret_cast<uint4*>(g.out[0]);
  uint4* o1 = reinterpret_cast<uint4*>(g.out[1]);
  if (W > 1) {
    uint4* mine = stage(r);
    for (long v = lo + t; v < hi; v += NT) mine[v] = v < v0 ? s0[v] : s1[v - v0];
    signal_all(a, b, k + 1u);
    if (!wait_all(a, b, k + 1u, kXgmiPhaseGather)) return;
  }
  for (long v = lo + t; v < hi; v += NT) {
    for (int d = 0; d < W; ++d) {
      const int q = (r + d) % W;                      // stagger peers across links (d = 0: my own rows)
      const uint4 x = d == 0 ? (v < v0 ? s0[v] : s1[v - v0]) : stage(q)[v];
      if (v < v0) o0[(long)q * v0 + v] = x;
      else o1[(long)q * v1 + (v - v0)] = x;
    }
  }
  if (t == 0) a.seq[b] = k + 1u;
}


// The data-parallel exchange of the fused update launch (optim_pack.h kModeDp) for one job slot: this
// thread's 4 values v of the slot's gradient are pushed into row `rank` of every PEER's inbox (remote
// xGMI stores, posted), published (system-scope fence + release flag store into every peer's signal
// word of the slot), then every peer's flag is awaited in my own signal words (local polls, bounded:
// the error word on expiry, no hang) and the W rows are summed in rank order -- the peers' from my
// inbox, mine from registers: the same bytes in the same order on every rank, so the replicas stay
// bit-identical. W = 1: v itself, no traffic. Inbox parity alternates per call of a slot: a rank
// reaches call k + 2 of a slot only after every peer flagged call k + 1, i.e. finished reading call k
// (stream order). Every thread of the block calls it (two barriers); `live`: this thread holds an
// element (the others neither push nor read).
DQN_DEV float4 dpx_sum(const DpExchange& X, int slot, int t, float4 v, bool live) {
  const int W = X.world, r = X.rank;
  if (W == 1) return v;
  const uint32_t k = X.seq[slot];
  const long stride = (long)X.slots * kDpxSlotElems;                    // one source rank's rows
  const long base = (long)(k & 1u) * W * stride + (long)slot * kDpxSlotElems + 4 * t;
  if (live) {
    for (int q = 1; q < W; ++q) {
      const int d = r + q < W ? r + q : r + q - W;                      // (peers staggered across links)
      *reinterpret_cast<float4*>(X.inbox[d] + base + (long)r * stride) = v;
    }
  }
  __threadfence_system();
  __syncthreads();
  if (t < W && t != r) store_rel(X.sig[t] + r * kDpxMaxSlots + slot, k + 1u);
  if (t < W && t != r) {
    const uint32_t* f = X.sig[r] + t * kDpxMaxSlots + slot;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t seen;
    while ((int32_t)((seen = load_acq(f)) - (k + 1u)) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kXgmiTimeoutTicks) {
        const int code = (int)(0x80000000u | ((uint32_t)kXgmiPhaseDpx << 24) | ((uint32_t)t << 16) | (uint32_t)slot);
        if (atomicCAS(X.err, 0, code) == 0) {
          X.err[1] = (int)(k + 1u);
          X.err[2] = (int)seen;
          X.err[3] = (int)k;
        }
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");                     // system scope, every thread
  const float* in = X.inbox[r] + base;
  float4 acc = (r == 0 || !live) ? v : *reinterpret_cast<const float4*>(in);
  for (int q0 = 1; q0 < W; q0 += 2) {                                 // 2 rows in flight, summed in order
    float4 x[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = q0 + u < W ? q0 + u : 0;
      x[u] = (q == r || !live) ? v : *reinterpret_cast<const float4*>(in + (long)q * stride);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (q0 + u >= W) break;
      acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w;
    }
  }
  if (t == 0) X.seq[slot] = k + 1u;                 // (every thread read it before the barriers)
  return acc;
}

}  // namespace dqn
