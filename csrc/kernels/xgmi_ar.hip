// Peer-to-peer gradient all-reduce over xGMI (reference message M3, the per-step
// gradient push of the async PS, /root/reference/src/network.py:198-202, here a
// synchronous sum across data-parallel ranks).
//
// Every rank owns one fine-grained (uncached) HBM region, IPC-mapped into every
// peer: [signal words][staging, 2 parities]. One launch does a two-shot all-reduce
// entirely with direct loads over the point-to-point xGMI mesh:
//   A  copy (fp32 or bf16) my gradient into my staging buffer, signal "A done"
//   B  reduce-scatter: my 1/W slice = sum over ranks of their staging slice, written
//      back to my gradient and to my staging slice, signal "B done"
//   C  all-gather: every other slice is read from its owner's staging buffer
// so each link carries 2*S/W bytes (S = message bytes) instead of a ring's 2(W-1)
// latency hops, and the kernel is an ordinary launch: it is captured in the learner's
// HIP graph with no host involvement.
//
// Synchronisation is per block: block b of every rank handles the same chunk of every
// slice, so block b only waits for block b of its peers (no grid barrier, no
// co-residency requirement beyond "each rank eventually runs block b"). Flags are
// monotonically increasing per-block sequence numbers (2k+1 after A, 2k+2 after B of
// call k), written with system-scope release stores into the PEER's signal words and
// polled with system-scope acquire loads. Staging alternates parity per call, so a
// slow peer still reading call k's staging never sees call k+1's writes (a rank can
// only reach call k+2 after every peer passed A of call k+1).
// Every spin has a wall-clock bound (s_memrealtime, 100 MHz): on expiry the block sets
// the error word and returns instead of hanging the GPU; the host checks the word.
#include "common.h"
#include "../include/dqn_kernels.h"
#include "xgmi_dev.h"

namespace dqn {

namespace {

constexpr int kThreads = 256;
struct F4 { float x, y, z, w; };

template <bool BF16>
DQN_DEV void put4(void* stage, long v, F4 f) {
  if constexpr (BF16) {
    uint2 u;
    u.x = (uint32_t)f2bf(f.x) | ((uint32_t)f2bf(f.y) << 16);
    u.y = (uint32_t)f2bf(f.z) | ((uint32_t)f2bf(f.w) << 16);
    reinterpret_cast<uint2*>(stage)[v] = u;
  } else {
    reinterpret_cast<float4*>(stage)[v] = make_float4(f.x, f.y, f.z, f.w);
  }
}

template <bool BF16>
DQN_DEV F4 get4(const void* stage, long v) {
  if constexpr (BF16) {
    const uint2 u = reinterpret_cast<const uint2*>(stage)[v];
    return F4{bf2f((uint16_t)(u.x & 0xffff)), bf2f((uint16_t)(u.x >> 16)), bf2f((uint16_t)(u.y & 0xffff)),
              bf2f((uint16_t)(u.y >> 16))};
  } else {
    const float4 q = reinterpret_cast<const float4*>(stage)[v];
    return F4{q.x, q.y, q.z, q.w};
  }
}

template <bool BF16>
DQN_DEV F4 round_wire(F4 f) {           // the value every rank ends with: wire precision
  if constexpr (BF16) {
    return F4{bf2f(f2bf(f.x)), bf2f(f2bf(f.y)), bf2f(f2bf(f.z)), bf2f(f2bf(f.w))};
  } else {
    return f;
  }
}

// WC: compile-time world size (0: runtime) so the per-peer loads of phases B/C are
// unrolled and all in flight at once (remote xGMI loads are ~1 us round trips)
template <bool BF16, int WC>
__global__ __launch_bounds__(kThreads) void xgmi_allreduce_kernel(XgmiArgs a) {
  const int b = blockIdx.x, G = gridDim.x, t = threadIdx.x;
  const int W = WC ? WC : a.world, r = a.rank;
  const uint32_t k = a.seq[b];                       // calls completed by this block
  const int par = (int)(k & 1u);
  const long esz = BF16 ? 2 : 4;
  auto stage = [&](int q) -> char* { return reinterpret_cast<char*>(a.data[q]) + (long)par * a.cap * esz; };
  // float4 vector i of the reduced vector (ranged: the concatenation of a.nr pieces of a.grad).
  // rc: the caller's range cursor -- every thread walks increasing i within a slice, so the
  // cursor only moves forward (amortised O(1) per vector instead of a scan of the ranges)
  auto first_range = [&](long i) -> int {          // (block-uniform: the start of a block's chunk)
    int q = 0;
    while (q + 1 < a.nr && 4 * i >= a.rpre[q + 1]) ++q;
    return q;
  };
  auto gv = [&](long i, int& rc) -> float4* {
    if (a.nr <= 0) return reinterpret_cast<float4*>(a.grad) + i;
    const long e = 4 * i;
    while (rc + 1 < a.nr && e >= a.rpre[rc + 1]) ++rc;
    return reinterpret_cast<float4*>(a.grad + a.rlo[rc] + (e - a.rpre[rc]));
  };
  const long nv = a.n / 4;                           // float4 vectors (host: n % (4 W) == 0)
  const long sv = nv / W;                            // vectors per slice
  // block b's share of every slice: [lo, hi) in slice-local vector units
  const long per = (sv + G - 1) / G;
  const long lo = per * b < sv ? per * b : sv;
  const long hi = per * (b + 1) < sv ? per * (b + 1) : sv;
  DQN_ASSERT(a.n % (4L * W) == 0 && a.n <= a.cap && b < kXgmiMaxBlocks);

  // ---- A: my gradient -> my staging (all slices, block b's chunk of each)
  char* mine = stage(r);
  for (int s = 0; s < W; ++s) {
    int rc = first_range((long)s * sv + lo);
    for (long v = lo + t; v < hi; v += kThreads) {
      const long i = (long)s * sv + v;
      const float4 g = *gv(i, rc);
      put4<BF16>(mine, i, F4{g.x, g.y, g.z, g.w});
    }
  }
  signal_all(a, b, 2u * k + 1u);
  if (!wait_all(a, b, 2u * k + 1u, kXgmiPhaseReduceScatter)) return;

  // ---- B: reduce my slice over all ranks' staging (fixed rank order: identical sums everywhere)
  int rcb = first_range((long)r * sv + lo);
  for (long v = lo + t; v < hi; v += kThreads) {
    const long i = (long)r * sv + v;
    F4 acc{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < (WC ? WC : kXgmiMaxRanks); ++q) {
      if (!WC && q >= W) break;
      const F4 x = get4<BF16>(stage(q), i);
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    }
    acc = round_wire<BF16>(acc);
    put4<BF16>(mine, i, acc);
    *gv(i, rcb) = make_float4(acc.x, acc.y, acc.z, acc.w);
  }
  signal_all(a, b, 2u * k + 2u);
  if (!wait_all(a, b, 2u * k + 2u, kXgmiPhaseAllGather)) return;

  // ---- C: gather the other slices from their owners (one range cursor per peer slice)
  int rcs[WC ? WC : kXgmiMaxRanks];
#pragma unroll
  for (int d = 1; d < (WC ? WC : kXgmiMaxRanks); ++d)
    rcs[d] = (!WC && d >= W) ? 0 : first_range((long)((r + d) % W) * sv + lo);
  for (long v = lo + t; v < hi; v += kThreads) {
#pragma unroll
    for (int d = 1; d < (WC ? WC : kXgmiMaxRanks); ++d) {
      if (!WC && d >= W) break;
      const int q = (r + d) % W;                      // stagger peers across links
      const long i = (long)q * sv + v;
      const F4 x = get4<BF16>(stage(q), i);
      *gv(i, rcs[d]) = make_float4(x.x, x.y, x.z, x.w);
    }
  }
  if (t == 0) a.seq[b] = k + 1u;
}

// All-gather of two segments: xgmi_dev.h xgmi_gather_block (also run as a side duty of the
// fc dgrad launch, qnet.hip), one block per chunk
__global__ __launch_bounds__(kThreads) void xgmi_allgather_kernel(XgmiGatherArgs g) {
  xgmi_gather_block(g, blockIdx.x, gridDim.x);
}

// Self-test of the update exchange (xgmi_dev.h dpx_sum), the exact protocol of the fused update's
// dependent jobs: block = slot, 512 threads x 4 values, v = rank-stamped small integers (exact in
// fp32), the sum written to out[slot][2048]; thread t of a slot is live unless (t + slot) % 7 == 0
// (dead lanes neither push nor read, as the partial tiles' outside lanes).
__global__ __launch_bounds__(512) void dpx_selftest_kernel(DpExchange x, float* out, int call) {
  const int s = blockIdx.x, t = threadIdx.x;
  const float base = (float)((s * 512 + t) % 97 + call);
  const float4 v = make_float4(base + x.rank, base + 2 * x.rank, base + 3 * x.rank, base + 4 * x.rank);
  const bool live = (t + s) % 7 != 0;
  const float4 r = dpx_sum(x, s, t, v, live);
  if (live) reinterpret_cast<float4*>(out + (long)s * kDpxSlotElems)[t] = r;
}

}  // namespace

}  // namespace dqn

int launch_xgmi_allgather(const dqn::XgmiGatherArgs& g, int blocks, hipStream_t st) {
  const dqn::XgmiArgs& a = g.x;
  if (blocks < 1 || blocks > dqn::kXgmiMaxBlocks || a.world < 1 || a.world > dqn::kXgmiMaxRanks) return 1;
  if (g.bytes[0] % 16 != 0 || g.bytes[1] % 16 != 0 || g.bytes[0] + g.bytes[1] > a.cap) return 2;
  hipLaunchKernelGGL(dqn::xgmi_allgather_kernel, dim3(blocks), dim3(dqn::kThreads), 0, st, g);
  return 0;
}

int launch_dpx_selftest(const dqn::DpExchange& x, float* out, int slots, int call, hipStream_t st) {
  if (slots < 1 || slots > x.slots || x.world < 1 || x.world > dqn::kXgmiMaxRanks) return 1;
  hipLaunchKernelGGL(dqn::dpx_selftest_kernel, dim3(slots), dim3(512), 0, st, x, out, call);
  return 0;
}

int launch_xgmi_allreduce(const dqn::XgmiArgs& a, int blocks, hipStream_t st) {
  if (blocks < 1 || blocks > dqn::kXgmiMaxBlocks || a.world < 1 || a.world > dqn::kXgmiMaxRanks) return 1;
  if (a.n % (4L * a.world) != 0 || a.n > a.cap) return 2;
#define XGMI_LAUNCH(WC)                                                                                   \
  do {                                                                                                    \
    if (a.bf16)                                                                                           \
      hipLaunchKernelGGL((dqn::xgmi_allreduce_kernel<true, WC>), dim3(blocks), dim3(dqn::kThreads), 0, st, a); \
    else                                                                                                  \
      hipLaunchKernelGGL((dqn::xgmi_allreduce_kernel<false, WC>), dim3(blocks), dim3(dqn::kThreads), 0, st, a); \
  } while (0)
  switch (a.world) {
    case 2: XGMI_LAUNCH(2); break;
    case 4: XGMI_LAUNCH(4); break;
    case 8: XGMI_LAUNCH(8); break;
    default: XGMI_LAUNCH(0); break;
  }
#undef XGMI_LAUNCH
  return 0;
}
