// Asynchronous parameter server over xGMI peer memory (the reference's default training mode:
// every worker pushes its gradient to the PS-held variables with no locking and reads back
// whatever the PS holds, /root/reference/src/network.py:184-202, src/main.py:105-129).
//
// Data moves GPU to GPU by one-sided peer access: rank 0 (the PS) exports one fine-grained
// HBM region holding a gradient slot and a parameter snapshot per worker; workers map it
// (HIP IPC). Control words live in a small host-shared page mapped into every rank's GPU
// address space (hipHostRegister): the PS host thread polls the workers' push words without
// touching the GPU, and the workers' GPUs poll the PS's done words. Per worker step, on the
// worker's stream with no host synchronisation (graph-capturable):
//   ps_push_kernel   grad -> PS slot (peer stores), then the last block publishes
//                    push word = (seq << 4) | kind with a system-scope release
//   ps_wait_kernel   one block waits for done word >= (seq << 4) (system-scope acquire, bounded)
//   ps_copy_kernel   then snapshot -> local flat and the int64 global step
// PS, per arrival (host loop): the fused optimizer reads the gradient slot in place, then
//   ps_publish_kernel  flat -> that worker's snapshot, step, then done word = (seq << 4) | st
#include "common.h"

namespace dqn {
namespace {

constexpr int kPsThreads = 256;
constexpr uint64_t kPsStop = 1;             // done-word status: the PS stopped (no parameters)

DQN_DEV uint64_t ld_acquire_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
DQN_DEV void st_release_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// dst[i] = src[i] (float4 vectors), grid-stride; then the grid's last block (arrival ticket)
// stores `word` with a system-scope release after every block's stores are visible system-wide
__global__ void __launch_bounds__(kPsThreads)
ps_push_kernel(const float4* __restrict__ grad, float4* __restrict__ slot, long n4, uint64_t* push_word,
               int64_t* seq, int kind, int32_t* ticket) {
  for (long i = (long)blockIdx.x * kPsThreads + threadIdx.x; i < n4; i += (long)gridDim.x * kPsThreads)
    slot[i] = grad[i];
  __threadfence_system();                   // this thread's peer stores, before its block's arrival
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (int)gridDim.x - 1) {          // every block's stores are done
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int64_t s = seq[0] + 1;          // this worker's push number (device-side: graph replays)
      seq[0] = s;
      __threadfence_system();
      st_release_sys(push_word, ((uint64_t)s << 4) | (uint64_t)kind);
    }
  }
}

// Segmented push (--ps_lowrank): up to kPsSegs (src, dst, 16-byte-multiple length) pieces -- the flat
// gradient outside the fc weight tensors, and the fc layer's factors (its input rows X and dL/dh rows,
// rank <= B) written into the fc weight region of the slot -- then the push word as ps_push_kernel.
constexpr int kPsSegs = 6;
struct PsSegs {
  const float4* src[kPsSegs];
  float4* dst[kPsSegs];
  long n4[kPsSegs];          // float4 vectors per piece
  long start[kPsSegs + 1];   // prefix sums of n4
  int n;
};

__global__ void __launch_bounds__(kPsThreads)
ps_push_segs_kernel(PsSegs sg, uint64_t* push_word, int64_t* seq, int kind, int32_t* ticket) {
  const long total = sg.start[sg.n];
  for (long i = (long)blockIdx.x * kPsThreads + threadIdx.x; i < total; i += (long)gridDim.x * kPsThreads) {
    int k = 0;
    while (k + 1 < sg.n && i >= sg.start[k + 1]) ++k;
    const long j = i - sg.start[k];
    sg.dst[k][j] = sg.src[k][j];
  }
  __threadfence_system();                   // this thread's peer stores, before its block's arrival
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (int)gridDim.x - 1) {
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int64_t s = seq[0] + 1;
      seq[0] = s;
      __threadfence_system();
      st_release_sys(push_word, ((uint64_t)s << 4) | (uint64_t)kind);
    }
  }
}

// Wait for the PS's answer to push number seq[0] in ONE block (ps_wait_kernel), then copy the
// snapshot -> flat (+ the global step) with the whole grid (ps_copy_kernel), in stream order. (A
// single kernel whose every block spun on the answer kept ~512 spinning workgroups on the GPU for
// the whole server round trip -- the other workers' and the server's kernels waited behind them:
// 153 us per pull, profiles/r5_async_ps_trace.md.) Status kPsStop: the PS stopped, nothing is
// copied and stopped[0] is set. A wait longer than timeout_ns sets err[0] (checked by the host)
// instead of spinning forever. gate[1] = the answer's status for the copy kernel (-1: timed out).
__global__ void __launch_bounds__(64)
ps_wait_kernel(const uint64_t* done_word, const int64_t* seq, int64_t* gate, int32_t* err, int32_t* stopped,
               long long timeout_ns) {
  if (threadIdx.x != 0) return;
  const int64_t want = seq[0];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t limit = (uint64_t)(timeout_ns / 10);       // 100 MHz counter
  int ok = 1;
  uint64_t v = ld_acquire_sys(done_word);
  while ((int64_t)(v >> 4) < want) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > limit) { ok = 0; break; }
    __builtin_amdgcn_s_sleep(8);
    v = ld_acquire_sys(done_word);
  }
  const int64_t st = ok ? (int64_t)(v & 15) : -1;
  if (!ok) err[0] = 1;
  if (st == (int64_t)kPsStop) stopped[0] = 1;
  gate[1] = st;
  gate[0] = want;
}

__global__ void __launch_bounds__(kPsThreads)
ps_copy_kernel(float4* __restrict__ flat, const float4* __restrict__ snap, long n4, int64_t* step,
               const int64_t* snap_step, const int64_t* gate) {
  if (gate[1] != 0) return;                                 // stopped / timed out: nothing to copy
  for (long i = (long)blockIdx.x * kPsThreads + threadIdx.x; i < n4; i += (long)gridDim.x * kPsThreads)
    flat[i] = snap[i];
  if (blockIdx.x == 0 && threadIdx.x == 0 && step != nullptr) step[0] = snap_step[0];
}

// PS: flat -> worker snapshot (+ step), then done word = value (system-scope release, last block).
// echo != nullptr: value = (*echo & ~15) | (value & 15), i.e. the push number the worker published in
// its push word -- the launch then has fixed arguments and replays from a captured graph per worker
// (the native server thread, csrc/ps_server.cpp); the worker pushes again only after this answer.
__global__ void __launch_bounds__(kPsThreads)
ps_publish_kernel(float4* __restrict__ snap, const float4* __restrict__ flat, long n4, int64_t* snap_step,
                  const int64_t* step, uint64_t* done_word, uint64_t value, int32_t* ticket, const uint64_t* echo) {
  if (flat != nullptr)
    for (long i = (long)blockIdx.x * kPsThreads + threadIdx.x; i < n4; i += (long)gridDim.x * kPsThreads)
      snap[i] = flat[i];
  if (blockIdx.x == 0 && threadIdx.x == 0 && step != nullptr) snap_step[0] = step[0];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (int)gridDim.x - 1) {
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (echo != nullptr) value = (ld_acquire_sys(echo) & ~(uint64_t)15) | (value & 15);
      __threadfence_system();
      st_release_sys(done_word, value);
    }
  }
}

int ps_grid(long n4) {
  const long g = (n4 + kPsThreads * 4 - 1) / (kPsThreads * 4);
  return (int)(g < 1 ? 1 : (g > 512 ? 512 : g));
}

}  // namespace
}  // namespace dqn

void launch_ps_push(const float* grad, float* slot, long n, uint64_t* push_word, int64_t* seq, int kind,
                    int32_t* ticket, hipStream_t st) {
  const long n4 = n / 4;
  hipLaunchKernelGGL(dqn::ps_push_kernel, dim3(dqn::ps_grid(n4)), dim3(dqn::kPsThreads), 0, st,
                     reinterpret_cast<const float4*>(grad), reinterpret_cast<float4*>(slot), n4, push_word, seq, kind,
                     ticket);
}

void launch_ps_pull(float* flat, const float* snap, long n, int64_t* step, const int64_t* snap_step,
                    const uint64_t* done_word, const int64_t* seq, int64_t* gate, int32_t* err, int32_t* stopped,
                    long long timeout_ns, hipStream_t st) {
  const long n4 = n / 4;
  hipLaunchKernelGGL(dqn::ps_wait_kernel, dim3(1), dim3(64), 0, st, done_word, seq, gate, err, stopped, timeout_ns);
  hipLaunchKernelGGL(dqn::ps_copy_kernel, dim3(dqn::ps_grid(n4)), dim3(dqn::kPsThreads), 0, st,
                     reinterpret_cast<float4*>(flat), reinterpret_cast<const float4*>(snap), n4, step, snap_step, gate);
}

void launch_ps_publish(float* snap, const float* flat, long n, int64_t* snap_step, const int64_t* step,
                       uint64_t* done_word, uint64_t value, int32_t* ticket, const uint64_t* echo, hipStream_t st) {
  const long n4 = n / 4;
  hipLaunchKernelGGL(dqn::ps_publish_kernel, dim3(flat != nullptr ? dqn::ps_grid(n4) : 1), dim3(dqn::kPsThreads),
                     0, st, reinterpret_cast<float4*>(snap), reinterpret_cast<const float4*>(flat), n4, snap_step,
                     step, done_word, value, ticket, echo);
}

int launch_ps_push_segs(const void* const* src, void* const* dst, const long* nbytes, int n, uint64_t* push_word,
                        int64_t* seq, int kind, int32_t* ticket, hipStream_t st) {
  if (n < 1 || n > dqn::kPsSegs) return -1;
  dqn::PsSegs sg{};
  sg.n = n;
  sg.start[0] = 0;
  for (int k = 0; k < n; ++k) {
    if (nbytes[k] % 16 != 0 || (reinterpret_cast<uintptr_t>(src[k]) & 15) || (reinterpret_cast<uintptr_t>(dst[k]) & 15))
      return -2;
    sg.src[k] = reinterpret_cast<const float4*>(src[k]);
    sg.dst[k] = reinterpret_cast<float4*>(dst[k]);
    sg.n4[k] = nbytes[k] / 16;
    sg.start[k + 1] = sg.start[k] + sg.n4[k];
  }
  hipLaunchKernelGGL(dqn::ps_push_segs_kernel, dim3(dqn::ps_grid(sg.start[n])), dim3(dqn::kPsThreads), 0, st, sg,
                     push_word, seq, kind, ticket);
  return 0;
}
