// Launchers for the gfx950 HIP kernels (raw pointers + stream; no torch types,
// so the .hip translation units compile without the torch headers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dqn { struct TrunkSample; }   // dqn_nets_k.h

// Optional outputs of the sampling kernels: per-sample scalars and the frame-slot
// tables of s and s' (so conv1 can read the frame ring directly). st_slots == nullptr: skip.
struct SampleOut {
  const int32_t* state_idx; const int32_t* next_idx; int K;
  const int32_t* actions; const float* rewards; const float* dones; const float* gammas;
  int32_t* a_out; float* r_out; float* d_out; float* g_out;
  int32_t* st_slots; int32_t* nx_slots;
};
// Prioritized replay inside the optimizer launch's extra block (optim.hip): update the
// priorities of this step's batch, then draw the next step's prioritized sample.
struct PerStep {
  float* sum; float* mn; float* maxp; int P, levels;
  const int32_t* upd_idx; const float* upd_td; float alpha, eps;   // this step's batch / |TD|
  int64_t* rng; const int32_t* size; const int64_t* step;          // next sample: rng, replay size, global_step
  float beta0, beta_steps;
  int32_t* idx_out; float* w_out; SampleOut so; int B;
  // fused acting: the actors' ins_n new transitions (ring slots ending at the advanced
  // cursor ins_cursor[0], capacity ins_cap) enter the tree at max priority in the same climb
  const int64_t* ins_cursor; int ins_n, ins_cap;
};
void launch_replay_sample_uniform(const int32_t* size, int64_t* rng, int32_t* out, int B, const SampleOut& so,
                                  hipStream_t st);
struct GatherScalars {   // optional per-sample scalar gather (a_out == nullptr: skip)
  const int32_t* actions; const float* rewards; const float* dones; const float* gammas;
  int32_t* a_out; float* r_out; float* d_out; float* g_out;
};
void launch_replay_gather_frames(const uint8_t* frames, const int32_t* state_idx, const int32_t* next_idx,
                                 const int32_t* idx, uint8_t* s, uint8_t* ns, int B, int HW, int K,
                                 const GatherScalars& sc, hipStream_t st);
void launch_sumtree_set(float* sum, float* mn, float* maxp, const int32_t* idx, const float* td, float alpha,
                        float eps, int use_max, int n, int P, hipStream_t st);
void launch_sumtree_sample(const float* sum, const float* mn, int64_t* rng, const int32_t* size,
                           const float* beta, int32_t* idx_out, float* w_out, int B, int P, const SampleOut& so,
                           const int64_t* sched_step, float beta0, float beta_steps, hipStream_t st);
void launch_optimizer_step(int op, float* w, const float* g, float* s0, float* s1, float* beta_pow,
                           int64_t* step, int32_t* ticket, const float* hp9, float lr, float reg, int reg_end,
                           float grad_scale, int n, float* tgt, int tfreq, hipStream_t st);
// The fc (hidden dense) layer's weight gradient formed inside the optimizer launch (optim.hip):
// dW[k][n] = sum_{m < M} x[m][k] dh[m][col + n] for the update jobs that carry a dH column
// (UpdJob.fc_col >= 0), and the fc bias gradient sum_m dh[m][col + n] -- never written to the
// flat gradient. x / dh are act_t rows (the fc input rows and dL/d(fc pre-activation) rows of
// this rank, or the all-gathered rows of every rank under the low-rank DP exchange).
struct FcFuse {
  const void* x;
  const void* dh;
  int M, ldx, ldh;
};
// dp: nullptr or a dqn::DpLaunch (WG launches under data parallelism: the dependent jobs exchange
// their gradients with every rank inside the launch, see DpExchange below)
void launch_optim_pack(int op, float* w, const float* g, float* s0, float* s1, float* beta_pow, int64_t* step,
                       int32_t* ticket, const float* hp9, float lr, float reg, int reg_end, float grad_scale,
                       const void* jobs, int njobs, void* packed, float* tgt, void* tgt_packed, int tfreq, int max_grid,
                       const float* noise, float* eff, const float* gnoise, float* noise_dst, int noise_n,
                       const dqn::TrunkSample* smp, const PerStep* per, const float* tnoise, float* teff, void* tpk,
                       int64_t* noise_rng, const FcFuse* fc, const float* part, const void* wg, int wg_blocks,
                       const void* dp, void* tsg, int no_pack, hipStream_t st);
// 1 when this build's optimizer launch can form the fc weight gradient itself (16-bit builds)
int optim_fc_fuse();
// probe launches (DQN_OPT_PROF=1): per-block [start, ready, end] s_memrealtime stamps of the last launch
int optim_timeline_read(int64_t* out, int nblocks);
// ... and [8] phase stamps inside each of the first weight-gradient tiles of a fused launch
int optim_tile_phases_read(int64_t* out, int nblocks);
// standard-normal noise (Box-Muller over Philox keyed by rng[0], counter rng[1], bumped)
void launch_noise_normal(float* out0, float* out1, int n, int64_t* rng, hipStream_t st);
int upd_job_ints();
void optim_prof_read(int64_t* out16);   // optim_pack phase stamps (DQN_OPT_PROF=1)
void launch_target_update(float* dst, const float* src, float tau, const int64_t* step, int freq, int n,
                          float* dst2, const float* src2, int n2, hipStream_t st);
void launch_step_bump(int64_t* step, hipStream_t st);
void launch_td_loss_scalar(const float* q, const float* qn_t, const float* qn_o, const int32_t* act,
                           const float* rew, const float* done, const float* gam, const float* wts,
                           float* loss, float* dq, float* prio, int B, int A, int huber, float delta,
                           hipStream_t st);
void launch_td_loss_c51(const float* lg, const float* lgn_t, const float* lgn_o, const int32_t* act,
                        const float* rew, const float* done, const float* gam, const float* wts, float* loss,
                        float* dlg, float* prio, int B, int A, int N, float vmin, float vmax, hipStream_t st);
void launch_preprocess_batch(const uint8_t* in, uint8_t* out, int N, int Hs, int Ws, int H, int W, hipStream_t st);
void launch_actor_step(const float* q, uint8_t* frames, int32_t* stacks, int64_t* cursor, int32_t* size_dev,
                       int32_t* state_idx, int32_t* next_idx, int32_t* actions, float* rewards, float* dones,
                       float* gammas, float* eps, int64_t* rng, int32_t* ticket, int64_t* frames_done, int E,
                       int A, int K, int HW, int C, int F, float gamma, float p_done, hipStream_t st);
void launch_stack_states(const uint8_t* frames, const int32_t* stacks, uint8_t* out, int E, int HW, int K,
                         hipStream_t st);

// Peer-to-peer (xGMI) two-shot all-reduce, csrc/kernels/xgmi_ar.hip.
namespace dqn {
constexpr int kXgmiMaxRanks = 16;
constexpr int kXgmiMaxBlocks = 256;
constexpr int kXgmiMaxRanges = 8;
struct XgmiArgs {
  void* data[kXgmiMaxRanks];       // every rank's staging buffer (2 parities x cap elements), peer-mapped
  uint32_t* sig[kXgmiMaxRanks];    // every rank's signal words [kXgmiMaxRanks][kXgmiMaxBlocks], peer-mapped
  uint32_t* seq;                   // this rank's per-block call counters [kXgmiMaxBlocks]
  int* err;                        // [4]: the first timed-out wait (xgmi_dev.h wait_all), 0 = none
  float* grad;                     // local gradient (in: my addend, out: the sum)
  long n;                          // elements to reduce (n % (4 * world) == 0)
  // nr > 0: the reduced vector is the concatenation of nr ranges grad[rlo[r], rlo[r] + len_r)
  // (rpre: exclusive prefix sums of the lengths, rpre[nr] = n; every length % 4 == 0), so several
  // disjoint pieces of one flat buffer are summed in ONE launch
  int nr;
  long rlo[kXgmiMaxRanges];
  long rpre[kXgmiMaxRanges + 1];
  long cap;                        // staging capacity per parity, elements
  int rank, world, bf16;
};
}  // namespace dqn
int launch_xgmi_allreduce(const dqn::XgmiArgs& a, int blocks, hipStream_t st);
namespace dqn {
// all-gather of two byte segments (the low-rank DP exchange: fc input rows + dH rows):
// out[s] = [rank 0's src[s] | rank 1's | ...], x.cap = staging bytes per parity
struct XgmiGatherArgs {
  XgmiArgs x;                      // data / sig / seq / err / cap / rank / world (grad, n, bf16 unused)
  const void* src[2];
  void* out[2];
  long bytes[2];                   // per-rank segment bytes (multiples of 16)
};
}  // namespace dqn
int launch_xgmi_allgather(const dqn::XgmiGatherArgs& a, int blocks, hipStream_t st);
namespace dqn {
// Data-parallel exchange INSIDE the fused weight-gradient + update launch (optim_pack.h kModeDp):
// every update job whose gradient the launch's own weight-gradient tiles produce (conv layers,
// output layer) pushes its 2048-value gradient slot into every rank's inbox, raises its flag in
// every rank's signal words, waits for all ranks' flags and sums the W slots in rank order
// (bit-identical on every rank), then updates. No all-reduce launch between backward and update.
constexpr int kDpxMaxSlots = 1024;     // dependent update jobs per launch (signal words per source rank)
constexpr int kDpxSlotElems = 2048;    // one job's gradient: a 32 x 64 tile or a <= 2048-element chunk
struct DpExchange {
  float* inbox[kXgmiMaxRanks];     // every rank's inbox, peer-mapped: [2 parities][world][slots][kDpxSlotElems]
  uint32_t* sig[kXgmiMaxRanks];    // every rank's signal words [kXgmiMaxRanks (source)][kDpxMaxSlots]
  uint32_t* seq;                   // this rank's per-slot call counters [kDpxMaxSlots]
  int* err;                        // [4]: the first timed-out wait (phase kXgmiPhaseDpx), 0 = none
  int rank, world, slots;          // slots: inbox capacity in jobs per source rank
};
// launch-time view: the device descriptor + where the dependent jobs sit in the job table
// ([first, first + n)) and how many blocks run them (blocks < n: each block takes jobs
// first + b, first + b + blocks, ... in order -- ranks sharing one GPU in the rehearsals)
struct DpLaunch {
  const DpExchange* x;
  int first, n, blocks;
};
}  // namespace dqn
// the exchange protocol's self-test (xgmi_ar.hip): slots blocks of rank-stamped values, sums -> out
int launch_dpx_selftest(const dqn::DpExchange& x, float* out, int slots, int call, hipStream_t st);

// Asynchronous parameter server over xGMI peer memory, csrc/kernels/async_ps.hip.
void launch_ps_push(const float* grad, float* slot, long n, uint64_t* push_word, int64_t* seq, int kind,
                    int32_t* ticket, hipStream_t st);
int launch_ps_push_segs(const void* const* src, void* const* dst, const long* nbytes, int n, uint64_t* push_word,
                        int64_t* seq, int kind, int32_t* ticket, hipStream_t st);
void launch_ps_pull(float* flat, const float* snap, long n, int64_t* step, const int64_t* snap_step,
                    const uint64_t* done_word, const int64_t* seq, int64_t* gate, int32_t* err, int32_t* stopped,
                    long long timeout_ns, hipStream_t st);
void launch_ps_publish(float* snap, const float* flat, long n, int64_t* snap_step, const int64_t* step,
                       uint64_t* done_word, uint64_t value, int32_t* ticket, const uint64_t* echo, hipStream_t st);

// Fused MLP Q-network (reference SimpleNetwork), csrc/kernels/mlp.hip.
namespace dqn {
constexpr int kMlpMaxLayers = 4;
constexpr int kMlpMaxWidth = 64;
constexpr int kMlpThreads = 128;
struct MlpArgs {
  const float* w_on;               // online flat parameters (TF layouts: dense W [in, out])
  const float* w_tg;               // target flat parameters
  int L, A, P;                     // layers, actions, flat length
  int Hs, Ds, sw;                  // LDS row strides (activations, deltas) and max layer width
  int fin[kMlpMaxLayers], fout[kMlpMaxLayers], act[kMlpMaxLayers];   // act: 0 none, 1 tanh, 2 relu
  int w_off[kMlpMaxLayers], b_off[kMlpMaxLayers];
  const float* x;                  // states [B, fin0]
  const float* xn;                 // next states [B, fin0]
  const int32_t* act_idx;
  const float* rew; const float* done; const float* gam; const float* wts;   // wts may be null
  float* loss; float* prio; float* grad; float* q_out;
  int B, double_dqn, huber;
  float delta, in_scale;
};
}  // namespace dqn
size_t mlp_train_lds_bytes(const dqn::MlpArgs& a);
int launch_mlp(const dqn::MlpArgs& a, int train, hipStream_t st);
