// Argument structs + launchers of the Q-network kernels (csrc/kernels/qnet.hip).
// Plain C++ (no torch types) so both the HIP TU and the torch binding TU include it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dqn_act.h"

namespace dqn {

// Up to 4 network instances per launch (grid.y / grid.z): online(s), target(s'),
// online(s') for Double DQN, and the device actors' states when acting is fused
// into the learner step.
constexpr int kMaxInst = 4;

// One packing job: fp32 master tensor (TF layout) -> bf16 MFMA B-fragments
// [K/32][N/16][64][8] (mode 0..2) or a contiguous fp32 copy (mode 3, biases).
struct PackJob {
  int src_off;   // element offset in the fp32 flat buffer
  int K, N;      // logical B operand shape [K][N] (mode 3: K = length)
  int dst_off;   // element offset (bf16 units) in the packed buffer
  int dst_N16;   // n-tiles per k-step row of the destination (>= nt_off + N/16)
  int nt_off;    // n-tile offset (concatenation along N)
  int ks_off;    // k-step offset (concatenation along K)
  int mode;      // 0 natural [K][N]; 1 conv dgrad (p0 taps, p1 CIN, p2 COUT); 2 dense transpose (p0 = OUT); 3 fp32 copy
  int p0, p1, p2, pad;
};

// Implicit-GEMM arguments (up to 3 instances: online(s), target(s'), online(s')).
struct ConvArgs {
  const void* in[kMaxInst];
  const void* w[kMaxInst];          // packed bf16 B fragments
  const float* bias[kMaxInst];
  void* out[kMaxInst];
  const void* mask[kMaxInst];       // ReLU mask source for dgrad epilogues
  float scale[kMaxInst];
  int M, N, K, N16;          // GEMM shape; N16 = n-tiles per k-step of the packed B
  int ldo;                   // output row stride (elements)
  int IH, IW, OH, OW, pad_t, pad_l;
  const void* frames;        // frame ring [F][H*W] u8 for the frame-slot conv1 loader
  int frame_hw;
  // optional side duties of the launch (null = off): zero [zero_ptr, +zero_n) (a gradient range
  // the conv weight gradients later accumulate into with atomics), and (block 0) loss_out[0] =
  // loss_mul * sum of loss_parts[0..nparts) (the scalar head's per-tile loss partials)
  float* zero_ptr; int zero_n;
  const float* loss_parts; int nparts;
  float* loss_out; float loss_mul;
  // noisy nets: draw the next noise samples (noise_normals4 at the stream's current counter,
  // spread over the launch's blocks) into nz_out0[0, nz_n) | nz_out1[0, nz_n); the counter is
  // advanced later by the fused optimizer's last block (every block of this launch read it)
  float* nz_out0; float* nz_out1; int nz_n;
  const int64_t* nz_rng;
  // data parallelism, low-rank exchange: the blocks of grid.z == gth_z run the xgmi all-gather of
  // the fc factors (the first gth_blocks of them; args: a device XgmiGatherArgs) beside the GEMM
  const void* gth; int gth_blocks, gth_z;
  // noisy nets, factorised target fc forward (fz_w2 != null; dense forward kind only): instance
  // fz_inst computes relu(scale * (X Wmu + f(eps_out) * ((X * f(eps_in)) Wsigma)) + bias) from the
  // mu fragments in w[fz_inst] and the sigma fragments in fz_w2 (f(x) = sgn(x) sqrt|x|; eps from
  // fz_noise, column halves [0, fz_nsplit) / [fz_nsplit, N) with their own eps_in / eps_out offsets)
  const void* fz_w2; const float* fz_noise; int fz_inst, fz_nsplit; int fz_ein[2], fz_eout[2];
};

struct WgradArgs {
  const void* dz;            // dZ rows [M][ldz] bf16 (gradient w.r.t. the layer pre-activation)
  int ldz;
  float* dw; float* db;      // columns [0, nsplit)
  float* dw2; float* db2;    // columns [nsplit, N) (dueling concatenation), may be null
  int nsplit, N;
  int MC, KB, NB;            // rows per block, K-range per block, N-range per block
  float scale;
  int atomic;
  int mloop;                 // > 1: each block sums this many consecutive M-chunks (no atomics)
  int db_zero;               // store 0 into db / db2 (the low-rank DP member on ranks != 0)
  // deterministic partials (grouped conv members): chunk group c (mloop consecutive M-chunks)
  // stores its sum plainly at part + c * pstride ([K][N] weights, then [N] bias); the fused
  // optimizer sums the groups in a fixed order (no atomics: run-to-run bit-identical)
  float* part;
  int pstride;
};

// Device actor step (eps-greedy + synthetic env + replay append), see actor.hip.
struct ActorArgs {
  const float* q;          // [E, A] online Q of the current states
  uint8_t* frames;         // [F, HW]
  int32_t* stacks;         // [E, K] frame slots of each env's current state
  int64_t* cursor;         // [3]: next transition slot, next frame slot, size
  int32_t* size_dev;       // [1]
  int32_t* state_idx;      // [C, K]
  int32_t* next_idx;       // [C]
  int32_t* actions;        // [C]
  float* rewards;          // [C]
  float* dones;            // [C]
  float* gammas;           // [C]
  float* eps;              // [3]: eps, eps_min, decay
  int64_t* rng;            // [2]
  int32_t* ticket;         // [1]
  int64_t* frames_done;    // [1] env-frame counter
  int E, A, K, HW, C, F;
  float gamma, p_done;
  // prioritized replay (tsum != nullptr): new transitions enter the sum-tree with the max priority
  float* tsum; float* tmin; float* tmaxp;
  int tP, tlevels;
};

struct HeadArgs {
  int B, A, HID, dueling, huber, infer;
  float delta;
  const void* h[3];
  const void* pw[3];         // packed bf16 head fragments (plain output / advantage), [HID/32][N16][64][8]
  const void* pwv[3];        // packed value-head fragments (dueling, N = 1)
  int N16;                   // action n-tiles of pw
  const float* w[3]; const float* b[3];
  const float* wv[3]; const float* bv[3];
  const int32_t* act; const float* rew; const float* done; const float* gam; const float* wts;
  float* loss; float* prio; float* q_out;
  float* dw; float* db; float* dwv; float* dbv;
  void* dh;
  float* zero_ptr; int zero_n;   // grad range zeroed in-kernel (conv wgrads accumulate atomically)
  int has_actor;                 // infer mode: run the fused actor step on the Q tile
  ActorArgs actor;
  const void* act_h;             // training mode + fused acting: the actors' hidden layer [E][HH]
  int act_E;                     //   (an extra workgroup runs the acting step), 0 = off
  int atoms;                     // C51 head (rainbow.hip): atoms per action, support [vmin, vmax]
  float vmin, vmax;
  int64_t* prof;                 // optional s_memtime phase stamps of block 0 (profiling)
  const float* lgi[3];           // C51: precomputed logits rows [B][KD] per instance (one igemm over the
                                 // combined output layer: logits | pad | dueling value logits at VO)
  const float* act_lgi;          // C51 + fused acting: the actors' logits rows [E][KD]
  // scalar heads (head_loss_kernel): per-16-sample-tile loss partials (summed by the fc dgrad
  // launch) and dL/dQ as act_t [B][64] (plain / advantage in columns 0..31, value in 32), the dZ
  // operand of the output layer's grouped weight-gradient members; dH goes to dh.
  // C51 (c51_train_kernel): per-block loss partials and dL/dlogits as act_t [B][KD] (plain /
  // advantage at [0, NO), value at [VO, VO + atoms), VO = NO rounded up to 32), the A operand
  // of the dH igemm and the dZ of the output layer's weight-gradient members
  float* loss_parts;
  void* dq16;
};

// Fused fc forward + scalar head (fc_head.hip): the output layer is folded into the fc launch's
// epilogue (per-tile partial Q values stored into qacc [instance][Mpad][32][N / 16]), the last
// block to arrive on a row group's counter (cnt [ngroups + 1], zero on entry and left zero; the
// last one is the fused actors') sums them in tile order and runs the TD loss / dQ / dH tail.
struct FoldArgs {
  float* qacc;
  int32_t* cnt;
  int Mpad, ngroups, nlearn;
  int64_t* prof;             // optional: s_memrealtime stamps [block][8] (scripts/probe_fold.py)
  // spin (every block of the launch resident at once): the online instance's blocks wait for
  // their group's dQ (tail -> dqg fp32 [Mpad][32] + epoch word dq_epoch[group], never reset) and
  // each writes its own 16x16 dH tile; else the tail computes the group's whole dH
  int spin;
  float* dqg;
  int32_t* dq_epoch;
  float* zero_ptr;           // side duty: block 0 zeroes [zero_ptr, +zero_n) (the step's dgrad-chain
  int zero_n;                // counters; 16-byte aligned, zero_n % 4 == 0)
  // spin mode: a dH-tile block whose dQ wait expires (1 s) stores 0x1000000 | group here and skips
  // its dH write instead of using stale dQ (read by Learner._device_checks). dq_epoch[ngroups + 1].
  int32_t* err;
  int dbg_no_publish;        // test hook (DQN_DEBUG_FOLD_NO_PUBLISH): the tails never publish dQ
  int two_per_cu;            // spin mode may run two blocks per CU (KernelTuning.fold_two_per_cu)
};

// The Nature dgrad chain in ONE launch (qnet.hip dgrad_chain_kernel): block ranges run
//   stage 0  fc dgrad        dz3 = (dH W_fc^T) * (x3 > 0)      (+ the fc dgrad's side duties)
//   stage 1  conv3 dgrad     dz2 = dgrad(dz3) * (x2 > 0)
//   stage 2  conv2 dgrad     dz1 = parity-class dgrad(dz2) * (x1 > 0)
// in dispatch order; a stage-1 block waits for the stage-0 row groups of its samples, a stage-2
// block for the stage-1 blocks of its sample (counters in cnt, one per 32 ints: [gx0] row groups |
// [B] samples | [1] error flag; zeroed by the step's fc forward launch). Stage 0 / 1 outputs are full 128-byte
// lines per block row, stored write-through.
struct ChainArgs {
  ConvArgs a[3];
  int n0, n1, n2;            // blocks per stage
  int gx0, gy0;              // stage-0 grid (16-sample row groups, 64-column tiles)
  int rows1;                 // stage-1 output rows per sample
  int B;
  int32_t* cnt;
};

// One tensor of the noisy-net parameter mix (rainbow.hip): eff[mu_off + k*N + n] =
// mu + sigma * f(noise[ein_off + k]) * f(noise[eout_off + n]); sigma_off < 0: plain
// copy; ein_off < 0: bias (no input factor).
struct NoisyJob {
  int mu_off, sigma_off, K, N, ein_off, eout_off, pad0, pad1;
};

// Fused per-sample Nature trunk (trunk.hip): conv1 -> conv2 -> conv3 in one launch.
// Fused uniform sampling inside the trunk launch (size == nullptr: off). Every sampled
// workgroup re-derives the batch (sample_dev.h), takes its own transition's frame slots,
// instance 0 writes the per-sample outputs the head / wgrad read, and the last workgroup
// to arrive (ticket) advances the rng counter.
struct TrunkSample {
  const int32_t* size; int64_t* rng; int32_t* ticket;
  const int32_t* state_idx; const int32_t* next_idx;            // replay [C][4], [C]
  const int32_t* actions; const float* rewards; const float* dones; const float* gammas;
  int32_t* idx_out; int32_t* a_out; float* r_out; float* d_out; float* g_out;
  int32_t* st_slots; int32_t* nx_slots;                          // [B][4]
  int B, ninst;                    // samples drawn; leading instances that use them
};

struct TrunkArgs {
  const uint8_t* frames;           // frame ring [F][84*84] (slot path)
  const int32_t* slots[kMaxInst];  // [B][4] frame slots per instance (or nullptr -> states)
  const uint8_t* states[kMaxInst]; // [B][84][84][4] NHWC stacks per instance (materialised path)
  const void* w1[kMaxInst]; const void* w2[kMaxInst]; const void* w3[kMaxInst];   // packed bf16 fragments
  const float* b1[kMaxInst]; const float* b2[kMaxInst]; const float* b3[kMaxInst];
  act_t* x1[kMaxInst]; act_t* x2[kMaxInst]; act_t* x3[kMaxInst];   // activations out ([B][...] NHWC)
  int M[kMaxInst];                 // valid samples per instance (the fused actor's E < B)
  float scale;                     // input scale folded into conv1
  int64_t* prof;                   // optional [ninst][B][8] s_memtime phase stamps (profiling)
  TrunkSample smp;                 // fused sampling (smp.size == nullptr: use `slots`)
};

// Reference `cnn` (SAME convs + 2x2 max-pools), per-sample fused kernels (cnn.hip).
struct CnnFwdArgs {
  const uint8_t* frames;
  const int32_t* slots[kMaxInst];
  const uint8_t* states[kMaxInst];
  const void* w1[kMaxInst]; const void* w2[kMaxInst]; const void* w3[kMaxInst];   // packed bf16 fwd fragments
  const float* b1[kMaxInst]; const float* b2[kMaxInst]; const float* b3[kMaxInst];
  act_t* a1; act_t* p1; act_t* a2; act_t* p2; act_t* a3;  // instance 0, for the backward
  act_t* x3[kMaxInst];                                        // [B][256] pooled fc inputs
  int M[kMaxInst];                                             // valid samples per instance
  float scale;
  int64_t* prof;             // probe only (scripts/probe_cnn.py): [block][8] s_memrealtime stamps
};

struct CnnBwdArgs {
  const act_t* dp3;                          // [B][256] d(pool3 out), masked by its ReLU
  const act_t* a1; const act_t* a2; const act_t* a3;   // post-ReLU pre-pool activations
  const void* w3d; const void* w2d;           // packed conv3 / conv2 dgrad fragments
  act_t* dz1; act_t* dz2; act_t* dz3;      // d(conv pre-activation) for the wgrads
  int64_t* prof;             // probe only (scripts/probe_cnn.py): [block][8] s_memrealtime stamps
};

// Grouped weight-gradient launch (qnet.hip): up to 4 independent layers.
constexpr int kMaxWgradMembers = 6;
struct WgradGroup {
  ConvArgs a[kMaxWgradMembers];
  WgradArgs g[kMaxWgradMembers];
  int kind[kMaxWgradMembers];
  int nblk[kMaxWgradMembers], gx[kMaxWgradMembers], gy[kMaxWgradMembers];     // filled by the launcher
  int n;
  // fused launches (optim.hip kModeWg): done counters (int32, 32 words apart, zero between
  // launches: [m] per member, then [kMaxWgradMembers + m * kWgSlots + s] per member K-range s <
  // kWgSlots - 1 and the member's bias, s = kWgSlots - 1), the member reading the current
  // minibatch's frame-slot tables (-1: none), and per (member, slot) the optimizer jobs its last
  // tile runs once that slot's gradient is complete (a contiguous range of the launch's job table)
  int32_t* done;
  int slots_member;
  int dep_first[kMaxWgradMembers][16 + 1], dep_count[kMaxWgradMembers][16 + 1];
};
constexpr int kWgSlots = 16 + 1;            // K-ranges (<= 16) + the bias
constexpr int kWgCounters = kMaxWgradMembers * (1 + kWgSlots);

enum LayerKind {
  L_NAT_CONV1_FWD = 1, L_NAT_CONV2_FWD = 2, L_NAT_CONV3_FWD = 3,
  L_DENSE_FWD_RELU = 4, L_DENSE_FWD_F32 = 5, L_DENSE_DGRAD = 6,
  L_NAT_CONV3_DGRAD = 7, L_NAT_CONV2_DGRAD = 8,
  L_NAT_CONV1_FRAMES = 9,   // conv1 reading the frame ring through a [B][4] slot table
  L_HEAD_WGRAD = 11,        // output layer weight gradient (grouped wgrad member: N <= 32)
  L_DENSE_WGRAD_LR = 12,    // fc weight gradient over all-gathered rows (64-row chunks summed per block)
};

}  // namespace dqn

void launch_pack(const float* src, void* dst, const dqn::PackJob* jobs_dev, int njobs, int max_threads,
                 void* dst2, const int64_t* step, int freq, hipStream_t st);
int launch_igemm(int kind, const dqn::ConvArgs& a, int ninst, hipStream_t st);
// -1: shapes outside the chained kernel (Nature fc / conv3 / conv2 dgrad, B <= 1024)
int launch_dgrad_chain(const dqn::ConvArgs& a0, const dqn::ConvArgs& a1, const dqn::ConvArgs& a2, int32_t* cnt, int B,
                       hipStream_t st);
int launch_wgrad(int kind, const dqn::ConvArgs& a, const dqn::WgradArgs& g, hipStream_t st);
int launch_wgrad_group(dqn::WgradGroup G, hipStream_t st);
// Plans G for the fused weight-gradient range of a split optimizer update (optim.hip kModeWg):
// fills nblk / gx / gy and every member's chunk grouping (conv members: conv_chunks 128-row chunks
// summed in registers per tile, one set of fp32 atomics per group) and atomic flag. Returns the
// total block count, or -1 when a member kind has no fused tile (16-bit builds only).
int wgrad_fused_plan(dqn::WgradGroup& G, int conv_chunks);
void launch_cnn_fwd(const dqn::CnnFwdArgs& a, int B, int ninst, hipStream_t st);
void launch_cnn_bwd(const dqn::CnnBwdArgs& a, int B, int parts, hipStream_t st);
void launch_head_loss(const dqn::HeadArgs& a, hipStream_t st);
// -1: shape outside the fused kernel's range (A <= 18, HID <= 512, E <= 16, 2-3 learner instances)
int launch_fc_head(const dqn::ConvArgs& a, const dqn::HeadArgs& h, const dqn::FoldArgs& f, hipStream_t st);
void launch_trunk_fwd(const dqn::TrunkArgs& a, int B, int ninst, hipStream_t st);
void launch_c51_head(const dqn::HeadArgs& a, hipStream_t st);
size_t c51_head_lds_bytes(const dqn::HeadArgs& a);
int c51_train_blocks(const dqn::HeadArgs& a);     // learner blocks = loss partials of the training head
void launch_noisy_mix(const float* flat, float* eff, const float* noise, const dqn::NoisyJob* jobs, int njobs,
                      int max_elems, hipStream_t st);
void launch_noisy_grad(float* grad, const float* noise, const dqn::NoisyJob* jobs, int njobs, int max_elems,
                       hipStream_t st);
