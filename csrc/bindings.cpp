// Python bindings of dist_dqn_amd._C: validates every operand on the host
// (device, dtype, contiguity, shapes the kernels assume) and launches on the
// current HIP stream, so the ops are captured correctly into HIP graphs.
#include <cstring>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "include/dqn_act.h"
#include "include/dqn_host.h"
#include "include/dqn_kernels.h"
#include "include/dqn_nets.h"
#include "include/dqn_nets_k.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " has wrong dtype: ", (t).scalar_type())
#define CHECK_T(t, dt) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, dt)

template <typename T>
T* ptr(const torch::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
template <class T>
T P(int64_t v) { return reinterpret_cast<T>(static_cast<intptr_t>(v)); }

// [] or [state_idx, next_idx, actions, rewards, dones, gammas, a_out, r_out, d_out, g_out, st_slots, nx_slots]
SampleOut sample_out(const std::vector<torch::Tensor>& v, int64_t B) {
  SampleOut so{};
  if (v.empty()) return so;
  TORCH_CHECK(v.size() == 12, "sample outputs: 12 tensors");
  for (auto& t : v) { CHECK_DEV(t); CHECK_CONTIG(t); }
  for (int i : {0, 1, 2, 6, 10, 11}) CHECK_DT(v[i], torch::kInt32);
  for (int i : {3, 4, 5, 7, 8, 9}) CHECK_DT(v[i], torch::kFloat32);
  const int K = (int)v[0].size(1);
  for (int i = 6; i < 10; ++i) TORCH_CHECK(v[i].numel() == B, "scalar outputs must be [B]");
  TORCH_CHECK(v[10].numel() == B * K && v[11].numel() == B * K, "slot tables must be [B, K]");
  so = SampleOut{ptr<int32_t>(v[0]), ptr<int32_t>(v[1]), K, ptr<int32_t>(v[2]), ptr<float>(v[3]),
                 ptr<float>(v[4]), ptr<float>(v[5]), ptr<int32_t>(v[6]), ptr<float>(v[7]), ptr<float>(v[8]),
                 ptr<float>(v[9]), ptr<int32_t>(v[10]), ptr<int32_t>(v[11])};
  return so;
}

void replay_sample_uniform(torch::Tensor size, torch::Tensor rng, torch::Tensor out, std::vector<torch::Tensor> so) {
  CHECK_T(size, torch::kInt32); CHECK_T(rng, torch::kInt64); CHECK_T(out, torch::kInt32);
  TORCH_CHECK(out.numel() >= 1 && out.numel() <= 1024, "sample batch must be in [1, 1024]");
  TORCH_CHECK(rng.numel() == 2, "rng state must be [seed, counter]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  launch_replay_sample_uniform(ptr<int32_t>(size), ptr<int64_t>(rng), ptr<int32_t>(out), (int)out.numel(),
                               sample_out(so, out.numel()), cur_stream());
}

void replay_gather_frames(torch::Tensor frames, torch::Tensor state_idx, torch::Tensor next_idx,
                          torch::Tensor idx, torch::Tensor s, torch::Tensor ns,
                          std::vector<torch::Tensor> scal) {
  // scal: [] or [actions, rewards, dones, gammas (replay columns), a_out, r_out, d_out, g_out]
  GatherScalars sc{};
  if (!scal.empty()) {
    TORCH_CHECK(scal.size() == 8, "scalars: 4 replay columns + 4 outputs");
    for (auto& t : scal) { CHECK_DEV(t); CHECK_CONTIG(t); }
    CHECK_DT(scal[0], torch::kInt32); CHECK_DT(scal[4], torch::kInt32);
    for (int i : {1, 2, 3, 5, 6, 7}) CHECK_DT(scal[i], torch::kFloat32);
    for (int i = 4; i < 8; ++i) TORCH_CHECK(scal[i].numel() == idx.numel(), "scalar output must be [B]");
    sc = GatherScalars{ptr<int32_t>(scal[0]), ptr<float>(scal[1]), ptr<float>(scal[2]), ptr<float>(scal[3]),
                       ptr<int32_t>(scal[4]), ptr<float>(scal[5]), ptr<float>(scal[6]), ptr<float>(scal[7])};
  }
  CHECK_T(frames, torch::kUInt8); CHECK_T(state_idx, torch::kInt32); CHECK_T(next_idx, torch::kInt32);
  CHECK_T(idx, torch::kInt32); CHECK_T(s, torch::kUInt8); CHECK_T(ns, torch::kUInt8);
  TORCH_CHECK(frames.dim() == 3 && state_idx.dim() == 2, "frames [F,H,W], state_idx [C,k]");
  const int K = (int)state_idx.size(1);
  const int HW = (int)(frames.size(1) * frames.size(2));
  const int B = (int)idx.numel();
  TORCH_CHECK(K >= 1 && K <= 4, "frames_per_state must be 1..4");
  TORCH_CHECK(HW % 4 == 0, "H*W must be a multiple of 4");
  TORCH_CHECK(s.numel() == (int64_t)B * HW * K && ns.numel() == s.numel(), "output size mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA g(frames.device());
  launch_replay_gather_frames(ptr<uint8_t>(frames), ptr<int32_t>(state_idx), ptr<int32_t>(next_idx),
                              ptr<int32_t>(idx), ptr<uint8_t>(s), ptr<uint8_t>(ns), B, HW, K, sc, cur_stream());
}

void sumtree_set(torch::Tensor sum, torch::Tensor mn, torch::Tensor maxp, torch::Tensor idx, torch::Tensor td,
                 double alpha, double eps, bool use_max, int64_t P) {
  CHECK_T(sum, torch::kFloat32); CHECK_T(mn, torch::kFloat32); CHECK_T(maxp, torch::kFloat32);
  CHECK_T(idx, torch::kInt32); CHECK_T(td, torch::kFloat32);
  TORCH_CHECK(sum.numel() == 2 * P && mn.numel() == 2 * P, "tree size must be 2P");
  TORCH_CHECK(use_max || td.numel() >= idx.numel(), "td must cover idx");
  c10::hip::HIPGuardMasqueradingAsCUDA g(sum.device());
  launch_sumtree_set(ptr<float>(sum), ptr<float>(mn), ptr<float>(maxp), ptr<int32_t>(idx), ptr<float>(td),
                     (float)alpha, (float)eps, use_max ? 1 : 0, (int)idx.numel(), (int)P, cur_stream());
}

void sumtree_sample(torch::Tensor sum, torch::Tensor mn, torch::Tensor rng, torch::Tensor size, torch::Tensor beta,
                    torch::Tensor idx_out, torch::Tensor w_out, int64_t P, std::vector<torch::Tensor> so,
                    double beta0, double beta_steps) {
  // beta: float32 [1] = the IS exponent itself, or int64 [1] = the device global_step of the
  // annealing schedule beta = min(1, beta0 + (1 - beta0) * step / beta_steps)
  CHECK_T(sum, torch::kFloat32); CHECK_T(mn, torch::kFloat32); CHECK_T(rng, torch::kInt64);
  CHECK_T(size, torch::kInt32); CHECK_T(idx_out, torch::kInt32); CHECK_T(w_out, torch::kFloat32);
  CHECK_DEV(beta); CHECK_CONTIG(beta);
  const bool sched = beta.scalar_type() == torch::kInt64;
  TORCH_CHECK(sched || beta.scalar_type() == torch::kFloat32, "beta: float32 value or int64 step");
  TORCH_CHECK(!sched || beta_steps >= 1.0, "beta schedule steps must be >= 1");
  TORCH_CHECK(idx_out.numel() <= 1024 && w_out.numel() == idx_out.numel(), "PER batch must be <= 1024");
  TORCH_CHECK(sum.numel() == 2 * P, "tree size must be 2P");
  c10::hip::HIPGuardMasqueradingAsCUDA g(sum.device());
  launch_sumtree_sample(ptr<float>(sum), ptr<float>(mn), ptr<int64_t>(rng), ptr<int32_t>(size),
                        sched ? nullptr : ptr<float>(beta), ptr<int32_t>(idx_out), ptr<float>(w_out),
                        (int)idx_out.numel(), (int)P, sample_out(so, idx_out.numel()),
                        sched ? ptr<int64_t>(beta) : nullptr, (float)beta0, (float)beta_steps, cur_stream());
}

void optimizer_step(int64_t op, torch::Tensor w, torch::Tensor grad, torch::Tensor s0, torch::Tensor s1,
                    torch::Tensor beta_pow, torch::Tensor ticket, double lr, double reg, int64_t reg_end,
                    double grad_scale, torch::Tensor step, bool has_step, std::vector<double> hp,
                    c10::optional<torch::Tensor> target, int64_t target_freq) {
  CHECK_T(w, torch::kFloat32); CHECK_T(grad, torch::kFloat32); CHECK_T(s0, torch::kFloat32);
  CHECK_T(s1, torch::kFloat32); CHECK_T(beta_pow, torch::kFloat32); CHECK_T(ticket, torch::kInt32);
  TORCH_CHECK(w.numel() % 4 == 0 && grad.numel() == w.numel(), "flat buffers must match and be /4");
  TORCH_CHECK(s0.numel() == w.numel() || s0.data_ptr() == w.data_ptr(), "slot 0 size");
  TORCH_CHECK(s1.numel() == w.numel() || s1.data_ptr() == w.data_ptr(), "slot 1 size");
  TORCH_CHECK(reg_end % 4 == 0 && reg_end <= w.numel(), "reg_end");
  TORCH_CHECK(hp.size() == 9, "9 hyper-parameters expected");
  TORCH_CHECK(ticket.numel() >= 2, "optimizer_step: ticket[1] is the slot flag word");
  if (has_step) { CHECK_T(step, torch::kInt64); }
  float h[9];
  for (int i = 0; i < 9; ++i) h[i] = (float)hp[i];
  float* tgt = nullptr;
  if (target.has_value() && target->defined()) {   // fused hard target sync (needs the device step)
    CHECK_T((*target), torch::kFloat32);
    TORCH_CHECK(target->numel() == w.numel() && has_step && target_freq >= 1, "target sync args");
    tgt = ptr<float>(*target);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(w.device());
  launch_optimizer_step((int)op, ptr<float>(w), ptr<float>(grad), ptr<float>(s0), ptr<float>(s1),
                        ptr<float>(beta_pow), has_step ? ptr<int64_t>(step) : nullptr, ptr<int32_t>(ticket), h,
                        (float)lr, (float)reg, (int)reg_end, (float)grad_scale, (int)w.numel(), tgt,
                        (int)target_freq, cur_stream());
}

// optimizer step fused with the executor's weight packing (optim.hip optim_pack_kernel)
void optim_pack(int64_t op, torch::Tensor w, torch::Tensor grad, torch::Tensor s0, torch::Tensor s1,
                torch::Tensor beta_pow, torch::Tensor ticket, double lr, double reg, int64_t reg_end,
                double grad_scale, torch::Tensor step, std::vector<double> hp, torch::Tensor jobs,
                torch::Tensor packed, c10::optional<torch::Tensor> target, c10::optional<torch::Tensor> target_packed,
                int64_t target_freq, int64_t max_grid, c10::optional<torch::Tensor> noise,
                c10::optional<torch::Tensor> eff, c10::optional<torch::Tensor> grad_noise,
                c10::optional<torch::Tensor> noise_dst, std::vector<int64_t> sample, std::vector<int64_t> per_p,
                std::vector<double> per_f, c10::optional<torch::Tensor> tnoise, c10::optional<torch::Tensor> teff,
                c10::optional<torch::Tensor> tpk, c10::optional<torch::Tensor> noise_rng, std::vector<int64_t> fc,
                int64_t part, int64_t wg, int64_t wg_blocks, std::vector<int64_t> dp, int64_t tsg, bool no_pack) {
  // wg / wg_blocks: the launch also computes the grouped weight gradients -- a device WgradGroup
  // (qnet_wgrad_plan) whose wg_blocks tiles follow the lead block; jobs with dep >= 0 wait for
  // their member (needs fc: the launch forms the fc gradients from FcFuse rows)
  // dp: [] or [device DpExchange (xgmi_dpx_args), first, n, blocks] (WG launches under data
  //   parallelism): the job table's dependent jobs [first, first + n) sum their gradient over every
  //   rank inside the launch, run by `blocks` blocks
  // part: 0 or the base of the grouped conv wgrad's partial buffer (jobs with part_n > 0 sum it)
  // fc: [] or [x ptr, dh ptr, M, ldx, ldh]: the launch forms the fc weight / bias gradient of the
  // jobs carrying a dH column from those act_t rows (optim.hip FcFuse) instead of reading `grad`
  // noise_rng (noisy nets): [seed, counter] of the noise stream whose next samples an earlier
  // launch of this step drew (the fc dgrad's noise duty); the last block advances the counter
  // tnoise / teff / tpk (noisy nets): mix + pack the target under tnoise in the same launch
  // per_p: [] or [sum, min, max_p, P, levels, upd_idx, upd_td, rng, size, step, idx_out, w_out,
  //   state_idx, next_idx, actions, rewards, dones, gammas, a_out, r_out, d_out, g_out, st_slots,
  //   nx_slots, B] ; per_f: [alpha, eps, beta0, beta_steps] — prioritized variant of `sample`
  // sample: [] or 16 pointers (TrunkSample order) + B: an extra block draws the next step's
  // uniform minibatch (frame-stacked replay, k = 4)
  // grad_noise: derive the sigma gradients from the mu gradients under that noise sample;
  // noise_dst: the last block copies `noise` there (next sample becomes the current one)
  // op -1: no optimizer update, only the (noisy) mix + pack of w (noise / eff given)
  // tsg: 0 or the sigma-fragment buffer (packed layout) of a factorised target (UpdJob.eff bit 1):
  //   update calls with tnoise write it at a sync step, mix-only calls on that target every time
  // no_pack: update only (no packed fragments / copies; the async-PS server)
  CHECK_T(w, torch::kFloat32); CHECK_T(grad, torch::kFloat32); CHECK_T(s0, torch::kFloat32);
  CHECK_T(s1, torch::kFloat32); CHECK_T(beta_pow, torch::kFloat32); CHECK_T(ticket, torch::kInt32);
  CHECK_T(step, torch::kInt64); CHECK_T(jobs, torch::kInt32); CHECK_T(packed, DQN_ACT_F32 ? torch::kFloat32 : DQN_ACT_F16 ? torch::kHalf : torch::kBFloat16);
  TORCH_CHECK(grad.numel() == w.numel() && hp.size() == 9, "optim_pack args");
  TORCH_CHECK(jobs.numel() % upd_job_ints() == 0, "optim_pack: job table size");
  TORCH_CHECK(ticket.numel() >= 17 * 32, "optim_pack: the end-of-launch arrival counters need the 17x32-word ticket");
  TORCH_CHECK(max_grid >= 1 && max_grid <= 65535, "optim_pack: max_grid");
  TORCH_CHECK(op >= -1 && op <= 7, "optim_pack: op (7 = rmsprop without momentum)");
  float* tgt = nullptr;
  void* tgtp = nullptr;
  if (target.has_value() && target->defined()) {
    CHECK_T((*target), torch::kFloat32);
    TORCH_CHECK(target->numel() == w.numel() && target_freq >= 1, "optim_pack: target sync args");
    tgt = ptr<float>(*target);
    if (target_packed.has_value() && target_packed->defined()) {   // noisy nets: fp32 target only
      TORCH_CHECK(target_packed->numel() == packed.numel(), "optim_pack: target packed size");
      tgtp = target_packed->data_ptr();
    }
  }
  const float* nz = nullptr;
  float* ef = nullptr;
  if (noise.has_value() && noise->defined()) {
    CHECK_T((*noise), torch::kFloat32);
    nz = ptr<float>(*noise);
  }
  if (eff.has_value() && eff->defined()) {
    CHECK_T((*eff), torch::kFloat32);
    TORCH_CHECK(eff->numel() == w.numel(), "optim_pack: eff size");
    ef = ptr<float>(*eff);
  }
  TORCH_CHECK(op >= 0 || tgt == nullptr, "optim_pack: mix-only call with a target");
  const float* gnz = nullptr;
  float* ndst = nullptr;
  int nn = 0;
  if (grad_noise.has_value() && grad_noise->defined()) {
    CHECK_T((*grad_noise), torch::kFloat32);
    TORCH_CHECK(nz != nullptr && grad_noise->numel() == noise->numel(), "optim_pack: grad_noise size");
    gnz = ptr<float>(*grad_noise);
  }
  if (noise_dst.has_value() && noise_dst->defined()) {
    CHECK_T((*noise_dst), torch::kFloat32);
    TORCH_CHECK(op >= 0 && nz != nullptr && noise_dst->numel() == noise->numel() &&
                noise_dst->data_ptr() != noise->data_ptr(), "optim_pack: noise_dst");
    ndst = ptr<float>(*noise_dst);
    nn = (int)noise_dst->numel();
  }
  dqn::TrunkSample smp{};
  if (!sample.empty()) {
    TORCH_CHECK(op >= 0 && sample.size() == 17, "optim_pack sample: 16 pointers + B (update calls only)");
    for (int i = 0; i < 16; ++i) TORCH_CHECK(sample[i] != 0, "optim_pack sample: null pointer");
    smp.size = P<const int32_t*>(sample[0]); smp.rng = P<int64_t*>(sample[1]); smp.ticket = P<int32_t*>(sample[2]);
    smp.state_idx = P<const int32_t*>(sample[3]); smp.next_idx = P<const int32_t*>(sample[4]);
    smp.actions = P<const int32_t*>(sample[5]); smp.rewards = P<const float*>(sample[6]);
    smp.dones = P<const float*>(sample[7]); smp.gammas = P<const float*>(sample[8]);
    smp.idx_out = P<int32_t*>(sample[9]); smp.a_out = P<int32_t*>(sample[10]); smp.r_out = P<float*>(sample[11]);
    smp.d_out = P<float*>(sample[12]); smp.g_out = P<float*>(sample[13]);
    smp.st_slots = P<int32_t*>(sample[14]); smp.nx_slots = P<int32_t*>(sample[15]);
    smp.B = (int)sample[16];
    smp.ninst = 0;
    TORCH_CHECK(smp.B >= 1 && smp.B <= 512, "optim_pack sample: 1 <= B <= 512 (one lane per sample)");
  }
  PerStep per{};
  if (!per_p.empty()) {
    TORCH_CHECK(op >= 0 && sample.empty() && (per_p.size() == 25 || per_p.size() == 28) && per_f.size() == 4,
                "optim_pack per: 25 (+3 insertion) ints + 4 floats (update calls only, not with a uniform sample)");
    for (int i : {0, 1, 2, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23})
      TORCH_CHECK(per_p[i] != 0, "optim_pack per: null pointer ", i);
    per.sum = P<float*>(per_p[0]); per.mn = P<float*>(per_p[1]); per.maxp = P<float*>(per_p[2]);
    per.P = (int)per_p[3]; per.levels = (int)per_p[4];
    per.upd_idx = P<const int32_t*>(per_p[5]); per.upd_td = P<const float*>(per_p[6]);
    per.rng = P<int64_t*>(per_p[7]); per.size = P<const int32_t*>(per_p[8]); per.step = P<const int64_t*>(per_p[9]);
    per.idx_out = P<int32_t*>(per_p[10]); per.w_out = P<float*>(per_p[11]);
    per.so = SampleOut{P<const int32_t*>(per_p[12]), P<const int32_t*>(per_p[13]), 4, P<const int32_t*>(per_p[14]),
                       P<const float*>(per_p[15]), P<const float*>(per_p[16]), P<const float*>(per_p[17]),
                       P<int32_t*>(per_p[18]), P<float*>(per_p[19]), P<float*>(per_p[20]), P<float*>(per_p[21]),
                       P<int32_t*>(per_p[22]), P<int32_t*>(per_p[23])};
    per.B = (int)per_p[24];
    if (per_p.size() == 28) {        // [cursor, n new transitions, capacity]: fused acting's PER insertion
      per.ins_cursor = P<const int64_t*>(per_p[25]);
      per.ins_n = (int)per_p[26];
      per.ins_cap = (int)per_p[27];
      TORCH_CHECK(per.ins_cursor != nullptr && per.ins_n >= 0 && per.ins_cap >= 1 && per.ins_n <= per.ins_cap &&
                      per.ins_cap <= per.P, "optim_pack per: bad insertion spec");
    }
    per.alpha = (float)per_f[0]; per.eps = (float)per_f[1]; per.beta0 = (float)per_f[2];
    per.beta_steps = (float)per_f[3];
    TORCH_CHECK(per.B >= 1 && per.B <= 64 && per.P >= 2 && (per.P & (per.P - 1)) == 0 &&
                (1 << per.levels) == per.P && per.levels <= 30 && per.beta_steps >= 1.f,
                "optim_pack per: 1 <= B <= 64 (one-wave tree update), P = 2^levels, beta_steps >= 1");
    TORCH_CHECK(per.B + per.ins_n <= 64, "optim_pack per: batch + inserted transitions <= 64 (one wave)");
  }
  const float* tnz = nullptr;
  float* tef = nullptr;
  void* tpkp = nullptr;
  if (tnoise.has_value() && tnoise->defined()) {
    CHECK_T((*tnoise), torch::kFloat32);
    TORCH_CHECK(op >= 0 && tgt != nullptr && nz != nullptr && tnoise->numel() == noise->numel() &&
                teff.has_value() && teff->defined() && tpk.has_value() && tpk->defined(),
                "optim_pack: target mix needs target, noise, teff, tpk");
    CHECK_T((*teff), torch::kFloat32);
    CHECK_T((*tpk), DQN_ACT_F32 ? torch::kFloat32 : DQN_ACT_F16 ? torch::kHalf : torch::kBFloat16);
    TORCH_CHECK(teff->numel() == w.numel() && tpk->numel() == packed.numel() && tpk->data_ptr() != packed.data_ptr(),
                "optim_pack: teff / tpk sizes");
    tnz = ptr<float>(*tnoise);
    tef = ptr<float>(*teff);
    tpkp = tpk->data_ptr();
  }
  int64_t* nrng = nullptr;
  if (noise_rng.has_value() && noise_rng->defined()) {
    CHECK_T((*noise_rng), torch::kInt64);
    TORCH_CHECK(op >= 0 && noise_rng->numel() >= 2, "optim_pack: noise_rng = [seed, counter] (update calls)");
    nrng = ptr<int64_t>(*noise_rng);
  }
  FcFuse ff{nullptr, nullptr, 0, 0, 0};
  if (!fc.empty()) {
    TORCH_CHECK(op >= 0 && fc.size() == 5 && fc[0] != 0 && fc[1] != 0 && fc[2] >= 1 && fc[2] <= 4096 &&
                    fc[3] % 8 == 0 && fc[4] % 8 == 0 && (fc[0] % 16) == 0 && (fc[1] % 16) == 0,
                "optim_pack fc: [x, dh, 1 <= M <= 4096, ldx % 8 == 0, ldh % 8 == 0], 16-byte aligned rows");
    TORCH_CHECK(optim_fc_fuse(), "optim_pack fc: not available in this build");
    TORCH_CHECK(ticket.numel() >= 17 * 32, "optim_pack fc: one block per job needs the 17x32-word ticket");
    ff = FcFuse{P<const void*>(fc[0]), P<const void*>(fc[1]), (int)fc[2], (int)fc[3], (int)fc[4]};
  }
  TORCH_CHECK(ticket.numel() >= 2, "optim_pack: ticket[1] is the slot flag word");
  if (wg != 0) {
    TORCH_CHECK(wg_blocks >= 1 && wg_blocks <= 16384 && !fc.empty() && op >= 0 && part == 0 && (wg % 16) == 0,
                "optim_pack wg: needs fc rows and an update, no partials");
  }
  dqn::DpLaunch dpl{nullptr, 0, 0, 0};
  if (!dp.empty()) {
    const int64_t nj = jobs.numel() / upd_job_ints();
    TORCH_CHECK(wg != 0 && dp.size() == 4 && dp[0] != 0 && (dp[0] % 16) == 0 && dp[2] >= 1 &&
                    dp[2] <= dqn::kDpxMaxSlots && dp[1] >= 0 && dp[1] + dp[2] <= nj && dp[3] >= 1 && dp[3] <= dp[2],
                "optim_pack dp: [device DpExchange, first, n, blocks] with a WG launch, the dependent jobs inside "
                "the table, 1 <= blocks <= n <= DPX_MAX_SLOTS");
    dpl = dqn::DpLaunch{P<const dqn::DpExchange*>(dp[0]), (int)dp[1], (int)dp[2], (int)dp[3]};
  }
  float h[9];
  for (int i = 0; i < 9; ++i) h[i] = (float)hp[i];
  c10::hip::HIPGuardMasqueradingAsCUDA g(w.device());
  launch_optim_pack((int)op, ptr<float>(w), ptr<float>(grad), ptr<float>(s0), ptr<float>(s1), ptr<float>(beta_pow),
                    ptr<int64_t>(step), ptr<int32_t>(ticket), h, (float)lr, (float)reg, (int)reg_end,
                    (float)grad_scale, jobs.data_ptr(), (int)(jobs.numel() / upd_job_ints()), packed.data_ptr(), tgt,
                    tgtp, (int)target_freq, (int)max_grid, nz, ef, gnz, ndst, nn, sample.empty() ? nullptr : &smp,
                    per_p.empty() ? nullptr : &per, tnz, tef, tpkp, nrng, fc.empty() ? nullptr : &ff,
                    reinterpret_cast<const float*>(part), reinterpret_cast<const void*>(wg), (int)wg_blocks,
                    dp.empty() ? nullptr : &dpl, reinterpret_cast<void*>(tsg), no_pack ? 1 : 0, cur_stream());
}

void noise_normal(torch::Tensor out0, c10::optional<torch::Tensor> out1, torch::Tensor rng) {
  CHECK_T(out0, torch::kFloat32); CHECK_T(rng, torch::kInt64);
  TORCH_CHECK(rng.numel() >= 2, "noise rng state is [seed, counter]");
  float* o1 = nullptr;
  if (out1.has_value() && out1->defined()) {
    CHECK_T((*out1), torch::kFloat32);
    TORCH_CHECK(out1->numel() == out0.numel(), "noise_normal: out1 size");
    o1 = ptr<float>(*out1);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(out0.device());
  launch_noise_normal(ptr<float>(out0), o1, (int)out0.numel(), ptr<int64_t>(rng), cur_stream());
}

void target_update(torch::Tensor dst, torch::Tensor src, double tau, torch::Tensor step, int64_t freq,
                   bool use_step, std::vector<torch::Tensor> extra) {
  CHECK_T(dst, torch::kFloat32); CHECK_T(src, torch::kFloat32);
  TORCH_CHECK(dst.numel() == src.numel() && dst.numel() % 4 == 0, "target/online size");
  if (use_step) { CHECK_T(step, torch::kInt64); }
  c10::hip::HIPGuardMasqueradingAsCUDA g(dst.device());
  float* d2 = nullptr;
  const float* s2 = nullptr;
  int n2 = 0;
  if (!extra.empty()) {   // second buffer pair in the same launch (packed bf16 weights, viewed as f32)
    TORCH_CHECK(extra.size() == 2, "extra = [dst2, src2]");
    CHECK_T(extra[0], torch::kFloat32); CHECK_T(extra[1], torch::kFloat32);
    TORCH_CHECK(extra[0].numel() == extra[1].numel() && extra[0].numel() % 4 == 0, "extra pair size");
    d2 = ptr<float>(extra[0]); s2 = ptr<float>(extra[1]); n2 = (int)extra[0].numel();
  }
  launch_target_update(ptr<float>(dst), ptr<float>(src), (float)tau, use_step ? ptr<int64_t>(step) : nullptr,
                       (int)freq, (int)dst.numel(), d2, s2, n2, cur_stream());
}

void td_loss_scalar(torch::Tensor q, torch::Tensor qn_t, c10::optional<torch::Tensor> qn_o, torch::Tensor act,
                    torch::Tensor rew, torch::Tensor done, torch::Tensor gam, c10::optional<torch::Tensor> wts,
                    torch::Tensor loss, torch::Tensor dq, torch::Tensor prio, bool huber, double delta) {
  CHECK_T(q, torch::kFloat32); CHECK_T(qn_t, torch::kFloat32); CHECK_T(act, torch::kInt32);
  CHECK_T(rew, torch::kFloat32); CHECK_T(done, torch::kFloat32); CHECK_T(gam, torch::kFloat32);
  CHECK_T(loss, torch::kFloat32); CHECK_T(dq, torch::kFloat32); CHECK_T(prio, torch::kFloat32);
  const int B = (int)q.size(0), A = (int)q.size(1);
  TORCH_CHECK(B >= 1 && B <= 1024, "TD-loss batch must be in [1, 1024]");
  TORCH_CHECK(qn_t.sizes() == q.sizes() && dq.sizes() == q.sizes(), "Q shapes");
  TORCH_CHECK(act.numel() == B && rew.numel() == B && done.numel() == B && gam.numel() == B && prio.numel() == B,
              "per-sample vectors must be [B]");
  const float* qo = nullptr;
  if (qn_o.has_value()) { CHECK_T((*qn_o), torch::kFloat32); TORCH_CHECK(qn_o->sizes() == q.sizes()); qo = ptr<float>(*qn_o); }
  const float* w = nullptr;
  if (wts.has_value()) { CHECK_T((*wts), torch::kFloat32); TORCH_CHECK(wts->numel() == B); w = ptr<float>(*wts); }
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  launch_td_loss_scalar(ptr<float>(q), ptr<float>(qn_t), qo, ptr<int32_t>(act), ptr<float>(rew), ptr<float>(done),
                        ptr<float>(gam), w, ptr<float>(loss), ptr<float>(dq), ptr<float>(prio), B, A, huber ? 1 : 0,
                        (float)delta, cur_stream());
}

void td_loss_c51(torch::Tensor lg, torch::Tensor lgn_t, c10::optional<torch::Tensor> lgn_o, torch::Tensor act,
                 torch::Tensor rew, torch::Tensor done, torch::Tensor gam, c10::optional<torch::Tensor> wts,
                 torch::Tensor loss, torch::Tensor dlg, torch::Tensor prio, double vmin, double vmax) {
  CHECK_T(lg, torch::kFloat32); CHECK_T(lgn_t, torch::kFloat32); CHECK_T(act, torch::kInt32);
  CHECK_T(rew, torch::kFloat32); CHECK_T(done, torch::kFloat32); CHECK_T(gam, torch::kFloat32);
  CHECK_T(loss, torch::kFloat32); CHECK_T(dlg, torch::kFloat32); CHECK_T(prio, torch::kFloat32);
  TORCH_CHECK(lg.dim() == 3, "logits must be [B, A, N]");
  const int B = (int)lg.size(0), A = (int)lg.size(1), N = (int)lg.size(2);
  TORCH_CHECK(N >= 2 && N <= 64, "C51 atoms must be in [2, 64] (one wave per sample)");
  TORCH_CHECK(lgn_t.sizes() == lg.sizes() && dlg.sizes() == lg.sizes(), "logit shapes");
  TORCH_CHECK(act.numel() == B && rew.numel() == B && done.numel() == B && gam.numel() == B && prio.numel() == B);
  const float* lo = nullptr;
  if (lgn_o.has_value()) { CHECK_T((*lgn_o), torch::kFloat32); TORCH_CHECK(lgn_o->sizes() == lg.sizes()); lo = ptr<float>(*lgn_o); }
  const float* w = nullptr;
  if (wts.has_value()) { CHECK_T((*wts), torch::kFloat32); TORCH_CHECK(wts->numel() == B); w = ptr<float>(*wts); }
  c10::hip::HIPGuardMasqueradingAsCUDA g(lg.device());
  launch_td_loss_c51(ptr<float>(lg), ptr<float>(lgn_t), lo, ptr<int32_t>(act), ptr<float>(rew), ptr<float>(done),
                     ptr<float>(gam), w, ptr<float>(loss), ptr<float>(dlg), ptr<float>(prio), B, A, N, (float)vmin,
                     (float)vmax, cur_stream());
}

void preprocess_batch(torch::Tensor in, torch::Tensor out) {
  CHECK_T(in, torch::kUInt8); CHECK_T(out, torch::kUInt8);
  TORCH_CHECK(in.dim() == 4 && in.size(3) == 3 && out.dim() == 3 && out.size(0) == in.size(0), "shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(in.device());
  launch_preprocess_batch(ptr<uint8_t>(in), ptr<uint8_t>(out), (int)in.size(0), (int)in.size(1), (int)in.size(2),
                          (int)out.size(1), (int)out.size(2), cur_stream());
}

void preprocess_host(torch::Tensor in, torch::Tensor out) {
  TORCH_CHECK(!in.is_cuda() && in.scalar_type() == torch::kUInt8 && in.is_contiguous() && in.dim() == 3 &&
              in.size(2) == 3, "host RGB uint8 [H, W, 3]");
  TORCH_CHECK(!out.is_cuda() && out.scalar_type() == torch::kUInt8 && out.is_contiguous() && out.dim() == 2);
  dqn_preprocess_host(ptr<uint8_t>(in), (int)in.size(0), (int)in.size(1), ptr<uint8_t>(out), (int)out.size(0),
                      (int)out.size(1));
}

void actor_step(torch::Tensor q, torch::Tensor frames, torch::Tensor stacks, torch::Tensor cursor,
                torch::Tensor size_dev, torch::Tensor state_idx, torch::Tensor next_idx, torch::Tensor actions,
                torch::Tensor rewards, torch::Tensor dones, torch::Tensor gammas, torch::Tensor eps, torch::Tensor rng,
                torch::Tensor ticket, torch::Tensor frames_done, double gamma, double p_done) {
  CHECK_T(q, torch::kFloat32); CHECK_T(frames, torch::kUInt8); CHECK_T(stacks, torch::kInt32);
  CHECK_T(cursor, torch::kInt64); CHECK_T(size_dev, torch::kInt32); CHECK_T(state_idx, torch::kInt32);
  CHECK_T(next_idx, torch::kInt32); CHECK_T(actions, torch::kInt32); CHECK_T(rewards, torch::kFloat32);
  CHECK_T(dones, torch::kFloat32); CHECK_T(gammas, torch::kFloat32); CHECK_T(eps, torch::kFloat32);
  CHECK_T(rng, torch::kInt64); CHECK_T(ticket, torch::kInt32); CHECK_T(frames_done, torch::kInt64);
  const int E = (int)q.size(0), A = (int)q.size(1), K = (int)stacks.size(1);
  const int F = (int)frames.size(0), HW = (int)(frames.size(1) * frames.size(2)), C = (int)state_idx.size(0);
  TORCH_CHECK(stacks.size(0) == E && state_idx.size(1) == K, "stack shapes");
  TORCH_CHECK(K >= 1 && K <= 4, "actor: frames_per_state must be 1..4");
  TORCH_CHECK(cursor.numel() == 3 && eps.numel() == 3 && rng.numel() == 2, "state vectors");
  TORCH_CHECK(F >= 2 * C + K, "frame ring must hold 2C + k frames");
  TORCH_CHECK(E >= 1 && E <= C, "env count");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  launch_actor_step(ptr<float>(q), ptr<uint8_t>(frames), ptr<int32_t>(stacks), ptr<int64_t>(cursor),
                    ptr<int32_t>(size_dev), ptr<int32_t>(state_idx), ptr<int32_t>(next_idx), ptr<int32_t>(actions),
                    ptr<float>(rewards), ptr<float>(dones), ptr<float>(gammas), ptr<float>(eps), ptr<int64_t>(rng),
                    ptr<int32_t>(ticket), ptr<int64_t>(frames_done), E, A, K, HW, C, F, (float)gamma, (float)p_done,
                    cur_stream());
}

void stack_states(torch::Tensor frames, torch::Tensor stacks, torch::Tensor out) {
  CHECK_T(frames, torch::kUInt8); CHECK_T(stacks, torch::kInt32); CHECK_T(out, torch::kUInt8);
  const int E = (int)stacks.size(0), K = (int)stacks.size(1), HW = (int)(frames.size(1) * frames.size(2));
  TORCH_CHECK(out.numel() == (int64_t)E * HW * K, "out must be [E, H, W, K]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(frames.device());
  launch_stack_states(ptr<uint8_t>(frames), ptr<int32_t>(stacks), ptr<uint8_t>(out), E, HW, K, cur_stream());
}

uint32_t crc32c(py::bytes data) {
  std::string s = data;
  return dqn_crc32c(reinterpret_cast<const uint8_t*>(s.data()), s.size());
}

void ring_init(torch::Tensor buf, int64_t cap, int64_t rec) {
  TORCH_CHECK(!buf.is_cuda() && buf.numel() >= (int64_t)dqn_ring_bytes(cap, rec), "ring buffer too small");
  dqn_ring_init(ptr<uint8_t>(buf), cap, rec);
}
int64_t ring_push(torch::Tensor buf, torch::Tensor recs, int64_t n) {
  return dqn_ring_push(ptr<uint8_t>(buf), ptr<uint8_t>(recs), n);
}
int64_t ring_pop(torch::Tensor buf, torch::Tensor out, int64_t max_n) {
  return dqn_ring_pop(ptr<uint8_t>(buf), ptr<uint8_t>(out), max_n);
}
int64_t ring_size(torch::Tensor buf) { return dqn_ring_size(ptr<uint8_t>(buf)); }

// ---------------------------------------------------------------- xGMI all-reduce
// Fine-grained (uncached) device memory: peers read/write it over xGMI with no stale
// cache lines (csrc/kernels/xgmi_ar.hip). Zeroed on allocation.
int64_t xgmi_alloc(int64_t nbytes) {
  TORCH_CHECK(nbytes > 0, "xgmi_alloc: size");
  void* p = nullptr;
  TORCH_CHECK(hipExtMallocWithFlags(&p, (size_t)nbytes, hipDeviceMallocUncached) == hipSuccess,
              "hipExtMallocWithFlags(uncached) failed");
  TORCH_CHECK(hipMemset(p, 0, (size_t)nbytes) == hipSuccess && hipDeviceSynchronize() == hipSuccess,
              "xgmi_alloc: memset");
  return reinterpret_cast<int64_t>(p);
}
void xgmi_free(int64_t p) { if (p) (void)hipFree(reinterpret_cast<void*>(p)); }
torch::Tensor xgmi_ipc_handle(int64_t p) {
  hipIpcMemHandle_t h;
  TORCH_CHECK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(p)) == hipSuccess, "hipIpcGetMemHandle failed");
  auto out = torch::empty({(int64_t)sizeof(h)}, torch::kUInt8);
  std::memcpy(out.data_ptr(), &h, sizeof(h));
  return out;
}
int64_t xgmi_ipc_open(torch::Tensor handle) {
  hipIpcMemHandle_t h;
  TORCH_CHECK(!handle.is_cuda() && handle.numel() == (int64_t)sizeof(h) && handle.scalar_type() == torch::kUInt8,
              "ipc handle: uint8 CPU tensor of the handle size");
  std::memcpy(&h, handle.data_ptr(), sizeof(h));
  void* p = nullptr;
  TORCH_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess, "hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}
void xgmi_ipc_close(int64_t p) { if (p) (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(p)); }

// ------------------------------------------------------ async PS over xGMI (async_ps.hip)
// A page-aligned host range (e.g. a shared /dev/shm mapping) registered for GPU access:
// returns its device address (kernels poll / publish the PS control words there).
int64_t host_register(int64_t p, int64_t nbytes) {
  TORCH_CHECK(p && nbytes > 0 && (p & 4095) == 0, "host_register: page-aligned range");
  TORCH_CHECK(hipHostRegister(reinterpret_cast<void*>(p), (size_t)nbytes, hipHostRegisterMapped) == hipSuccess,
              "hipHostRegister failed");
  void* d = nullptr;
  TORCH_CHECK(hipHostGetDevicePointer(&d, reinterpret_cast<void*>(p), 0) == hipSuccess,
              "hipHostGetDevicePointer failed");
  return reinterpret_cast<int64_t>(d);
}
void host_unregister(int64_t p) { if (p) (void)hipHostUnregister(reinterpret_cast<void*>(p)); }

// non-owning fp32 view of n floats of device memory at p (a peer-mapped / fine-grained region)
torch::Tensor tensor_from_ptr(int64_t p, int64_t n, int64_t device) {
  TORCH_CHECK(p && n > 0 && (p & 15) == 0, "tensor_from_ptr: 16-byte aligned pointer");
  return torch::from_blob(reinterpret_cast<void*>(p), {n},
                          torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, (int)device));
}

void ps_push(torch::Tensor grad, int64_t slot, int64_t push_word, torch::Tensor seq, int64_t kind,
             torch::Tensor ticket) {
  CHECK_T(grad, torch::kFloat32); CHECK_T(seq, torch::kInt64); CHECK_T(ticket, torch::kInt32);
  TORCH_CHECK(grad.numel() % 4 == 0 && slot && push_word && (slot & 15) == 0 && kind >= 0 && kind < 16,
              "ps_push args");
  c10::hip::HIPGuardMasqueradingAsCUDA g(grad.device());
  launch_ps_push(ptr<float>(grad), reinterpret_cast<float*>(slot), (long)grad.numel(),
                 reinterpret_cast<uint64_t*>(push_word), ptr<int64_t>(seq), (int)kind, ptr<int32_t>(ticket),
                 cur_stream());
}

// --ps_lowrank: the push as up to 6 pieces (raw device pointers, 16-byte aligned, lengths % 16 == 0)
void ps_push_segs(std::vector<int64_t> src, std::vector<int64_t> dst, std::vector<int64_t> nbytes, int64_t push_word,
                  torch::Tensor seq, int64_t kind, torch::Tensor ticket) {
  CHECK_T(seq, torch::kInt64); CHECK_T(ticket, torch::kInt32);
  TORCH_CHECK(src.size() == dst.size() && src.size() == nbytes.size() && push_word && kind >= 0 && kind < 16,
              "ps_push_segs args");
  std::vector<const void*> s(src.size());
  std::vector<void*> d(dst.size());
  std::vector<long> nb(nbytes.size());
  for (size_t k = 0; k < src.size(); ++k) {
    s[k] = reinterpret_cast<const void*>(src[k]);
    d[k] = reinterpret_cast<void*>(dst[k]);
    nb[k] = (long)nbytes[k];
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(seq.device());
  TORCH_CHECK(launch_ps_push_segs(s.data(), d.data(), nb.data(), (int)src.size(), reinterpret_cast<uint64_t*>(push_word),
                                  ptr<int64_t>(seq), (int)kind, ptr<int32_t>(ticket), cur_stream()) == 0,
              "ps_push_segs: 1..6 pieces, 16-byte aligned, lengths % 16 == 0");
}

// seq: int64 [2] = (push number, gate number) device words of this worker
void ps_pull(torch::Tensor flat, int64_t snap, torch::Tensor step, int64_t snap_step, int64_t done_word,
             torch::Tensor seq, torch::Tensor gate, torch::Tensor err, torch::Tensor stopped, int64_t timeout_ns) {
  CHECK_T(flat, torch::kFloat32); CHECK_T(step, torch::kInt64); CHECK_T(seq, torch::kInt64);
  CHECK_T(gate, torch::kInt64); CHECK_T(err, torch::kInt32); CHECK_T(stopped, torch::kInt32);
  TORCH_CHECK(gate.numel() >= 2, "ps_pull: gate = [seq, status]");
  TORCH_CHECK(flat.numel() % 4 == 0 && snap && snap_step && done_word && (snap & 15) == 0, "ps_pull args");
  c10::hip::HIPGuardMasqueradingAsCUDA g(flat.device());
  launch_ps_pull(ptr<float>(flat), reinterpret_cast<const float*>(snap), (long)flat.numel(), ptr<int64_t>(step),
                 reinterpret_cast<const int64_t*>(snap_step), reinterpret_cast<const uint64_t*>(done_word),
                 ptr<int64_t>(seq), ptr<int64_t>(gate), ptr<int32_t>(err), ptr<int32_t>(stopped), (long long)timeout_ns,
                 cur_stream());
}

// flat / step undefined: signal only (e.g. STOP)
// echo != 0: the done word takes the push number from that (host-shared) push word, see the kernel
void ps_publish(int64_t snap, c10::optional<torch::Tensor> flat, int64_t snap_step, c10::optional<torch::Tensor> step,
                int64_t done_word, int64_t value, torch::Tensor ticket, int64_t n, int64_t echo) {
  CHECK_T(ticket, torch::kInt32);
  const float* f = nullptr;
  const int64_t* s = nullptr;
  if (flat.has_value() && flat->defined()) {
    CHECK_T((*flat), torch::kFloat32);
    TORCH_CHECK(flat->numel() == n && n % 4 == 0 && snap && (snap & 15) == 0, "ps_publish: flat");
    f = ptr<float>(*flat);
  }
  if (step.has_value() && step->defined()) {
    CHECK_T((*step), torch::kInt64);
    s = ptr<int64_t>(*step);
  }
  TORCH_CHECK(done_word && (s == nullptr || snap_step), "ps_publish args");
  c10::hip::HIPGuardMasqueradingAsCUDA g(ticket.device());
  launch_ps_publish(reinterpret_cast<float*>(snap), f, (long)n, reinterpret_cast<int64_t*>(snap_step), s,
                    reinterpret_cast<uint64_t*>(done_word), (uint64_t)value, ptr<int32_t>(ticket),
                    reinterpret_cast<const uint64_t*>(echo), cur_stream());
}

// grad: fp32 GPU slice to reduce in place; data/sig: one pointer per rank (mine included)
// ranges (optional): [lo0, hi0, lo1, hi1, ...] element ranges of grad summed as ONE vector
void xgmi_allreduce(torch::Tensor grad, std::vector<int64_t> data, std::vector<int64_t> sig, int64_t seq,
                    int64_t err, int64_t cap, int64_t rank, int64_t world, bool bf16, int64_t blocks,
                    std::vector<int64_t> ranges) {
  CHECK_T(grad, torch::kFloat32);
  TORCH_CHECK(world >= 1 && world <= dqn::kXgmiMaxRanks && rank >= 0 && rank < world, "xgmi: rank/world");
  TORCH_CHECK((int64_t)data.size() == world && (int64_t)sig.size() == world && seq && err, "xgmi: pointers");
  int64_t n = grad.numel();
  const int nr = (int)(ranges.size() / 2);
  TORCH_CHECK(ranges.size() % 2 == 0 && nr <= dqn::kXgmiMaxRanges, "xgmi: at most ", dqn::kXgmiMaxRanges, " ranges");
  if (nr > 0) {
    n = 0;
    int64_t prev = 0;
    for (int r = 0; r < nr; ++r) {
      const int64_t lo = ranges[2 * r], hi = ranges[2 * r + 1];
      TORCH_CHECK(lo >= prev && hi > lo && hi <= grad.numel() && lo % 4 == 0 && (hi - lo) % 4 == 0,
                  "xgmi: ranges ascending, disjoint, inside the buffer, multiples of 4");
      prev = hi;
      n += hi - lo;
    }
  }
  TORCH_CHECK(n % (4 * world) == 0 && n <= cap, "xgmi: n % (4 world) and capacity");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(grad.data_ptr()) & 15) == 0, "xgmi: 16-byte aligned gradient");
  TORCH_CHECK(blocks >= 1 && blocks <= dqn::kXgmiMaxBlocks, "xgmi: blocks");
  dqn::XgmiArgs a{};
  for (int i = 0; i < world; ++i) {
    TORCH_CHECK(data[i] && sig[i], "xgmi: null peer pointer");
    a.data[i] = reinterpret_cast<void*>(data[i]);
    a.sig[i] = reinterpret_cast<uint32_t*>(sig[i]);
  }
  a.seq = reinterpret_cast<uint32_t*>(seq);
  a.err = reinterpret_cast<int*>(err);
  a.grad = ptr<float>(grad);
  a.n = n;
  a.nr = nr;
  int64_t pre = 0;
  for (int r = 0; r < nr; ++r) {
    a.rlo[r] = ranges[2 * r];
    a.rpre[r] = pre;
    pre += ranges[2 * r + 1] - ranges[2 * r];
  }
  a.rpre[nr] = pre;
  a.cap = cap;
  a.rank = (int)rank; a.world = (int)world; a.bf16 = bf16 ? 1 : 0;
  c10::hip::HIPGuardMasqueradingAsCUDA g(grad.device());
  TORCH_CHECK(launch_xgmi_allreduce(a, (int)blocks, cur_stream()) == 0, "xgmi: launch arguments");
}

// srcs / outs: two segments each (byte pointers); bytes: per-rank segment sizes; cap: staging
// bytes per parity of this channel
void xgmi_allgather(std::vector<int64_t> srcs, std::vector<int64_t> outs, std::vector<int64_t> bytes,
                    std::vector<int64_t> data, std::vector<int64_t> sig, int64_t seq, int64_t err, int64_t cap,
                    int64_t rank, int64_t world, int64_t blocks, int64_t device) {
  TORCH_CHECK(world >= 1 && world <= dqn::kXgmiMaxRanks && rank >= 0 && rank < world, "xgmi gather: rank/world");
  TORCH_CHECK((int64_t)data.size() == world && (int64_t)sig.size() == world && seq && err, "xgmi gather: pointers");
  TORCH_CHECK(srcs.size() == 2 && outs.size() == 2 && bytes.size() == 2, "xgmi gather: two segments");
  TORCH_CHECK(blocks >= 1 && blocks <= dqn::kXgmiMaxBlocks, "xgmi gather: blocks");
  dqn::XgmiGatherArgs g{};
  for (int i = 0; i < world; ++i) {
    TORCH_CHECK(data[i] && sig[i], "xgmi gather: null peer pointer");
    g.x.data[i] = reinterpret_cast<void*>(data[i]);
    g.x.sig[i] = reinterpret_cast<uint32_t*>(sig[i]);
  }
  for (int s = 0; s < 2; ++s) {
    TORCH_CHECK(srcs[s] && outs[s] && bytes[s] >= 0 && bytes[s] % 16 == 0 && (srcs[s] & 15) == 0 && (outs[s] & 15) == 0,
                "xgmi gather: 16-byte aligned segments, sizes % 16 == 0");
    g.src[s] = reinterpret_cast<const void*>(srcs[s]);
    g.out[s] = reinterpret_cast<void*>(outs[s]);
    g.bytes[s] = bytes[s];
  }
  TORCH_CHECK(bytes[0] + bytes[1] <= cap, "xgmi gather: payload exceeds the channel's staging");
  g.x.seq = reinterpret_cast<uint32_t*>(seq);
  g.x.err = reinterpret_cast<int*>(err);
  g.x.cap = cap;
  g.x.rank = (int)rank; g.x.world = (int)world;
  c10::hip::HIPGuardMasqueradingAsCUDA guard((c10::DeviceIndex)device);
  TORCH_CHECK(launch_xgmi_allgather(g, (int)blocks, cur_stream()) == 0, "xgmi gather: launch arguments");
}

// the XgmiGatherArgs bytes (CPU uint8) of a gather over this channel: the fc dgrad launch's
// gather side duty reads them from device memory (copied there by the caller)
torch::Tensor xgmi_gather_args(std::vector<int64_t> srcs, std::vector<int64_t> outs, std::vector<int64_t> bytes,
                               std::vector<int64_t> data, std::vector<int64_t> sig, int64_t seq, int64_t err,
                               int64_t cap, int64_t rank, int64_t world) {
  TORCH_CHECK(world >= 1 && world <= dqn::kXgmiMaxRanks && rank >= 0 && rank < world, "xgmi gather: rank/world");
  TORCH_CHECK((int64_t)data.size() == world && (int64_t)sig.size() == world && seq && err, "xgmi gather: pointers");
  TORCH_CHECK(srcs.size() == 2 && outs.size() == 2 && bytes.size() == 2, "xgmi gather: two segments");
  dqn::XgmiGatherArgs g{};
  for (int i = 0; i < world; ++i) {
    TORCH_CHECK(data[i] && sig[i], "xgmi gather: null peer pointer");
    g.x.data[i] = reinterpret_cast<void*>(data[i]);
    g.x.sig[i] = reinterpret_cast<uint32_t*>(sig[i]);
  }
  for (int q = 0; q < 2; ++q) {
    TORCH_CHECK(srcs[q] && outs[q] && bytes[q] >= 0 && bytes[q] % 16 == 0 && (srcs[q] & 15) == 0 && (outs[q] & 15) == 0,
                "xgmi gather: 16-byte aligned segments, sizes % 16 == 0");
    g.src[q] = reinterpret_cast<const void*>(srcs[q]);
    g.out[q] = reinterpret_cast<void*>(outs[q]);
    g.bytes[q] = bytes[q];
  }
  TORCH_CHECK(bytes[0] + bytes[1] <= cap, "xgmi gather: payload exceeds the channel's staging");
  g.x.seq = reinterpret_cast<uint32_t*>(seq);
  g.x.err = reinterpret_cast<int*>(err);
  g.x.cap = cap;
  g.x.rank = (int)rank; g.x.world = (int)world;
  auto out = torch::empty({(int64_t)sizeof(g)}, torch::kUInt8);
  std::memcpy(out.data_ptr(), &g, sizeof(g));
  return out;
}

// the DpExchange bytes (CPU uint8) of an exchange channel: every rank's inbox / signal-word base
// (peer-mapped), this rank's per-slot counters and error word; the fused update launch reads them
// from device memory (copied there by the caller)
torch::Tensor xgmi_dpx_args(std::vector<int64_t> inbox, std::vector<int64_t> sig, int64_t seq, int64_t err,
                            int64_t rank, int64_t world, int64_t slots, int64_t cap) {
  TORCH_CHECK(world >= 1 && world <= dqn::kXgmiMaxRanks && rank >= 0 && rank < world, "xgmi dpx: rank/world");
  TORCH_CHECK((int64_t)inbox.size() == world && (int64_t)sig.size() == world && seq && err, "xgmi dpx: pointers");
  // (cap: the channel's elements per parity; the kernel addresses [2 parities][world][slots][elems])
  TORCH_CHECK(slots >= 1 && slots <= dqn::kDpxMaxSlots && world * slots * (int64_t)dqn::kDpxSlotElems <= cap,
              "xgmi dpx: slots exceed the channel's inbox");
  dqn::DpExchange x{};
  for (int i = 0; i < world; ++i) {
    TORCH_CHECK(inbox[i] && sig[i] && (inbox[i] & 15) == 0, "xgmi dpx: null / misaligned peer pointer");
    x.inbox[i] = reinterpret_cast<float*>(inbox[i]);
    x.sig[i] = reinterpret_cast<uint32_t*>(sig[i]);
  }
  x.seq = reinterpret_cast<uint32_t*>(seq);
  x.err = reinterpret_cast<int*>(err);
  x.rank = (int)rank; x.world = (int)world; x.slots = (int)slots;
  auto out = torch::empty({(int64_t)sizeof(x)}, torch::kUInt8);
  std::memcpy(out.data_ptr(), &x, sizeof(x));
  return out;
}

// one call of the exchange self-test over the channel described by `args` (xgmi_dpx_args bytes, CPU)
void xgmi_dpx_selftest(torch::Tensor args, torch::Tensor out, int64_t slots, int64_t call) {
  TORCH_CHECK(args.numel() == (int64_t)sizeof(dqn::DpExchange) && !args.is_cuda(), "dpx selftest: args bytes");
  CHECK_T(out, torch::kFloat32);
  dqn::DpExchange x;
  std::memcpy(&x, args.data_ptr(), sizeof(x));
  TORCH_CHECK(slots >= 1 && slots <= x.slots && out.numel() >= slots * (int64_t)dqn::kDpxSlotElems, "dpx selftest: slots");
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  TORCH_CHECK(launch_dpx_selftest(x, ptr<float>(out), (int)slots, (int)call, cur_stream()) == 0, "dpx selftest launch");
}

// ---------------------------------------------------------------- fused MLP
// ints: [L, A, P, Hs, Ds, sw, B, double, huber, fin x4, fout x4, act x4, w_off x4, b_off x4]
// ptrs: [w_on, w_tg, x, xn, act, rew, done, gam, wts, loss, prio, grad, q_out] (0 = unused)
void mlp(int64_t train, std::vector<int64_t> ints, std::vector<int64_t> ptrs, std::vector<double> flts,
         torch::Tensor like) {
  constexpr int NL = dqn::kMlpMaxLayers;
  TORCH_CHECK(ints.size() == 9 + 5 * NL && ptrs.size() == 13 && flts.size() == 2, "mlp: argument counts");
  CHECK_DEV(like);
  dqn::MlpArgs a{};
  a.L = (int)ints[0]; a.A = (int)ints[1]; a.P = (int)ints[2]; a.Hs = (int)ints[3]; a.Ds = (int)ints[4];
  a.sw = (int)ints[5]; a.B = (int)ints[6]; a.double_dqn = (int)ints[7]; a.huber = (int)ints[8];
  for (int l = 0; l < NL; ++l) {
    a.fin[l] = (int)ints[9 + l]; a.fout[l] = (int)ints[9 + NL + l]; a.act[l] = (int)ints[9 + 2 * NL + l];
    a.w_off[l] = (int)ints[9 + 3 * NL + l]; a.b_off[l] = (int)ints[9 + 4 * NL + l];
  }
  a.w_on = P<const float*>(ptrs[0]); a.w_tg = P<const float*>(ptrs[1]);
  a.x = P<const float*>(ptrs[2]); a.xn = P<const float*>(ptrs[3]); a.act_idx = P<const int32_t*>(ptrs[4]);
  a.rew = P<const float*>(ptrs[5]); a.done = P<const float*>(ptrs[6]); a.gam = P<const float*>(ptrs[7]);
  a.wts = P<const float*>(ptrs[8]); a.loss = P<float*>(ptrs[9]); a.prio = P<float*>(ptrs[10]);
  a.grad = P<float*>(ptrs[11]); a.q_out = P<float*>(ptrs[12]);
  a.delta = (float)flts[0]; a.in_scale = (float)flts[1];
  if (train) {
    TORCH_CHECK(a.w_on && a.w_tg && a.x && a.xn && a.act_idx && a.rew && a.done && a.gam && a.loss && a.prio &&
                a.grad, "mlp train: null operand");
  } else {
    TORCH_CHECK(a.w_on && a.x && a.q_out, "mlp forward: null operand");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(like.device());
  const int rc = launch_mlp(a, (int)train, cur_stream());
  TORCH_CHECK(rc == 0, "mlp: unsupported shape (code ", rc, ")");
}
int64_t mlp_lds_bytes(std::vector<int64_t> ints) {
  dqn::MlpArgs a{};
  a.P = (int)ints[0]; a.Hs = (int)ints[1]; a.Ds = (int)ints[2];
  return (int64_t)mlp_train_lds_bytes(a);
}

}  // namespace

void register_infer_server(pybind11::module_& m);   // infer_server.cpp
void register_ingest_server(pybind11::module_& m);  // ingest_server.cpp
void register_ps_server(pybind11::module_& m);      // ps_server.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "dist_dqn_amd native extension (gfx950 HIP kernels + C++ host runtime)";
  m.def("replay_sample_uniform", &replay_sample_uniform);
  m.def("mlp", &mlp);
  m.def("mlp_lds_bytes", &mlp_lds_bytes);
  m.def("xgmi_alloc", &xgmi_alloc);
  m.def("host_register", &host_register);
  m.def("host_unregister", &host_unregister);
  m.def("tensor_from_ptr", &tensor_from_ptr);
  m.def("ps_push", &ps_push);
  m.def("ps_push_segs", &ps_push_segs);
  m.def("ps_pull", &ps_pull);
  m.def("ps_publish", &ps_publish, pybind11::arg("snap"), pybind11::arg("flat"), pybind11::arg("snap_step"),
        pybind11::arg("step"), pybind11::arg("done_word"), pybind11::arg("value"), pybind11::arg("ticket"),
        pybind11::arg("n"), pybind11::arg("echo") = 0);
  m.def("xgmi_free", &xgmi_free);
  m.def("xgmi_ipc_handle", &xgmi_ipc_handle);
  m.def("xgmi_ipc_open", &xgmi_ipc_open);
  m.def("xgmi_ipc_close", &xgmi_ipc_close);
  m.def("xgmi_allreduce", &xgmi_allreduce, pybind11::arg("grad"), pybind11::arg("data"), pybind11::arg("sig"),
        pybind11::arg("seq"), pybind11::arg("err"), pybind11::arg("cap"), pybind11::arg("rank"), pybind11::arg("world"),
        pybind11::arg("bf16"), pybind11::arg("blocks"), pybind11::arg("ranges") = std::vector<int64_t>{});
  m.def("xgmi_allgather", &xgmi_allgather);
  m.def("xgmi_gather_args", &xgmi_gather_args);
  m.def("xgmi_dpx_args", &xgmi_dpx_args);
  m.def("xgmi_dpx_selftest", &xgmi_dpx_selftest);
  m.attr("DPX_MAX_SLOTS") = dqn::kDpxMaxSlots;
  m.attr("DPX_SLOT_ELEMS") = dqn::kDpxSlotElems;
  m.attr("XGMI_MAX_BLOCKS") = dqn::kXgmiMaxBlocks;
  m.attr("XGMI_SIG_WORDS") = dqn::kXgmiMaxRanks * dqn::kXgmiMaxBlocks;
  m.def("replay_gather_frames", &replay_gather_frames);
  m.def("sumtree_set", &sumtree_set);
  m.def("sumtree_sample", &sumtree_sample);
  m.def("optimizer_step", &optimizer_step, pybind11::arg("op"), pybind11::arg("w"), pybind11::arg("grad"),
        pybind11::arg("s0"), pybind11::arg("s1"), pybind11::arg("beta_pow"), pybind11::arg("ticket"), pybind11::arg("lr"),
        pybind11::arg("reg"), pybind11::arg("reg_end"), pybind11::arg("grad_scale"), pybind11::arg("step"),
        pybind11::arg("has_step"), pybind11::arg("hp"), pybind11::arg("target") = pybind11::none(),
        pybind11::arg("target_freq") = 1);
  m.def("target_update", &target_update);
  m.def("optim_pack", &optim_pack, pybind11::arg("op"), pybind11::arg("w"), pybind11::arg("grad"),
        pybind11::arg("s0"), pybind11::arg("s1"), pybind11::arg("beta_pow"), pybind11::arg("ticket"),
        pybind11::arg("lr"), pybind11::arg("reg"), pybind11::arg("reg_end"), pybind11::arg("grad_scale"),
        pybind11::arg("step"), pybind11::arg("hp"), pybind11::arg("jobs"), pybind11::arg("packed"),
        pybind11::arg("target"), pybind11::arg("target_packed"), pybind11::arg("target_freq"),
        pybind11::arg("max_grid"), pybind11::arg("noise"), pybind11::arg("eff"), pybind11::arg("grad_noise"),
        pybind11::arg("noise_dst"), pybind11::arg("sample"), pybind11::arg("per_p"), pybind11::arg("per_f"),
        pybind11::arg("tnoise"), pybind11::arg("teff"), pybind11::arg("tpk"), pybind11::arg("noise_rng"),
        pybind11::arg("fc"), pybind11::arg("part"), pybind11::arg("wg") = 0, pybind11::arg("wg_blocks") = 0,
        pybind11::arg("dp") = std::vector<int64_t>{}, pybind11::arg("tsg") = 0, pybind11::arg("no_pack") = false);
  m.def("noise_normal", &noise_normal);
  m.attr("UPD_JOB_INTS") = upd_job_ints();
  m.def("optim_prof", []() {
    std::vector<int64_t> v(16, 0);
    optim_prof_read(v.data());
    return v;
  }, "optim_pack s_memtime phase stamps of blocks 0 and 1 (DQN_OPT_PROF=1 launches)");
  m.def("optim_timeline", [](int64_t nblocks) {
    std::vector<int64_t> v(3 * (size_t)std::max<int64_t>(nblocks, 0), 0);
    const int n = optim_timeline_read(v.data(), (int)nblocks);
    v.resize(3 * (size_t)n);
    return v;
  }, "per-block [start, ready, end] s_memrealtime stamps (100 MHz) of the last DQN_OPT_PROF=1 optim_pack launch");
  m.def("optim_tile_phases", [](int64_t nblocks) {
    std::vector<int64_t> v(8 * (size_t)std::max<int64_t>(nblocks, 0), 0);
    const int n = optim_tile_phases_read(v.data(), (int)nblocks);
    v.resize(8 * (size_t)n);
    return v;
  }, "[8] s_memrealtime phase stamps of each of the first weight-gradient tiles of the last probe launch");
  m.attr("OPTIM_FC_FUSE") = optim_fc_fuse();
  m.def("td_loss_scalar", &td_loss_scalar);
  m.def("td_loss_c51", &td_loss_c51);
  m.def("preprocess_batch", &preprocess_batch);
  m.def("preprocess_host", &preprocess_host);
  m.def("actor_step", &actor_step);
  m.def("stack_states", &stack_states);
  m.def("crc32c", &crc32c);
  m.def("ring_bytes", [](int64_t cap, int64_t rec) { return (int64_t)dqn_ring_bytes(cap, rec); });
  m.def("ring_init", &ring_init);
  m.def("ring_push", &ring_push);
  m.def("ring_pop", &ring_pop);
  m.def("ring_size", &ring_size);
  register_net_ops(m);
  register_infer_server(m);
  register_ingest_server(m);
  register_ps_server(m);
}
