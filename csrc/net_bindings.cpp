// Bindings for the Q-network kernels (csrc/kernels/qnet.hip).
//
// The Python executor (dist_dqn_amd/ops/executor.py) builds a static launch
// plan once per (architecture, batch): it validates every buffer's shape,
// dtype and device there, then hands raw device addresses to these entry
// points, which only assemble the argument structs and launch on the current
// HIP stream (so the whole step can be captured into one HIP graph).
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "include/dqn_nets.h"
#include "include/dqn_nets_k.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

template <typename T>
T P(int64_t v) { return reinterpret_cast<T>(static_cast<intptr_t>(v)); }

void pack(int64_t src, int64_t dst, int64_t jobs, int64_t njobs, int64_t max_threads, int64_t dst2, int64_t step,
          int64_t freq) {
  TORCH_CHECK(dst2 == 0 || (step != 0 && freq >= 1), "pack: a second destination needs the device step");
  launch_pack(P<const float*>(src), P<void*>(dst), P<const dqn::PackJob*>(jobs), (int)njobs, (int)max_threads,
              P<void*>(dst2), P<const int64_t*>(step), (int)freq, cur_stream());
}

dqn::ConvArgs conv_args(const std::vector<int64_t>& in, const std::vector<int64_t>& w,
                        const std::vector<int64_t>& bias, const std::vector<int64_t>& out,
                        const std::vector<int64_t>& mask, const std::vector<double>& scale,
                        const std::vector<int64_t>& d) {
  TORCH_CHECK(d.size() == 11 || d.size() == 13, "dims: M, N, K, N16, ldo, IH, IW, OH, OW, pad_t, pad_l[, frames, hw]");
  TORCH_CHECK(in.size() >= 1 && in.size() <= (size_t)dqn::kMaxInst, "1..4 instances");
  dqn::ConvArgs a{};
  for (size_t i = 0; i < in.size(); ++i) {
    a.in[i] = P<const void*>(in[i]);
    a.w[i] = i < w.size() ? P<const void*>(w[i]) : nullptr;
    a.bias[i] = i < bias.size() ? P<const float*>(bias[i]) : nullptr;
    a.out[i] = i < out.size() ? P<void*>(out[i]) : nullptr;
    a.mask[i] = i < mask.size() ? P<const void*>(mask[i]) : nullptr;
    a.scale[i] = i < scale.size() ? (float)scale[i] : 1.f;
  }
  a.M = (int)d[0]; a.N = (int)d[1]; a.K = (int)d[2]; a.N16 = (int)d[3]; a.ldo = (int)d[4];
  a.IH = (int)d[5]; a.IW = (int)d[6]; a.OH = (int)d[7]; a.OW = (int)d[8]; a.pad_t = (int)d[9]; a.pad_l = (int)d[10];
  if (d.size() == 13) { a.frames = P<const void*>(d[11]); a.frame_hw = (int)d[12]; }
  return a;
}

// aux = [] or [zero_ptr (16 B aligned), zero_n (% 4 == 0), loss_parts, nparts (<= 64), loss_out]
// with aux_f = [loss_mul]: the launch's side duties (ConvArgs)
void igemm(int64_t kind, std::vector<int64_t> in, std::vector<int64_t> w, std::vector<int64_t> bias,
           std::vector<int64_t> out, std::vector<int64_t> mask, std::vector<double> scale, std::vector<int64_t> dims,
           std::vector<int64_t> aux, std::vector<double> aux_f, std::vector<int64_t> fz) {
  dqn::ConvArgs a = conv_args(in, w, bias, out, mask, scale, dims);
  // fz = [] or [instance, sigma fragments, noise, nsplit, ein0, eout0, ein1, eout1]: the dense forward's
  // factorised noisy instance (qnet.hip fc_fwd_fz_kernel)
  if (!fz.empty()) {
    TORCH_CHECK(kind == dqn::L_DENSE_FWD_RELU && fz.size() == 8 && fz[0] >= 0 && fz[0] < (int64_t)in.size() && fz[1] != 0 &&
                    fz[2] != 0 && fz[1] % 16 == 0 && a.M >= 1 && a.M <= 32 && a.N % 16 == 0 && a.N16 == a.N / 16 &&
                    a.K % 32 == 0 && a.K >= 8 * 32 && a.K <= 4096 && fz[3] % 16 == 0 && fz[3] >= 16 && fz[3] <= a.N &&
                    fz[4] >= 0 && fz[5] >= 0 && fz[6] >= 0 && fz[7] >= 0,
                "igemm fz: dense forward, [inst, w2, noise, nsplit % 16, ein0, eout0, ein1, eout1], M <= 32, "
                "N % 16 == 0, K % 32 == 0, 256 <= K <= 4096");
    a.fz_inst = (int)fz[0];
    a.fz_w2 = P<const void*>(fz[1]);
    a.fz_noise = P<const float*>(fz[2]);
    a.fz_nsplit = (int)fz[3];
    a.fz_ein[0] = (int)fz[4]; a.fz_eout[0] = (int)fz[5]; a.fz_ein[1] = (int)fz[6]; a.fz_eout[1] = (int)fz[7];
  }
  if (!aux.empty()) {
    // + optional noise duty [out0, out1, n, rng]: the next noisy-net samples at the stream's counter
    // + optional gather duty [gth (device XgmiGatherArgs), gth_blocks] at the end
    size_t na = aux.size();
    if (na == 7 || na == 11) {
      TORCH_CHECK(aux[na - 2] != 0 && aux[na - 1] >= 1 && aux[na - 1] <= 256, "igemm gather duty: args, 1..256 blocks");
      a.gth = P<const void*>(aux[na - 2]);
      a.gth_blocks = (int)aux[na - 1];
      a.gth_z = (int)in.size();
      aux.resize(na - 2);
    }
    TORCH_CHECK((aux.size() == 5 || aux.size() == 9) && aux_f.size() == 1 && aux[0] % 16 == 0 && aux[1] % 4 == 0 &&
                aux[3] <= 64, "igemm aux = [zero_ptr, zero_n, loss_parts, nparts, loss_out(, nz_out0, nz_out1, "
                "nz_n, nz_rng)(, gth, gth_blocks)], [loss_mul]");
    if (aux.size() == 9) {
      TORCH_CHECK(aux[5] != 0 && aux[7] >= 1 && aux[8] != 0, "igemm noise duty: out0, n, rng");
      a.nz_out0 = P<float*>(aux[5]); a.nz_out1 = P<float*>(aux[6]); a.nz_n = (int)aux[7];
      a.nz_rng = P<const int64_t*>(aux[8]);
    }
    a.zero_ptr = P<float*>(aux[0]); a.zero_n = (int)aux[1];
    a.loss_parts = P<const float*>(aux[2]); a.nparts = (int)aux[3]; a.loss_out = P<float*>(aux[4]);
    a.loss_mul = (float)aux_f[0];
    TORCH_CHECK(a.loss_parts == nullptr || a.loss_out != nullptr, "igemm aux: loss output");
  }
  TORCH_CHECK(launch_igemm((int)kind, a, (int)in.size(), cur_stream()) == 0, "unknown igemm kind ", kind);
}

// The Nature dgrad chain in one launch (qnet.hip dgrad_chain_kernel): the fc dgrad (with its aux
// side duties, as igemm), the conv3 dgrad and the conv2 parity dgrad; cnt: int32 counters, one per
// 32 ints ((ceil(B / 16) + B + 1) * 32, zeroed by the step's fc forward launch)
void dgrad_chain(int64_t in0, int64_t w0, int64_t out0, int64_t mask0, std::vector<int64_t> dims0,
                 std::vector<int64_t> aux0, std::vector<double> aux_f0, int64_t w1, int64_t out1, int64_t mask1,
                 std::vector<int64_t> dims1, int64_t w2, int64_t out2, int64_t mask2, std::vector<int64_t> dims2,
                 int64_t cnt, int64_t B) {
  dqn::ConvArgs a0 = conv_args({in0}, {w0}, {}, {out0}, {mask0}, {1.0}, dims0);
  TORCH_CHECK((aux0.size() == 5 || aux0.size() == 9) && aux_f0.size() == 1 && aux0[0] % 16 == 0 && aux0[1] % 4 == 0 &&
                  aux0[3] <= 64, "dgrad_chain aux = [zero_ptr, zero_n, loss_parts, nparts, loss_out(, noise)]");
  a0.zero_ptr = P<float*>(aux0[0]); a0.zero_n = (int)aux0[1];
  a0.loss_parts = P<const float*>(aux0[2]); a0.nparts = (int)aux0[3]; a0.loss_out = P<float*>(aux0[4]);
  a0.loss_mul = (float)aux_f0[0];
  if (aux0.size() == 9) {
    TORCH_CHECK(aux0[5] != 0 && aux0[7] >= 1 && aux0[8] != 0, "dgrad_chain noise duty: out0, n, rng");
    a0.nz_out0 = P<float*>(aux0[5]); a0.nz_out1 = P<float*>(aux0[6]); a0.nz_n = (int)aux0[7];
    a0.nz_rng = P<const int64_t*>(aux0[8]);
  }
  TORCH_CHECK(a0.loss_parts == nullptr || a0.loss_out != nullptr, "dgrad_chain aux: loss output");
  dqn::ConvArgs a1 = conv_args({out0}, {w1}, {}, {out1}, {mask1}, {1.0}, dims1);
  dqn::ConvArgs a2 = conv_args({out1}, {w2}, {}, {out2}, {mask2}, {1.0}, dims2);   // out2 = 0: two stages
  TORCH_CHECK(launch_dgrad_chain(a0, a1, a2, P<int32_t*>(cnt), (int)B, cur_stream()) == 0,
              "dgrad_chain: shapes outside the chained kernel");
}

void wgrad(int64_t kind, int64_t in, std::vector<int64_t> dims, int64_t dz, int64_t ldz, int64_t dw, int64_t db,
           int64_t dw2, int64_t db2, int64_t nsplit, int64_t N, int64_t MC, int64_t KB, int64_t NB, double scale,
           bool atomic, int64_t mloop, bool db_zero) {
  dqn::ConvArgs a = conv_args({in}, {}, {}, {}, {}, {1.0}, dims);
  dqn::WgradArgs g{};
  g.mloop = (int)mloop; g.db_zero = db_zero ? 1 : 0;
  TORCH_CHECK(mloop >= 1 && mloop <= 64, "wgrad: 1 <= mloop <= 64");
  g.dz = P<const void*>(dz); g.ldz = (int)ldz;
  g.dw = P<float*>(dw); g.db = P<float*>(db); g.dw2 = P<float*>(dw2); g.db2 = P<float*>(db2);
  g.nsplit = (int)nsplit; g.N = (int)N; g.MC = (int)MC; g.KB = (int)KB; g.NB = (int)NB;
  g.scale = (float)scale; g.atomic = atomic ? 1 : 0;
  TORCH_CHECK(KB % 16 == 0 && NB % 16 == 0 && MC % 32 == 0, "wgrad tiling");
  TORCH_CHECK((KB / 16) * (NB / 16) <= 48, "wgrad: at most 48 output tiles per block");
  TORCH_CHECK(launch_wgrad((int)kind, a, g, cur_stream()) == 0, "unknown wgrad kind ", kind);
}

dqn::HeadArgs head_args(const std::vector<int64_t>& ints, const std::vector<int64_t>& h,
                        const std::vector<int64_t>& w, const std::vector<int64_t>& b, const std::vector<int64_t>& wv,
                        const std::vector<int64_t>& bv, const std::vector<int64_t>& io, const std::vector<int64_t>& pw,
                        const std::vector<int64_t>& pwv, const std::vector<int64_t>& zero,
                        const std::vector<int64_t>& actor, const std::vector<double>& actor_f, int64_t act_h = 0) {
  // ints: B, A, HID, dueling, huber, infer
  // io: act, rew, done, gam, wts, loss, prio, q_out, dw, db, dwv, dbv, dh
  TORCH_CHECK(ints.size() == 6 && io.size() == 13, "head args");
  TORCH_CHECK(ints[1] >= 1 && ints[1] <= 32, "1..32 actions");
  TORCH_CHECK(ints[2] % 128 == 0, "head hidden size must be a multiple of 128");
  dqn::HeadArgs a{};
  a.B = (int)ints[0]; a.A = (int)ints[1]; a.HID = (int)ints[2]; a.dueling = (int)ints[3]; a.huber = (int)ints[4];
  a.infer = (int)ints[5];
  a.atoms = 1; a.vmin = 0.f; a.vmax = 0.f;
  for (size_t i = 0; i < 3; ++i) {
    a.h[i] = i < h.size() ? P<const void*>(h[i]) : nullptr;
    a.w[i] = i < w.size() ? P<const float*>(w[i]) : nullptr;
    a.b[i] = i < b.size() ? P<const float*>(b[i]) : nullptr;
    a.wv[i] = i < wv.size() ? P<const float*>(wv[i]) : nullptr;
    a.bv[i] = i < bv.size() ? P<const float*>(bv[i]) : nullptr;
    a.pw[i] = i < pw.size() ? P<const void*>(pw[i]) : nullptr;
    a.pwv[i] = i < pwv.size() ? P<const void*>(pwv[i]) : nullptr;
  }
  a.N16 = (a.A + 15) / 16;
  if (!zero.empty()) {
    TORCH_CHECK(zero.size() == 2 && zero[1] % 4 == 0 && zero[0] % 16 == 0, "zero = [ptr (16B aligned), n % 4 == 0]");
    a.zero_ptr = P<float*>(zero[0]); a.zero_n = (int)zero[1];
  }
  if (!actor.empty()) {
    // actor = 15 pointers (ActorArgs order, q unused) + E, A, K, HW, C, F
    //         [+ PER tree: sum, min, max_p, P, levels] ; actor_f = gamma, p_done
    TORCH_CHECK((actor.size() == 21 || actor.size() == 26) && actor_f.size() == 2, "fused actor args");
    dqn::ActorArgs& x = a.actor;
    x.q = nullptr; x.frames = P<uint8_t*>(actor[1]); x.stacks = P<int32_t*>(actor[2]);
    x.cursor = P<int64_t*>(actor[3]); x.size_dev = P<int32_t*>(actor[4]); x.state_idx = P<int32_t*>(actor[5]);
    x.next_idx = P<int32_t*>(actor[6]); x.actions = P<int32_t*>(actor[7]); x.rewards = P<float*>(actor[8]);
    x.dones = P<float*>(actor[9]); x.gammas = P<float*>(actor[10]); x.eps = P<float*>(actor[11]);
    x.rng = P<int64_t*>(actor[12]); x.ticket = P<int32_t*>(actor[13]); x.frames_done = P<int64_t*>(actor[14]);
    x.E = (int)actor[15]; x.A = (int)actor[16]; x.K = (int)actor[17]; x.HW = (int)actor[18]; x.C = (int)actor[19];
    x.F = (int)actor[20]; x.gamma = (float)actor_f[0]; x.p_done = (float)actor_f[1];
    if (actor.size() == 26) {
      x.tsum = P<float*>(actor[21]); x.tmin = P<float*>(actor[22]); x.tmaxp = P<float*>(actor[23]);
      x.tP = (int)actor[24]; x.tlevels = (int)actor[25];
      TORCH_CHECK(x.tsum && x.tmin && x.tmaxp && x.tP >= x.C && (1 << x.tlevels) == x.tP && x.tlevels <= 30,
                  "actor PER tree: P = 2^levels >= capacity");
    }
    TORCH_CHECK(x.A == a.A, "actor action count");
    TORCH_CHECK(x.F >= 2 * x.C + x.K, "frame ring must hold 2C + k frames");
    TORCH_CHECK(x.K >= 1 && x.K <= 4 && x.E >= 1 && x.E <= 64, "fused actor: 1 <= K <= 4, 1 <= E <= 64");
    if (a.infer) {                 // acting launch: the batch IS the env batch
      TORCH_CHECK(x.E == a.B, "actor env batch must be the inference batch");
      a.has_actor = 1;
    } else {                       // learner launch + one fused acting workgroup
      TORCH_CHECK(act_h != 0 && x.E >= 1 && x.E <= a.B, "fused acting needs the actors' hidden layer, E <= B");
      a.act_h = P<const void*>(act_h);
      a.act_E = x.E;
    }
  }
  a.act = P<const int32_t*>(io[0]); a.rew = P<const float*>(io[1]); a.done = P<const float*>(io[2]);
  a.gam = P<const float*>(io[3]); a.wts = P<const float*>(io[4]);
  a.loss = P<float*>(io[5]); a.prio = P<float*>(io[6]); a.q_out = P<float*>(io[7]);
  a.dw = P<float*>(io[8]); a.db = P<float*>(io[9]); a.dwv = P<float*>(io[10]); a.dbv = P<float*>(io[11]);
  a.dh = P<void*>(io[12]);
  return a;
}

// members: per layer [kind, in, dz, ldz, dw, db, dw2, db2, nsplit, N] + dims (11 or 13) + scale
static dqn::WgradGroup build_group(const std::vector<std::vector<int64_t>>& members,
                                   const std::vector<std::vector<int64_t>>& dims, const std::vector<double>& scales) {
  TORCH_CHECK(members.size() >= 1 && members.size() <= (size_t)dqn::kMaxWgradMembers &&
              dims.size() == members.size() && scales.size() == members.size(), "1..6 group members");
  dqn::WgradGroup G{};
  G.n = (int)members.size();
  for (int i = 0; i < G.n; ++i) {
    const auto& m = members[i];
    TORCH_CHECK(m.size() == 10 || m.size() == 13,
                "member = [kind, in, dz, ldz, dw, db, dw2, db2, nsplit, N] (+ [part, pstride, mloop])");
    G.kind[i] = (int)m[0];
    G.a[i] = conv_args({m[1]}, {}, {}, {}, {}, {1.0}, dims[i]);
    dqn::WgradArgs& g = G.g[i];
    g.dz = P<const void*>(m[2]); g.ldz = (int)m[3];
    g.dw = P<float*>(m[4]); g.db = P<float*>(m[5]); g.dw2 = P<float*>(m[6]); g.db2 = P<float*>(m[7]);
    g.nsplit = (int)m[8]; g.N = (int)m[9]; g.scale = (float)scales[i];
    g.mloop = 1;
    if (m.size() == 13 && m[10] != 0) {          // deterministic partial member
      g.part = P<float*>(m[10]); g.pstride = (int)m[11]; g.mloop = (int)m[12];
      TORCH_CHECK(g.mloop >= 1 && g.mloop <= 64 && g.nsplit == g.N && g.dw2 == nullptr, "partial member args");
    }
  }
  return G;
}

void wgrad_group(std::vector<std::vector<int64_t>> members, std::vector<std::vector<int64_t>> dims,
                 std::vector<double> scales) {
  const dqn::WgradGroup G = build_group(members, dims, scales);
  const int rc = launch_wgrad_group(G, cur_stream());
  TORCH_CHECK(rc != -3, "wgrad group: partial members need 128-row chunks and pstride >= K*N + N");
  TORCH_CHECK(rc == 0, "unknown wgrad kind in group");
}

// The fused weight-gradient range of a split optimizer update (optim.hip kModeWg): the planned
// group as bytes (the caller keeps a device copy for the launches) and its block count.
// done: device int32 counters (>= 32 * kWgCounters words, zeroed; the launch leaves them zero).
// deps: [member, slot, first job, job count] per (member, K-range slot / bias slot kWgSlots - 1):
// the job-table ranges waiting on the slot (recorded in the plan; the jobs carry UpdJob.dep).
std::tuple<torch::Tensor, int64_t> wgrad_plan(std::vector<std::vector<int64_t>> members,
                                              std::vector<std::vector<int64_t>> dims, std::vector<double> scales,
                                              torch::Tensor done, std::vector<std::vector<int64_t>> deps,
                                              int64_t conv_chunks) {
  TORCH_CHECK(conv_chunks >= 1 && conv_chunks <= 64, "wgrad_plan: conv_chunks");
  TORCH_CHECK(done.is_cuda() && done.scalar_type() == torch::kInt32 && done.is_contiguous() &&
                  done.numel() >= 32 * (int64_t)dqn::kWgCounters, "wgrad_plan: done counters");
  dqn::WgradGroup G = build_group(members, dims, scales);
  G.done = done.data_ptr<int32_t>();
  for (const auto& d : deps) {
    TORCH_CHECK(d.size() == 4 && d[0] >= 0 && d[0] < G.n && d[1] >= 0 && d[1] < dqn::kWgSlots && d[2] >= 0 && d[3] >= 1,
                "wgrad_plan: dep = [member, slot, first, count]");
    G.dep_first[d[0]][d[1]] = (int)d[2];
    G.dep_count[d[0]][d[1]] = (int)d[3];
  }
  const int total = wgrad_fused_plan(G, (int)conv_chunks);
  TORCH_CHECK(total > 0, "wgrad_plan: a member has no fused tile (16-bit builds; conv / head members only)");
  for (int i = 0; i < G.n; ++i)
    TORCH_CHECK(G.gy[i] <= dqn::kWgSlots - 1, "wgrad_plan: more K-ranges than counter slots");
  torch::Tensor t = torch::empty({(int64_t)sizeof(dqn::WgradGroup)}, torch::kUInt8);
  memcpy(t.data_ptr(), &G, sizeof(G));
  return {t, (int64_t)total};
}

// ptrs (4 per group): slots, states, w1, w2, w3, b1, b2, b3, x3, then a1, p1, a2, p2, a3; M as in trunk
void cnn_fwd(int64_t frames, std::vector<int64_t> ptrs, int64_t B, int64_t ninst, double scale,
             std::vector<int64_t> M, int64_t prof) {
  constexpr int I = dqn::kMaxInst;
  TORCH_CHECK(ptrs.size() == 9 * I + 5 && ninst >= 1 && ninst <= I && B >= 1 && M.size() <= (size_t)I, "cnn_fwd args");
  dqn::CnnFwdArgs a{};
  a.frames = P<const uint8_t*>(frames);
  for (int i = 0; i < I; ++i) {
    a.slots[i] = P<const int32_t*>(ptrs[0 * I + i]); a.states[i] = P<const uint8_t*>(ptrs[1 * I + i]);
    a.w1[i] = P<const void*>(ptrs[2 * I + i]); a.w2[i] = P<const void*>(ptrs[3 * I + i]);
    a.w3[i] = P<const void*>(ptrs[4 * I + i]);
    a.b1[i] = P<const float*>(ptrs[5 * I + i]); a.b2[i] = P<const float*>(ptrs[6 * I + i]);
    a.b3[i] = P<const float*>(ptrs[7 * I + i]);
    a.x3[i] = P<act_t*>(ptrs[8 * I + i]);
    a.M[i] = i < (int)M.size() ? (int)M[i] : 0;
    TORCH_CHECK(a.M[i] >= 0 && a.M[i] <= B, "cnn_fwd: per-instance sample count");
    if (i < ninst) {
      TORCH_CHECK((a.slots[i] != nullptr && a.frames != nullptr) || a.states[i] != nullptr, "cnn_fwd input");
      TORCH_CHECK(a.w1[i] && a.w2[i] && a.w3[i] && a.b1[i] && a.b2[i] && a.b3[i] && a.x3[i], "cnn_fwd weights/out");
    }
  }
  a.a1 = P<act_t*>(ptrs[9 * I + 0]); a.p1 = P<act_t*>(ptrs[9 * I + 1]); a.a2 = P<act_t*>(ptrs[9 * I + 2]);
  a.p2 = P<act_t*>(ptrs[9 * I + 3]); a.a3 = P<act_t*>(ptrs[9 * I + 4]);
  a.prof = P<int64_t*>(prof);
  TORCH_CHECK(a.a1 == nullptr || (a.p1 && a.a2 && a.p2 && a.a3), "cnn_fwd: keep all activations or none");
  a.scale = (float)scale;
  launch_cnn_fwd(a, (int)B, (int)ninst, cur_stream());
}

// ptrs: dp3, a1, a2, a3, w3d, w2d, dz1, dz2, dz3
void cnn_bwd(std::vector<int64_t> ptrs, int64_t B, int64_t prof, int64_t parts) {
  TORCH_CHECK(ptrs.size() == 9 && B >= 1 && (parts == 1 || parts == 2 || parts == 4), "cnn_bwd args (parts 1, 2, 4)");
  for (auto p : ptrs) TORCH_CHECK(p != 0, "cnn_bwd: null pointer");
  dqn::CnnBwdArgs a{};
  a.dp3 = P<const act_t*>(ptrs[0]); a.a1 = P<const act_t*>(ptrs[1]); a.a2 = P<const act_t*>(ptrs[2]);
  a.a3 = P<const act_t*>(ptrs[3]); a.w3d = P<const void*>(ptrs[4]); a.w2d = P<const void*>(ptrs[5]);
  a.dz1 = P<act_t*>(ptrs[6]); a.dz2 = P<act_t*>(ptrs[7]); a.dz3 = P<act_t*>(ptrs[8]);
  a.prof = P<int64_t*>(prof);
  launch_cnn_bwd(a, (int)B, (int)parts, cur_stream());
}

// Scalar head. qp = [loss_parts, dq16]: per-16-sample-tile loss partials (training; summed by
// the fc dgrad launch's aux duty) and dQ as act_t [B][64] (the output layer's wgrad dZ); dH goes
// to io[12]. h = the learner instances' hidden layers (online(s), target(s')[, online(s')]) or,
// infer, the one instance; pw / pwv = their packed output-layer fragments.
void head_loss(std::vector<int64_t> ints, std::vector<double> flts, std::vector<int64_t> h, std::vector<int64_t> w,
               std::vector<int64_t> b, std::vector<int64_t> wv, std::vector<int64_t> bv, std::vector<int64_t> io,
               std::vector<int64_t> pw, std::vector<int64_t> pwv, std::vector<int64_t> qp,
               std::vector<int64_t> actor, std::vector<double> actor_f, int64_t act_h, int64_t prof) {
  TORCH_CHECK(flts.size() == 1, "flts = [huber delta]");
  TORCH_CHECK(qp.size() == 2, "qp = [loss_parts, dq16]");
  dqn::HeadArgs a = head_args(ints, h, w, b, wv, bv, io, pw, pwv, {}, actor, actor_f, act_h);
  a.prof = P<int64_t*>(prof);
  a.delta = (float)flts[0];
  a.loss_parts = P<float*>(qp[0]);
  a.dq16 = P<void*>(qp[1]);
  const int ninst = a.infer ? 1 : (a.h[2] != nullptr ? 3 : 2);
  for (int i = 0; i < ninst; ++i) TORCH_CHECK(a.h[i] && a.pw[i] && a.b[i] && (!a.dueling || (a.pwv[i] && a.bv[i])),
                                              "head: instance ", i, " pointers");
  TORCH_CHECK(a.infer || (a.dq16 && a.loss_parts && a.dh && a.w[0] && (!a.dueling || a.wv[0]) && a.B <= 1024),
              "head: training outputs / online output layer");
  TORCH_CHECK(a.HID <= 512 && a.A <= 32, "scalar head: hidden width <= 512, A <= 32");
  TORCH_CHECK(!a.has_actor || a.actor.E <= 64, "head: acting E <= 64");
  launch_head_loss(a, cur_stream());
}

// Fused fc forward + scalar head (fc_head.hip): fc args as igemm (instances: the learner's, then
// the fused actors'), head args as head_loss (h = the learner instances' hidden rows = the fc
// outputs), fold = [qacc, cnt, Mpad, nlearn]: the fp32 partial-Q slots ([ninst][Mpad][32][N / 16])
// and the row-group counters (>= Mpad / 16 + 1 int32, zeroed; left zero).
void fc_head(std::vector<int64_t> in, std::vector<int64_t> w, std::vector<int64_t> bias, std::vector<int64_t> out,
             std::vector<int64_t> dims, std::vector<int64_t> ints, std::vector<double> flts, std::vector<int64_t> h,
             std::vector<int64_t> hw, std::vector<int64_t> hb, std::vector<int64_t> hwv, std::vector<int64_t> hbv,
             std::vector<int64_t> io, std::vector<int64_t> qp, std::vector<int64_t> actor, std::vector<double> actor_f,
             int64_t act_h, std::vector<int64_t> fold, int64_t prof, bool two_per_cu) {
  // two_per_cu: spin mode may run two blocks per CU (the executor's KernelTuning.fold_two_per_cu)
  dqn::ConvArgs a = conv_args(in, w, bias, out, {}, std::vector<double>(in.size(), 1.0), dims);
  TORCH_CHECK(flts.size() == 1 && qp.size() == 2 && (fold.size() == 4 || fold.size() == 6 || fold.size() == 8),
              "fc_head: flts = [delta], qp, fold = [qacc, cnt, Mpad, nlearn(, dqg, dq_epoch(, zero_ptr, zero_n))]");
  dqn::HeadArgs hd = head_args(ints, h, hw, hb, hwv, hbv, io, {}, {}, {}, actor, actor_f, act_h);
  TORCH_CHECK(!hd.infer, "fc_head: training launches only");
  hd.delta = (float)flts[0];
  hd.loss_parts = P<float*>(qp[0]);
  hd.dq16 = P<void*>(qp[1]);
  dqn::FoldArgs f{};
  f.qacc = P<float*>(fold[0]);
  f.cnt = P<int32_t*>(fold[1]);
  f.Mpad = (int)fold[2];
  f.nlearn = (int)fold[3];
  f.ngroups = (a.M + 15) / 16;
  f.prof = P<int64_t*>(prof);
  f.two_per_cu = two_per_cu ? 1 : 0;
  if (fold.size() >= 6 && fold[4] != 0) {     // spin mode: the online blocks write their own dH tiles
    f.spin = 1;
    f.dqg = P<float*>(fold[4]);
    f.dq_epoch = P<int32_t*>(fold[5]);
    f.err = f.dq_epoch + f.ngroups + 1;       // the epoch buffer holds ngroups + 2 words
    f.dbg_no_publish = std::getenv("DQN_DEBUG_FOLD_NO_PUBLISH") != nullptr ? 1 : 0;
  }
  if (fold.size() == 8 && fold[6] != 0) {      // zero duty (the step's dgrad-chain counters)
    TORCH_CHECK(fold[6] % 16 == 0 && fold[7] % 4 == 0, "fc_head: zero range 16-byte aligned, n % 4 == 0");
    f.zero_ptr = P<float*>(fold[6]);
    f.zero_n = (int)fold[7];
  }
  TORCH_CHECK(f.qacc && f.cnt && (f.nlearn == 2 || f.nlearn == 3), "fc_head: fold buffers, 2-3 learner instances");
  TORCH_CHECK((int)in.size() == f.nlearn + (hd.act_E > 0 ? 1 : 0) && out.size() == in.size() && bias.size() == in.size() &&
                  w.size() == in.size(), "fc_head: one fc input / weights / bias / output per instance");
  TORCH_CHECK(a.M == hd.B && a.ldo == a.N, "fc_head: fc rows = the minibatch, dense output rows");
  for (int i = 0; i < f.nlearn; ++i)
    TORCH_CHECK(hd.h[i] == a.out[i] && hd.w[i] && hd.b[i] && (!hd.dueling || (hd.wv[i] && hd.bv[i])),
                "fc_head: instance ", i, " head pointers (h = the fc output)");
  TORCH_CHECK(hd.act_E == 0 || hd.act_h == a.out[f.nlearn], "fc_head: the actors' h is the last fc output");
  TORCH_CHECK(hd.dq16 && hd.loss_parts && hd.dh && hd.prio, "fc_head: training outputs");
  TORCH_CHECK(launch_fc_head(a, hd, f, cur_stream()) == 0,
              "fc_head: shape outside the fused kernel (A <= 18, HID <= 512 and % 64 == 0, E <= 16)");
}

// C51 head: ints as head_loss; dist = [atoms]; flts = [v_min, v_max]; lg = the instances' logits
// rows (one igemm over the combined output layer: KD floats per row, rainbow.hip c51_kd)
void c51_head(std::vector<int64_t> ints, std::vector<int64_t> dist, std::vector<double> flts, std::vector<int64_t> h,
              std::vector<int64_t> w, std::vector<int64_t> b, std::vector<int64_t> wv, std::vector<int64_t> bv,
              std::vector<int64_t> io, std::vector<int64_t> pw, std::vector<int64_t> pwv, std::vector<int64_t> zero,
              std::vector<int64_t> actor, std::vector<double> actor_f, int64_t prof, std::vector<int64_t> lg,
              int64_t act_h, std::vector<int64_t> qp) {
  // training + actor: fused acting; lg then carries one more entry, the actors' logits.
  // qp (training): [loss_parts (>= c51_train_blocks floats), dout16 act_t [B][KD]]
  TORCH_CHECK(dist.size() == 1 && flts.size() == 2, "c51 args");
  dqn::HeadArgs a = head_args(ints, h, w, b, wv, bv, io, pw, pwv, zero, actor, actor_f, act_h);
  a.atoms = (int)dist[0]; a.vmin = (float)flts[0]; a.vmax = (float)flts[1];
  TORCH_CHECK(a.atoms >= 2 && a.atoms <= 64, "C51: 2..64 atoms (one wave64 lane per atom)");
  TORCH_CHECK(a.vmax > a.vmin, "C51 support");
  TORCH_CHECK(c51_head_lds_bytes(a) <= 160 * 1024, "C51 head: batch too large for one workgroup's LDS");
  if (!a.infer) {
    TORCH_CHECK(qp.size() == 2 && qp[0] != 0 && qp[1] != 0 && io[6] != 0, "C51 training: loss partials, dout16, prio");
    a.loss_parts = P<float*>(qp[0]);
    a.dq16 = P<void*>(qp[1]);
  }
  a.prof = P<int64_t*>(prof);
  if (a.act_E > 0) {
    TORCH_CHECK(!lg.empty(), "c51 fused acting: the actors' logits");
    a.act_lgi = P<const float*>(lg.back());
    lg.pop_back();
  }
  TORCH_CHECK(a.infer ? lg.size() == 1 : (lg.size() == 2 || lg.size() == 3), "c51: logits of every instance");
  for (size_t i = 0; i < lg.size(); ++i) a.lgi[i] = P<const float*>(lg[i]);
  launch_c51_head(a, cur_stream());
}

void noisy_mix(int64_t flat, int64_t eff, int64_t noise, int64_t jobs, int64_t njobs, int64_t max_elems) {
  launch_noisy_mix(P<const float*>(flat), P<float*>(eff), P<const float*>(noise), P<const dqn::NoisyJob*>(jobs),
                   (int)njobs, (int)max_elems, cur_stream());
}

void noisy_grad(int64_t grad, int64_t noise, int64_t jobs, int64_t njobs, int64_t max_elems) {
  TORCH_CHECK(noise != 0, "noisy_grad needs the noise vector");
  launch_noisy_grad(P<float*>(grad), P<const float*>(noise), P<const dqn::NoisyJob*>(jobs), (int)njobs,
                    (int)max_elems, cur_stream());
}

// ptrs per instance (4 entries each, 0 = absent): slots, states, w1, w2, w3, b1, b2, b3, x1, x2, x3;
// M: valid samples per instance (empty = all B)
void trunk(int64_t frames, std::vector<int64_t> ptrs, int64_t B, int64_t ninst, double scale, int64_t prof,
           std::vector<int64_t> M, std::vector<int64_t> sample) {
  constexpr int I = dqn::kMaxInst;
  TORCH_CHECK(ptrs.size() == 11 * I && ninst >= 1 && ninst <= I && B >= 1 && M.size() <= (size_t)I, "trunk args");
  dqn::TrunkArgs a{};
  a.frames = P<const uint8_t*>(frames);
  for (int i = 0; i < I; ++i) {
    a.slots[i] = P<const int32_t*>(ptrs[0 * I + i]);
    a.states[i] = P<const uint8_t*>(ptrs[1 * I + i]);
    a.w1[i] = P<const void*>(ptrs[2 * I + i]); a.w2[i] = P<const void*>(ptrs[3 * I + i]);
    a.w3[i] = P<const void*>(ptrs[4 * I + i]);
    a.b1[i] = P<const float*>(ptrs[5 * I + i]); a.b2[i] = P<const float*>(ptrs[6 * I + i]);
    a.b3[i] = P<const float*>(ptrs[7 * I + i]);
    a.x1[i] = P<act_t*>(ptrs[8 * I + i]); a.x2[i] = P<act_t*>(ptrs[9 * I + i]); a.x3[i] = P<act_t*>(ptrs[10 * I + i]);
    a.M[i] = i < (int)M.size() ? (int)M[i] : 0;
    TORCH_CHECK(a.M[i] >= 0 && a.M[i] <= B, "trunk: per-instance sample count");
    if (i < ninst) {
      TORCH_CHECK((a.slots[i] != nullptr && a.frames != nullptr) || a.states[i] != nullptr, "trunk input");
      TORCH_CHECK(a.w1[i] && a.w2[i] && a.w3[i] && a.b1[i] && a.b2[i] && a.b3[i] && a.x3[i], "trunk weights/out");
    }
  }
  a.scale = (float)scale;
  a.prof = P<int64_t*>(prof);
  // sample: [] or 16 pointers (TrunkSample order) + ninst_sampled; the replay must be
  // frame-stacked with k = 4 (int4 slot rows)
  if (!sample.empty()) {
    TORCH_CHECK(sample.size() == 17, "trunk sample: 16 pointers + sampled instances");
    for (int i = 0; i < 16; ++i) TORCH_CHECK(sample[i] != 0, "trunk sample: null pointer");
    dqn::TrunkSample& s = a.smp;
    s.size = P<const int32_t*>(sample[0]); s.rng = P<int64_t*>(sample[1]); s.ticket = P<int32_t*>(sample[2]);
    s.state_idx = P<const int32_t*>(sample[3]); s.next_idx = P<const int32_t*>(sample[4]);
    s.actions = P<const int32_t*>(sample[5]); s.rewards = P<const float*>(sample[6]);
    s.dones = P<const float*>(sample[7]); s.gammas = P<const float*>(sample[8]);
    s.idx_out = P<int32_t*>(sample[9]); s.a_out = P<int32_t*>(sample[10]); s.r_out = P<float*>(sample[11]);
    s.d_out = P<float*>(sample[12]); s.g_out = P<float*>(sample[13]);
    s.st_slots = P<int32_t*>(sample[14]); s.nx_slots = P<int32_t*>(sample[15]);
    s.B = (int)B;
    s.ninst = (int)sample[16];
    TORCH_CHECK(B >= 1 && B <= 512 && s.ninst >= 1 && s.ninst <= ninst && a.frames != nullptr,
                "trunk sample: 1 <= B <= 512 (one lane per sample), sampled instances <= ninst");
    for (int i = 0; i < s.ninst; ++i) TORCH_CHECK(a.M[i] == 0 || a.M[i] == B, "sampled instances use all B");
  }
  launch_trunk_fwd(a, (int)B, (int)ninst, cur_stream());
}

}  // namespace

void register_net_ops(pybind11::module_& m) {
  m.def("qnet_trunk", &trunk, pybind11::arg("frames"), pybind11::arg("ptrs"), pybind11::arg("B"),
        pybind11::arg("ninst"), pybind11::arg("scale"), pybind11::arg("prof") = 0,
        pybind11::arg("M") = std::vector<int64_t>{}, pybind11::arg("sample") = std::vector<int64_t>{});
  m.def("qnet_pack", &pack, pybind11::arg("src"), pybind11::arg("dst"), pybind11::arg("jobs"), pybind11::arg("njobs"),
        pybind11::arg("max_threads"), pybind11::arg("dst2") = 0, pybind11::arg("step") = 0, pybind11::arg("freq") = 1);
  m.def("qnet_igemm", &igemm, pybind11::arg("kind"), pybind11::arg("inp"), pybind11::arg("w"), pybind11::arg("bias"),
        pybind11::arg("out"), pybind11::arg("mask"), pybind11::arg("scale"), pybind11::arg("dims"),
        pybind11::arg("aux") = std::vector<int64_t>{}, pybind11::arg("aux_f") = std::vector<double>{},
        pybind11::arg("fz") = std::vector<int64_t>{});
  m.def("qnet_wgrad", &wgrad, pybind11::arg("kind"), pybind11::arg("in"), pybind11::arg("dims"), pybind11::arg("dz"), pybind11::arg("ldz"),
        pybind11::arg("dw"), pybind11::arg("db"), pybind11::arg("dw2"), pybind11::arg("db2"), pybind11::arg("nsplit"), pybind11::arg("N"), pybind11::arg("MC"),
        pybind11::arg("KB"), pybind11::arg("NB"), pybind11::arg("scale"), pybind11::arg("atomic"), pybind11::arg("mloop") = 1,
        pybind11::arg("db_zero") = false);
  m.def("qnet_dgrad_chain", &dgrad_chain);
  m.def("qnet_fc_head", &fc_head, pybind11::arg("inp"), pybind11::arg("w"), pybind11::arg("bias"),
        pybind11::arg("out"), pybind11::arg("dims"), pybind11::arg("ints"), pybind11::arg("flts"), pybind11::arg("h"),
        pybind11::arg("hw"), pybind11::arg("hb"), pybind11::arg("hwv"), pybind11::arg("hbv"), pybind11::arg("io"),
        pybind11::arg("qp"), pybind11::arg("actor"), pybind11::arg("actor_f"), pybind11::arg("act_h"),
        pybind11::arg("fold"), pybind11::arg("prof") = 0, pybind11::arg("two_per_cu") = true);
  m.def("qnet_head_loss", &head_loss, pybind11::arg("ints"), pybind11::arg("flts"), pybind11::arg("h"),
        pybind11::arg("w"), pybind11::arg("b"), pybind11::arg("wv"), pybind11::arg("bv"), pybind11::arg("io"),
        pybind11::arg("pw"), pybind11::arg("pwv"), pybind11::arg("qp"), pybind11::arg("actor"),
        pybind11::arg("actor_f"), pybind11::arg("act_h") = 0, pybind11::arg("prof") = 0);
  m.def("qnet_wgrad_group", &wgrad_group);
  m.def("qnet_wgrad_plan", &wgrad_plan, pybind11::arg("members"), pybind11::arg("dims"), pybind11::arg("scales"),
        pybind11::arg("done"), pybind11::arg("deps"), pybind11::arg("conv_chunks") = 2);
  m.attr("WG_COUNTERS") = (int)dqn::kWgCounters;
  m.attr("WG_SLOTS") = (int)dqn::kWgSlots;
  m.def("qnet_cnn_fwd", &cnn_fwd, pybind11::arg("frames"), pybind11::arg("ptrs"), pybind11::arg("B"),
        pybind11::arg("ninst"), pybind11::arg("scale"), pybind11::arg("M") = std::vector<int64_t>{},
        pybind11::arg("prof") = 0);
  m.def("qnet_cnn_bwd", &cnn_bwd, pybind11::arg("ptrs"), pybind11::arg("B"), pybind11::arg("prof") = 0,
        pybind11::arg("parts") = 1);
  m.def("qnet_c51_head", &c51_head, pybind11::arg("ints"), pybind11::arg("dist"), pybind11::arg("flts"),
        pybind11::arg("h"), pybind11::arg("w"), pybind11::arg("b"), pybind11::arg("wv"), pybind11::arg("bv"),
        pybind11::arg("io"), pybind11::arg("pw"), pybind11::arg("pwv"), pybind11::arg("zero"), pybind11::arg("actor"),
        pybind11::arg("actor_f"), pybind11::arg("prof") = 0, pybind11::arg("lg") = std::vector<int64_t>{},
        pybind11::arg("act_h") = 0, pybind11::arg("qp") = std::vector<int64_t>{});
  m.def("qnet_noisy_mix", &noisy_mix);
  m.def("qnet_noisy_grad", &noisy_grad);
  m.attr("NOISY_JOB_INTS") = (int)(sizeof(dqn::NoisyJob) / sizeof(int));
  m.attr("PACK_JOB_INTS") = (int)(sizeof(dqn::PackJob) / sizeof(int));
}
