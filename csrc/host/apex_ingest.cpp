// Ape-X ingest: one call per actor moves every pending transition record of its SPSC ring
// (spsc_ring.cpp) straight into the HBM replay's pinned staging buffers (replay/device.py
// _StageSet): the observation frame into the frame staging, the frame-slot stack and the
// n-step fold into the transition columns. Replaces a per-record Python loop (one
// begin_episode / add_step call and two numpy copies per env frame) with a memcpy per frame.
//
// Semantics match DeviceReplay.begin_episode / add_step / add_step_nstep with
// replay.nstep.NStepAccumulator (the Python path the vector-observation envs keep):
//   RESET  a new frame slot, duplicated k times as the stack; the n-step window is cleared
//   STEP   a new frame slot s; the transition (stack, action, reward) enters the window;
//          done -> every window entry is emitted (oldest first) with next = s, done = 1;
//          window full (n) -> the oldest is emitted with R = sum gamma^i r_i, gamma^n
//          stack <- stack[1:] + [s]
// The call stops BEFORE a record the staging could not hold (a frame, plus up to n
// transitions): the caller flushes the staging and calls again.
//
// actor_state (int32, caller-owned, zero-initialised): [k] stack | [1] window length |
//   [n][k] window stacks | [n] window actions | [n] window rewards (float bits)
#include <cmath>
#include <cstring>

#include "../include/dqn_host.h"

namespace {
struct Record {                      // actors/apex.py HEADER (16 bytes) + payload
  uint8_t kind, done;
  uint16_t pad;
  int32_t action;
  float reward, ret;
};
static_assert(sizeof(Record) == 16, "record header");
constexpr uint8_t kReset = 0;

int64_t alloc_frame(DqnIngestStage* st, const uint8_t* src, int64_t bytes) {
  std::memcpy(st->frames + st->nf * bytes, src, (size_t)bytes);
  st->nf += 1;
  const int64_t slot = st->f_next;
  st->f_next = (st->f_next + 1) % st->num_frames;
  return slot;
}

void emit(DqnIngestStage* st, const int32_t* stack, int k, int32_t next, int32_t action, float R, float done,
          float g) {
  const int64_t i = st->nt++;
  std::memcpy(st->sidx + i * k, stack, sizeof(int32_t) * (size_t)k);
  st->nidx[i] = next;
  st->act[i] = action;
  st->rew[i] = R;
  st->done[i] = done;
  st->gam[i] = g;
}
}  // namespace

void dqn_apex_ingest(uint8_t* ring, int64_t max_n, int32_t* S, int k, int nstep, double gamma, int64_t frame_bytes,
                     DqnIngestStage* st, float* returns, int64_t returns_cap, DqnIngestOut* out) {
  out->consumed = out->frames = out->episodes = out->n_returns = out->stage_full = 0;
  uint64_t tail, avail, cap, rb;
  const uint8_t* data = dqn_ring_peek(ring, &tail, &avail, &cap, &rb);
  const uint64_t m = max_n >= 0 && (uint64_t)max_n < avail ? (uint64_t)max_n : avail;
  int32_t* stack = S;
  int32_t& wlen = S[k];
  int32_t* wst = S + k + 1;                       // [nstep][k]
  int32_t* wact = wst + (int64_t)nstep * k;       // [nstep]
  float* wrew = reinterpret_cast<float*>(wact + nstep);
  uint64_t i = 0;
  for (; i < m; ++i) {
    const uint8_t* rec = data + ((tail + i) % cap) * rb;
    Record h;
    std::memcpy(&h, rec, sizeof(h));
    const uint8_t* obs = rec + sizeof(Record);
    if (st->nf + 1 > st->frames_cap || st->nt + nstep > st->trans_cap) {
      out->stage_full = 1;
      break;
    }
    const int32_t slot = (int32_t)alloc_frame(st, obs, frame_bytes);
    if (h.kind == kReset) {
      for (int c = 0; c < k; ++c) stack[c] = slot;
      wlen = 0;
      continue;
    }
    // the transition from the current stack enters the n-step window
    std::memcpy(wst + (int64_t)wlen * k, stack, sizeof(int32_t) * (size_t)k);
    wact[wlen] = h.action;
    wrew[wlen] = h.reward;
    wlen += 1;
    auto emit_front = [&](bool done) {           // oldest entry, R over the whole window
      double R = 0.0, g = 1.0;                  // (double, as the Python accumulator)
      for (int j = 0; j < wlen; ++j) {
        R += g * (double)wrew[j];
        g *= gamma;
      }
      emit(st, wst, k, slot, wact[0], (float)R, done ? 1.f : 0.f, (float)g);
      std::memmove(wst, wst + k, sizeof(int32_t) * (size_t)(wlen - 1) * k);
      std::memmove(wact, wact + 1, sizeof(int32_t) * (size_t)(wlen - 1));
      std::memmove(wrew, wrew + 1, sizeof(float) * (size_t)(wlen - 1));
      wlen -= 1;
    };
    if (h.done) {
      while (wlen > 0) emit_front(true);
    } else if (wlen >= nstep) {
      emit_front(false);
    }
    for (int c = 0; c + 1 < k; ++c) stack[c] = stack[c + 1];
    stack[k - 1] = slot;
    out->frames += 1;
    if (!std::isnan(h.ret)) {
      out->episodes += 1;
      if (out->n_returns < returns_cap) returns[out->n_returns++] = h.ret;
    }
  }
  dqn_ring_release(ring, i);
  out->consumed = (int64_t)i;
}
