// C ABI of the host runtime for ctypes (dist_dqn_amd/native/hostlib.py), so CPU
// actor processes can use the rings, mailboxes and preprocessing without
// importing torch or the HIP runtime (libdqn_host has no GPU dependency).
#include "../include/dqn_host.h"

extern "C" {
size_t dqnh_ring_bytes(uint64_t cap, uint64_t rec) { return dqn_ring_bytes(cap, rec); }
void dqnh_ring_init(uint8_t* b, uint64_t cap, uint64_t rec) { dqn_ring_init(b, cap, rec); }
int64_t dqnh_ring_push(uint8_t* b, const uint8_t* r, int64_t n) { return dqn_ring_push(b, r, n); }
int64_t dqnh_ring_pop(uint8_t* b, uint8_t* o, int64_t m) { return dqn_ring_pop(b, o, m); }
int64_t dqnh_ring_size(uint8_t* b) { return dqn_ring_size(b); }

int64_t dqnh_mbox_stride(int64_t sb) { return dqn_mbox_stride(sb); }
size_t dqnh_mbox_region_bytes(int64_t n, int64_t sb) { return dqn_mbox_region_bytes(n, sb); }
void dqnh_mbox_init(uint8_t* r, int64_t n, int64_t sb) { dqn_mbox_init(r, n, sb); }
void dqnh_mbox_set_stop(uint8_t* r, int64_t v) { dqn_mbox_set_stop(r, v); }
int64_t dqnh_mbox_stopped(uint8_t* r) { return dqn_mbox_stopped(r); }
int64_t dqnh_mbox_request(uint8_t* r, int64_t i, int64_t sb, const uint8_t* s, int64_t t) {
  return dqn_mbox_request(r, i, sb, s, t);
}
int64_t dqnh_mbox_collect(uint8_t* r, int64_t n, int64_t sb, uint8_t* os, int32_t* oi, uint64_t* oq, int64_t mb) {
  return dqn_mbox_collect(r, n, sb, os, oi, oq, mb);
}
void dqnh_mbox_respond(uint8_t* r, int64_t sb, const int32_t* ids, const uint64_t* q, const int32_t* a, int64_t m) {
  dqn_mbox_respond(r, sb, ids, q, a, m);
}

void dqnh_preprocess(const uint8_t* rgb, int Hs, int Ws, uint8_t* out, int H, int W) {
  dqn_preprocess_host(rgb, Hs, Ws, out, H, W);
}
uint32_t dqnh_crc32c(const uint8_t* d, size_t n) { return dqn_crc32c(d, n); }

// stage / out: int64 arrays in DqnIngestStage / DqnIngestOut field order (pointers as int64)
void dqnh_apex_ingest(uint8_t* ring, int64_t max_n, int32_t* actor_state, int k, int nstep, double gamma,
                      int64_t frame_bytes, int64_t* stage, float* returns, int64_t returns_cap, int64_t* out) {
  DqnIngestStage st;
  st.frames = reinterpret_cast<uint8_t*>(stage[0]); st.frames_cap = stage[1]; st.nf = stage[2];
  st.sidx = reinterpret_cast<int32_t*>(stage[3]); st.nidx = reinterpret_cast<int32_t*>(stage[4]);
  st.act = reinterpret_cast<int32_t*>(stage[5]); st.rew = reinterpret_cast<float*>(stage[6]);
  st.done = reinterpret_cast<float*>(stage[7]); st.gam = reinterpret_cast<float*>(stage[8]);
  st.trans_cap = stage[9]; st.nt = stage[10]; st.f_next = stage[11]; st.num_frames = stage[12];
  DqnIngestOut o;
  dqn_apex_ingest(ring, max_n, actor_state, k, nstep, gamma, frame_bytes, &st, returns, returns_cap, &o);
  stage[2] = st.nf; stage[10] = st.nt; stage[11] = st.f_next;
  out[0] = o.consumed; out[1] = o.frames; out[2] = o.episodes; out[3] = o.n_returns; out[4] = o.stage_full;
}

// Every actor ring in ONE call (actors first..n-1, in order): stops at a full staging with
// out[5] = the actor to resume with (its ring position and state are kept), else out[5] = n.
// out[0..3] accumulate over the actors; out[4] = stage full.
void dqnh_apex_ingest_many(int64_t n, const int64_t* rings, int32_t* states, int64_t state_words, int64_t first,
                           int64_t max_n, int k, int nstep, double gamma, int64_t frame_bytes, int64_t* stage,
                           float* returns, int64_t returns_cap, int64_t* out) {
  int64_t acc[4] = {0, 0, 0, 0};
  int64_t a = first;
  int64_t tmp[5];
  out[4] = 0;
  for (; a < n; ++a) {
    dqnh_apex_ingest(reinterpret_cast<uint8_t*>(rings[a]), max_n, states + a * state_words, k, nstep, gamma,
                     frame_bytes, stage, returns + acc[3], returns_cap - acc[3], tmp);
    for (int j = 0; j < 4; ++j) acc[j] += tmp[j];
    if (tmp[4]) { out[4] = 1; break; }
  }
  for (int j = 0; j < 4; ++j) out[j] = acc[j];
  out[5] = a;
}
}
