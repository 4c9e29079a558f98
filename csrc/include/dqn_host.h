// Host-side (CPU) native runtime pieces of dist_dqn_amd.
#pragma once
#include <cstddef>
#include <cstdint>

void dqn_preprocess_host(const uint8_t* rgb, int Hs, int Ws, uint8_t* out, int H, int W);
uint32_t dqn_crc32c(const uint8_t* data, size_t n);

size_t dqn_ring_bytes(uint64_t capacity, uint64_t record_bytes);
void dqn_ring_init(uint8_t* buf, uint64_t capacity, uint64_t record_bytes);
int64_t dqn_ring_push(uint8_t* buf, const uint8_t* recs, int64_t n);
int64_t dqn_ring_pop(uint8_t* buf, uint8_t* out, int64_t max_n);
int64_t dqn_ring_size(uint8_t* buf);

// Actor <-> inference-server mailboxes (mailbox.cpp)
int64_t dqn_mbox_stride(int64_t state_bytes);
size_t dqn_mbox_region_bytes(int64_t n, int64_t state_bytes);
void dqn_mbox_init(uint8_t* region, int64_t n, int64_t state_bytes);
void dqn_mbox_set_stop(uint8_t* region, int64_t v);
int64_t dqn_mbox_stopped(uint8_t* region);
int64_t dqn_mbox_request(uint8_t* region, int64_t i, int64_t state_bytes, const uint8_t* state, int64_t timeout_us);
int64_t dqn_mbox_collect(uint8_t* region, int64_t n, int64_t state_bytes, uint8_t* out_states, int32_t* out_ids,
                         uint64_t* out_seq, int64_t max_batch);
void dqn_mbox_respond(uint8_t* region, int64_t state_bytes, const int32_t* ids, const uint64_t* seq,
                      const int32_t* actions, int64_t m);

// In-place consumption of a ring (apex_ingest.cpp): records [tail, tail + avail) are read where
// they lie, then released with dqn_ring_release.
const uint8_t* dqn_ring_peek(uint8_t* buf, uint64_t* tail, uint64_t* avail, uint64_t* cap, uint64_t* rec_bytes);
void dqn_ring_release(uint8_t* buf, uint64_t n);

// Ape-X ingest (apex_ingest.cpp): one actor's ring straight into the replay's pinned staging.
struct DqnIngestStage {
  uint8_t* frames; int64_t frames_cap; int64_t nf;      // frame staging [frames_cap][HW], fill count
  int32_t* sidx; int32_t* nidx; int32_t* act; float* rew; float* done; float* gam;
  int64_t trans_cap; int64_t nt;                         // transition staging columns, fill count
  int64_t f_next; int64_t num_frames;                    // replay frame-slot cursor / ring size
};
struct DqnIngestOut {
  int64_t consumed, frames, episodes, n_returns, stage_full;
};
void dqn_apex_ingest(uint8_t* ring, int64_t max_n, int32_t* actor_state, int k, int nstep, double gamma,
                     int64_t frame_bytes, DqnIngestStage* st, float* returns, int64_t returns_cap, DqnIngestOut* out);
