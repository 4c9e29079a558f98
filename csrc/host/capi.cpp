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
}
