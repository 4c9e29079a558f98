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
