// Actor-side frame preprocessing in C++ (reference: cv2.cvtColor + cv2.resize,
// /root/reference/src/utils.py:39-45). Same fixed-point arithmetic as the
// numpy oracle (dist_dqn_amd/utils/image.py) and the HIP kernel; coefficient
// tables are cached per (src, dst) shape.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "../include/dqn_host.h"

namespace {

struct Axis {
  std::vector<int> s, c0;
};

Axis make_axis(int src, int dst) {
  Axis a;
  a.s.resize(dst);
  a.c0.resize(dst);
  const double scale = (double)src / (double)dst;
  for (int d = 0; d < dst; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int si = (int)std::floor(f);
    f -= (float)si;
    if (si < 0) { si = 0; f = 0.f; }
    if (si >= src - 1) { si = src - 1; f = 0.f; }
    a.s[d] = si;
    a.c0[d] = (int)std::nearbyint((1.f - f) * 2048.f);
  }
  return a;
}

const Axis& axis_cached(int src, int dst) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, Axis> cache;
  std::lock_guard<std::mutex> g(mu);
  auto key = std::make_pair(src, dst);
  auto it = cache.find(key);
  if (it == cache.end()) it = cache.emplace(key, make_axis(src, dst)).first;
  return it->second;
}

}  // namespace

void dqn_preprocess_host(const uint8_t* rgb, int Hs, int Ws, uint8_t* out, int H, int W) {
  std::vector<int> gray((size_t)Hs * Ws);
  for (int i = 0; i < Hs * Ws; ++i) {
    const uint8_t* p = rgb + (size_t)i * 3;
    gray[i] = (4899 * p[0] + 9617 * p[1] + 1868 * p[2] + (1 << 13)) >> 14;
  }
  const Axis& ax = axis_cached(Ws, W);
  const Axis& ay = axis_cached(Hs, H);
  std::vector<int> rows((size_t)Hs * W);
  // horizontal pass on every source row that is needed
  std::vector<char> need(Hs, 0);
  for (int y = 0; y < H; ++y) {
    need[ay.s[y]] = 1;
    need[std::min(ay.s[y] + 1, Hs - 1)] = 1;
  }
  for (int sy = 0; sy < Hs; ++sy) {
    if (!need[sy]) continue;
    const int* g = gray.data() + (size_t)sy * Ws;
    int* r = rows.data() + (size_t)sy * W;
    for (int x = 0; x < W; ++x) {
      const int s0 = ax.s[x], s1 = std::min(s0 + 1, Ws - 1), c0 = ax.c0[x];
      r[x] = g[s0] * c0 + g[s1] * (2048 - c0);
    }
  }
  for (int y = 0; y < H; ++y) {
    const int s0 = ay.s[y], s1 = std::min(s0 + 1, Hs - 1), c0 = ay.c0[y];
    const int* r0 = rows.data() + (size_t)s0 * W;
    const int* r1 = rows.data() + (size_t)s1 * W;
    for (int x = 0; x < W; ++x) {
      long long v = ((long long)r0[x] * c0 + (long long)r1[x] * (2048 - c0) + (1 << 21)) >> 22;
      out[(size_t)y * W + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
  }
}

// CRC32C (Castagnoli), slicing-by-1 table; used by the TF event-file writer.
uint32_t dqn_crc32c(const uint8_t* data, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
      table[i] = c;
    }
    init = true;
  }
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = table[(c ^ data[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}
