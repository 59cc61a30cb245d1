// uwvk_synth.cpp — counter-based normal variates for the synthetic logs of the
// benches and tests (host only, no device code).
//
// The reference ships no driver and no data; the
// synthetic mission of uwvk.synth draws its sensor noise here.  Every variate
// is a pure function of (seed, global instance id, stream, index), so a shard
// [lo, hi) of the batch reproduces exactly the rows of the full batch (the
// instance-sharded multi-GPU runs rely on that), and the cost is linear in the
// numbers drawn with no per-instance set-up.
//
//   block  = Philox4x32-10(key = (seed_lo ^ seed_hi, instance_lo ^ (stream << 24)),
//                          counter = (b, instance_hi, stream, 0x5eed))
//   u1, u2 = 53-bit uniforms from the block's two 64-bit halves, u1 in (0, 1]
//   normal[2 b], normal[2 b + 1] = sqrt(-2 ln u1) (cos, sin)(2 pi u2)   (Box-Muller)
//
// uwvk.synth._normal_np is an independent numpy restatement of the same map
// (tests/test_synth.py holds the two to 1e-14).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "../../include/uwvk.h"

namespace {

struct P4 {
  uint32_t v[4];
};

inline void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  const uint64_t p = (uint64_t)a * b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

inline P4 philox10(P4 c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo(0xD2511F53u, c.v[0], hi0, lo0);
    mulhilo(0xCD9E8D57u, c.v[2], hi1, lo1);
    c = P4{{hi1 ^ c.v[1] ^ k0, lo1, hi0 ^ c.v[3] ^ k1, lo0}};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

void fill_rows(uint64_t seed, int64_t i0, int64_t i1, int64_t first, uint32_t stream, int64_t count, double* out) {
  const double two_pi = 6.283185307179586476925286766559;
  const double inv53 = 1.0 / 9007199254740992.0;  // 2^-53
  for (int64_t j = i0; j < i1; j++) {
    const uint64_t inst = (uint64_t)(first + j);
    const uint32_t k0 = (uint32_t)seed ^ (uint32_t)(seed >> 32);
    const uint32_t k1 = (uint32_t)inst ^ (stream << 24);
    double* o = out + j * count;
    for (int64_t b = 0; 2 * b < count; b++) {
      const P4 r = philox10(P4{{(uint32_t)b, (uint32_t)(inst >> 32), stream, 0x5eedu}}, k0, k1);
      const uint64_t a = ((uint64_t)r.v[0] << 32 | r.v[1]) >> 11;
      const uint64_t c = ((uint64_t)r.v[2] << 32 | r.v[3]) >> 11;
      const double u1 = (double)(a + 1) * inv53;  // (0, 1]
      const double u2 = (double)c * inv53;        // [0, 1)
      const double rad = std::sqrt(-2.0 * std::log(u1));
      const double th = two_pi * u2;
      o[2 * b] = rad * std::cos(th);
      if (2 * b + 1 < count) o[2 * b + 1] = rad * std::sin(th);
    }
  }
}

}  // namespace

extern "C" uwvk_status uwvk_synth_normal(uint64_t seed, int64_t first_instance, int64_t batch, uint32_t stream,
                                         int64_t count, double* out) {
  if (!out || batch < 0 || count < 0 || first_instance < 0 || stream >= 256) return UWVK_EINVAL;
  if (batch == 0 || count == 0) return UWVK_OK;
  const int64_t work = batch * count;
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  nt = (unsigned)std::min<int64_t>(nt, std::max<int64_t>(1, work / 65536));
  nt = (unsigned)std::min<int64_t>(nt, batch);
  if (nt <= 1) {
    fill_rows(seed, 0, batch, first_instance, stream, count, out);
    return UWVK_OK;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; t++) {
    const int64_t a = batch * t / nt, b = batch * (t + 1) / nt;
    th.emplace_back(fill_rows, seed, a, b, first_instance, stream, count, out);
  }
  for (auto& x : th) x.join();
  return UWVK_OK;
}
