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
// (tests/test_synth.py holds the two to 1e-14).  uwvk_synth_normal_at draws a
// window [offset, offset + count) of the same sequences, optionally written
// record-major ([record][instance][group]: the logs' epoch-major layout), so a
// log can be generated in epoch segments that are bitwise slices of the whole.
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

// the two variates of block b: (cos, sin) halves of one Box-Muller pair; every
// path computes both (the same libm sincos call), so a variate's bits do not
// depend on which path or window drew it
inline void box_muller(uint64_t seed, uint64_t inst, uint32_t stream, int64_t b, double* v0, double* v1) {
  const double two_pi = 6.283185307179586476925286766559;
  const double inv53 = 1.0 / 9007199254740992.0;  // 2^-53
  const uint32_t k0 = (uint32_t)seed ^ (uint32_t)(seed >> 32);
  const uint32_t k1 = (uint32_t)inst ^ (stream << 24);
  const P4 r = philox10(P4{{(uint32_t)b, (uint32_t)(inst >> 32), stream, 0x5eedu}}, k0, k1);
  const uint64_t a = ((uint64_t)r.v[0] << 32 | r.v[1]) >> 11;
  const uint64_t c = ((uint64_t)r.v[2] << 32 | r.v[3]) >> 11;
  const double u1 = (double)(a + 1) * inv53;  // (0, 1]
  const double u2 = (double)c * inv53;        // [0, 1)
  const double rad = std::sqrt(-2.0 * std::log(u1));
  const double th = two_pi * u2;
  *v0 = rad * std::cos(th);
  *v1 = rad * std::sin(th);
}

// variates [offset, offset + count) of instances lo..hi (rows of `count`), or,
// group > 0, records lo..hi of `group` variates for every instance, written
// record-major: out[(r * batch + j) * group + g] = variate offset + r * group + g
void fill(uint64_t seed, int64_t first, int64_t batch, uint32_t stream, int64_t offset, int64_t count, int group,
          int64_t lo, int64_t hi, double* out) {
  const int64_t rows = group ? batch : 1;
  for (int64_t u = lo; u < hi; u++)
    for (int64_t jj = 0; jj < rows; jj++) {
      // group 0: u is the instance, one run of `count`; group > 0: u is the record
      const int64_t j = group ? jj : u;
      const int64_t n = group ? group : count;
      const int64_t e0 = group ? offset + u * group : offset;
      double* o = group ? out + (u * batch + j) * group : out + j * count;
      const uint64_t inst = (uint64_t)(first + j);
      for (int64_t i = 0; i < n;) {
        const int64_t e = e0 + i;
        double v0, v1;
        box_muller(seed, inst, stream, e >> 1, &v0, &v1);
        if (e & 1) {
          o[i++] = v1;
        } else {
          o[i++] = v0;
          if (i < n) o[i++] = v1;
        }
      }
    }
}

uwvk_status normal_at(uint64_t seed, int64_t first_instance, int64_t batch, uint32_t stream, int64_t offset,
                      int64_t count, int32_t group, double* out) {
  if (!out || batch < 0 || count < 0 || first_instance < 0 || offset < 0 || stream >= 256 || group < 0)
    return UWVK_EINVAL;
  if (group > 0 && count % group) return UWVK_EINVAL;
  if (batch == 0 || count == 0) return UWVK_OK;
  const int64_t work = batch * count;
  const int64_t units = group ? count / group : batch;  // split over records or over instances
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  nt = (unsigned)std::min<int64_t>(nt, std::max<int64_t>(1, work / 65536));
  nt = (unsigned)std::min<int64_t>(nt, units);
  if (nt <= 1) {
    fill(seed, first_instance, batch, stream, offset, count, group, 0, units, out);
    return UWVK_OK;
  }
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; t++) {
    const int64_t a = units * t / nt, b = units * (t + 1) / nt;
    th.emplace_back(fill, seed, first_instance, batch, stream, offset, count, group, a, b, out);
  }
  for (auto& x : th) x.join();
  return UWVK_OK;
}

}  // namespace

extern "C" uwvk_status uwvk_synth_normal(uint64_t seed, int64_t first_instance, int64_t batch, uint32_t stream,
                                         int64_t count, double* out) {
  return normal_at(seed, first_instance, batch, stream, 0, count, 0, out);
}

extern "C" uwvk_status uwvk_synth_normal_at(uint64_t seed, int64_t first_instance, int64_t batch, uint32_t stream,
                                            int64_t offset, int64_t count, int32_t group, double* out) {
  return normal_at(seed, first_instance, batch, stream, offset, count, group, out);
}
