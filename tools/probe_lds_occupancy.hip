// Probe: how many 64-thread workgroups of a given static LDS size run at once
// on one gfx950 CU (the PSP epoch kernel's 13,184 B per instance gave 11 per
// CU in the timeline, not the 12 that 160 KiB / 13,184 B suggests).
// Each block spins ~60 us on the wall clock and records start, end and CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int BYTES>
__global__ __launch_bounds__(64) void k_probe(unsigned long long* out) {
  __shared__ double buf[BYTES / 8];
  buf[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  double acc = buf[(threadIdx.x + 1) & 63];
  while (wall_clock64() - t0 < 6000) acc = acc * 0.999 + 1.0;  // 100 MHz clock: 60 us
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    out[blockIdx.x * 4 + 0] = t0;
    out[blockIdx.x * 4 + 1] = t1;
    out[blockIdx.x * 4 + 2] = ((unsigned long long)xcc << 32) | (unsigned)__smid();
    out[blockIdx.x * 4 + 3] = (unsigned long long)(acc > 1e300);
  }
}

template <int BYTES>
static void run(unsigned long long* d, int nblk) {
  hipLaunchKernelGGL(k_probe<BYTES>, dim3(nblk), dim3(64), 0, 0, d);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h((size_t)nblk * 4);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  // max concurrency per CU: sweep events
  std::vector<std::pair<unsigned long long, std::pair<unsigned long long, int>>> ev;
  for (int b = 0; b < nblk; b++) {
    ev.push_back({h[b * 4 + 2], {h[b * 4 + 0], +1}});
    ev.push_back({h[b * 4 + 2], {h[b * 4 + 1], -1}});
  }
  std::sort(ev.begin(), ev.end(), [](auto& a, auto& b) {
    if (a.first != b.first) return a.first < b.first;
    if (a.second.first != b.second.first) return a.second.first < b.second.first;
    return a.second.second < b.second.second;  // ends before starts at equal time
  });
  int best = 0, cur = 0, cus = 0;
  unsigned long long key = ~0ull;
  std::vector<int> per;
  for (auto& e : ev) {
    if (e.first != key) { if (key != ~0ull) per.push_back(best); key = e.first; cur = 0; best = 0; }
    cur += e.second.second;
    best = std::max(best, cur);
  }
  per.push_back(best);
  std::sort(per.begin(), per.end());
  printf("LDS %6d B/block: %zu CUs seen, concurrent blocks per CU min %d median %d max %d\n", BYTES, per.size(),
         per.front(), per[per.size() / 2], per.back());
}

int main() {
  unsigned long long* d;
  const int nblk = 256 * 24;
  hipMalloc(&d, (size_t)nblk * 4 * 8);
  run<12288>(d, nblk);
  run<12800>(d, nblk);
  run<13056>(d, nblk);
  run<13184>(d, nblk);
  run<13312>(d, nblk);
  run<13568>(d, nblk);
  run<13648>(d, nblk);
  run<16384>(d, nblk);
  run<20480>(d, nblk);
  return 0;
}
