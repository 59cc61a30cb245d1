// probe_lmask.hip — per-lane value of __builtin_amdgcn_inverse_ballot_w64 for
// constant masks whose 64-bit value is a sign-extended 32-bit literal
// (0xffffffffffffffe0: lanes 5..63) and for masks the compiler splits into two
// 32-bit halves; checks every lane on the host.  Decides whether constant lane
// masks (the PSP_LMASK experiment) are safe to materialise on gfx950.
// Build: hipcc -O3 --offload-arch=gfx950 tools/probe_lmask.hip -o tools/probe_lmask
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <unsigned long long M>
__global__ void k_mask(int* out) {
  const int l = threadIdx.x;
  out[l] = __builtin_amdgcn_inverse_ballot_w64(M) ? 1 : 0;
}
template <unsigned long long M>
__global__ void k_mask_branch(int* out) {
  const int l = threadIdx.x;
  int v = 0;
  if (__builtin_amdgcn_inverse_ballot_w64(M)) v = 1;
  out[l] = v;
}

// the mask materialised by an s_mov_b64 with the literal (as the PSP kernel's
// code generation did for sign-extendable values), then used as the condition
__global__ void k_mask_smov64(int* out) {
  const int l = threadIdx.x;
  unsigned long long m;
  asm volatile("s_mov_b64 %0, 0xffffffffffffffe0" : "=s"(m));
  out[l] = __builtin_amdgcn_inverse_ballot_w64(m) ? 1 : 0;
}

template <unsigned long long M>
static int check(int* d, const char* name) {
  int h[2][64];
  hipLaunchKernelGGL(k_mask<M>, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h[0], d, 64 * 4, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(k_mask_branch<M>, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h[1], d, 64 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int v = 0; v < 2; v++)
    for (int l = 0; l < 64; l++) bad += h[v][l] != (int)((M >> l) & 1ull);
  std::printf("%-28s 0x%016llx  select/branch mismatching lanes: %d\n", name, M, bad);
  return bad;
}

int main() {
  int* d;
  hipMalloc(&d, 64 * 4);
  int bad = 0;
  bad += check<0xffffffffffffffe0ull>(d, "lanes >= 5 (sext literal)");
  bad += check<0xfffffffffffff000ull>(d, "lanes >= 12 (sext literal)");
  bad += check<0xffffffff80000000ull>(d, "lanes >= 31 (sext literal)");
  bad += check<0x001fffffffffffc7ull>(d, "l < 53 && !(3<=l<6)");
  bad += check<0x00000000fffffff0ull>(d, "4 <= l < 32");
  bad += check<0x0000000000000fc0ull>(d, "6 <= l < 12");
  {
    int h[64];
    hipLaunchKernelGGL(k_mask_smov64, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, 64 * 4, hipMemcpyDeviceToHost);
    int b = 0, hi = 0;
    for (int l = 0; l < 64; l++) {
      b += h[l] != (int)((0xffffffffffffffe0ull >> l) & 1ull);
      hi += l >= 32 ? h[l] : 0;
    }
    std::printf("%-28s 0x%016llx  mismatching lanes: %d (lanes 32..63 set: %d of 32)\n", "s_mov_b64 literal (asm)",
                0xffffffffffffffe0ull, b, hi);
    bad += b;
  }
  std::printf(bad ? "MISMATCH\n" : "all lanes match\n");
  hipFree(d);
  return bad ? 1 : 0;
}
