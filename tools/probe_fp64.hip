// Hardware probe for gfx950 fp64 paths used by the batched UKF engine:
//  (1) v_mfma_f64_16x16x4_f64 operand / accumulator lane maps (checked with
//      asymmetric integer data against a host GEMM),
//  (2) fp64 throughput: MFMA-only, VALU-FMA-only and both interleaved,
//  (3) fp64 transcendental cost (sqrt, sincos, atan2) per lane-op.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void layout_k(const double* A /*16x4 row-major*/, const double* B /*4x16*/, double* C /*16x16*/) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int i = 0; i < 4; i++) C[((l >> 4) + 4 * i) * 16 + (l & 15)] = acc[i];
}

template <int MODE>
__global__ void tput_k(double* out, int iters, double seed) {
  int l = threadIdx.x;
  double a = seed + l, b = seed * 0.5 + l;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double v0 = a, v1 = b, v2 = a + 1, v3 = b + 1, v4 = a + 2, v5 = b + 2, v6 = a + 3, v7 = b + 3;
  for (int i = 0; i < iters; i++) {
    if (MODE == 0 || MODE == 2) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
    if (MODE == 1 || MODE == 2) {
#pragma unroll
      for (int r = 0; r < 8; r++) {
        v0 = fma(v0, 1.0000001, a); v1 = fma(v1, 0.9999999, b);
        v2 = fma(v2, 1.0000001, a); v3 = fma(v3, 0.9999999, b);
        v4 = fma(v4, 1.0000001, a); v5 = fma(v5, 0.9999999, b);
        v6 = fma(v6, 1.0000001, a); v7 = fma(v7, 0.9999999, b);
      }
    }
  }
  double s = c0[0] + c1[1] + c2[2] + c3[3] + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
  out[blockIdx.x * blockDim.x + l] = s;
}

template <int OP>
__global__ void transc_k(double* out, int iters, double seed) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  double x = 1e-3 * (g & 1023) + seed, acc = 0;
  for (int i = 0; i < iters; i++) {
    if (OP == 0) acc += sqrt(x + acc * 1e-30);
    if (OP == 1) { double s, c; sincos(x + acc * 1e-30, &s, &c); acc += s + c; }
    if (OP == 2) acc += atan2(x + acc * 1e-30, 1.0 - x);
    if (OP == 3) acc += 1.0 / (x + acc * 1e-30);
    x += 1e-7;
  }
  out[g] = acc;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  printf("device %s arch %s CUs %d clock %d kHz\n", p.name, p.gcnArchName, p.multiProcessorCount, p.clockRate);
  // (1) layout
  std::vector<double> A(64), B(64), C(256), R(256, 0.0);
  for (int i = 0; i < 16; i++) for (int k = 0; k < 4; k++) A[i * 4 + k] = 1 + i + 17 * k;
  for (int k = 0; k < 4; k++) for (int j = 0; j < 16; j++) B[k * 16 + j] = 3 + 2 * j - 5 * k + (j * j) % 7;
  for (int i = 0; i < 16; i++) for (int j = 0; j < 16; j++) for (int k = 0; k < 4; k++) R[i * 16 + j] += A[i * 4 + k] * B[k * 16 + j];
  double *dA, *dB, *dC; CK(hipMalloc(&dA, 512)); CK(hipMalloc(&dB, 512)); CK(hipMalloc(&dC, 2048));
  CK(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice));
  layout_k<<<1, 64>>>(dA, dB, dC); CK(hipDeviceSynchronize());
  CK(hipMemcpy(C.data(), dC, 2048, hipMemcpyDeviceToHost));
  int bad = 0; for (int i = 0; i < 256; i++) bad += (C[i] != R[i]);
  printf("mfma_f64_16x16x4 layout: %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);
  // (2) throughput
  double* dout; CK(hipMalloc(&dout, 8 << 20));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int blocks = p.multiProcessorCount * 4 * 2, threads = 64, iters = 4096;
  for (int rep = 0; rep < 2; rep++) {
    float ms; 
    hipEventRecord(e0); tput_k<0><<<blocks, threads>>>(dout, iters, 1.0); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    double fl0 = (double)blocks * iters * 4 * 2048; printf("MFMA f64 only: %.2f TF/s (%.3f ms)\n", fl0 / ms / 1e9, ms);
    hipEventRecord(e0); tput_k<1><<<blocks, threads>>>(dout, iters, 1.0); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    double fl1 = (double)blocks * threads * iters * 64 * 2; printf("VALU f64 FMA only: %.2f TF/s (%.3f ms)\n", fl1 / ms / 1e9, ms);
    hipEventRecord(e0); tput_k<2><<<blocks, threads>>>(dout, iters, 1.0); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("MFMA+VALU interleaved: %.2f TF/s combined (%.3f ms)\n", (fl0 + fl1) / ms / 1e9, ms);
  }
  // (3) transcendentals
  const int tb = p.multiProcessorCount * 16, tt = 256, ti = 2048;
  const char* names[] = {"sqrt", "sincos", "atan2", "div"};
  for (int op = 0; op < 4; op++) {
    float ms; hipEventRecord(e0);
    if (op == 0) transc_k<0><<<tb, tt>>>(dout, ti, 0.1);
    if (op == 1) transc_k<1><<<tb, tt>>>(dout, ti, 0.1);
    if (op == 2) transc_k<2><<<tb, tt>>>(dout, ti, 0.1);
    if (op == 3) transc_k<3><<<tb, tt>>>(dout, ti, 0.1);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    double ops = (double)tb * tt * ti;
    printf("%s: %.1f Gop/s chip-wide -> %.1f SIMD-cycles per wave-op @2.4GHz\n", names[op], ops / ms / 1e6,
           (1024.0 * 2.4e9) / (ops / ms * 1e3 / 64));
  }
  return 0;
}
