// probe_rsq.hip — accuracy of gfx950's v_rsq_f64 / v_rcp_f64 against the
// correctly rounded result (host long double), with and without the Newton
// refinements the PSP kernels apply (uwvk_pose_dev.hpp rsqrt_f64, the
// v_rcp_f64 + 2 Newton steps of PSP_FAST & 8 / 32).  Decides whether the
// refinements are needed for the 1e-9 parity bar.
// Build: hipcc -O3 --offload-arch=gfx950 tools/probe_rsq.hip -o /tmp/probe_rsq
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

__global__ void k_probe(const double* x, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  const double r = __builtin_amdgcn_rsq(v);
  const double e = fma(-(v * r), r, 1.0);
  const double rn = fma(r * e, fma(0.375, e, 0.5), r);
  double c = __builtin_amdgcn_rcp(v);
  double c1 = fma(c, fma(-v, c, 1.0), c);
  double c2 = fma(c1, fma(-v, c1, 1.0), c1);
  out[6 * i + 0] = r;
  out[6 * i + 1] = rn;
  out[6 * i + 2] = c;
  out[6 * i + 3] = c1;
  out[6 * i + 4] = c2;
  out[6 * i + 5] = 1.0 / sqrt(v);
}

static double ulp_err(double got, long double ref) {
  const double rd = (double)ref;
  const double u = std::nextafter(rd, INFINITY) - rd;
  return (double)fabsl((long double)got - ref) / u;
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n);
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> ex(-30.0, 10.0), mant(1.0, 2.0);
  for (int i = 0; i < n; i++) x[i] = ldexp(mant(g), (int)std::floor(ex(g)));
  for (int i = 0; i < 4096; i++) x[i] = 0.99 + 0.01 * (i / 4096.0);  // the so3 log range of 1/w
  double *dx, *dout;
  hipMalloc(&dx, n * 8);
  hipMalloc(&dout, (size_t)n * 48);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dout, n);
  std::vector<double> o((size_t)n * 6);
  hipMemcpy(o.data(), dout, (size_t)n * 48, hipMemcpyDeviceToHost);
  const char* names[6] = {"v_rsq_f64", "rsq + Halley step (rsqrt_f64)", "v_rcp_f64", "rcp + 1 Newton",
                          "rcp + 2 Newton", "1.0 / sqrt (library)"};
  for (int k = 0; k < 6; k++) {
    double mx = 0, sum = 0;
    int exact = 0;
    for (int i = 0; i < n; i++) {
      const long double ref = (k == 2 || k == 3 || k == 4) ? 1.0L / (long double)x[i] : 1.0L / sqrtl((long double)x[i]);
      const double e = ulp_err(o[(size_t)6 * i + k], ref);
      mx = e > mx ? e : mx;
      sum += e;
      exact += e <= 0.5 ? 1 : 0;
    }
    printf("%-32s max %.3g ulp, mean %.3g ulp, correctly rounded %.4f\n", names[k], mx, sum / n, exact / (double)n);
  }
  return 0;
}
