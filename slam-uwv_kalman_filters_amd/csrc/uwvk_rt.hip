// uwvk_rt.hip — library-level entry points of the C ABI (device probe, memory
// helpers, status strings).  There is deliberately no CPU fallback anywhere in
// libuwvk.so: without a gfx950 device every handle creation fails loudly.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "../../include/uwvk.h"
#include "uwvk_dev.hpp"

static_assert(UWVK_EDEVICE == 5, "uwvk_dev.hpp edevice_status");
namespace uwvk {
// uwvk_last_device_error: the HIP error behind the thread's last UWVK_EDEVICE
thread_local char g_last_hip_error[160] = "";
void clear_hip_error() { g_last_hip_error[0] = 0; }
void note_hip_error(int err, const char* where) {
  std::snprintf(g_last_hip_error, sizeof(g_last_hip_error), "%s: %s (in %s)", hipGetErrorName((hipError_t)err),
                hipGetErrorString((hipError_t)err), where ? where : "?");
}
}  // namespace uwvk

__global__ void uwvk_probe_kernel(int* out) {
  if (threadIdx.x == 0) out[0] = 0x5a5a;
}

extern "C" {

int uwvk_abi_version(void) { return UWVK_ABI_VERSION; }

int uwvk_device_available(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return 0;
  uwvk::DeviceGuard g(device);
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return 0;
  if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0) return 0;
  if (hipSetDevice(device) != hipSuccess) return 0;
  // make sure this library's gfx950 code object actually loads and runs
  int* d = nullptr;
  int h = 0;
  if (hipMalloc(&d, sizeof(int)) != hipSuccess) return 0;
  hipLaunchKernelGGL(uwvk_probe_kernel, dim3(1), dim3(64), 0, 0, d);
  bool ok = hipGetLastError() == hipSuccess && hipMemcpy(&h, d, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(d);
  return ok && h == 0x5a5a;
}

const char* uwvk_last_device_error(void) { return uwvk::g_last_hip_error; }

const char* uwvk_status_string(uwvk_status s) {
  switch (s) {
    case UWVK_OK: return "UWVK_OK";
    case UWVK_EINVAL: return "UWVK_EINVAL: invalid argument";
    case UWVK_ENAN: return "UWVK_ENAN: measurement contains NaN/Inf";
    case UWVK_ENOTPD: return "UWVK_ENOTPD: covariance not positive definite";
    case UWVK_ENOMODEL: return "UWVK_ENOMODEL: Motion model is not initialized!";
    case UWVK_EDEVICE: return "UWVK_EDEVICE: no usable gfx950 device / HIP error";
    case UWVK_ENOMEM: return "UWVK_ENOMEM: device allocation failed";
    case UWVK_ENOTINIT: return "UWVK_ENOTINIT: filter state not initialised";
    case UWVK_ESCHEDULE: return "UWVK_ESCHEDULE: a tail-chunk hand-off timed out (re-initialise the flagged instances)";
  }
  return "UWVK_?";
}

uwvk_status uwvk_device_malloc(int device, size_t bytes, void** out) {
  int n = 0;
  if (!out) return UWVK_EINVAL;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return UWVK_EDEVICE;
  uwvk::DeviceGuard g(device);
  return hipMalloc(out, bytes ? bytes : 16) == hipSuccess ? UWVK_OK : UWVK_ENOMEM;
}
uwvk_status uwvk_device_free(void* p) {
  uwvk::clear_hip_error();
  return hipFree(p) == hipSuccess ? UWVK_OK : UWVK_EDEVICE;
}
// Synchronous with ALL device work: every handle launches on its own
// non-blocking stream, which the null-stream hipMemcpy does not wait for, so
// a read after run_log(sync = 0) would otherwise race the epoch kernels.
// The device that owns the buffer is made current first (hipDeviceSynchronize
// waits for the CURRENT device only, and a one-process multi-GPU caller may
// have another device current).
static int owner_device(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) return -1;
  return a.type == hipMemoryTypeDevice ? a.device : -1;
}
uwvk_status uwvk_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  uwvk::DeviceGuard g(owner_device(dst));
  if (hipDeviceSynchronize() != hipSuccess) return UWVK_EDEVICE;
  return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? UWVK_OK : UWVK_EDEVICE;
}
uwvk_status uwvk_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  uwvk::DeviceGuard g(owner_device(src));
  if (hipDeviceSynchronize() != hipSuccess) return UWVK_EDEVICE;
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? UWVK_OK : UWVK_EDEVICE;
}
// Stream-ordered: queued on `stream` (a handle's uwvk_*_stream), behind
// everything already queued there; returns once the copy has completed.
uwvk_status uwvk_memcpy_h2d_on(void* dst, const void* src, size_t bytes, void* stream) {
  uwvk::clear_hip_error();
  hipStream_t st = (hipStream_t)stream;
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
  return (uwvk_status)uwvk::launch_sync_status(e, st, "uwvk_memcpy_h2d_on");
}
uwvk_status uwvk_memcpy_d2h_on(void* dst, const void* src, size_t bytes, void* stream) {
  uwvk::clear_hip_error();
  hipStream_t st = (hipStream_t)stream;
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
  return (uwvk_status)uwvk::launch_sync_status(e, st, "uwvk_memcpy_d2h_on");
}

}  // extern "C"
