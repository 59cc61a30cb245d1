// uwvk_comm.hip — the engine's one collective: the ensemble-statistics
// all-reduce of instance-sharded runs, over RCCL
// (xGMI between the GPUs of a node).  Thin wrappers so that C / C++ callers
// need no RCCL headers: a communicator is an opaque void* (ncclComm_t).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "../../include/uwvk.h"

extern "C" {

int uwvk_comm_unique_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

uwvk_status uwvk_comm_unique_id(char* id) {
  if (!id) return UWVK_EINVAL;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return UWVK_EDEVICE;
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return UWVK_OK;
}

uwvk_status uwvk_comm_init(int nranks, const char* id, int rank, int device, void** comm) {
  if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) return UWVK_EINVAL;
  *comm = nullptr;
  if (hipSetDevice(device) != hipSuccess) return UWVK_EDEVICE;
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  if (ncclCommInitRank(&c, nranks, u, rank) != ncclSuccess) return UWVK_EDEVICE;
  *comm = (void*)c;
  return UWVK_OK;
}

void uwvk_comm_destroy(void* comm) {
  if (comm) (void)ncclCommDestroy((ncclComm_t)comm);
}

// in-place sum of n doubles in device memory, on `stream`, over `comm`
uwvk_status uwvk_comm_allreduce_sum_device(void* comm, double* d_buf, int64_t n, void* stream) {
  if (!comm || !d_buf || n < 0) return UWVK_EINVAL;
  if (ncclAllReduce(d_buf, d_buf, (size_t)n, ncclDouble, ncclSum, (ncclComm_t)comm, (hipStream_t)stream) !=
      ncclSuccess)
    return UWVK_EDEVICE;
  return UWVK_OK;
}

}  // extern "C"
