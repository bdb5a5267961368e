// comm.cpp -- RCCL over xGMI: the multi-GPU replacement of StorageClient's per-host RPC
// scatter/gather (src/storage/client/StorageClient.inl:74-159).  One process per GPU; every
// collective runs on the context's stream so it orders with the expansion kernels.
#include <rccl/rccl.h>

#include <vector>

#include "engine.h"

namespace nbg {

#define NBG_NCCL(x)                                                                        \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess) throw Error(NBG_E_COMM, std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

static ncclComm_t comm_of(Ctx& c) {
  if (c.world == 1) return nullptr;
  if (!c.comm) throw Error(NBG_E_STATE, "nbg_comm_init was not called");
  return static_cast<ncclComm_t>(c.comm);
}

int32_t comm_unique_id(uint8_t out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return NBG_E_COMM;
  memcpy(out, &id, 128);
  return NBG_OK;
}

void comm_init(Ctx& c, const uint8_t id_bytes[128]) {
  if (c.world == 1) return;
  ncclUniqueId id;
  memcpy(&id, id_bytes, 128);
  NBG_HIP(hipSetDevice(c.device));
  ncclComm_t comm;
  NBG_NCCL(ncclCommInitRank(&comm, c.world, id, c.rank));
  c.comm = comm;
}

void comm_destroy(Ctx& c) {
  if (c.comm) ncclCommDestroy(static_cast<ncclComm_t>(c.comm));
  c.comm = nullptr;
}

void comm_allgather_bytes(Ctx& c, const void* send, size_t bytes_each, void* recv) {
  if (c.world == 1) {
    NBG_HIP(hipMemcpyAsync(recv, send, bytes_each, hipMemcpyDeviceToDevice, c.stream));
    return;
  }
  NBG_NCCL(ncclAllGather(send, recv, bytes_each, ncclUint8, comm_of(c), c.stream));
}

// all-to-all with per-peer byte counts (grouped point-to-point: on xGMI every peer pair has
// its own link, so the 7 transfers of an 8-GPU exchange run concurrently)
void comm_alltoallv_bytes(Ctx& c, const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                          const size_t* recv_bytes, const size_t* recv_off) {
  if (c.world == 1) {
    if (send_bytes[0])
      NBG_HIP(hipMemcpyAsync(static_cast<uint8_t*>(recv) + recv_off[0],
                             static_cast<const uint8_t*>(send) + send_off[0], send_bytes[0],
                             hipMemcpyDeviceToDevice, c.stream));
    return;
  }
  ncclComm_t comm = comm_of(c);
  NBG_NCCL(ncclGroupStart());
  for (int p = 0; p < c.world; p++) {
    if (send_bytes[p])
      NBG_NCCL(ncclSend(static_cast<const uint8_t*>(send) + send_off[p], send_bytes[p], ncclUint8, p, comm, c.stream));
    if (recv_bytes[p])
      NBG_NCCL(ncclRecv(static_cast<uint8_t*>(recv) + recv_off[p], recv_bytes[p], ncclUint8, p, comm, c.stream));
  }
  NBG_NCCL(ncclGroupEnd());
}

void comm_allreduce_sum_i64(Ctx& c, int64_t* d_vals, size_t n) {
  if (c.world == 1) return;
  NBG_NCCL(ncclAllReduce(d_vals, d_vals, n, ncclInt64, ncclSum, comm_of(c), c.stream));
}

}  // namespace nbg
