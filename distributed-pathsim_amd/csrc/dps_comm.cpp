// RCCL over xGMI behind the C ABI: one communicator per
// process (one rank per GPU), bootstrapped from a unique id that one rank
// creates and the launcher shares out of band (torch.distributed's store /
// gloo carries the 128 bytes; no tensor data goes through PyTorch).  The
// collectives replace the Spark shuffle that brings per-target counts back to
// the driver (DPathSim_APVPA.py:86,107 -- .count() -- and :146-168): a gather
// of every rank's finished top-k block to the root, a broadcast, and the
// all-gather of the ranks' C^T tile slices (N > 1 build).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "dps_host.hpp"

namespace {

int nccl_ret(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return DPS_OK;
  dps::set_error("%s: %s", what, ncclGetErrorString(r));
  return DPS_ERR_HIP;
}

}  // namespace

extern "C" {

int dps_comm_id_bytes(void) { return static_cast<int>(sizeof(ncclUniqueId)); }

int dps_comm_get_id(uint8_t* id_out) {
  DPS_REQUIRE(id_out, DPS_ERR_INVALID, "null id_out");
  ncclUniqueId id;
  if (int rc = nccl_ret(ncclGetUniqueId(&id), "ncclGetUniqueId")) return rc;
  std::memcpy(id_out, &id, sizeof(id));
  return DPS_OK;
}

int dps_comm_init(void** comm_out, int32_t nranks, int32_t rank, const uint8_t* id) {
  DPS_REQUIRE(comm_out && id, DPS_ERR_INVALID, "null comm_out / id");
  DPS_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, DPS_ERR_INVALID,
              "bad rank %d of %d", rank, nranks);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm = nullptr;
  if (int rc = nccl_ret(ncclCommInitRank(&comm, nranks, uid, rank), "ncclCommInitRank")) return rc;
  *comm_out = comm;
  return DPS_OK;
}

int dps_comm_destroy(void* comm) {
  if (!comm) return DPS_OK;
  return nccl_ret(ncclCommDestroy(static_cast<ncclComm_t>(comm)), "ncclCommDestroy");
}

int dps_bcast(void* comm, void* buf, size_t bytes, int32_t root, void* stream) {
  DPS_REQUIRE(comm, DPS_ERR_INVALID, "null comm");
  DPS_REQUIRE(buf || bytes == 0, DPS_ERR_INVALID, "null buffer");
  return nccl_ret(ncclBroadcast(buf, buf, bytes, ncclUint8, root, static_cast<ncclComm_t>(comm),
                                static_cast<hipStream_t>(stream)),
                  "ncclBroadcast");
}

int dps_gather(void* comm, const void* send, void* recv, size_t bytes, int32_t root, void* stream) {
  DPS_REQUIRE(comm, DPS_ERR_INVALID, "null comm");
  DPS_REQUIRE(send || bytes == 0, DPS_ERR_INVALID, "null send buffer");
  return nccl_ret(ncclGather(send, recv, bytes, ncclUint8, root, static_cast<ncclComm_t>(comm),
                             static_cast<hipStream_t>(stream)),
                  "ncclGather");
}

int dps_allgather(void* comm, const void* send, void* recv, size_t bytes, void* stream) {
  DPS_REQUIRE(comm, DPS_ERR_INVALID, "null comm");
  DPS_REQUIRE((send && recv) || bytes == 0, DPS_ERR_INVALID, "null buffer");
  return nccl_ret(ncclAllGather(send, recv, bytes, ncclUint8, static_cast<ncclComm_t>(comm),
                                static_cast<hipStream_t>(stream)),
                  "ncclAllGather");
}

}  // extern "C"
