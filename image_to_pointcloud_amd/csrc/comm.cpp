// Device-side collectives of the tile-parallel panorama mode (BASELINE configs[3]):
// an RCCL communicator owned by the C ABI, and the band unprojection whose counter exchange
// (RCCL all-reduces) and window-candidate all-gather run on the call's own stream -- no host callback,
// so a whole band call (sweeps, all-reduces, unprojection) can be captured into a HIP graph.
//   i2pc_comm_unique_id / i2pc_comm_create / i2pc_comm_destroy : ncclGetUniqueId /
//       ncclCommInitRank / ncclCommDestroy (the caller ships the 128-byte id from rank 0 to
//       the others, e.g. with torch.distributed.broadcast_object_list)
//   i2pc_unproject_band_rccl : i2pc_unproject_band with the exchange done by RCCL over xGMI
#include "common.h"

#include <rccl/rccl.h>

#include <cstring>

struct i2pc_comm {
  ncclComm_t comm;
  int nranks, rank;
};

namespace {

// hist SUM; counters rows 0-1 SUM, row 2 MIN, row 3 MAX (the i2pc_exchange_fn contract)
int rccl_exchange(void* user, uint32_t* hist, int64_t hist_words, int64_t* counters, int batch, void* stream) {
  auto* c = static_cast<i2pc_comm*>(user);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (ncclGroupStart() != ncclSuccess) return 1;
  ncclResult_t r = hist_words > 0 ? ncclAllReduce(hist, hist, (size_t)hist_words, ncclUint32, ncclSum, c->comm, s)
                                  : ncclSuccess;
  if (r == ncclSuccess && counters) {
    r = ncclAllReduce(counters, counters, 2 * (size_t)batch, ncclInt64, ncclSum, c->comm, s);
    if (r == ncclSuccess) r = ncclAllReduce(counters + 2 * batch, counters + 2 * batch, batch, ncclInt64, ncclMin, c->comm, s);
    if (r == ncclSuccess) r = ncclAllReduce(counters + 3 * batch, counters + 3 * batch, batch, ncclInt64, ncclMax, c->comm, s);
  }
  const ncclResult_t e = ncclGroupEnd();
  if (r != ncclSuccess || e != ncclSuccess) {
    i2pc::set_error(I2PC_ELAUNCH, "RCCL all-reduce failed: %s", ncclGetErrorString(r != ncclSuccess ? r : e));
    return 1;
  }
  return 0;
}

// the window-selection band mode's candidate lists: every rank's `words` into recv [nranks][words]
int rccl_gather(void* user, const uint32_t* send, uint32_t* recv, int64_t words, void* stream) {
  auto* c = static_cast<i2pc_comm*>(user);
  const ncclResult_t r = ncclAllGather(send, recv, (size_t)words, ncclUint32, c->comm, static_cast<hipStream_t>(stream));
  if (r != ncclSuccess) {
    i2pc::set_error(I2PC_ELAUNCH, "RCCL all-gather failed: %s", ncclGetErrorString(r));
    return 1;
  }
  return 0;
}

}  // namespace

using namespace i2pc;

extern "C" int i2pc_comm_unique_id(void* out, int nbytes) {
  clear_error();
  I2PC_REQUIRE(out && nbytes >= (int)sizeof(ncclUniqueId), "need a %d-byte buffer", (int)sizeof(ncclUniqueId));
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return set_error(I2PC_ELAUNCH, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  std::memcpy(out, &id, sizeof id);
  return I2PC_OK;
}

extern "C" int i2pc_comm_create(const void* unique_id, int nranks, int rank, i2pc_comm** comm) {
  clear_error();
  I2PC_REQUIRE(unique_id && comm && nranks > 0 && rank >= 0 && rank < nranks, "bad arguments");
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof id);
  ncclComm_t c;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
  if (r != ncclSuccess) return set_error(I2PC_ELAUNCH, "ncclCommInitRank: %s", ncclGetErrorString(r));
  *comm = new i2pc_comm{c, nranks, rank};
  return I2PC_OK;
}

extern "C" void i2pc_comm_destroy(i2pc_comm* comm) {
  if (!comm) return;
  (void)ncclCommDestroy(comm->comm);
  delete comm;
}

extern "C" int i2pc_unproject_band_rccl(const float* depth, int dep_h, int dep_w, const uint8_t* image_band,
                                        int channels, int img_h, int img_w, int row0, int row1,
                                        const i2pc_unproject_params* params, float* xyz_band, uint8_t* rgb_band,
                                        double* bbox, double* stats, void* workspace, size_t workspace_bytes,
                                        i2pc_comm* comm, void* stream) {
  clear_error();
  I2PC_REQUIRE(comm != nullptr, "comm is NULL");
  // window selection: one sweep, then the counters all-reduced and the candidate lists all-gathered
  return i2pc_unproject_band_w(depth, dep_h, dep_w, image_band, channels, img_h, img_w, row0, row1, params, xyz_band,
                               rgb_band, bbox, stats, workspace, workspace_bytes, comm->nranks, rccl_exchange,
                               rccl_gather, comm, stream);
}
