// qd_comm.hip — the RCCL side of the C-ABI for hosts without torch.distributed: one communicator per
// process (one process per GPU), used for the single sum-reduce of a sharded result (the 2DES
// ensemble grid / waiting-time stack).  The Python host uses torch.distributed
// (backend "nccl" = RCCL) for the same collective; both sum complex128 buffers as 2n float64.
#include "qd_common.hpp"

#include <rccl/rccl.h>

#include <mutex>

namespace qd {
namespace {
std::mutex g_comm_mu;
ncclComm_t g_comm = nullptr;
}  // namespace
}  // namespace qd

using namespace qd;

#define QD_NCCL(call)                                                                                        \
  do {                                                                                                       \
    ncclResult_t _r = (call);                                                                                \
    if (_r != ncclSuccess) {                                                                                 \
      ::qd::set_error("RCCL error %s at %s:%d (%s)", ncclGetErrorString(_r), __FILE__, __LINE__, #call);  \
      return QD_ERCCL;                                                                                       \
    }                                                                                                        \
  } while (0)

extern "C" int qd_comm_unique_id(void* uid) {
  QD_CHECK_ARG(uid != nullptr, "qd_comm_unique_id: null pointer");
  static_assert(sizeof(ncclUniqueId) == QD_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  QD_NCCL(ncclGetUniqueId(&id));
  std::memcpy(uid, &id, sizeof(id));
  return QD_OK;
}

extern "C" int qd_comm_init(int nranks, int rank, const void* uid) {
  QD_CHECK_ARG(uid != nullptr, "qd_comm_init: null unique id");
  QD_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "qd_comm_init: rank %d of %d", rank, nranks);
  std::lock_guard<std::mutex> lk(g_comm_mu);
  QD_CHECK_ARG(g_comm == nullptr, "qd_comm_init: communicator already initialised (qd_comm_destroy first)");
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  QD_NCCL(ncclCommInitRank(&g_comm, nranks, id, rank));
  return QD_OK;
}

extern "C" int qd_reduce_sum(qd_c128* buf, size_t n, int root, void* stream) {
  QD_CHECK_ARG(buf != nullptr || n == 0, "qd_reduce_sum: null buffer");
  std::lock_guard<std::mutex> lk(g_comm_mu);
  QD_CHECK_ARG(g_comm != nullptr, "qd_reduce_sum: no communicator (qd_comm_init)");
  int nr = 0;
  QD_NCCL(ncclCommCount(g_comm, &nr));
  QD_CHECK_ARG(root >= 0 && root < nr, "qd_reduce_sum: root %d of %d ranks", root, nr);
  if (n == 0) return QD_OK;
  // in place: every rank contributes buf, the root receives the sum (complex = two float64 lanes)
  QD_NCCL(ncclReduce(buf, buf, 2 * n, ncclFloat64, ncclSum, root, g_comm, (hipStream_t)stream));
  return QD_OK;
}

extern "C" int qd_comm_destroy(void) {
  std::lock_guard<std::mutex> lk(g_comm_mu);
  if (g_comm) {
    ncclResult_t r = ncclCommDestroy(g_comm);
    g_comm = nullptr;
    if (r != ncclSuccess) {
      set_error("RCCL error %s in ncclCommDestroy", ncclGetErrorString(r));
      return QD_ERCCL;
    }
  }
  return QD_OK;
}
