// sa_rccl.cpp — the one exchange step of the multi-GPU path: the masked
// partial sums (uint64) of every GPU's clients reduced to the server GPU with
// RCCL over xGMI.  Replaces the RayFed/Ray object-store `.to(server)` transfer
// of masked arrays plus the server's np.sum (sfl/distributed/op_strategy.py:
// 131-141, sfl/security/aggregation/sparse_plain_aggregator.py:86-94).
// uint64 addition is associative mod 2^64, so every RCCL algorithm/order
// yields the bit-exact masked sum.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include "../../include/sfl_sa.h"
#include "sa_internal.h"

static_assert(sizeof(ncclUniqueId) <= SA_UNIQUE_ID_BYTES, "unique id size");

#define SA_NCCL_CHECK(expr)                                                          \
  do {                                                                               \
    ncclResult_t r_ = (expr);                                                        \
    if (r_ != ncclSuccess) {                                                         \
      sa_set_error("%s failed: %s", #expr, ncclGetErrorString(r_));                  \
      return SA_ERR_RCCL;                                                            \
    }                                                                                \
  } while (0)

extern "C" int sa_comm_unique_id(void* id_out, int cap) {
  if (!id_out || cap < (int)sizeof(ncclUniqueId)) {
    sa_set_error("sa_comm_unique_id: buffer too small (%d < %d)", cap, (int)sizeof(ncclUniqueId));
    return SA_ERR_ARG;
  }
  ncclUniqueId id;
  SA_NCCL_CHECK(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof(id));
  return SA_OK;
}

extern "C" int sa_comm_init(void** comm, const void* id, int nranks, int rank, int device) {
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) {
    sa_set_error("sa_comm_init: bad arguments");
    return SA_ERR_ARG;
  }
  SA_HIP_CHECK(hipSetDevice(device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  SA_NCCL_CHECK(ncclCommInitRank(&c, nranks, uid, rank));
  *comm = (void*)c;
  return SA_OK;
}

extern "C" int sa_comm_reduce_u64(void* comm, const uint64_t* send, uint64_t* recv, uint64_t n,
                                  int root, void* stream) {
  if (!comm || !send) {
    sa_set_error("sa_comm_reduce_u64: bad arguments");
    return SA_ERR_ARG;
  }
  // non-root ranks without a receive buffer reduce in place: RCCL is handed
  // a valid buffer on every rank whatever algorithm it picks
  uint64_t* rb = recv ? recv : const_cast<uint64_t*>(send);
  SA_NCCL_CHECK(ncclReduce(send, rb, (size_t)n, ncclUint64, ncclSum, root, (ncclComm_t)comm,
                           (hipStream_t)stream));
  return SA_OK;
}

extern "C" int sa_comm_allreduce_u64(void* comm, const uint64_t* send, uint64_t* recv,
                                     uint64_t n, void* stream) {
  if (!comm || !send || !recv) {
    sa_set_error("sa_comm_allreduce_u64: bad arguments");
    return SA_ERR_ARG;
  }
  SA_NCCL_CHECK(ncclAllReduce(send, recv, (size_t)n, ncclUint64, ncclSum, (ncclComm_t)comm,
                              (hipStream_t)stream));
  return SA_OK;
}

// The sharded server (ReduceScatter, decode the shards in
// parallel, Gather float64): rank r receives the masked sum of elements
// [r*count, (r+1)*count) of send.  In place when recv == send + r*count.
extern "C" int sa_comm_reduce_scatter_u64(void* comm, const uint64_t* send, uint64_t* recv,
                                          uint64_t count, void* stream) {
  if (!comm || !send || !recv) {
    sa_set_error("sa_comm_reduce_scatter_u64: bad arguments");
    return SA_ERR_ARG;
  }
  SA_NCCL_CHECK(ncclReduceScatter(send, recv, (size_t)count, ncclUint64, ncclSum, (ncclComm_t)comm,
                                  (hipStream_t)stream));
  return SA_OK;
}

// The sharded server's exchange as direct transfers over the point-to-point
// xGMI links: rank r sends shard p of `send` (count elements at send +
// p*count) to rank p and receives rank p's shard r into recv + p*count, for
// every p != r, in one grouped ncclSend/ncclRecv round; recv's slot r is not
// written (the caller's own shard stays in send).  The caller then sums the
// world shards (sa_sum_u64).  The same bytes as sa_comm_reduce_scatter_u64,
// each shard crossing exactly one link, instead of RCCL's reduce-scatter
// schedule (rings or trees of partial sums).
extern "C" int sa_comm_alltoall_u64(void* comm, const uint64_t* send, uint64_t* recv, uint64_t count,
                                    void* stream) {
  if (!comm || !send || !recv) {
    sa_set_error("sa_comm_alltoall_u64: bad arguments");
    return SA_ERR_ARG;
  }
  ncclComm_t c = (ncclComm_t)comm;
  int rank = 0, nranks = 0;
  SA_NCCL_CHECK(ncclCommUserRank(c, &rank));
  SA_NCCL_CHECK(ncclCommCount(c, &nranks));
  if (count == 0 || nranks == 1) return SA_OK;
  hipStream_t s = (hipStream_t)stream;
  SA_NCCL_CHECK(ncclGroupStart());
  for (int k = 1; k < nranks; ++k) {  // peers in ring order from this rank: every link busy at once
    const int to = (rank + k) % nranks, from = (rank - k + nranks) % nranks;
    ncclResult_t e = ncclSend(send + (size_t)to * count, (size_t)count, ncclUint64, to, c, s);
    if (e == ncclSuccess) e = ncclRecv(recv + (size_t)from * count, (size_t)count, ncclUint64, from, c, s);
    if (e != ncclSuccess) {
      ncclGroupEnd();
      sa_set_error("sa_comm_alltoall_u64: send/recv with rank %d/%d failed: %s", to, from, ncclGetErrorString(e));
      return SA_ERR_RCCL;
    }
  }
  SA_NCCL_CHECK(ncclGroupEnd());
  return SA_OK;
}

// float64 shards to the server: root's recv[r*count, (r+1)*count) = rank r's
// send (one grouped ncclSend/ncclRecv round; root's own shard is a device copy
// unless it is already in place).  recv is only read on root (may be NULL
// elsewhere).
extern "C" int sa_comm_gather_f64(void* comm, const double* send, double* recv, uint64_t count,
                                  int root, void* stream) {
  if (!comm || !send) {
    sa_set_error("sa_comm_gather_f64: bad arguments");
    return SA_ERR_ARG;
  }
  ncclComm_t c = (ncclComm_t)comm;
  int rank = 0, nranks = 0;
  SA_NCCL_CHECK(ncclCommUserRank(c, &rank));
  SA_NCCL_CHECK(ncclCommCount(c, &nranks));
  if (root < 0 || root >= nranks || (rank == root && !recv)) {
    sa_set_error("sa_comm_gather_f64: bad root %d or missing receive buffer (world %d)", root, nranks);
    return SA_ERR_ARG;
  }
  if (count == 0) return SA_OK;
  hipStream_t s = (hipStream_t)stream;
  if (rank != root) {
    SA_NCCL_CHECK(ncclSend(send, (size_t)count, ncclFloat64, root, c, s));
    return SA_OK;
  }
  double* own = recv + (size_t)root * count;
  if (own != send) SA_HIP_CHECK(hipMemcpyAsync(own, send, count * sizeof(double), hipMemcpyDeviceToDevice, s));
  SA_NCCL_CHECK(ncclGroupStart());
  for (int r = 0; r < nranks; ++r) {
    if (r == root) continue;
    ncclResult_t e = ncclRecv(recv + (size_t)r * count, (size_t)count, ncclFloat64, r, c, s);
    if (e != ncclSuccess) {
      ncclGroupEnd();
      sa_set_error("ncclRecv from rank %d failed: %s", r, ncclGetErrorString(e));
      return SA_ERR_RCCL;
    }
  }
  SA_NCCL_CHECK(ncclGroupEnd());
  return SA_OK;
}

extern "C" int sa_comm_destroy(void* comm) {
  if (!comm) return SA_OK;
  SA_NCCL_CHECK(ncclCommDestroy((ncclComm_t)comm));
  return SA_OK;
}

extern "C" int sa_comm_info(void* comm, int* nranks, int* rank, int* device) {
  if (!comm) {
    sa_set_error("sa_comm_info: bad arguments (comm is NULL)");
    return SA_ERR_ARG;
  }
  int v = 0;
  if (nranks) {
    SA_NCCL_CHECK(ncclCommCount((ncclComm_t)comm, &v));
    *nranks = v;
  }
  if (rank) {
    SA_NCCL_CHECK(ncclCommUserRank((ncclComm_t)comm, &v));
    *rank = v;
  }
  if (device) {
    SA_NCCL_CHECK(ncclCommCuDevice((ncclComm_t)comm, &v));
    *device = v;
  }
  return SA_OK;
}
