// Native RCCL collectives of the item-sharded step (host code; one process
// per GPU, xGMI inside a node).
//
// The multi-GPU step's exchanges (csrc/emb_shard.hip, csrc/sampled_shard.hip,
// DESIGN §5) are small — tens of KB to a few MB per rank — and sit between
// kernels of a few microseconds, so what they cost is latency, not bytes.
// Through torch.distributed each collective ran on the process group's own
// stream: the compute stream's event waited on there, the RCCL kernel, an
// event waited on back on the compute stream — two cross-stream hops
// (≈ 10–15 µs each on MI355X) plus the process group's host bookkeeping, per
// collective.  Here the collectives are enqueued by ncclGroupStart / ncclSend /
// ncclRecv / ncclGroupEnd (or the one-call collectives) directly on the
// caller's stream — the stream the producing and consuming kernels run on —
// so they are ordered by the stream alone, with the counts of the variable
// all-to-all taken from host arrays (the splits come from the host batch,
// recommenders/hip/dist.py host_routes).
//
// The communicator is this library's own (ncclCommInitRank over a unique id
// that rank 0 makes and the host process group broadcasts), beside torch's.
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>

#include "common.h"

namespace {

inline int rc(ncclResult_t r) { return r == ncclSuccess ? RG_OK : RG_ERR_LAUNCH; }

ncclDataType_t dtype_of(int code) {
  switch (code) {
    case 0: return ncclUint8;
    case 1: return ncclInt32;
    case 2: return ncclFloat32;
    case 3: return ncclFloat16;
    case 4: return ncclInt64;
    default: return ncclUint8;
  }
}

int elem_size(int code) { return code == 0 ? 1 : code == 3 ? 2 : code == 4 ? 8 : 4; }

}  // namespace

extern "C" int rg_comm_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

extern "C" int rg_comm_unique_id(void* out) {
  if (!out) return RG_ERR_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return RG_ERR_LAUNCH;
  std::memcpy(out, &id, sizeof(id));
  return RG_OK;
}

// device: the HIP device this rank drives (made current before the init)
extern "C" int rg_comm_init(const void* id, int world, int rank, int device, void** comm) {
  if (!id || !comm || world <= 0 || rank < 0 || rank >= world || device < 0) return RG_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return RG_ERR_LAUNCH;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  if (ncclCommInitRank(&c, world, u, rank) != ncclSuccess) return RG_ERR_LAUNCH;
  *comm = c;
  return RG_OK;
}

extern "C" int rg_comm_destroy(void* comm) {
  if (!comm) return RG_ERR_ARG;
  return rc(ncclCommDestroy(static_cast<ncclComm_t>(comm)));
}

// Variable all-to-all: send_counts[q] elements of `send` (consecutive, in rank
// order) go to rank q; recv_counts[q] elements from rank q land consecutively
// in `recv`.  Counts are HOST arrays of world int64; dtype: 0 u8, 1 i32,
// 2 f32, 3 f16, 4 i64.  Every pair is one send / recv in one group (empty ones
// skipped), enqueued on `stream`.
extern "C" int rg_comm_alltoallv(void* comm, const void* send, const int64_t* send_counts, void* recv,
                                 const int64_t* recv_counts, int dtype, hipStream_t stream) {
  if (!comm || !send_counts || !recv_counts) return RG_ERR_ARG;
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  int world = 0;
  if (ncclCommCount(c, &world) != ncclSuccess) return RG_ERR_LAUNCH;
  const ncclDataType_t dt = dtype_of(dtype);
  const int es = elem_size(dtype);
  int64_t so = 0, ro = 0;
  for (int q = 0; q < world; ++q) {
    if (send_counts[q] < 0 || recv_counts[q] < 0) return RG_ERR_ARG;
    so += send_counts[q];
    ro += recv_counts[q];
  }
  if ((so && !send) || (ro && !recv)) return RG_ERR_ARG;
  if (ncclGroupStart() != ncclSuccess) return RG_ERR_LAUNCH;
  so = ro = 0;
  int err = RG_OK;
  for (int q = 0; q < world && err == RG_OK; ++q) {
    if (send_counts[q] > 0)
      err = rc(ncclSend(static_cast<const char*>(send) + so * es, (size_t)send_counts[q], dt, q, c, stream));
    if (err == RG_OK && recv_counts[q] > 0)
      err = rc(ncclRecv(static_cast<char*>(recv) + ro * es, (size_t)recv_counts[q], dt, q, c, stream));
    so += send_counts[q];
    ro += recv_counts[q];
  }
  const int e2 = rc(ncclGroupEnd());
  return err != RG_OK ? err : e2;
}

// Sum all-reduce of n elements (in place when send == recv)
extern "C" int rg_comm_allreduce(void* comm, const void* send, void* recv, int64_t n, int dtype, hipStream_t stream) {
  if (!comm || n < 0 || (n && (!send || !recv)) || dtype == 0) return RG_ERR_ARG;
  if (n == 0) return RG_OK;
  return rc(ncclAllReduce(send, recv, (size_t)n, dtype_of(dtype), ncclSum, static_cast<ncclComm_t>(comm), stream));
}

// recv (world · n) <- every rank's send (n), rank-major
extern "C" int rg_comm_allgather(void* comm, const void* send, void* recv, int64_t n, int dtype, hipStream_t stream) {
  if (!comm || n < 0 || (n && (!send || !recv))) return RG_ERR_ARG;
  if (n == 0) return RG_OK;
  return rc(ncclAllGather(send, recv, (size_t)n, dtype_of(dtype), static_cast<ncclComm_t>(comm), stream));
}

// recv (n) <- slice `rank` of the elementwise sum over ranks of send (world · n)
extern "C" int rg_comm_reduce_scatter(void* comm, const void* send, void* recv, int64_t n, int dtype,
                                      hipStream_t stream) {
  if (!comm || n < 0 || (n && (!send || !recv)) || dtype == 0) return RG_ERR_ARG;
  if (n == 0) return RG_OK;
  return rc(ncclReduceScatter(send, recv, (size_t)n, dtype_of(dtype), ncclSum, static_cast<ncclComm_t>(comm),
                              stream));
}
