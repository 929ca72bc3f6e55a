// ms_comm_loopback.h — TEST-ONLY stand-in for the RCCL calls of ms_comm.cpp
// (`make comm-loopback`, -DMS_COMM_LOOPBACK; never part of the product
// libminisched_gpu.so, which links RCCL).
//
// RCCL refuses two ranks of one communicator on the same GPU, so on a 1-GPU box
// the library's world > 1 code (slice_of offsets, padded combine buffers, the
// G-way candidate gather, per-rank bind commits) could otherwise only run with
// world = 1. This loopback lets G contexts of ONE process, each driven by its
// own host thread (one thread per rank, as SURVEY §8(b) "Threading" describes
// for the real library), form a communicator on one device:
//   * init: an in-process rendezvous keyed by the id bytes (blocks until all
//     `world` ranks joined, like ncclCommInitRank);
//   * each collective: every rank records a "send ready" event on its stream
//     and posts its buffers; once all ranks posted (host barrier), each rank's
//     stream waits for every rank's event and runs the combine for its OWN
//     output (element-wise MAX over the ranks' send buffers / copies of their
//     slices); a second barrier + event wait makes the collective complete on a
//     rank's stream only after every rank finished reading its send buffer, as
//     a ring collective completes.
// Every wait is on an event recorded earlier in host order, and all blocking is
// on the host (bounded: a missing rank returns ncclSystemError after 120 s), so
// no device queue ever spins on a value.
#pragma once

#include <rccl/rccl.h>  // types only (ncclComm_t, ncclUniqueId, enums); nothing is linked

#include <hip/hip_runtime.h>

extern "C" {
ncclResult_t lb_ncclGetUniqueId(ncclUniqueId *id);
ncclResult_t lb_ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank);
ncclResult_t lb_ncclCommDestroy(ncclComm_t comm);
ncclResult_t lb_ncclReduceScatter(const void *sendbuff, void *recvbuff, size_t recvcount, ncclDataType_t datatype,
                                  ncclRedOp_t op, ncclComm_t comm, hipStream_t stream);
ncclResult_t lb_ncclAllGather(const void *sendbuff, void *recvbuff, size_t sendcount, ncclDataType_t datatype,
                              ncclComm_t comm, hipStream_t stream);
ncclResult_t lb_ncclAllToAll(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t datatype,
                             ncclComm_t comm, hipStream_t stream);
ncclResult_t lb_ncclGroupStart();
ncclResult_t lb_ncclGroupEnd();
const char *lb_ncclGetErrorString(ncclResult_t result);
// Collectives completed by all ranks of all loopback communicators since the
// library was loaded (exported for the loopback tests: proof that the world > 1
// path really exchanged data).
unsigned long long lb_collectives_issued(void);
}
