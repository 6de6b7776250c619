/*
 * hccl.h — MI355X-native drop-in for the reducing half of HCCL's operator surface.
 *
 * Each entry point below keeps the exact name, argument order, argument meaning and
 * return-code behaviour of the reference's declaration, so a caller linked against
 * HCCL links against libhccl_amd.so unchanged:
 *
 *   HcclAllReduce      replaces /root/reference/include/hccl.h:35-37  (impl all_reduce_op.cc:23-52)
 *   HcclReduceScatter  replaces /root/reference/include/hccl.h:67-69  (impl reduce_scatter_op.cc:23-72)
 *   HcclReduceScatterV replaces /root/reference/include/hccl.h:87-89  (impl reduce_scatter_v_op.cc:24-83)
 *   HcclReduce         replaces /root/reference/include/hccl.h:245-247 (impl reduce_op.cc:23-54)
 *
 * The communicator calls are the hcomm functions the reference's callers use
 * (examples/02_collectives/01_allreduce/main.cc:75,100,122; test/st/.../all_reduce_testcase.cc:80);
 * they are external to the reference repo and are implemented here over RCCL:
 *
 *   HcclGetRootInfo, HcclCommInitRootInfo, HcclCommInitClusterInfo, HcclCommInitAll, HcclCommDestroy,
 *   HcclGetRankSize, HcclGetRankId
 *
 * Semantics: stream-ordered and asynchronous with respect to the host, like the reference
 * (op_common.cc:962-970): work is enqueued behind everything already on `stream`, internal
 * streams are joined back into `stream` before return, and the host never blocks.
 */
#ifndef HCCL_AMD_HCCL_H_
#define HCCL_AMD_HCCL_H_

#include "hccl_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* AllReduce: recvBuf[i] = op over ranks of sendBuf[i], count elements. In-place allowed. */
extern HcclResult HcclAllReduce(void* sendBuf, void* recvBuf, uint64_t count, HcclDataType dataType,
                                HcclReduceOp op, HcclComm comm, aclrtStream stream);

/* ReduceScatter: sendBuf holds rankSize blocks of recvCount; rank r receives the reduce of block r. */
extern HcclResult HcclReduceScatter(void* sendBuf, void* recvBuf, uint64_t recvCount, HcclDataType dataType,
                                    HcclReduceOp op, HcclComm comm, aclrtStream stream);

/* ReduceScatterV: rank q's block of sendBuf is sendCounts[q] elements at sendDispls[q] (uint64 arrays of rankSize
 * entries); rank r receives the reduce of every rank's block r, sendCounts[r] elements (recvCount must hold them).
 * Replaces /root/reference/include/hccl.h:87-89 (reduce_scatter_v_op.cc:24-83).
 * Per-rank contract: the argument checks are local and run before any collective work, like the reference's. One
 * addition has no reference counterpart: sendCounts[rank] > recvCount returns HCCL_E_PARA on that rank alone (the
 * reference would overrun recvBuf). Its peers are not told: they wait in the collective until HCCL_EXEC_TIMEOUT
 * fails their communicators (HCCL_E_TIMEOUT, then HCCL_E_SUSPENDING), so every rank must pass consistent counts. */
extern HcclResult HcclReduceScatterV(void* sendBuf, const void* sendCounts, const void* sendDispls, void* recvBuf,
                                     uint64_t recvCount, HcclDataType dataType, HcclReduceOp op, HcclComm comm,
                                     aclrtStream stream);

/* Reduce: recvBuf on `root` receives the reduce of every rank's sendBuf (recvBuf must be non-null everywhere). */
extern HcclResult HcclReduce(void* sendBuf, void* recvBuf, uint64_t count, HcclDataType dataType, HcclReduceOp op,
                             uint32_t root, HcclComm comm, aclrtStream stream);

/* AllGather: recvBuf holds rankSize blocks of sendCount, block r = rank r's sendBuf (replaces
 * /root/reference/include/hccl.h:120-121; the gather half of AllReduce and of config C4's RS + AG). */
extern HcclResult HcclAllGather(void* sendBuf, void* recvBuf, uint64_t sendCount, HcclDataType dataType,
                                HcclComm comm, aclrtStream stream);

/* Communicator management (hcomm surface used by the reference's callers). */
extern HcclResult HcclGetRootInfo(HcclRootInfo* rootInfo);
extern HcclResult HcclCommInitRootInfo(uint32_t nRanks, const HcclRootInfo* rootInfo, uint32_t rank,
                                       HcclComm* comm);
/* Rank `rank` of the communicator described by the rank table file `clusterInfo` (JSON, docs/.../cluster_info_config/rank_table_config_a2.md;
 * test/st/algorithm/testcase/all_reduce_testcase.cc:80). The rank runs on its entry's device_id. Rank 0 publishes the
 * transport's unique id over TCP at the rank-0 server's host_ip (else HCCL_IF_IP, else 127.0.0.1 for one server) and
 * the rank-0 device's host_port (else HCCL_IF_BASE_PORT, default 60000), waiting at most HCCL_CONNECT_TIMEOUT + 20 s. */
extern HcclResult HcclCommInitClusterInfo(const char* clusterInfo, uint32_t rank, HcclComm* comm);
/* One communicator per listed device in this process (single-node batch creation); comms[i] is rank i on
 * devices[i]. Drive each rank from its own host thread. */
extern HcclResult HcclCommInitAll(uint32_t ndev, int32_t* devices, HcclComm* comms);
/* Destroys the communicator. Its outstanding work is flushed first (ncclCommFinalize, bounded by HCCL_EXEC_TIMEOUT;
 * past it the communicator is aborted). If a HIP graph captured on a collective of this communicator is still alive,
 * the call returns HCCL_SUCCESS at once and the teardown runs when the last such graph is destroyed: the graph holds
 * the communicator's staging and RCCL plans (RCCL's own destroy would wait for the graph). The handle is invalid on
 * return either way. */
extern HcclResult HcclCommDestroy(HcclComm comm);
extern HcclResult HcclGetRankSize(HcclComm comm, uint32_t* rankSize);
extern HcclResult HcclGetRankId(HcclComm comm, uint32_t* rank);
/* Asynchronous error of the communicator (CANN hccl_comm.h; polled by framework watchdogs such as torch_npu's
 * ProcessGroupHCCL). Non-blocking. *asyncError = HCCL_E_TIMEOUT after a one-sided barrier wait exceeded its bound,
 * or after a collective on the RCCL path ran past HCCL_EXEC_TIMEOUT once started (default 1836 s, 0 = never; the
 * communicator's watchdog then aborts RCCL), the transport's error after an RCCL asynchronous failure, else
 * HCCL_SUCCESS. Once the first
 * collective entry has observed such an error (and returned it), every later collective on the communicator returns
 * HCCL_E_SUSPENDING: the reference's status gate, src/ops/op_common/op_common.cc:89-97. */
extern HcclResult HcclGetCommAsyncError(HcclComm comm, HcclResult* asyncError);

#ifdef __cplusplus
}
#endif
#endif /* HCCL_AMD_HCCL_H_ */
