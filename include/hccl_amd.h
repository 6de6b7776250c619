/*
 * hccl_amd.h — extension C ABI of libhccl_amd.so (everything that is not in the reference's hccl.h).
 *
 * 1. The inner reduce primitive. In the reference every reducing schedule ends in
 *    LocalReduce (/root/reference/src/ops/op_common/template/wrapper/alg_data_trans_wrapper.cc:901-928),
 *    which enqueues hcomm's HcommLocalReduceOnThread(thread, dst, src, count, dtype, op) = "dst = src (+) dst"
 *    (call site :924-926; stub semantics test/st/algorithm/utils/src/hccl_proxy/hccl_stub.cc:648-677), or, for
 *    64-bit dtypes and PROD, runs AicpuReduce on the AICPU core (:1254-1353). HcclAmdLocalReduce replaces both
 *    with one HIP kernel family on a HIP stream. Element rule, identical to AicpuReduceTemplate (:1313-1353):
 *        SUM  dst = src + dst          PROD dst = src * dst   (integers wrap, two's complement)
 *        MAX  dst = (src < dst) ? dst : src    (std::max(src, dst): ties and NaN give src)
 *        MIN  dst = (dst < src) ? dst : src    (std::min(src, dst): ties and NaN give src)
 *    fp16 is computed through fp32 with round-to-nearest-even (AicpuReduceFp16, :1232-1252); bf16 the same way.
 *
 * 2. The schedule IR. Every collective is compiled to a per-rank list of HcclAmdIrOp records. The same records
 *    are executed by the HIP/RCCL executor and replayed by the CPU oracle (oracle/), so the association order of
 *    every reduced element is fixed by the IR and checked bit-for-bit.
 *
 * 3. A loopback world: nRanks communicators inside one process on the current device whose "links" are
 *    device-to-device copies. It runs the exact executor the RCCL path runs and is how the multi-rank schedules
 *    are tested on a single MI355X (the reference's analogue is its host simulator, test/st/algorithm).
 */
#ifndef HCCL_AMD_EXT_H_
#define HCCL_AMD_EXT_H_

#include "hccl_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- local reduce primitive */

/* dst[i] = src[i] (op) dst[i], i < count. Mirrors HcommLocalReduceOnThread(thread, dst, src, count, dt, op). */
extern HcclResult HcclAmdLocalReduce(void* dst, const void* src, uint64_t count, HcclDataType dataType,
                                     HcclReduceOp op, aclrtStream stream);

/* out[i] = src[i] (op) dst[i]: the out-of-place form (3 streams: 2 reads, 1 write). out may alias dst or src. */
extern HcclResult HcclAmdLocalReduce2(void* out, const void* src, const void* dst, uint64_t count,
                                      HcclDataType dataType, HcclReduceOp op, aclrtStream stream);

/* Ordered n-ary fold in one pass: acc = srcs[0]; for j = 1..nsrc-1: acc = srcs[j] (op) acc; out = acc.
 * 1 <= nsrc <= HCCL_AMD_IR_MAX_SRC. out may alias any srcs[j]. */
extern HcclResult HcclAmdLocalReduceN(void* out, const void* const* srcs, uint32_t nsrc, uint64_t count,
                                      HcclDataType dataType, HcclReduceOp op, aclrtStream stream);

/* Tuning knobs for the streaming reduce kernels (process-wide; 0 = default for every field).
 * blocksPerCu: workgroups of 256 threads per CU in the persistent grid. unroll: 16-B vectors per lane per
 * iteration (1, 2, 4 or 8). cachePolicy: 1 = plain, 2 = nt loads, 3 = nt stores, 4 = nt loads + stores,
 * 5 = nt loads + stores with contiguous per-workgroup tile runs. */
extern HcclResult HcclAmdSetReduceLaunch(uint32_t blocksPerCu, uint32_t unroll, uint32_t cachePolicy);

/* Operand pipelining of the ordered n-ary fold (process-wide, tuning): 0 = default, 1 = serial (operand j+1 loaded
 * after operand j is folded), 2 = prefetch (operand j+1 loaded before operand j is folded), 3 = every operand of a tile
 * loaded before the first combine (compile-time operand count, 3..8). The fold order is the same in every mode. */
extern HcclResult HcclAmdSetFoldMode(uint32_t mode);

/* Byte size of one element of dataType, 0 if unknown (DATATYPE_SIZE_TABLE, alg_param.h:43-61). */
extern uint32_t HcclAmdDataTypeSize(HcclDataType dataType);

extern const char* HcclAmdGetErrorString(HcclResult code);

/* ---------------------------------------------------------------- schedule IR */

#define HCCL_AMD_IR_MAX_SRC 16

typedef enum {
    HCCL_AMD_IR_COPY = 0,   /* dst <- src[0] */
    HCCL_AMD_IR_REDUCE = 1, /* dst <- fold(src[0..nsrc)) with the LocalReduceN order */
    HCCL_AMD_IR_SEND = 2,   /* send src[0] (count elements) to peer */
    HCCL_AMD_IR_RECV = 3    /* receive count elements from peer into dst */
} HcclAmdIrKind;

typedef enum {
    HCCL_AMD_BUF_INPUT = 0,   /* user sendBuf */
    HCCL_AMD_BUF_OUTPUT = 1,  /* user recvBuf */
    HCCL_AMD_BUF_SCRATCH = 2  /* per-communicator staging ("CCL buffer") */
} HcclAmdBuf;

typedef struct {
    int32_t kind;   /* HcclAmdIrKind */
    int32_t peer;   /* SEND / RECV peer rank, else -1 */
    int32_t nsrc;   /* number of valid src entries */
    int32_t group;  /* SEND/RECV records with equal group are posted together (one RCCL group) */
    uint64_t count; /* elements */
    int32_t dstBuf; /* HcclAmdBuf, -1 for SEND */
    int32_t reserved;
    uint64_t dstOff; /* element offset */
    int32_t srcBuf[HCCL_AMD_IR_MAX_SRC];
    uint64_t srcOff[HCCL_AMD_IR_MAX_SRC];
} HcclAmdIrOp;

typedef enum {
    HCCL_AMD_OP_ALLREDUCE = 0,
    HCCL_AMD_OP_REDUCE_SCATTER = 1,
    HCCL_AMD_OP_REDUCE = 2,
    HCCL_AMD_OP_ALLGATHER = 3, /* the second half of AllReduce as an operator (count = sendCount) */
    HCCL_AMD_OP_REDUCE_SCATTER_V = 4 /* per-rank counts and displacements (HcclAmdBuildScheduleV) */
} HcclAmdOpType;

typedef enum {
    HCCL_AMD_ALGO_AUTO = 0,         /* reference selector policy (all_reduce_auto_selector.cc:517-550) */
    HCCL_AMD_ALGO_MESH_ONESHOT = 1, /* order O1: own input first, then ascending ranks */
    HCCL_AMD_ALGO_MESH_TWOSHOT = 2, /* AllReduce: order O2 (ascending from rank 0); RS/Reduce: O1 */
    HCCL_AMD_ALGO_RING = 3,         /* ring reduce-scatter (+ ring all-gather) */
    HCCL_AMD_ALGO_RHD = 4,          /* recursive halving / doubling (power-of-two rank counts) */
    HCCL_AMD_ALGO_NHR = 5,          /* AllReduce: the reference's NHR template, order O5 (any rank count) */
    HCCL_AMD_ALGO_ORDER_PRESERVED = 6, /* AllReduce / ReduceScatter: HCCL_DETERMINISTIC=STRICT tree, order O4 */
    HCCL_AMD_ALGO_IPC_TWOSHOT = 7,     /* AllReduce: one kernel over peer-mapped staging (AIV GM_IN model), O2 */
    HCCL_AMD_ALGO_MESH_CHUNK = 8,      /* AllReduce / ReduceScatter: the reference's MeshChunk templates, order O6
                                          (owner first, then the peers in a per-sub-slice rotated order) */
    HCCL_AMD_ALGO_IPC = 9,             /* the one-sided kernel in the order family the auto selector picks (one-shot
                                          O1 / two-shot O2 / MeshChunk O6 ...): the auto path's bits over IPC */
    HCCL_AMD_ALGO_AIV = 10,            /* the reference's AIV engine (HCCL_OP_EXPANSION_MODE=AIV): SelectAivAlgo's
                                          choice and orders on the one-sided kernel; what it does not match runs
                                          the auto (AICPU) selection, as the reference falls back */
    HCCL_AMD_ALGO_AIV_ONLY = 11,       /* the AIV engine with no fallback (OpExecuteConfig::AIV_ONLY): no 8 MiB x n
                                          bound, and what SelectAivAlgo does not match returns HCCL_E_NOT_SUPPORT */
    HCCL_AMD_ALGO_IPC_RHD = 12         /* AllReduce, power-of-two n: HCCL_AMD_ALGO_RHD's bits from one one-shot launch
                                          of the one-sided kernel (one barrier instead of 2 log2 n transport steps);
                                          anything else, or no peer mappings, runs HCCL_AMD_ALGO_RHD */
} HcclAmdAlgo;

/* Variant of the reference's AIV engine a call takes (HcclAmdSelectAivAlgo). */
typedef enum {
    HCCL_AMD_AIV_NOT_MATCHED = 0,       /* SelectAivAlgo does not match: the AICPU engine runs */
    HCCL_AMD_AIV_AR_ONESHOT = 1,        /* aiv_all_reduce_mesh_1d_oneshot.h:33-48, order O2 */
    HCCL_AMD_AIV_AR_TWOSHOT_LARGE = 2,  /* aiv_all_reduce_mesh_1d_twoshot.h:145-181: O1 over groupSize * n
                                           balanced slices, rank r owning [r * groupSize, (r + 1) * groupSize) */
    HCCL_AMD_AIV_AR_TWOSHOT_SMALL = 3,  /* aiv_all_reduce_mesh_1d_twoshot.h:224-271: O2 over ceil(count / n) */
    HCCL_AMD_AIV_RS_BIGDATA = 4,        /* aiv_reduce_scatter_mesh_1d_bigdata.h:85-101: O2 */
    HCCL_AMD_AIV_RS_LOCAL_TREE = 5      /* aiv_reduce_scatter_local_tree.h:138-172: O4 (pow-2 tree) */
} HcclAmdAivVariant;

/* The AIV-engine variant an operation would take (opType ALLREDUCE or REDUCE_SCATTER; count = recvCount for
 * ReduceScatter) on nRanks ranks with `coreLimit` vector cores (0 = HCCL_AMD_AIV_CORE_LIMIT, default 48) and the CCL
 * buffer HCCL_BUFFSIZE. flags: bit 0 = HCCL_DETERMINISTIC=strict, bit 1 = AIV_ONLY (HCCL_AMD_ALGO_AIV_ONLY).
 * *groupSize (may be NULL) receives the slices per rank of HCCL_AMD_AIV_AR_TWOSHOT_LARGE (1 otherwise). Returns an
 * HcclAmdAivVariant. */
extern int32_t HcclAmdSelectAivAlgo(int32_t opType, uint32_t nRanks, uint64_t count, HcclDataType dataType,
                                    HcclReduceOp op, uint32_t coreLimit, int32_t flags, uint32_t* groupSize);

/* Build rank `rank`'s schedule. If ops == NULL only *numOps is written. scratchElems receives the number of
 * scratch elements the schedule addresses. pieceBytes = 0 picks the default pipelining granule. */
extern HcclResult HcclAmdBuildSchedule(int32_t opType, int32_t algo, uint32_t nRanks, uint32_t rank, uint64_t count,
                                       HcclDataType dataType, uint32_t root, uint64_t pieceBytes, HcclAmdIrOp* ops,
                                       uint64_t capacity, uint64_t* numOps, int32_t* algoUsed,
                                       uint64_t* scratchElems);

/* ReduceScatterV schedule of rank `rank`: rank q's block of every input is [sendDispls[q], sendDispls[q] +
 * sendCounts[q]) elements (nRanks entries each); the mesh template's order O1
 * (ins_temp_reduce_scatter_v_mesh_1D.cc:107-146). Same output conventions as HcclAmdBuildSchedule. */
extern HcclResult HcclAmdBuildScheduleV(uint32_t nRanks, uint32_t rank, const uint64_t* sendCounts,
                                        const uint64_t* sendDispls, HcclDataType dataType, uint64_t pieceBytes,
                                        HcclAmdIrOp* ops, uint64_t capacity, uint64_t* numOps,
                                        uint64_t* scratchElems);

/* The algorithm HCCL_AMD_ALGO_AUTO selects for an operation of `bytes` bytes per rank (ReduceScatter: recvCount
 * bytes) on nRanks ranks; special = 64-bit data type or PROD (the reference selectors' isDataTypeOrReduceTypeSpecial).
 * Mirrors AllReduceAutoSelector / ReduceScatterAutoSelector / ReduceAutoSelector for a single-node MESH_1D. */
extern int32_t HcclAmdSelectAlgo(int32_t opType, uint32_t nRanks, uint64_t bytes, int32_t special);

/* The rings HCCL_AMD_ALGO_RING runs on nRanks ranks: arc-disjoint directed Hamiltonian cycles (n-1 of them for
 * n <= 8 except 4 and 6, where n-2 is the maximum). Writes up to `capacity` cycles of nRanks ranks each, row-major,
 * into cycles (may be NULL) and returns the number of rings (0 for nRanks == 0). */
extern int32_t HcclAmdRingTable(uint32_t nRanks, uint32_t* cycles, uint32_t capacity);

/* The concurrent instances HCCL_AMD_ALGO_RHD runs on a power-of-two nRanks (n-1 of them, one per XOR matching of
 * the ranks): for each instance the real rank of every virtual rank, row-major (nRanks entries per instance), up to
 * `capacity` instances. Returns the number of instances (0 when nRanks is not a power of two or exceeds 16). */
extern int32_t HcclAmdRhdTable(uint32_t nRanks, uint32_t* realOfVirtual, uint32_t capacity);

/* The executor's plan for one rank's IR, without running it (host only; what Execute issues on the GPU): units in
 * issue order, each a transport group (stream 0, the link stream) or a batch of folds / a copy (stream 1, the reduce
 * stream), with the unit of the other stream it waits for (hipStreamWaitEvent), derived from RAW / WAR / WAW conflicts
 * of the units' byte ranges at the buffer base addresses bufBase[HcclAmdBuf] (equal bases model in-place calls). */
typedef struct {
    int32_t stream;   /* 0 = link, 1 = reduce */
    int32_t isComm;   /* 1: SEND/RECV group */
    uint64_t firstOp; /* IR records [firstOp, firstOp + numOps) */
    uint64_t numOps;
    int64_t waitUnit; /* unit index on the other stream, or -1 */
} HcclAmdUnitPlan;
extern HcclResult HcclAmdExecutorPlan(const HcclAmdIrOp* ops, uint64_t numOps, uint32_t elemSize,
                                      const uint64_t* bufBase, HcclAmdUnitPlan* units, uint64_t capacity,
                                      uint64_t* numUnits);

/* ---------------------------------------------------------------- communicator extensions */

/* nRanks communicators on the current HIP device, joined by device-to-device copies. comms[r] is rank r.
 * Each rank must be driven from its own host thread (collectives rendezvous like real ranks). */
extern HcclResult HcclAmdCommInitLoopback(uint32_t nRanks, HcclComm* comms);

/* Force the schedule family for subsequent collectives on comm (HCCL_AMD_ALGO_AUTO restores the selector). */
extern HcclResult HcclAmdCommSetAlgo(HcclComm comm, int32_t algo);

/* Workgroups per launch of the one-sided IPC kernel (1..512; 0 restores the default, which grows with the call's
 * bytes from 16 to 256). Must be equal on every rank of the communicator (block b synchronises with block b of each
 * peer). A loopback world uses at most 128 per rank unless set here. Either way the launch is capped at the blocks
 * the device holds at once, divided by the ranks that share it. */
extern HcclResult HcclAmdCommSetIpcBlocks(HcclComm comm, uint32_t blocks);

/* Pipelining granule (bytes per piece) for subsequent collectives on comm; 0 restores the default. */
extern HcclResult HcclAmdCommSetPieceBytes(HcclComm comm, uint64_t pieceBytes);

/* Algorithm the last collective on comm executed (HcclAmdAlgo), or -1. A collective that the small-call rule
 * (HCCL_AMD_CFG_SMALL_IPC_BYTES) put on the one-sided kernel reports HCCL_AMD_ALGO_IPC (the auto family's order) or,
 * for an AllReduce asked for RHD, HCCL_AMD_ALGO_IPC_RHD (RHD's order). */
extern int32_t HcclAmdCommLastAlgo(HcclComm comm);

/* Configuration. A communicator reads the environment once, when it is created (the reference parses its environment
 * once, InitEnvConfig, src/common/alg_env_config.cc:176); no collective reads it. HcclAmdCommSetConfig changes one
 * entry of comm afterwards: keys marked (=) must be equal on every rank of the communicator, as the environment
 * variables they stand for must be. HCCL_E_PARA for an unknown key or a value out of range. */
typedef enum {
    HCCL_AMD_CFG_DETERMINISTIC_STRICT = 0, /* (=) HCCL_DETERMINISTIC=strict: 1, else 0 */
    HCCL_AMD_CFG_EXPANSION_MODE_AIV = 1,   /* (=) HCCL_OP_EXPANSION_MODE=AIV: 1, else 0 */
    HCCL_AMD_CFG_AIV_CORE_LIMIT = 2,       /* (=) HCCL_AMD_AIV_CORE_LIMIT, 1..4096 (default 48) */
    HCCL_AMD_CFG_SINGLE_STREAM_BYTES = 3,  /* HCCL_AMD_SINGLE_STREAM_BYTES: programs up to this per-rank payload run
                                              on the caller's stream alone (default 1 MiB) */
    HCCL_AMD_CFG_SMALL_IPC_BYTES = 4,      /* (=) HCCL_AMD_SMALL_IPC_BYTES: an AllReduce of auto or RHD family, or a
                                              ReduceScatter or Reduce of auto family, with at most this many input
                                              bytes per rank runs on the one-sided kernel, same bits (default 1 MiB;
                                              0 = never) */
    HCCL_AMD_CFG_PLAN_CACHE = 5,           /* HCCL_AMD_PLAN_CACHE: compiled-collective cache on (1, default) / off (0) */
    HCCL_AMD_CFG_GRAPH_CACHE = 6,          /* HCCL_AMD_GRAPH_CACHE: executor graphs kept, 0..1024 (default 16) */
    HCCL_AMD_CFG_IPC_LIGHT_FENCE = 7,      /* (=) HCCL_AMD_IPC_LIGHT_FENCE: -1 per mode (default), 0 system, 1 light */
    HCCL_AMD_CFG_IPC_NT = 8,               /* (=) HCCL_AMD_IPC_NT: non-temporal loads and stores (default 1) */
    HCCL_AMD_CFG_IPC_THREADS = 9,          /* (=) HCCL_AMD_IPC_THREADS: 256 (default) or 512 */
    HCCL_AMD_CFG_IPC_TILE_KIB = 10,        /* (=) HCCL_AMD_IPC_TILE_KIB: 0 = one window per block (default) */
    HCCL_AMD_CFG_IPC_TIMEOUT_MS = 11,      /* HCCL_AMD_IPC_TIMEOUT_MS, else HCCL_EXEC_TIMEOUT's AIV rule (HcclAmdIpcTimeoutMs) */
    HCCL_AMD_CFG_IPC_STAGING_MIB = 12,     /* (=) HCCL_AMD_IPC_STAGING_MIB: the one-sided kernel's large staging tier,
                                              MiB per area (four areas per rank), 16..1000, or 0 (default) for
                                              HCCL_BUFFSIZE / 2, so that the tier holds 2 x HCCL_BUFFSIZE; read when
                                              the tier is set up (HcclAmdCommDeviceBytes) */
    /* 13 is retired (HCCL_AMD_IPC_STAGING_CACHED, an r03 diagnostic): HCCL_E_PARA */
    HCCL_AMD_CFG_IPC_TRACE = 14,           /* HCCL_AMD_IPC_TRACE: phase stamps (diagnostics); at the IPC set-up */
    HCCL_AMD_CFG_IPC_L2_SCRUB = 15,        /* HCCL_AMD_IPC_L2_SCRUB: L2 maintenance at the IPC set-up (default 1) */
    HCCL_AMD_CFG_FOLD_TIMING = 16,         /* HCCL_AMD_FOLD_TIMING: time the executor's folds (diagnostics; calls run
                                              eagerly, HcclAmdCommFoldTiming reads the last one) */
    HCCL_AMD_CFG_IPC_LL_BYTES = 17,        /* (=) HCCL_AMD_IPC_LL_BYTES, 0..65536 (default 65536): one-shot
                                              AllReduces of at most this many bytes per rank run in the LL form (data
                                              and flag in one 8-byte store, no barrier; same bits); 0 = off */
    HCCL_AMD_CFG_COUNT = 18
} HcclAmdConfigKey;
extern HcclResult HcclAmdCommSetConfig(HcclComm comm, int32_t key, int64_t value);
extern HcclResult HcclAmdCommGetConfig(HcclComm comm, int32_t key, int64_t* value);
/* Re-reads comm's whole configuration from the environment, as at its creation (for test harnesses that keep one
 * communicator across cases with different environments; never called by a collective). */
extern HcclResult HcclAmdCommReloadConfig(HcclComm comm);

/* The folds of comm's last executor program while HCCL_AMD_CFG_FOLD_TIMING is on (diagnostics: the fold's operating
 * point inside a program, on staging a transport group has just written). Waits for that program's end. *folds = fold
 * launches (a batch counts once), *foldBytes = their algorithmic bytes (sum over records of (operands + 1) x count x
 * element size), *foldUs = the sum of their durations (HIP events around each launch on its stream), *spanUs = the
 * program's span on the caller's stream. HCCL_E_NOT_SUPPORT when no timed program ran (timing off, the one-sided
 * kernel, a capture). */
extern HcclResult HcclAmdCommFoldTiming(HcclComm comm, uint64_t* folds, uint64_t* foldBytes, double* foldUs,
                                        double* spanUs);


/* Runs one rank's IR program on comm's executor: what every collective runs after it has built its schedule (SEND/RECV
 * groups on the transport, folds and copies on the reduce stream, the cross-stream waits derived from the records'
 * byte ranges; singleStream != 0 puts everything on `stream` in program order). Collective over the peers the program
 * names, whose programs must post matching groups. For custom schedules and for testing the transport and executor.
 * Records are checked for form (kind, operand count, peer < rank count, buffer ids; staging inside the communicator's
 * staging); the extents of sendBuf / recvBuf are the caller's contract. */
extern HcclResult HcclAmdCommExecute(HcclComm comm, const HcclAmdIrOp* ops, uint64_t numOps, void* sendBuf,
                                     void* recvBuf, HcclDataType dataType, HcclReduceOp op, int32_t singleStream,
                                     aclrtStream stream);

/* Compiled-collective cache of comm: a call whose schedule parameters (operation, family, ranks, count, type, root,
 * piece size, buffer size) match an earlier one reuses its schedule and, for the same overlap of sendBuf / recvBuf /
 * staging, its executor plan (up to 32 entries, least recently used evicted; HCCL_AMD_PLAN_CACHE=0 disables it).
 * *hits and *misses count the RCCL-path calls that reused or built one. */
extern HcclResult HcclAmdCommCompileStats(HcclComm comm, uint64_t* hits, uint64_t* misses);

/* Executor graphs of comm (RCCL path, two-stream programs): *launches = calls served by one hipGraphLaunch of a
 * captured program, *captures = programs captured. A compiled collective runs eagerly the first time; later calls with
 * the same buffers, stream, dtype and op replay its graph. HCCL_AMD_GRAPH_CACHE = graphs kept per communicator
 * (default 16, least recently used evicted; 0 = every call eager). */
extern HcclResult HcclAmdCommGraphStats(HcclComm comm, uint64_t* launches, uint64_t* captures);

/* Status of the IPC path of comm (synchronous read). Bit 0: a cross-rank wait exceeded the communicator's bound
 * (HCCL_AMD_CFG_IPC_TIMEOUT_MS: HCCL_AMD_IPC_TIMEOUT_MS, else HCCL_EXEC_TIMEOUT's AIV rule, default 1091 s) — the
 * results of that and every later IPC collective on comm are invalid (sticky: the communicator is failed, as after an
 * asynchronous error). Bits 8-15: bit length of the longest wait of the last IPC collective, in polls (diagnostic;
 * 0 = no block ever waited). */
extern HcclResult HcclAmdCommIpcStatus(HcclComm comm, uint32_t* status);

/* One-sided launches of comm that ran in the LL form so far (HCCL_AMD_CFG_IPC_LL_BYTES; synchronous read of the
 * device's LL sequence word; in a loopback world the launches count on rank 0's communicator, which issues them). */
extern HcclResult HcclAmdCommIpcLlLaunches(HcclComm comm, uint32_t* launches);

/* Phase timeline of the one-sided kernel (diagnostics). With HCCL_AMD_IPC_TRACE=1 set when comm makes its first IPC
 * call, every launch stamps, per rank and workgroup, 8 s_memrealtime values (100 MHz) of its last staging round:
 * entry, round start, phase 0 issued, barrier 1 passed, phase 1 issued, barrier 2 passed, phase 2 issued, exit.
 * Synchronises the device and copies the last launch's stamps into stamps[rank][block][8] (cap >= 16 x 512 x 8
 * entries; in a loopback world call it on rank 0, which issues the world's launch); *blocks = workgroups per rank of
 * that launch. HCCL_E_NOT_SUPPORT when tracing is off. */
extern HcclResult HcclAmdCommIpcTrace(HcclComm comm, uint64_t* stamps, uint64_t cap, uint32_t* blocks);

/* The barrier wait bound of the one-sided kernel in ms, as the next IPC call would take it from the environment:
 * HCCL_AMD_IPC_TIMEOUT_MS if set (1 .. 3600000), else HCCL_EXEC_TIMEOUT by the reference's AIV-mode rule (seconds,
 * at most two decimals; 0, above 1091 or unset = 1091 s). A wait past it fails the communicator (HcclGetCommAsyncError). */
extern uint64_t HcclAmdIpcTimeoutMs(void);

/* Parse and validate a rank table (as HcclCommInitClusterInfo does): *nRanks = number of ranks, *deviceId = the
 * device_id of `rank`. HCCL_E_PARA for a malformed table or a rank outside it. */
extern HcclResult HcclAmdRankTableInfo(const char* clusterInfo, uint32_t rank, uint32_t* nRanks, int32_t* deviceId);

/* The last HcclCommInitClusterInfo of this process: *stage = 0 (none, or it failed before the unique-id exchange
 * completed), 1 (the transport's unique id was exchanged over TCP; *idDigest = FNV-1a 64 of the 128-byte id, the same
 * on every rank of a good exchange), 2 (the RCCL communicator was then created). Diagnostics for bootstrap tests. */
extern HcclResult HcclAmdLastBootstrap(uint64_t* idDigest, int32_t* stage);

/* The rank-table TCP exchange alone (host only, no device): rank 0 serves the 128 bytes at id128 to every other
 * rank of the table, which receive them into id128. Same addresses and bounds as HcclCommInitClusterInfo. */
extern HcclResult HcclAmdBootstrapExchangeId(const char* clusterInfo, uint32_t rank, void* id128);

/* Host time by category, accumulated while HCCL_AMD_HOST_PROFILE=1 (read at library load): ns[i] and calls[i] for
 * i < n of the categories below; reset != 0 zeroes them afterwards. Diagnostics of the enqueue cost. */
enum {
    HCCL_AMD_HP_EXECUTE = 0, /* a whole Execute call */
    HCCL_AMD_HP_GROUP = 1,   /* transport groups (ncclGroupStart .. ncclGroupEnd) */
    HCCL_AMD_HP_FOLD = 2,    /* fold launches */
    HCCL_AMD_HP_COPY = 3,    /* copy launches */
    HCCL_AMD_HP_RECORD = 4,  /* unit event records */
    HCCL_AMD_HP_WAIT = 5,    /* cross-stream waits */
    HCCL_AMD_HP_PLAN = 6,    /* planning outside the compiled-collective cache */
    HCCL_AMD_HP_ENTRY = 7,   /* a whole collective call past its argument checks (HcclAllReduce, HcclReduceScatter,
                                HcclReduceScatterV, HcclReduce, HcclAllGather): lock, selection, every enqueue */
    HCCL_AMD_HP_IPC = 8,     /* the one-sided kernel's host side: launch arguments and the launch (RunIpcPlan) */
    HCCL_AMD_HP_COUNT = 9
};
extern HcclResult HcclAmdHostProfile(uint64_t* ns, uint64_t* calls, uint32_t n, int32_t reset);

/* Communicators whose HcclCommDestroy is waiting for the graphs captured on them to be destroyed. */
extern uint32_t HcclAmdCommPendingDestroys(void);

/* RCCL's p2p channel settings of this process as requested through the environment: *perPeer =
 * NCCL_NCHANNELS_PER_PEER, *minP2pChannels = NCCL_MIN_P2P_NCHANNELS (0 when unset). Opt-in: only when
 * HCCL_AMD_P2P_CHANNELS_PER_PEER=k > 0 does the library, when it is loaded, set NCCL_NCHANNELS_PER_PEER = k rounded
 * up to a power of two and
 * NCCL_MIN_P2P_NCHANNELS = (the per-peer value in effect) x 7 rounded up to a power of two, at most 64, each unless the
 * caller set it (RCCL's p2p kernel streams about 43 GB/s per channel, an xGMI link 76.8 GB/s per direction). RCCL reads
 * them once per process, at its first communicator, so these are requests: RCCL's INIT log says what it set up.
 * Child processes inherit them. */
extern HcclResult HcclAmdRcclP2pChannels(uint32_t* perPeer, uint32_t* minP2pChannels);

/* The executor staging of comm (diagnostics): *ptr = its device address (NULL until allocated), *bytes = its size. */
extern HcclResult HcclAmdCommScratch(HcclComm comm, void** ptr, uint64_t* bytes);

/* The device memory the library holds for comm now, in bytes: the executor staging (2 x HCCL_BUFFSIZE, allocated by
 * the first collective that runs a schedule) plus the one-sided kernel's allocations (flags and LL area, status words
 * and unpack area at its first call; the small staging tier, n x HCCL_AMD_SMALL_IPC_BYTES per area, and the large
 * one, 2 x HCCL_BUFFSIZE, each at the first call that needs it). RCCL's own buffers are not included. */
extern HcclResult HcclAmdCommDeviceBytes(HcclComm comm, uint64_t* bytes);

/* The one-sided path's uncached allocations outlive the communicator that made them: a destroyed communicator's
 * blocks stay with the process and serve the next communicator's set-up of the same size on the same device. *bytes =
 * the idle blocks' total size. They are never freed while the process runs: freeing memory allocated with
 * hipDeviceMallocUncached corrupts later GPU work on this stack (lost operands and memory aperture violations after
 * such frees), so release != 0 returns HCCL_E_NOT_SUPPORT after reporting. A block serves
 * only a request of its own size: communicators of other sizes (rank count, HCCL_BUFFSIZE) allocate their own. */
extern HcclResult HcclAmdIpcIdleStaging(int32_t release, uint64_t* bytes);

/* Enqueues on `stream` a system-scope write-back and invalidate of every XCD's L2 of the current device (one
 * workgroup per CU runs buffer_wbl2 sc0 sc1 / buffer_inv sc0 sc1) and waits for it. Diagnostics: a kernel launched
 * after it reads every line from memory. */
extern HcclResult HcclAmdL2Maintain(aclrtStream stream);

/* Enqueues on `stream` a read of `words` 4-byte words at device address p by 256 workgroups (dealt over the XCDs),
 * each reading the whole range with plain loads (nonTemporal = 0) or non-temporal loads (1) and comparing it with the
 * device array `expect`. out (device, 768 uint32) receives {mismatching words, zero words, XCC id} per workgroup.
 * Diagnostics: which XCDs see stale or unwritten lines of a buffer. */
extern HcclResult HcclAmdDiagReadByXcc(const void* p, const void* expect, uint64_t words, int32_t nonTemporal,
                                       void* out, aclrtStream stream);

/* Blocking host all-gather supplied by the caller's bootstrap (a TCP store, MPI, torch.distributed gloo ...):
 * gathers `bytes` bytes from every rank into all[nRanks * bytes] in rank order; returns 0 on success. */
typedef int32_t (*HcclAmdHostAllGatherFn)(void* ctx, const void* mine, uint64_t bytes, void* all);

/* Rank `rank` of an IPC-only communicator on the current HIP device, bootstrapped through `fn` instead of RCCL.
 * Its data path is the one-sided kernel over peer-mapped memory opened with hipIpcOpenMemHandle:
 * HCCL_AMD_ALGO_IPC_TWOSHOT (the default on such a communicator), HCCL_AMD_ALGO_IPC_RHD when RHD or IPC_RHD is set
 * (AllReduce, power-of-two ranks), otherwise HCCL_AMD_ALGO_IPC whatever family is set. Every operator has an IPC form,
 * HcclReduceScatterV included (per-rank blocks, order O1).
 * Ranks may share a device (separate processes), which is how the rank-mode IPC path is tested on one GPU.
 * `fn` and `ctx` must stay valid for the communicator's lifetime. */
extern HcclResult HcclAmdCommInitHostExchange(uint32_t nRanks, uint32_t rank, HcclAmdHostAllGatherFn fn, void* ctx,
                                              HcclComm* comm);

/* A stand-in for one rank of an nRanks-rank communicator on one GPU (benchmark and test harnesses; never a data
 * path): rank `rank`'s schedules run through a one-rank RCCL communicator with every peer mapped onto itself. Each
 * transport group's sends are paired with its receives of the same size (RCCL pairs messages to itself in posting
 * order), so every program keeps the schedule's shape (groups, pieces, staging, folds, waits, graph capture) and runs
 * through RCCL's kernels, while the data no longer means the collective. Sends and receives of a group whose sizes
 * differ (a ragged last chunk) are paired in order at the smaller size; a surplus on either side is dropped. The
 * one-sided kernel is unavailable (HCCL_E_NOT_SUPPORT; the small-call rule falls back to the schedule). */
extern HcclResult HcclAmdCommInitSelfLoop(uint32_t nRanks, uint32_t rank, HcclComm* comm);

#ifdef __cplusplus
}
#endif
#endif /* HCCL_AMD_EXT_H_ */
