// ops.cc — the operator surface of include/hccl.h plus the communicator extensions of include/hccl_amd.h.
//
// Each entry point keeps the reference's validation order and return codes:
//   HcclAllReduce      all_reduce_op.cc:23-52, AllReduceInitAndCheck :107-133, CheckAllReduceInputPara :135-157
//   HcclReduceScatter  reduce_scatter_op.cc:23-72, CheckReduceScatterInputPara
//   HcclReduce         reduce_op.cc:23-54, ReduceInitAndCheck, CheckReduceInputPara :106-127
//   CheckCount / CheckDataType / CheckReduceOp / SingleRankProc   op_common.cc:2902-3098
// then build this rank's schedule (schedule.cc) and run it (executor.cc).
#include <strings.h>

#include <algorithm>

#include <cstring>

#include "comm.h"

namespace hccl_amd {

namespace {

constexpr uint64_t kSysMaxCount = 0x7FFFFFFFFull;  // SYS_MAX_COUNT, hccl_common.h:42

HcclResult CheckCount(uint64_t count) { return count > kSysMaxCount ? HCCL_E_PARA : HCCL_SUCCESS; }

// CheckDataType(dataType, needReduce = true), op_common.cc:2913-2950
HcclResult CheckReduceDataType(HcclDataType dt) { return IsReduceDataType(dt) ? HCCL_SUCCESS : HCCL_E_NOT_SUPPORT; }

// CheckReduceOp, op_common.cc:2977-2998: PROD only on INT8/INT32/INT64/UINT64/FP16/FP32/FP64. An op outside
// {SUM, PROD, MAX, MIN} has no reference check at the entry (it fails deep in the template); it is HCCL_E_PARA here.
HcclResult CheckReduceOp(HcclDataType dt, HcclReduceOp op)
{
    if (op == HCCL_REDUCE_PROD) {
        switch (dt) {
            case HCCL_DATA_TYPE_INT8:
            case HCCL_DATA_TYPE_INT32:
            case HCCL_DATA_TYPE_INT64:
            case HCCL_DATA_TYPE_UINT64:
            case HCCL_DATA_TYPE_FP16:
            case HCCL_DATA_TYPE_FP32:
            case HCCL_DATA_TYPE_FP64: return HCCL_SUCCESS;
            default: return HCCL_E_NOT_SUPPORT;
        }
    }
    if (op != HCCL_REDUCE_SUM && op != HCCL_REDUCE_MAX && op != HCCL_REDUCE_MIN) return HCCL_E_PARA;
    return HCCL_SUCCESS;
}

// HCCL_DETERMINISTIC=strict (alg_env_config.cc:1036-1076; CommConfig::strict) with fp16/fp32/bf16/fp64, SUM/PROD and
// more than two ranks selects the order-preserved tree (IsNeedStrictModeForOrderPreserved, order_preserved_common.h:
// 63-73). At n <= 8 the reference runs it as InsTempReduceScatterOrderPreservedLevel1 (reduce_scatter_auto_selector.cc:
// 406-413), whose tree is the same O4 (schedule.cc ReduceScatterTree).
bool NeedStrictOrder(const Comm& c, int32_t opType, HcclDataType dt, HcclReduceOp op)
{
    const uint32_t nRanks = c.nRanks;
    if (!c.cfg.strict) return false;
    if (opType != HCCL_AMD_OP_ALLREDUCE && opType != HCCL_AMD_OP_REDUCE_SCATTER) return false;
    const bool fp = dt == HCCL_DATA_TYPE_FP16 || dt == HCCL_DATA_TYPE_FP32 || dt == HCCL_DATA_TYPE_BFP16 ||
                    dt == HCCL_DATA_TYPE_FP64;
    return fp && (op == HCCL_REDUCE_SUM || op == HCCL_REDUCE_PROD) && nRanks > 2;
}

// isDataTypeOrReduceTypeSpecial of the selectors (all_reduce_auto_selector.cc:525-528,
// reduce_scatter_auto_selector.cc:477): 64-bit data or PROD.
bool IsSpecialForSelector(HcclDataType dt, HcclReduceOp op)
{
    return dt == HCCL_DATA_TYPE_INT64 || dt == HCCL_DATA_TYPE_UINT64 || dt == HCCL_DATA_TYPE_FP64 ||
           op == HCCL_REDUCE_PROD;
}

// Pipelining granule of a call: the communicator's (HcclAmdCommSetPieceBytes) if set. Otherwise the schedule's default
// for the two-stream executor, and one piece per slice (as far as the staging holds) for the single-stream one, where
// pieces cannot overlap anything and each costs a transport group (about 10 us of host time per group, RCCL self-loop
// programs: profiles/r02_rccl_selfloop_latency*.jsonl). Pieces never change a fold order: every order is fixed per
// executor loop and slice, and a piece only splits a slice's elements.
uint64_t PieceBytesFor(const Comm& c, bool singleStream, uint64_t payload)
{
    if (c.pieceBytes != 0) return c.pieceBytes;
    return singleStream ? std::max<uint64_t>(payload, 128) : 0;  // no slice is larger than the payload
}

// A pointer a kernel of this device may dereference: device memory, or host memory registered and mapped for it.
bool DeviceAccessible(const void* p)
{
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // an unregistered host pointer reports an error: clear it
        return false;
    }
    // registered host memory counts only where the device addresses it at the host pointer itself (the copy kernel is
    // handed that pointer); a registration mapped elsewhere goes to hipMemcpyAsync
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ||
           (a.type == hipMemoryTypeHost && a.devicePointer == p);
}

// The one-rank collective's copy (SingleRankProc). The library's copy kernel when both buffers are device-accessible;
// hipMemcpyAsync otherwise, which resolves pageable host memory where a kernel would fault the GPU.
HcclResult CopyUserBuffer(void* dst, const void* src, uint64_t bytes, hipStream_t stream)
{
    if (bytes == 0 || dst == src) return HCCL_SUCCESS;
    if (DeviceAccessible(dst) && DeviceAccessible(src)) return LaunchCopyBytes(dst, src, bytes, stream);
    HIP_CHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, stream));
    return HCCL_SUCCESS;
}

HcclResult RunCollective(Comm& c, int32_t opType, void* sendBuf, void* recvBuf, uint64_t count, HcclDataType dt,
                         HcclReduceOp op, uint32_t root, hipStream_t stream)
{
    const HostProfileScope hp(HCCL_AMD_HP_ENTRY);
    std::lock_guard<std::mutex> lk(c.mu);
    HCCL_CHK(c.Gate());  // a failed communicator takes no more work (op_common.cc:89-97)
    HIP_CHK(hipSetDevice(c.device));
    const EntryScope entry(c, stream);
    HCCL_CHK(entry.status());
    const uint32_t es = DataTypeSize(dt);
    if (c.nRanks == 1) {
        // SingleRankProc (op_common.cc:3042-3098): copy in -> out unless they are the same buffer.
        c.lastAlgo = HCCL_AMD_ALGO_AUTO;
        return CopyUserBuffer(recvBuf, sendBuf, count * es, stream);
    }
    ScheduleParams p;
    p.opType = opType;
    p.algo = c.algoOverride;
    // The AIV engine (HCCL_OP_EXPANSION_MODE=AIV, or forced per communicator): SelectAivAlgo's choice and its
    // kernels' orders on the one-sided kernel. What it does not match, or cannot run (no peer mappings, a capture
    // before the set-up), takes the AICPU engine's selection below, as the reference falls back
    // (AutoSelectorBase::ProcessAivConfig, auto_selector_base.cc:353-371).
    // AIV_ONLY (the reference's OpExecuteConfig::AIV_ONLY, a communicator's configured expansion mode) takes no
    // fallback: an operation the AIV engine does not match returns HCCL_E_NOT_SUPPORT (op_common.cc:115-122).
    const bool aivOnly = p.algo == HCCL_AMD_ALGO_AIV_ONLY;
    if (aivOnly || p.algo == HCCL_AMD_ALGO_AIV || (p.algo == HCCL_AMD_ALGO_AUTO && c.cfg.expansionAiv)) {
        IpcPlan plan{};
        const int32_t v = SelectAivPlan(opType, c.nRanks, count, dt, op, NeedStrictOrder(c, opType, dt, op), aivOnly,
                                        c.cclBytes, c.cfg.aivCoreLimit, &plan, nullptr);
        if (v != HCCL_AMD_AIV_NOT_MATCHED) {
            const HcclResult r = RunIpcPlan(c, opType, plan, sendBuf, recvBuf, count, dt, op, root, stream);
            if (r != HCCL_E_NOT_SUPPORT) {
                c.lastAlgo = aivOnly ? HCCL_AMD_ALGO_AIV_ONLY : HCCL_AMD_ALGO_AIV;
                return r;
            }
        }
        if (aivOnly) return HCCL_E_NOT_SUPPORT;
        p.algo = HCCL_AMD_ALGO_AUTO;
    }
    // RHD's bits from one launch of the one-sided kernel (AllReduce, power-of-two n). An IPC-only communicator asked for
    // RHD takes it too, so it keeps RHD's order. Anything else runs the RHD schedule (or its own fallbacks).
    if (p.algo == HCCL_AMD_ALGO_RHD && !c.transport->HasSendRecv()) p.algo = HCCL_AMD_ALGO_IPC_RHD;
    if (p.algo == HCCL_AMD_ALGO_IPC_RHD) {
        IpcPlan plan{};
        if (opType == HCCL_AMD_OP_ALLREDUCE && IpcPlanRhd(c.nRanks, &plan) == HCCL_SUCCESS) {
            const HcclResult r = RunIpcPlan(c, opType, plan, sendBuf, recvBuf, count, dt, op, root, stream);
            if (r != HCCL_E_NOT_SUPPORT) {
                c.lastAlgo = HCCL_AMD_ALGO_IPC_RHD;
                return r;
            }
        }
        p.algo = HCCL_AMD_ALGO_RHD;
    }
    // an IPC-only communicator (bootstrap transport without send/recv) runs every reducing op on the IPC kernel in
    // the auto family, whatever schedule family was asked for
    if (!c.transport->HasSendRecv() && p.algo != HCCL_AMD_ALGO_IPC_TWOSHOT) p.algo = HCCL_AMD_ALGO_IPC;
    if (p.algo == HCCL_AMD_ALGO_AUTO && NeedStrictOrder(c, opType, dt, op)) {
        p.algo = HCCL_AMD_ALGO_ORDER_PRESERVED;
    }
    // Small collectives take the one-sided kernel (HCCL_AMD_SMALL_IPC_BYTES, default 1 MiB per rank): one launch with
    // one or two cross-rank barriers instead of the transport groups of a schedule, each of which costs a group launch
    // (1 KiB one-shot over RCCL: 29-32 us, an 8-rank RHD: 81.5 us; profiles/r03_host_cost_rccl_selfloop.jsonl,
    // r02_rccl_selfloop_latency.jsonl). The reference runs small data on its vector cores the same way
    // (all_reduce_auto_selector.cc:591-683; a task costs it 1-2 us, cost_model.cc:240-245). The bits do not change: the
    // auto family runs in the auto family's order (HCCL_AMD_ALGO_IPC), RHD in RHD's (HCCL_AMD_ALGO_IPC_RHD). Every rank
    // decides alike (count, dtype and the (=) config are equal on every rank); a call the kernel cannot take (no peer
    // mappings, a capture before the set-up) runs the schedule.
    // ReduceScatter and Reduce take the rule too (r05), in the auto family's order only (the one-sided kernel has no
    // RHD form of them); the threshold applies to the rank's input (ReduceScatter: n blocks).
    const bool reducing = opType == HCCL_AMD_OP_ALLREDUCE || opType == HCCL_AMD_OP_REDUCE_SCATTER ||
                          opType == HCCL_AMD_OP_REDUCE;
    const uint64_t inBytes = count * es * (opType == HCCL_AMD_OP_REDUCE_SCATTER ? c.nRanks : 1);
    if (reducing && c.transport->HasSendRecv() && !c.ipc.unavailable && inBytes <= c.cfg.smallIpcBytes &&
        (p.algo == HCCL_AMD_ALGO_AUTO || (opType == HCCL_AMD_OP_ALLREDUCE && p.algo == HCCL_AMD_ALGO_RHD))) {
        IpcPlan plan{};
        HcclResult r = HCCL_E_NOT_SUPPORT;
        int32_t ran = HCCL_AMD_ALGO_IPC;
        if (p.algo == HCCL_AMD_ALGO_RHD) {
            ran = HCCL_AMD_ALGO_IPC_RHD;
            if (IpcPlanRhd(c.nRanks, &plan) == HCCL_SUCCESS) {
                r = RunIpcPlan(c, opType, plan, sendBuf, recvBuf, count, dt, op, root, stream);
            }
        } else {
            const int32_t family = SelectAlgo(opType, c.nRanks, count * es, IsSpecialForSelector(dt, op));
            r = RunIpcCollective(c, opType, family, sendBuf, recvBuf, count, dt, op, root, stream);
        }
        if (r != HCCL_E_NOT_SUPPORT) {
            c.lastAlgo = ran;
            return r;
        }
    }
    if (p.algo == HCCL_AMD_ALGO_IPC_TWOSHOT || p.algo == HCCL_AMD_ALGO_IPC) {
        // the order family of the one-sided kernel: IPC_TWOSHOT fixes AllReduce two-shot (O2), mesh ReduceScatter
        // and two-shot Reduce; IPC takes whatever the auto selector takes, so its bits are the auto path's
        // (AllGather moves data only: the family does not matter)
        const uint64_t bytes = count * es;
        const int32_t family =
            p.algo == HCCL_AMD_ALGO_IPC
                ? SelectAlgo(opType, c.nRanks, bytes, IsSpecialForSelector(dt, op))
                : (opType == HCCL_AMD_OP_REDUCE_SCATTER ? HCCL_AMD_ALGO_MESH_ONESHOT : HCCL_AMD_ALGO_MESH_TWOSHOT);
        HcclResult r = RunIpcCollective(c, opType, family, sendBuf, recvBuf, count, dt, op, root, stream);
        if (r != HCCL_E_NOT_SUPPORT) {
            c.lastAlgo = p.algo;
            return r;
        }
        // no peer mappings, or a capturing stream: the RCCL schedule with the same order, if there is RCCL
        if (!c.transport->HasSendRecv()) return HCCL_E_NOT_SUPPORT;
        p.algo = opType == HCCL_AMD_OP_ALLGATHER ? HCCL_AMD_ALGO_MESH_ONESHOT : family;
    }
    HCCL_CHK(c.EnsureScratch());
    p.nRanks = c.nRanks;
    p.rank = c.rank;
    p.count = count;
    p.elemSize = es;
    p.root = root;
    p.scratchCapBytes = c.scratchBytes;
    p.cclBytes = c.cclBytes;
    p.special = IsSpecialForSelector(dt, op);
    void* bufs[3] = {sendBuf, recvBuf, c.scratch};
    const uint64_t payload = count * es * (opType == HCCL_AMD_OP_REDUCE_SCATTER ? c.nRanks : 1);
    const bool single = payload <= c.cfg.singleStreamBytes;
    p.pieceBytes = PieceBytesFor(c, single, payload);
    const CompiledSchedule* cs = nullptr;
    HCCL_CHK(CompileCollective(c, p, bufs, !single, &cs));
    const Schedule& s = cs->sched;
    if (s.scratchElems * es > c.scratchBytes) {
        HCCL_AMD_ERR("schedule needs %llu B of staging, communicator has %llu B",
                     (unsigned long long)(s.scratchElems * es), (unsigned long long)c.scratchBytes);
        return HCCL_E_INTERNAL;
    }
    c.lastAlgo = s.algo;
    HCCL_AMD_LOG("rank %u op %d algo %d count %llu ops %zu", c.rank, opType, s.algo, (unsigned long long)count,
                 s.ops.size());
    // single-stream programs replay from the executor graph cache too (RCCL path, the key's second call on)
    return RunCompiled(c, *cs, bufs, dt, op, stream, single);
}

// ReduceScatterV (reduce_scatter_v_op.cc:24-83, ReduceScatterVOutPlaceCommon :285-330): the mesh template's order
// over per-rank blocks; the output holds counts[rank] elements.
HcclResult RunReduceScatterV(Comm& c, void* sendBuf, const uint64_t* counts, const uint64_t* displs, void* recvBuf,
                             HcclDataType dt, HcclReduceOp op, hipStream_t stream)
{
    const HostProfileScope hp(HCCL_AMD_HP_ENTRY);
    std::lock_guard<std::mutex> lk(c.mu);
    HCCL_CHK(c.Gate());
    HIP_CHK(hipSetDevice(c.device));
    const EntryScope entry(c, stream);
    HCCL_CHK(entry.status());
    // ReduceScatterVAutoSelector::SelectAicpuAlgo (reduce_scatter_v_auto_selector.cc:180-197): UINT64 and FP64 have
    // no algorithm
    if (dt == HCCL_DATA_TYPE_UINT64 || dt == HCCL_DATA_TYPE_FP64) return HCCL_E_NOT_SUPPORT;
    // The one-sided kernel runs it over per-rank blocks (kIpcGeomV) in the same order O1 (own block first, then the
    // other ranks ascending): on an IPC-only communicator, which has no send/recv path, and when the communicator's
    // family is IPC / IPC_TWOSHOT. Without peer mappings an IPC-only communicator answers NOT_SUPPORT.
    const bool ipcOnly = !c.transport->HasSendRecv();
    if (c.nRanks > 1 &&
        (ipcOnly || c.algoOverride == HCCL_AMD_ALGO_IPC || c.algoOverride == HCCL_AMD_ALGO_IPC_TWOSHOT)) {
        IpcPlan plan{};
        plan.kind = kIpcReduceScatter;
        plan.order = kIpcO1;
        plan.geom = kIpcGeomV;
        const HcclResult r = RunIpcPlan(c, HCCL_AMD_OP_REDUCE_SCATTER, plan, sendBuf, recvBuf, counts[c.rank], dt, op,
                                        0, stream, counts, displs);
        if (r != HCCL_E_NOT_SUPPORT) {
            c.lastAlgo = ipcOnly ? HCCL_AMD_ALGO_IPC : c.algoOverride;
            return r;
        }
        if (ipcOnly) return HCCL_E_NOT_SUPPORT;
    }
    const uint32_t es = DataTypeSize(dt);
    HCCL_CHK(c.EnsureScratch());
    ScheduleParams p;
    p.opType = HCCL_AMD_OP_REDUCE_SCATTER_V;
    p.nRanks = c.nRanks;
    p.rank = c.rank;
    p.counts.assign(counts, counts + c.nRanks);
    p.displs.assign(displs, displs + c.nRanks);
    p.count = counts[c.rank];
    p.elemSize = es;
    p.scratchCapBytes = c.scratchBytes;
    p.cclBytes = c.cclBytes;
    void* bufs[3] = {sendBuf, recvBuf, c.scratch};
    uint64_t payload = 0;
    for (uint32_t q = 0; q < c.nRanks; ++q) payload += counts[q] * es;
    const bool single = c.nRanks == 1 || payload <= c.cfg.singleStreamBytes;
    p.pieceBytes = PieceBytesFor(c, single, payload);
    const CompiledSchedule* cs = nullptr;
    HCCL_CHK(CompileCollective(c, p, bufs, !single, &cs));
    const Schedule& s = cs->sched;
    if (s.scratchElems * es > c.scratchBytes) return HCCL_E_INTERNAL;
    c.lastAlgo = s.algo;
    return RunCompiled(c, *cs, bufs, dt, op, stream, single);
}

}  // namespace

}  // namespace hccl_amd

using namespace hccl_amd;

extern "C" {

// ------------------------------------------------------------------------------------------------ operators

HcclResult HcclAllReduce(void* sendBuf, void* recvBuf, uint64_t count, HcclDataType dataType, HcclReduceOp op,
                         HcclComm comm, aclrtStream stream)
{
    if (count == 0) return HCCL_SUCCESS;  // all_reduce_op.cc:37
    if (stream == nullptr || comm == nullptr || sendBuf == nullptr || recvBuf == nullptr) return HCCL_E_PTR;
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PARA;
    if (c->rank >= c->nRanks) return HCCL_E_PARA;  // HcomCheckUserRank
    HCCL_CHK(CheckCount(count));
    HCCL_CHK(CheckReduceDataType(dataType));
    HCCL_CHK(CheckReduceOp(dataType, op));
    return RunCollective(*c, HCCL_AMD_OP_ALLREDUCE, sendBuf, recvBuf, count, dataType, op, 0,
                         static_cast<hipStream_t>(stream));
}

HcclResult HcclReduceScatter(void* sendBuf, void* recvBuf, uint64_t recvCount, HcclDataType dataType,
                             HcclReduceOp op, HcclComm comm, aclrtStream stream)
{
    if (recvCount == 0) return HCCL_SUCCESS;  // reduce_scatter_op.cc:47
    if (stream == nullptr || comm == nullptr || sendBuf == nullptr || recvBuf == nullptr) return HCCL_E_PTR;
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PARA;
    if (c->rank >= c->nRanks) return HCCL_E_PARA;
    HCCL_CHK(CheckCount(recvCount));
    HCCL_CHK(CheckReduceDataType(dataType));
    HCCL_CHK(CheckReduceOp(dataType, op));
    return RunCollective(*c, HCCL_AMD_OP_REDUCE_SCATTER, sendBuf, recvBuf, recvCount, dataType, op, 0,
                         static_cast<hipStream_t>(stream));
}

HcclResult HcclReduceScatterV(void* sendBuf, const void* sendCounts, const void* sendDispls, void* recvBuf,
                              uint64_t recvCount, HcclDataType dataType, HcclReduceOp op, HcclComm comm,
                              aclrtStream stream)
{
    // CheckReduceScatterVInputParam (reduce_scatter_v_op.cc:155-183): stream, comm, sendCounts, sendDispls, then
    // recvBuf when recvCount > 0 (sendBuf is not checked there: a rank may send nothing)
    if (stream == nullptr || comm == nullptr || sendCounts == nullptr || sendDispls == nullptr) return HCCL_E_PTR;
    if (recvCount > 0 && recvBuf == nullptr) return HCCL_E_PTR;
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PARA;
    const uint64_t* counts = static_cast<const uint64_t*>(sendCounts);
    const uint64_t* displs = static_cast<const uint64_t*>(sendDispls);
    bool any = false;
    for (uint32_t q = 0; q < c->nRanks; ++q) any = any || counts[q] != 0;
    if (!any) return HCCL_SUCCESS;  // every sendCounts entry 0: success (:45-53)
    if (c->rank >= c->nRanks) return HCCL_E_PARA;  // HcomCheckUserRank
    HCCL_CHK(CheckCount(recvCount));
    HCCL_CHK(CheckReduceDataType(dataType));
    HCCL_CHK(CheckReduceOp(dataType, op));
    for (uint32_t q = 0; q < c->nRanks; ++q) {
        HCCL_CHK(CheckCount(counts[q]));
        // a block whose end does not fit in 64 bits would wrap the schedule's offsets onto other memory
        if (displs[q] > UINT64_MAX / 16 - counts[q]) return HCCL_E_PARA;
    }
    // The template writes sendCounts[rank] elements to recvBuf (PostCopy, ins_temp_reduce_scatter_v_mesh_1D.cc:
    // 107-146); a smaller recvCount would overrun it, so it is refused here (the reference has no such check).
    if (counts[c->rank] > recvCount) return HCCL_E_PARA;
    if (sendBuf == nullptr) return HCCL_E_PTR;  // some rank's block is non-empty: the input is read
    return RunReduceScatterV(*c, sendBuf, counts, displs, recvBuf, dataType, op, static_cast<hipStream_t>(stream));
}

HcclResult HcclReduce(void* sendBuf, void* recvBuf, uint64_t count, HcclDataType dataType, HcclReduceOp op,
                      uint32_t root, HcclComm comm, aclrtStream stream)
{
    if (count == 0) return HCCL_SUCCESS;  // reduce_op.cc:42
    // CheckReduceInputPara order: comm, sendBuf, recvBuf, stream (reduce_op.cc:106-127)
    if (comm == nullptr || sendBuf == nullptr || recvBuf == nullptr || stream == nullptr) return HCCL_E_PTR;
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PARA;
    HCCL_CHK(CheckCount(count));
    HCCL_CHK(CheckReduceDataType(dataType));
    HCCL_CHK(CheckReduceOp(dataType, op));
    if (root >= c->nRanks) return HCCL_E_PARA;     // HcomCheckUserRank(rankSize, root)
    if (c->rank >= c->nRanks) return HCCL_E_PARA;  // HcomCheckUserRank(rankSize, userRank)
    return RunCollective(*c, HCCL_AMD_OP_REDUCE, sendBuf, recvBuf, count, dataType, op, root,
                         static_cast<hipStream_t>(stream));
}

HcclResult HcclAllGather(void* sendBuf, void* recvBuf, uint64_t sendCount, HcclDataType dataType, HcclComm comm,
                         aclrtStream stream)
{
    // all_gather_op.cc:22-50, AllGatherInitAndCheck :97-122
    if (sendCount == 0) return HCCL_SUCCESS;
    if (stream == nullptr || comm == nullptr || sendBuf == nullptr || recvBuf == nullptr) return HCCL_E_PTR;
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PARA;
    HCCL_CHK(CheckCount(sendCount));
    // CheckDataType(dataType, needReduce = false): every valid type but INT128
    if (DataTypeSize(dataType) == 0 || dataType == HCCL_DATA_TYPE_INT128) return HCCL_E_NOT_SUPPORT;
    if (c->rank >= c->nRanks) return HCCL_E_PARA;
    return RunCollective(*c, HCCL_AMD_OP_ALLGATHER, sendBuf, recvBuf, sendCount, dataType, HCCL_REDUCE_SUM, 0,
                         static_cast<hipStream_t>(stream));
}

// ------------------------------------------------------------------------------------------------ communicators

static const char kRootMagic[8] = {'H', 'C', 'C', 'L', 'A', 'M', 'D', '1'};

HcclResult HcclGetRootInfo(HcclRootInfo* rootInfo)
{
    if (rootInfo == nullptr) return HCCL_E_PTR;
    std::memset(rootInfo->internal, 0, sizeof rootInfo->internal);
    std::memcpy(rootInfo->internal, kRootMagic, sizeof kRootMagic);
    return RcclGetUniqueId(rootInfo->internal + 8);
}

HcclResult HcclCommInitRootInfo(uint32_t nRanks, const HcclRootInfo* rootInfo, uint32_t rank, HcclComm* comm)
{
    if (rootInfo == nullptr || comm == nullptr) return HCCL_E_PTR;
    if (nRanks == 0 || rank >= nRanks || nRanks > HCCL_AMD_IR_MAX_SRC) return HCCL_E_PARA;
    if (std::memcmp(rootInfo->internal, kRootMagic, sizeof kRootMagic) != 0) return HCCL_E_PARA;
    int dev = 0;
    HIP_CHK(hipGetDevice(&dev));
    auto c = std::make_unique<Comm>();
    c->rank = rank;
    c->nRanks = nRanks;
    HCCL_CHK(c->Init(dev));
    HcclResult err = HCCL_SUCCESS;
    c->transport = MakeRcclTransport(const_cast<char*>(rootInfo->internal + 8), nRanks, rank, &err);
    if (c->transport == nullptr) return err == HCCL_SUCCESS ? HCCL_E_INTERNAL : err;
    HCCL_CHK(c->StartWatchdog());
    *comm = c.release();
    return HCCL_SUCCESS;
}

HcclResult HcclCommDestroy(HcclComm comm)
{
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PTR;
    c->magic = 0;  // no further use through this handle, whether torn down now or later
    // A graph captured on this communicator still holds its staging and RCCL plans, and ncclCommDestroy would wait
    // for that graph to be destroyed: the teardown then runs when the last such graph goes (watchdog.cc).
    if (DeferDestroy(c)) return HCCL_SUCCESS;
    delete c;
    return HCCL_SUCCESS;
}

HcclResult HcclGetCommAsyncError(HcclComm comm, HcclResult* asyncError)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || asyncError == nullptr) return HCCL_E_PTR;
    *asyncError = c->PollAsyncError();  // lock-free: a watchdog thread never waits behind a collective
    return HCCL_SUCCESS;
}

uint64_t HcclAmdIpcTimeoutMs(void) { return IpcTimeoutTicks() / 100000; }

HcclResult HcclGetRankSize(HcclComm comm, uint32_t* rankSize)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || rankSize == nullptr) return HCCL_E_PTR;
    *rankSize = c->nRanks;
    return HCCL_SUCCESS;
}

HcclResult HcclGetRankId(HcclComm comm, uint32_t* rank)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || rank == nullptr) return HCCL_E_PTR;
    *rank = c->rank;
    return HCCL_SUCCESS;
}

HcclResult HcclAmdCommInitLoopback(uint32_t nRanks, HcclComm* comms)
{
    if (comms == nullptr) return HCCL_E_PTR;
    if (nRanks == 0 || nRanks > HCCL_AMD_IR_MAX_SRC) return HCCL_E_PARA;
    int dev = 0;
    HIP_CHK(hipGetDevice(&dev));
    auto world = MakeLoopbackWorld(nRanks);
    std::vector<std::unique_ptr<Comm>> made;
    for (uint32_t r = 0; r < nRanks; ++r) {
        auto c = std::make_unique<Comm>();
        c->rank = r;
        c->nRanks = nRanks;
        HCCL_CHK(c->Init(dev));
        c->transport = MakeLoopbackTransport(world, r);
        made.push_back(std::move(c));
    }
    for (uint32_t r = 0; r < nRanks; ++r) comms[r] = made[r].release();
    return HCCL_SUCCESS;
}

HcclResult HcclAmdCommInitHostExchange(uint32_t nRanks, uint32_t rank, HcclAmdHostAllGatherFn fn, void* ctx,
                                       HcclComm* comm)
{
    if (fn == nullptr || comm == nullptr) return HCCL_E_PTR;
    if (nRanks == 0 || rank >= nRanks || nRanks > kIpcMaxRanks) return HCCL_E_PARA;
    int dev = 0;
    HIP_CHK(hipGetDevice(&dev));
    auto c = std::make_unique<Comm>();
    c->rank = rank;
    c->nRanks = nRanks;
    HCCL_CHK(c->Init(dev));
    c->transport = MakeHostExchangeTransport(fn, ctx);
    c->algoOverride = HCCL_AMD_ALGO_IPC_TWOSHOT;
    *comm = c.release();
    return HCCL_SUCCESS;
}

HcclResult HcclAmdCommInitSelfLoop(uint32_t nRanks, uint32_t rank, HcclComm* comm)
{
    if (comm == nullptr) return HCCL_E_PTR;
    if (nRanks == 0 || rank >= nRanks || nRanks > HCCL_AMD_IR_MAX_SRC) return HCCL_E_PARA;
    int dev = 0;
    HIP_CHK(hipGetDevice(&dev));
    auto c = std::make_unique<Comm>();
    c->rank = rank;
    c->nRanks = nRanks;
    HCCL_CHK(c->Init(dev));
    HcclResult err = HCCL_SUCCESS;
    c->transport = MakeRcclSelfLoopTransport(&err);
    if (c->transport == nullptr) return err == HCCL_SUCCESS ? HCCL_E_INTERNAL : err;
    c->ipc.unavailable = true;  // no peers to map: the one-sided kernel answers NOT_SUPPORT
    HCCL_CHK(c->StartWatchdog());
    *comm = c.release();
    return HCCL_SUCCESS;
}

HcclResult HcclAmdCommSetAlgo(HcclComm comm, int32_t algo)
{
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PTR;
    if (algo < HCCL_AMD_ALGO_AUTO || algo > HCCL_AMD_ALGO_IPC_RHD) return HCCL_E_PARA;
    c->algoOverride = algo;
    return HCCL_SUCCESS;
}

HcclResult HcclAmdCommSetIpcBlocks(HcclComm comm, uint32_t blocks)
{
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PTR;
    if (blocks > kIpcMaxBlocks) return HCCL_E_PARA;
    c->ipcBlocks = blocks;
    return HCCL_SUCCESS;
}

HcclResult HcclAmdCommSetPieceBytes(HcclComm comm, uint64_t pieceBytes)
{
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PTR;
    c->pieceBytes = pieceBytes;
    return HCCL_SUCCESS;
}

int32_t HcclAmdCommLastAlgo(HcclComm comm)
{
    Comm* c = AsComm(comm);
    return c == nullptr ? -1 : c->lastAlgo;
}

HcclResult HcclAmdCommSetConfig(HcclComm comm, int32_t key, int64_t value)
{
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PTR;
    std::lock_guard<std::mutex> lk(c->mu);
    return SetConfigEntry(c->cfg, key, value);
}

HcclResult HcclAmdCommReloadConfig(HcclComm comm)
{
    Comm* c = AsComm(comm);
    if (c == nullptr) return HCCL_E_PTR;
    std::lock_guard<std::mutex> lk(c->mu);
    c->cfg = ReadCommConfig();
    return HCCL_SUCCESS;
}

HcclResult HcclAmdCommGetConfig(HcclComm comm, int32_t key, int64_t* value)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || value == nullptr) return HCCL_E_PTR;
    std::lock_guard<std::mutex> lk(c->mu);
    return GetConfigEntry(c->cfg, key, value);
}

HcclResult HcclAmdCommDeviceBytes(HcclComm comm, uint64_t* bytes)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || bytes == nullptr) return HCCL_E_PTR;
    std::lock_guard<std::mutex> lk(c->mu);
    *bytes = c->DeviceBytes();
    return HCCL_SUCCESS;
}

HcclResult HcclAmdIpcIdleStaging(int32_t release, uint64_t* bytes)
{
    if (bytes == nullptr) return HCCL_E_PTR;
    *bytes = IpcIdleBytes();
    // Freeing memory allocated with hipDeviceMallocUncached corrupts later GPU work on this stack (DESIGN.md §5b, item
    // 5; profiles/r06_release_stress.txt): the idle blocks stay with the process.
    return release != 0 ? HCCL_E_NOT_SUPPORT : HCCL_SUCCESS;
}

HcclResult HcclAmdCommScratch(HcclComm comm, void** ptr, uint64_t* bytes)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || ptr == nullptr || bytes == nullptr) return HCCL_E_PTR;
    std::lock_guard<std::mutex> lk(c->mu);
    *ptr = c->scratch;
    *bytes = c->scratch != nullptr ? c->scratchBytes : 0;
    return HCCL_SUCCESS;
}

HcclResult HcclAmdRcclP2pChannels(uint32_t* perPeer, uint32_t* minP2pChannels)
{
    if (perPeer == nullptr || minP2pChannels == nullptr) return HCCL_E_PTR;
    RcclP2pChannels(perPeer, minP2pChannels);
    return HCCL_SUCCESS;
}

HcclResult HcclAmdL2Maintain(aclrtStream stream) { return ScrubL2(static_cast<hipStream_t>(stream)); }

HcclResult HcclAmdCommExecute(HcclComm comm,const HcclAmdIrOp* ops, uint64_t numOps, void* sendBuf, void* recvBuf,
                              HcclDataType dataType, HcclReduceOp op, int32_t singleStream, aclrtStream stream)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || stream == nullptr || (ops == nullptr && numOps != 0)) return HCCL_E_PTR;
    HCCL_CHK(CheckReduceDataType(dataType));
    HCCL_CHK(CheckReduceOp(dataType, op));
    const uint64_t es = DataTypeSize(dataType);
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->scratch == nullptr) {
        // no staging until a program asks for it
        for (uint64_t i = 0; i < numOps; ++i) {
            bool uses = ops[i].kind != HCCL_AMD_IR_SEND && ops[i].dstBuf == HCCL_AMD_BUF_SCRATCH;
            for (int j = 0; j < ops[i].nsrc && j < HCCL_AMD_IR_MAX_SRC; ++j) {
                uses = uses || ops[i].srcBuf[j] == HCCL_AMD_BUF_SCRATCH;
            }
            if (uses) {
                HCCL_CHK(c->EnsureScratch());
                break;
            }
        }
    }
    // Every record must be well formed; staging references must lie inside the communicator's staging (the user
    // buffers' extents are the caller's contract, as for the collectives).
    auto bufOk = [&](int32_t b, uint64_t off, uint64_t cnt) {
        if (b == HCCL_AMD_BUF_INPUT) return sendBuf != nullptr;
        if (b == HCCL_AMD_BUF_OUTPUT) return recvBuf != nullptr;
        if (b != HCCL_AMD_BUF_SCRATCH || c->scratch == nullptr) return false;
        return off <= c->scratchBytes / es && cnt <= c->scratchBytes / es - off;
    };
    for (uint64_t i = 0; i < numOps; ++i) {
        const HcclAmdIrOp& o = ops[i];
        const bool p2p = o.kind == HCCL_AMD_IR_SEND || o.kind == HCCL_AMD_IR_RECV;
        if (o.kind < HCCL_AMD_IR_COPY || o.kind > HCCL_AMD_IR_RECV) return HCCL_E_PARA;
        if (p2p && (o.peer < 0 || static_cast<uint32_t>(o.peer) >= c->nRanks)) return HCCL_E_PARA;
        const int32_t wantSrc = o.kind == HCCL_AMD_IR_RECV ? 0 : (o.kind == HCCL_AMD_IR_REDUCE ? -1 : 1);
        if ((wantSrc >= 0 && o.nsrc != wantSrc) || (wantSrc < 0 && (o.nsrc < 1 || o.nsrc > HCCL_AMD_IR_MAX_SRC))) {
            return HCCL_E_PARA;
        }
        if (o.kind != HCCL_AMD_IR_SEND && !bufOk(o.dstBuf, o.dstOff, o.count)) return HCCL_E_PARA;
        for (int j = 0; j < o.nsrc; ++j) {
            if (!bufOk(o.srcBuf[j], o.srcOff[j], o.count)) return HCCL_E_PARA;
        }
    }
    HCCL_CHK(c->Gate());
    HIP_CHK(hipSetDevice(c->device));
    const EntryScope entry(*c, static_cast<hipStream_t>(stream));
    HCCL_CHK(entry.status());
    void* bufs[3] = {sendBuf, recvBuf, c->scratch};
    const CompiledSchedule* cs = nullptr;
    HCCL_CHK(CompileProgram(*c, ops, numOps, static_cast<uint32_t>(es), bufs, &cs));
    return RunCompiled(*c, *cs, bufs, dataType, op, static_cast<hipStream_t>(stream), singleStream != 0);
}

HcclResult HcclAmdCommCompileStats(HcclComm comm, uint64_t* hits, uint64_t* misses)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || hits == nullptr || misses == nullptr) return HCCL_E_PTR;
    std::lock_guard<std::mutex> lk(c->mu);
    *hits = c->compileHits;
    *misses = c->compileMisses;
    return HCCL_SUCCESS;
}

int32_t HcclAmdRingTable(uint32_t nRanks, uint32_t* cycles, uint32_t capacity)
{
    if (nRanks == 0) return 0;
    const std::vector<std::vector<uint32_t>> t = RingTable(nRanks);
    for (uint32_t k = 0; cycles != nullptr && k < t.size() && k < capacity; ++k) {
        std::memcpy(cycles + size_t(k) * nRanks, t[k].data(), nRanks * sizeof(uint32_t));
    }
    return static_cast<int32_t>(t.size());
}

int32_t HcclAmdRhdTable(uint32_t nRanks, uint32_t* realOfVirtual, uint32_t capacity)
{
    if (nRanks == 0) return 0;
    const std::vector<std::vector<uint32_t>> t = RhdTable(nRanks);
    for (uint32_t k = 0; realOfVirtual != nullptr && k < t.size() && k < capacity; ++k) {
        std::memcpy(realOfVirtual + size_t(k) * nRanks, t[k].data(), nRanks * sizeof(uint32_t));
    }
    return static_cast<int32_t>(t.size());
}

HcclResult HcclAmdExecutorPlan(const HcclAmdIrOp* ops, uint64_t numOps, uint32_t elemSize, const uint64_t* bufBase,
                               HcclAmdUnitPlan* units, uint64_t capacity, uint64_t* numUnits)
{
    if ((ops == nullptr && numOps != 0) || bufBase == nullptr || numUnits == nullptr) return HCCL_E_PTR;
    if (elemSize == 0) return HCCL_E_PARA;
    const std::vector<HcclAmdIrOp> v(ops, ops + numOps);
    void* bufs[3];
    for (int i = 0; i < 3; ++i) bufs[i] = reinterpret_cast<void*>(static_cast<uintptr_t>(bufBase[i]));
    const std::vector<UnitPlan> plan = PlanUnits(v, bufs, elemSize);
    *numUnits = plan.size();
    if (units == nullptr) return HCCL_SUCCESS;
    if (capacity < plan.size()) return HCCL_E_PARA;
    for (size_t i = 0; i < plan.size(); ++i) {
        units[i].stream = plan[i].stream;
        units[i].isComm = plan[i].isComm ? 1 : 0;
        units[i].firstOp = plan[i].first;
        units[i].numOps = plan[i].count;
        units[i].waitUnit = plan[i].waitUnit;
    }
    return HCCL_SUCCESS;
}

int32_t HcclAmdSelectAivAlgo(int32_t opType, uint32_t nRanks, uint64_t count, HcclDataType dataType, HcclReduceOp op,
                             uint32_t coreLimit, int32_t flags, uint32_t* groupSize)
{
    return SelectAivPlan(opType, nRanks, count, dataType, op, (flags & 1) != 0, (flags & 2) != 0, CclBytesDefault(),
                         coreLimit != 0 ? coreLimit : ReadCommConfig().aivCoreLimit, nullptr, groupSize);
}

HcclResult HcclAmdBuildScheduleV(uint32_t nRanks, uint32_t rank, const uint64_t* sendCounts,
                                 const uint64_t* sendDispls, HcclDataType dataType, uint64_t pieceBytes,
                                 HcclAmdIrOp* ops, uint64_t capacity, uint64_t* numOps, uint64_t* scratchElems)
{
    if (numOps == nullptr || sendCounts == nullptr || sendDispls == nullptr) return HCCL_E_PTR;
    const uint32_t es = DataTypeSize(dataType);
    if (es == 0) return HCCL_E_NOT_SUPPORT;
    if (nRanks == 0 || rank >= nRanks) return HCCL_E_PARA;
    for (uint32_t q = 0; q < nRanks; ++q) {
        if (sendCounts[q] > UINT64_MAX / 16 || sendDispls[q] > UINT64_MAX / 16 - sendCounts[q]) return HCCL_E_PARA;
    }
    ScheduleParams p;
    p.opType = HCCL_AMD_OP_REDUCE_SCATTER_V;
    p.nRanks = nRanks;
    p.rank = rank;
    p.counts.assign(sendCounts, sendCounts + nRanks);
    p.displs.assign(sendDispls, sendDispls + nRanks);
    p.count = sendCounts[rank];
    p.elemSize = es;
    p.pieceBytes = pieceBytes;
    p.scratchCapBytes = ScratchBytesDefault();
    p.cclBytes = CclBytesDefault();
    Schedule s;
    HcclResult r = static_cast<HcclResult>(BuildSchedule(p, &s));
    if (r != HCCL_SUCCESS) return r;
    *numOps = s.ops.size();
    if (scratchElems != nullptr) *scratchElems = s.scratchElems;
    if (ops != nullptr) {
        if (capacity < s.ops.size()) return HCCL_E_PARA;
        std::memcpy(ops, s.ops.data(), s.ops.size() * sizeof(HcclAmdIrOp));
    }
    return HCCL_SUCCESS;
}

int32_t HcclAmdSelectAlgo(int32_t opType, uint32_t nRanks, uint64_t bytes, int32_t special)
{
    return SelectAlgo(opType, nRanks, bytes, special != 0);
}

HcclResult HcclAmdBuildSchedule(int32_t opType, int32_t algo, uint32_t nRanks, uint32_t rank, uint64_t count,
                                HcclDataType dataType, uint32_t root, uint64_t pieceBytes, HcclAmdIrOp* ops,
                                uint64_t capacity, uint64_t* numOps, int32_t* algoUsed, uint64_t* scratchElems)
{
    if (numOps == nullptr) return HCCL_E_PTR;
    uint32_t es = DataTypeSize(dataType);
    if (es == 0) return HCCL_E_NOT_SUPPORT;
    ScheduleParams p;
    p.opType = opType;
    p.algo = algo;
    p.nRanks = nRanks;
    p.rank = rank;
    p.count = count;
    p.elemSize = es;
    p.root = root;
    p.pieceBytes = pieceBytes;
    p.scratchCapBytes = ScratchBytesDefault();
    p.cclBytes = CclBytesDefault();
    p.special = IsSpecialForSelector(dataType, HCCL_REDUCE_SUM);  // the op is not an argument here
    Schedule s;
    HcclResult r = static_cast<HcclResult>(BuildSchedule(p, &s));
    if (r != HCCL_SUCCESS) return r;
    *numOps = s.ops.size();
    if (algoUsed != nullptr) *algoUsed = s.algo;
    if (scratchElems != nullptr) *scratchElems = s.scratchElems;
    if (ops != nullptr) {
        if (capacity < s.ops.size()) return HCCL_E_PARA;
        std::memcpy(ops, s.ops.data(), s.ops.size() * sizeof(HcclAmdIrOp));
    }
    return HCCL_SUCCESS;
}

}  // extern "C"
