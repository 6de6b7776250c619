// ipc.cc — host side of the one-sided AllReduce (ipc_kernels.hip): peer-mapped staging set-up and launch.
//
// Set-up (collective, on the first IPC AllReduce of a communicator): every rank allocates uncached staging and a
// flag array, exports them with hipIpcGetMemHandle, all-gathers the handles over the communicator (ncclAllGather)
// and opens every peer's with hipIpcOpenMemHandle — the reference's channel set-up that hands each rank its peers'
// CCL buffers (ChannelInfo.remoteCclMem, alg_param.h:434-448; AIV GM_IN[r], aiv_communication_base_v2.h:121-150).
// In a loopback world the ranks share a device and the raw pointers are exchanged instead, and the whole world runs
// as one launch (all ranks' blocks must be resident together, which separate per-rank launches on 4 hardware queues
// would not guarantee).
#include <cstring>

#include "comm.h"

namespace hccl_amd {

namespace {

struct Exported {
    hipIpcMemHandle_t stg;
    hipIpcMemHandle_t flags;
};

struct RawPtrs {
    void* stg;
    uint32_t* flags;
};

HcclResult IpcSetup(Comm& c)
{
    IpcState& s = c.ipc;
    if (s.ready) return HCCL_SUCCESS;
    const uint32_t n = c.nRanks, me = c.rank;
    s.blocks = kIpcBlocks;
    s.stgInBytes = kIpcStagingBytes;
    s.stgResBytes = kIpcStagingBytes / n + 4096;
    const size_t flagBytes = size_t(s.blocks) * kIpcMaxRanks * sizeof(uint32_t);
    HIP_CHK(hipExtMallocWithFlags(&s.stg, s.stgInBytes + s.stgResBytes, hipDeviceMallocUncached));
    HIP_CHK(hipExtMallocWithFlags(reinterpret_cast<void**>(&s.flags), flagBytes, hipDeviceMallocUncached));
    HIP_CHK(hipMalloc(reinterpret_cast<void**>(&s.status), sizeof(uint32_t)));
    HIP_CHK(hipMemset(s.flags, 0, flagBytes));
    HIP_CHK(hipMemset(s.status, 0, sizeof(uint32_t)));
    HIP_CHK(hipDeviceSynchronize());
    if (c.transport->SharedDevice()) {
        RawPtrs mine{s.stg, s.flags};
        std::vector<RawPtrs> all(n);
        HCCL_CHK(c.transport->AllGatherHost(&mine, sizeof mine, all.data()));
        for (uint32_t r = 0; r < n; ++r) {
            s.peerStg[r] = all[r].stg;
            s.peerFlags[r] = all[r].flags;
        }
    } else {
        Exported mine{};
        HIP_CHK(hipIpcGetMemHandle(&mine.stg, s.stg));
        HIP_CHK(hipIpcGetMemHandle(&mine.flags, s.flags));
        std::vector<Exported> all(n);
        HCCL_CHK(c.transport->AllGatherHost(&mine, sizeof mine, all.data()));
        for (uint32_t r = 0; r < n; ++r) {
            if (r == me) {
                s.peerStg[r] = s.stg;
                s.peerFlags[r] = s.flags;
                continue;
            }
            HIP_CHK(hipIpcOpenMemHandle(&s.peerStg[r], all[r].stg, hipIpcMemLazyEnablePeerAccess));
            void* f = nullptr;
            HIP_CHK(hipIpcOpenMemHandle(&f, all[r].flags, hipIpcMemLazyEnablePeerAccess));
            s.peerFlags[r] = static_cast<uint32_t*>(f);
            s.opened[r] = true;
        }
    }
    s.epoch = 0;
    s.ready = true;
    return HCCL_SUCCESS;
}

}  // namespace

void IpcRelease(Comm& c)
{
    IpcState& s = c.ipc;
    for (uint32_t r = 0; r < kIpcMaxRanks; ++r) {
        if (s.opened[r]) {
            (void)hipIpcCloseMemHandle(s.peerStg[r]);
            (void)hipIpcCloseMemHandle(s.peerFlags[r]);
            s.opened[r] = false;
        }
    }
    if (s.stg != nullptr) (void)hipFree(s.stg);
    if (s.flags != nullptr) (void)hipFree(s.flags);
    if (s.status != nullptr) (void)hipFree(s.status);
    s = IpcState{};
}

HcclResult RunIpcAllReduce(Comm& c, const void* sendBuf, void* recvBuf, uint64_t count, HcclDataType dt,
                           HcclReduceOp op, hipStream_t stream)
{
    if ((reinterpret_cast<uintptr_t>(sendBuf) | reinterpret_cast<uintptr_t>(recvBuf)) & 15u) {
        return HCCL_E_NOT_SUPPORT;
    }
    const uint64_t es = DataTypeSize(dt);
    if (es == 0 || c.nRanks > kIpcMaxRanks) return HCCL_E_NOT_SUPPORT;
    HCCL_CHK(IpcSetup(c));
    IpcState& s = c.ipc;
    const uint32_t n = c.nRanks;
    const uint64_t unit = uint64_t(n) * (16 / es);
    const uint64_t roundElems = (s.stgInBytes / es) / unit * unit;
    const uint64_t rounds = (count + roundElems - 1) / roundElems;

    IpcArgs a{};
    for (uint32_t r = 0; r < n; ++r) {
        a.stgIn[r] = s.peerStg[r];
        a.stgRes[r] = static_cast<char*>(s.peerStg[r]) + s.stgInBytes;
        a.flags[r] = s.peerFlags[r];
    }
    a.n = n;
    a.count = count;
    a.roundElems = roundElems;
    a.epochBase = s.epoch;
    a.maxPolls = 1u << 22;  // ~ seconds of polling: a lost peer ends the kernel with status bit 0, never a hang
    a.status = s.status;
    s.epoch += static_cast<uint32_t>(3 * rounds);

    if (!c.transport->SharedDevice()) {
        a.me = static_cast<int32_t>(c.rank);
        a.in[c.rank] = sendBuf;
        a.out[c.rank] = recvBuf;
        HIP_CHK(hipMemsetAsync(s.status, 0, sizeof(uint32_t), stream));  // the status describes the last call
        return LaunchIpcAllReduce(a, s.blocks, 0, dt, op, stream);
    }

    // loopback world: one launch for every rank, issued by rank 0 behind every rank's stream
    struct Part {
        const void* in;
        void* out;
        hipEvent_t ready;
        uint32_t* status;
    };
    Part mine{sendBuf, recvBuf, nullptr, s.status};
    c.nextEvent = 0;
    HCCL_CHK(c.NextEvent(&mine.ready));
    HIP_CHK(hipEventRecord(mine.ready, stream));
    std::vector<Part> all(n);
    HCCL_CHK(c.transport->AllGatherHost(&mine, sizeof mine, all.data()));
    hipEvent_t done = nullptr;
    if (c.rank == 0) {
        a.me = -1;
        for (uint32_t r = 0; r < n; ++r) {
            a.in[r] = all[r].in;
            a.out[r] = all[r].out;
            HIP_CHK(hipStreamWaitEvent(stream, all[r].ready, 0));
        }
        HIP_CHK(hipMemsetAsync(s.status, 0, sizeof(uint32_t), stream));
        HCCL_CHK(LaunchIpcAllReduce(a, s.blocks, n, dt, op, stream));
        HCCL_CHK(c.NextEvent(&done));
        HIP_CHK(hipEventRecord(done, stream));
    }
    std::vector<hipEvent_t> dones(n);
    HCCL_CHK(c.transport->AllGatherHost(&done, sizeof done, dones.data()));
    if (c.rank != 0) HIP_CHK(hipStreamWaitEvent(stream, dones[0], 0));
    return HCCL_SUCCESS;
}

}  // namespace hccl_amd

using namespace hccl_amd;

extern "C" HcclResult HcclAmdCommIpcStatus(HcclComm comm, uint32_t* status)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || status == nullptr) return HCCL_E_PTR;
    *status = 0;
    if (!c->ipc.ready) return HCCL_SUCCESS;
    HIP_CHK(hipSetDevice(c->device));
    HIP_CHK(hipMemcpy(status, c->ipc.status, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return HCCL_SUCCESS;
}
