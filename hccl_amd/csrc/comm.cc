// comm.cc — communicator lifetime, RCCL transport (xGMI), loopback transport (single-device test world).
#include "comm.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

namespace hccl_amd {

// ------------------------------------------------------------------------------------------------ Comm

Comm* AsComm(HcclComm c)
{
    Comm* p = static_cast<Comm*>(c);
    if (p == nullptr || p->magic != 0x48434C41) return nullptr;
    return p;
}

uint64_t CclBytesDefault()
{
    // HCCL_BUFFSIZE in MB, default 200 (docs/zh/user_guide/hccl_env/HCCL_BUFFSIZE.md; the reference simulator's CCL
    // buffer, sim_npu.cc:47). It sizes the executor loops, and so the slicing of the ownership-dependent orders.
    const char* e = std::getenv("HCCL_BUFFSIZE");
    uint64_t mb = 200;
    if (e != nullptr && e[0] != '\0') {
        char* end = nullptr;
        unsigned long long v = std::strtoull(e, &end, 10);
        if (end != e && v > 0) mb = v;
    }
    return mb << 20;
}

// Every communicator holds 2 x HCCL_BUFFSIZE (HCCL_BUFFSIZE.md: "2*HCCL_BUFFSIZE", send and receive halves).
uint64_t ScratchBytesDefault() { return 2 * CclBytesDefault(); }

HcclResult Comm::Init(int dev)
{
    device = dev;
    cfg = ReadCommConfig();
    HIP_CHK(hipSetDevice(dev));
    int lo = 0, hi = 0;
    HIP_CHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // the link stream gets the higher priority: its kernels are short and gate every peer
    HIP_CHK(hipStreamCreateWithPriority(&commStream, hipStreamNonBlocking, hi));
    HIP_CHK(hipStreamCreateWithPriority(&reduceStream, hipStreamNonBlocking, lo));
    // the executor's staging is allocated by the first program that needs it (EnsureScratch)
    cclBytes = CclBytesDefault();
    scratchBytes = 2 * cclBytes;
    return HCCL_SUCCESS;
}

HcclResult Comm::EnsureScratch()
{
    if (scratch != nullptr) return HCCL_SUCCESS;
    HIP_CHK(hipSetDevice(device));
    // A first program may be issued under the caller's stream capture: an allocation is not a stream operation, and
    // the relaxed mode lets this thread make it whatever capture mode the caller chose (as a library's lazily made
    // workspace must).
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    HIP_CHK(hipThreadExchangeStreamCaptureMode(&mode));
    const hipError_t e = hipMalloc(&scratch, scratchBytes);
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (e != hipSuccess) {
        scratch = nullptr;
        HCCL_AMD_ERR("rank %u: executor staging of %llu B: %s", rank, (unsigned long long)scratchBytes,
                     hipGetErrorString(e));
        return HCCL_E_MEMORY;
    }
    return HCCL_SUCCESS;
}

uint64_t Comm::DeviceBytes() const { return (scratch != nullptr ? scratchBytes : 0) + IpcDeviceBytes(*this); }

// The executor's ordering events (a program's start, its cross-stream unit events and stream joins) keep the runtime's
// default system-scope fence: unlike the communicator's tail (EntryScope), they order data one stream's kernel or
// transport group wrote before another stream's kernel reads it (r05 measured them fence-free within 1 % behind RCCL
// groups and kept them).
HcclResult Comm::NextEvent(hipEvent_t* e)
{
    if (nextEvent == events.size()) {
        hipEvent_t ev;
        HIP_CHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        events.push_back(ev);
    }
    *e = events[nextEvent++];
    return HCCL_SUCCESS;
}

HcclResult Comm::PollAsyncError()
{
    const int32_t known = failCode.load(std::memory_order_acquire);
    if (known != HCCL_SUCCESS) return static_cast<HcclResult>(known);
    HcclResult e = HCCL_SUCCESS;
    const volatile uint32_t* w = failWord.load(std::memory_order_acquire);
    if (w != nullptr && *w != 0) {
        e = HCCL_E_TIMEOUT;  // an IPC barrier wait exceeded its bound (IpcTimeoutTicks)
    } else if (transport != nullptr) {
        e = transport->AsyncError();
    }
    if (e == HCCL_SUCCESS) return HCCL_SUCCESS;
    int32_t expected = HCCL_SUCCESS;  // the first error seen sticks, whichever thread saw it
    failCode.compare_exchange_strong(expected, e, std::memory_order_acq_rel);
    return static_cast<HcclResult>(failCode.load(std::memory_order_acquire));
}

HcclResult Comm::Gate()
{
    if (failed) return HCCL_E_SUSPENDING;
    const HcclResult e = PollAsyncError();
    if (e != HCCL_SUCCESS) {
        failed = true;
        HCCL_AMD_ERR("rank %u: communicator failed (%s); later collectives return HCCL_E_SUSPENDING", rank,
                     HcclAmdGetErrorString(e));
    }
    return e;
}

HcclResult Comm::StartWatchdog()
{
    if (transport == nullptr || !transport->Abortable()) return HCCL_SUCCESS;
    const char* e = std::getenv("HCCL_AMD_INJECT_STALL_GROUP");
    if (e != nullptr && *e != '\0') {
        stallAtGroup = std::strtoull(e, nullptr, 10);
        if (stallAtGroup != 0) {
            HIP_CHK(hipHostMalloc(reinterpret_cast<void**>(&stallHost), 64,
                                  hipHostMallocCoherent | hipHostMallocMapped));
            HIP_CHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&stallDev), stallHost, 0));
            *stallHost = 0;
        }
    }
    const uint64_t bound = RcclExecTimeoutMs();
    if (bound != 0) {
        watchdog = std::make_unique<Watchdog>(this, bound);
        HCCL_CHK(watchdog->Init());
    }
    return HCCL_SUCCESS;
}

// Teardown order (each step time-stamped on stderr with HCCL_AMD_TEARDOWN_TRACE=1): drain the communicator's streams
// while the watchdog still runs (a lost peer is aborted past the bound, so the drain ends), stop the watchdog, release
// the IPC mappings (collective), then RCCL (ncclCommFinalize bounded by the execution timeout, else ncclCommAbort).
Comm::~Comm()
{
    magic = 0;
    if (commStream != nullptr || reduceStream != nullptr) {
        (void)hipSetDevice(device);
    }
    TeardownTrace(rank, "sync link stream", true);
    if (commStream != nullptr) (void)hipStreamSynchronize(commStream);
    TeardownTrace(rank, "sync reduce stream", true);
    if (reduceStream != nullptr) (void)hipStreamSynchronize(reduceStream);
    TeardownTrace(rank, "sync last call + graphs", true);
    if (tail != nullptr) (void)hipEventSynchronize(tail);
    ReleaseGraphs(*this);
    TeardownTrace(rank, "stop watchdog", true);
    watchdog.reset();
    TeardownTrace(rank, "IPC quiesce + release", true);
    IpcQuiesce(*this);
    IpcRelease(*this);
    TeardownTrace(rank, "transport teardown", true);
    transport.reset();
    TeardownTrace(rank, "events, staging, streams", true);
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    for (hipEvent_t e : foldTiming.pool) (void)hipEventDestroy(e);
    if (scratch != nullptr) (void)hipFree(scratch);
    if (commStream != nullptr) (void)hipStreamDestroy(commStream);
    if (reduceStream != nullptr) (void)hipStreamDestroy(reduceStream);
    if (stallHost != nullptr) (void)hipHostFree(stallHost);
    if (tail != nullptr) (void)hipEventDestroy(tail);
    TeardownTrace(rank, "done", false);
}

// ------------------------------------------------------------------------------------------------ RCCL transport

namespace {

HcclResult FromNccl(ncclResult_t r, const char* what)
{
    if (r == ncclSuccess) return HCCL_SUCCESS;
    HCCL_AMD_ERR("%s: %s", what, ncclGetErrorString(r));
    switch (r) {
        case ncclInvalidArgument:
        case ncclInvalidUsage: return HCCL_E_PARA;
        case ncclSystemError: return HCCL_E_SYSCALL;
        case ncclRemoteError: return HCCL_E_REMOTE;
        default: return HCCL_E_INTERNAL;
    }
}

// Polls a non-blocking communicator until the call that returned `r` has finished, at most boundMs (0 = no bound).
// Returns ncclInProgress when the bound passed.
ncclResult_t WaitSettled(ncclComm_t comm, ncclResult_t r, uint64_t boundMs)
{
    if (r != ncclInProgress) return r;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) return ncclInternalError;
        if (r != ncclInProgress) return r;
        if (boundMs != 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(boundMs)) {
            return ncclInProgress;
        }
        if (spin < 1000) {
            std::this_thread::yield();
        } else {
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
}

class RcclTransport : public Transport {
public:
    // selfLoop: a one-rank RCCL communicator standing in for every peer (HcclAmdCommInitSelfLoop)
    explicit RcclTransport(ncclComm_t comm, bool selfLoop = false) : comm_(comm), selfLoop_(selfLoop) {}
    ~RcclTransport() override
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (comm_ == nullptr) return;
        if (localTeardown_) {
            (void)ncclCommAbort(comm_);  // a deferred teardown: no peer takes part any more
            comm_ = nullptr;
            return;
        }
        // ncclCommFinalize flushes this rank's outstanding work; bounded like any other wait on a peer
        ncclResult_t r = WaitSettled(comm_, ncclCommFinalize(comm_), RcclExecTimeoutMs());
        if (r == ncclSuccess) {
            (void)ncclCommDestroy(comm_);
        } else {
            HCCL_AMD_ERR("ncclCommFinalize: %s: aborting the communicator", ncclGetErrorString(r));
            (void)ncclCommAbort(comm_);
        }
        comm_ = nullptr;
    }
    HcclResult Group(const std::vector<P2pOp>& ops, hipStream_t stream) override
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (comm_ == nullptr) return HCCL_E_SUSPENDING;  // aborted by the watchdog
        std::vector<P2pOp> paired;
        const std::vector<P2pOp>* post = &ops;
        if (selfLoop_) {
            // every peer is this rank: each send is posted beside a receive of the same size, since RCCL pairs
            // messages to itself in posting order. Sends and receives whose sizes differ (a ring's ragged last chunk)
            // are paired in order at the smaller size, and a surplus on either side is dropped: the stand-in keeps
            // the program's shape, not its data.
            std::vector<P2pOp> sends, recvs;
            for (const P2pOp& o : ops) (o.isSend ? sends : recvs).push_back(o);
            std::vector<P2pOp> restSends;
            for (const P2pOp& o : sends) {
                auto it = std::find_if(recvs.begin(), recvs.end(), [&](const P2pOp& q) { return q.bytes == o.bytes; });
                if (it == recvs.end()) {
                    restSends.push_back(o);
                    continue;
                }
                paired.push_back({true, 0, o.ptr, o.bytes});
                paired.push_back({false, 0, it->ptr, it->bytes});
                recvs.erase(it);
            }
            for (size_t k = 0; k < restSends.size() && k < recvs.size(); ++k) {
                const uint64_t b = std::min(restSends[k].bytes, recvs[k].bytes);
                paired.push_back({true, 0, restSends[k].ptr, b});
                paired.push_back({false, 0, recvs[k].ptr, b});
            }
            post = &paired;
        }
        ncclResult_t r = ncclGroupStart();
        if (r != ncclSuccess) return FromNccl(r, "ncclGroupStart");
        for (const P2pOp& o : *post) {
            r = o.isSend ? ncclSend(o.ptr, o.bytes, ncclUint8, static_cast<int>(o.peer), comm_, stream)
                         : ncclRecv(o.ptr, o.bytes, ncclUint8, static_cast<int>(o.peer), comm_, stream);
            if (r != ncclSuccess && r != ncclInProgress) {
                (void)ncclGroupEnd();
                return FromNccl(r, o.isSend ? "ncclSend" : "ncclRecv");
            }
        }
        return Settle(ncclGroupEnd(), "ncclGroupEnd");
    }
    const char* Name() const override { return "rccl"; }
    bool Abortable() const override { return true; }
    void SetLocalTeardown(bool on) override
    {
        std::lock_guard<std::mutex> lk(mu_);
        localTeardown_ = on;
    }
    // hands the RCCL communicator over (to a transport of another kind around it)
    ncclComm_t Release()
    {
        std::lock_guard<std::mutex> lk(mu_);
        ncclComm_t c = comm_;
        comm_ = nullptr;
        return c;
    }
    // From the watchdog thread. The communicator is taken out under the lock and aborted outside it: RCCL's abort
    // raises the kernels' abort flag at once but then waits for the graphs holding its plans (the executor graph cache,
    // a user's captured graph) to go, and a thread entering Group / AllGatherHost meanwhile must get
    // HCCL_E_SUSPENDING instead of waiting on the lock.
    void Abort() override
    {
        ncclComm_t c = nullptr;
        {
            std::lock_guard<std::mutex> lk(mu_);
            c = comm_;
            comm_ = nullptr;
        }
        if (c != nullptr) (void)ncclCommAbort(c);
    }
    HcclResult AsyncError() override
    {
        // never waits behind a group being posted (HcclGetCommAsyncError is polled by watchdog threads)
        std::unique_lock<std::mutex> lk(mu_, std::try_to_lock);
        if (!lk.owns_lock() || comm_ == nullptr) return HCCL_SUCCESS;
        ncclResult_t a = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &a) != ncclSuccess) return HCCL_E_INTERNAL;
        return (a == ncclSuccess || a == ncclInProgress) ? HCCL_SUCCESS : FromNccl(a, "RCCL asynchronous error");
    }
    HcclResult AllGatherHost(const void* mine, size_t bytes, void* all) override
    {
        if (selfLoop_) return HCCL_E_NOT_SUPPORT;  // no peers to exchange with (the one-sided kernel is unavailable)
        std::lock_guard<std::mutex> lk(mu_);
        if (comm_ == nullptr) return HCCL_E_SUSPENDING;
        int n = 0;
        HcclResult r = FromNccl(ncclCommCount(comm_, &n), "ncclCommCount");
        if (r != HCCL_SUCCESS) return r;
        void* d = nullptr;
        hipStream_t s = nullptr;
        HIP_CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        if (hipMalloc(&d, bytes * (size_t(n) + 1)) != hipSuccess) {
            (void)hipStreamDestroy(s);
            return HCCL_E_MEMORY;
        }
        char* dAll = static_cast<char*>(d) + bytes;
        r = hipMemcpyAsync(d, mine, bytes, hipMemcpyHostToDevice, s) == hipSuccess ? HCCL_SUCCESS : HCCL_E_RUNTIME;
        if (r == HCCL_SUCCESS) r = Settle(ncclAllGather(d, dAll, bytes, ncclUint8, comm_, s), "ncclAllGather");
        if (r == HCCL_SUCCESS) {
            r = hipMemcpyAsync(all, dAll, bytes * size_t(n), hipMemcpyDeviceToHost, s) == hipSuccess ? HCCL_SUCCESS
                                                                                                   : HCCL_E_RUNTIME;
        }
        if (r == HCCL_SUCCESS) {
            // a host-side wait on peers: bounded by the execution timeout like the device-side ones
            const uint64_t bound = RcclExecTimeoutMs();
            const auto t0 = std::chrono::steady_clock::now();
            hipError_t q;
            while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
                if (bound != 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(bound)) {
                    HCCL_AMD_ERR("host all-gather over RCCL ran past HCCL_EXEC_TIMEOUT: aborting the communicator");
                    AbortLocked();
                    (void)hipStreamSynchronize(s);  // the aborted all-gather returns
                    q = hipSuccess;
                    r = HCCL_E_TIMEOUT;
                    break;
                }
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
            if (q != hipSuccess) r = HCCL_E_RUNTIME;
        }
        (void)hipStreamSynchronize(s);
        (void)hipFree(d);
        (void)hipStreamDestroy(s);
        return r;
    }

private:
    HcclResult Settle(ncclResult_t r, const char* what)  // mu_ held
    {
        r = WaitSettled(comm_, r, RcclExecTimeoutMs());
        if (r == ncclInProgress) {
            HCCL_AMD_ERR("%s did not complete within HCCL_EXEC_TIMEOUT: aborting the communicator", what);
            AbortLocked();
            return HCCL_E_TIMEOUT;
        }
        return FromNccl(r, what);
    }
    void AbortLocked()
    {
        if (comm_ == nullptr) return;
        (void)ncclCommAbort(comm_);  // RCCL's kernels of this communicator see the abort flag and return
        comm_ = nullptr;
    }
    std::mutex mu_;
    ncclComm_t comm_;
    bool selfLoop_ = false;
    bool localTeardown_ = false;
};

}  // namespace

HcclResult RcclGetUniqueId(void* id128)
{
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    HcclResult r = FromNccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
    if (r != HCCL_SUCCESS) return r;
    std::memcpy(id128, &id, sizeof id);
    return HCCL_SUCCESS;
}

namespace {

uint32_t g_p2pPerPeer = 0;  // what RCCL was configured with (0 = not yet)
uint32_t g_p2pMin = 0;

uint32_t EnvU32(const char* name, uint32_t dflt)
{
    const char* e = std::getenv(name);
    if (e == nullptr || *e == '\0') return dflt;
    const unsigned long v = std::strtoul(e, nullptr, 10);
    return v == 0 ? dflt : static_cast<uint32_t>(std::min<unsigned long>(v, 64));
}

uint32_t Pow2Up(uint32_t x)
{
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace

// Per-peer p2p channels of RCCL, opt-in. The schedules move their data with grouped ncclSend/ncclRecv, one
// message per peer per step, and RCCL's p2p kernel streams about 43 GB/s per channel
// (profiles/r02_rccl_p2p_channels_selfloop.jsonl: 176 / 345 / 650 GB/s at 4 / 8 / 16 channels per peer), below one
// 76.8 GB/s xGMI link per direction (cost_model.cc:78-79 prices the reference's links the same way); the reference
// sizes its channels per link explicitly (alg_param.h:434-448). RCCL reads NCCL_NCHANNELS_PER_PEER and
// NCCL_MIN_P2P_NCHANNELS once per process, at its first communicator, whoever creates it, and they then apply to every
// RCCL communicator of the process (torch.distributed's too), with a device-memory cost per channel that no run on this
// pool has measured at seven peers. So the library changes them only when asked: HCCL_AMD_P2P_CHANNELS_PER_PEER=k sets
// NCCL_NCHANNELS_PER_PEER=k unless the caller set it, and NCCL_MIN_P2P_NCHANNELS = (the per-peer value in effect) x 7
// (the peers of an 8-GPU node) rounded up to a power of two, at most 64, unless the caller set it. They are set when the
// library is loaded, before any thread of the library exists; a caller that loads it after starting threads of its own
// that read the environment should set the NCCL_* variables itself instead. bench.py opts in with 16 (r04: 4 made the
// one-GPU self-loop proxy of the RCCL path 1.7-2.9x slower, profiles/r04_span_channels.jsonl). HcclAmdRcclP2pChannels
// reports the values in the environment after this step (requested, not necessarily what RCCL used: RCCL's INIT log
// line "%d p2p channels, %d p2p channels per peer" says that, and bench.py's transport.p2p_channels carries it).
__attribute__((constructor)) void ConfigureRcclP2pChannels()
{
    const uint32_t per = EnvU32("HCCL_AMD_P2P_CHANNELS_PER_PEER", 0);
    if (per != 0) {
        if (std::getenv("NCCL_NCHANNELS_PER_PEER") == nullptr) {
            setenv("NCCL_NCHANNELS_PER_PEER", std::to_string(Pow2Up(per)).c_str(), 0);
        }
        const uint32_t inEffect = EnvU32("NCCL_NCHANNELS_PER_PEER", Pow2Up(per));
        if (std::getenv("NCCL_MIN_P2P_NCHANNELS") == nullptr) {
            setenv("NCCL_MIN_P2P_NCHANNELS", std::to_string(std::min<uint32_t>(64, Pow2Up(inEffect * 7))).c_str(), 0);
        }
    }
    g_p2pPerPeer = EnvU32("NCCL_NCHANNELS_PER_PEER", 0);
    g_p2pMin = EnvU32("NCCL_MIN_P2P_NCHANNELS", 0);
}

void RcclP2pChannels(uint32_t* perPeer, uint32_t* minP2p)
{
    *perPeer = g_p2pPerPeer;
    *minP2p = g_p2pMin;
}

std::unique_ptr<Transport> MakeRcclSelfLoopTransport(HcclResult* err)
{
    ncclUniqueId id;
    *err = FromNccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
    if (*err != HCCL_SUCCESS) return nullptr;
    std::unique_ptr<Transport> t = MakeRcclTransport(&id, 1, 0, err);
    if (t == nullptr) return nullptr;
    auto* rc = static_cast<RcclTransport*>(t.get());
    return std::make_unique<RcclTransport>(rc->Release(), true);
}

std::unique_ptr<Transport> MakeRcclTransport(void* uniqueId, uint32_t nRanks, uint32_t rank, HcclResult* err)
{
    ncclUniqueId id;
    std::memcpy(&id, uniqueId, sizeof id);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;  // non-blocking: every wait on a peer returns ncclInProgress and is ours to bound
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclCommInitRankConfig(&comm, static_cast<int>(nRanks), id, static_cast<int>(rank), &cfg);
    if (comm != nullptr) r = WaitSettled(comm, r, ConnectTimeoutMs());
    if (r == ncclInProgress) {
        HCCL_AMD_ERR("ncclCommInitRankConfig: rank %u of %u: not every rank joined within the connect timeout", rank,
                     nRanks);
        (void)ncclCommAbort(comm);
        *err = HCCL_E_TIMEOUT;
        return nullptr;
    }
    *err = FromNccl(r, "ncclCommInitRankConfig");
    if (*err != HCCL_SUCCESS) {
        if (comm != nullptr) (void)ncclCommAbort(comm);
        return nullptr;
    }
    return std::make_unique<RcclTransport>(comm);
}

HcclResult MakeRcclTransportsAll(uint32_t ndev, const int32_t* devices, std::vector<std::unique_ptr<Transport>>* out)
{
    // ncclCommInitAll's steps, with the communicators' config: one unique id, ncclCommInitRankConfig per device in a
    // group.
    ncclUniqueId id;
    HCCL_CHK(FromNccl(ncclGetUniqueId(&id), "ncclGetUniqueId"));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;  // non-blocking: every wait on a peer returns ncclInProgress and is ours to bound
    std::vector<ncclComm_t> comms(ndev, nullptr);
    int dev0 = 0;
    HIP_CHK(hipGetDevice(&dev0));
    ncclResult_t r = ncclGroupStart();
    for (uint32_t i = 0; i < ndev && r == ncclSuccess; ++i) {
        if (hipSetDevice(devices[i]) != hipSuccess) {
            r = ncclInvalidArgument;
            break;
        }
        r = ncclCommInitRankConfig(&comms[i], static_cast<int>(ndev), id, static_cast<int>(i), &cfg);
        if (r == ncclInProgress) r = ncclSuccess;
    }
    ncclResult_t e = ncclGroupEnd();
    (void)hipSetDevice(dev0);
    if (r == ncclSuccess) r = e == ncclInProgress ? ncclSuccess : e;
    for (uint32_t i = 0; i < ndev && r == ncclSuccess; ++i) {
        if (comms[i] != nullptr) r = WaitSettled(comms[i], ncclInProgress, ConnectTimeoutMs());
    }
    if (r != ncclSuccess) {
        for (ncclComm_t c : comms) {
            if (c != nullptr) (void)ncclCommAbort(c);
        }
        return r == ncclInProgress ? HCCL_E_TIMEOUT : FromNccl(r, "ncclCommInitRankConfig (all devices)");
    }
    out->clear();
    for (uint32_t i = 0; i < ndev; ++i) out->push_back(std::make_unique<RcclTransport>(comms[i]));
    return HCCL_SUCCESS;
}

// ------------------------------------------------------------------------------------------------ loopback

// nRanks ranks in one process on one device. A send posts {source, bytes, ready event} into the (from, to) FIFO;
// the receiver's stream waits for `ready`, copies device-to-device and records `done`; the sender's stream then
// waits for `done`, so a group completes exactly when an RCCL group would. Ranks rendezvous on the host like real
// ranks, so each must be driven from its own thread.
class LoopbackWorld {
public:
    struct Entry {
        const void* src = nullptr;
        uint64_t bytes = 0;
        hipEvent_t ready = nullptr;
        hipEvent_t done = nullptr;
        bool consumed = false;
        bool failed = false;
    };
    explicit LoopbackWorld(uint32_t n) : n_(n), boxes_(size_t(n) * n), slots_(n) {}
    ~LoopbackWorld()
    {
        // every rank's communicator has drained its streams before it released the world (~Comm)
        for (hipEvent_t e : retired_) (void)hipEventDestroy(e);
        if (failHost_ != nullptr) (void)hipHostFree(failHost_);
    }
    LoopbackWorld(const LoopbackWorld&) = delete;
    LoopbackWorld& operator=(const LoopbackWorld&) = delete;
    uint32_t n_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<std::deque<std::shared_ptr<Entry>>> boxes_;

    // host all-gather among the rank threads (generation-counted so that back-to-back exchanges cannot mix)
    std::vector<std::vector<char>> slots_;
    std::vector<char> result_;
    bool resultOk_ = false;
    uint32_t arrived_ = 0;
    uint64_t generation_ = 0;

    // the failure word of the world's IPC launches (Transport::SharedFailWord), allocated by the first rank to ask
    uint32_t* failHost_ = nullptr;
    uint32_t* failDev_ = nullptr;

    // Events of the links, retired once both sides have enqueued their waits on them. They were destroyed at once
    // before r05, right after another thread's stream had been told to wait on them: HIP may hand a
    // destroyed event's completion signal to a new event while a wait on it is still queued. They now live until the
    // world is torn down; past kRetiredMax the oldest completed ones go, far behind any wait still queued (r05 showed
    // the old lifetime was not the cause of the r03 stale operands, DESIGN.md §5b, but this is the lifetime HIP's
    // contract wants).
    static constexpr size_t kRetiredMax = 16384;
    std::deque<hipEvent_t> retired_;

    void Retire(hipEvent_t e)  // mu_ not held
    {
        if (e == nullptr) return;
        std::lock_guard<std::mutex> lk(mu_);
        retired_.push_back(e);
        while (retired_.size() > kRetiredMax && hipEventQuery(retired_.front()) == hipSuccess) {
            (void)hipEventDestroy(retired_.front());
            retired_.pop_front();
        }
    }

    uint32_t* FailWord(uint32_t** dev)
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (failHost_ == nullptr) {
            uint32_t* h = nullptr;
            if (hipHostMalloc(reinterpret_cast<void**>(&h), 64, hipHostMallocCoherent | hipHostMallocMapped) !=
                hipSuccess) {
                *dev = nullptr;
                return nullptr;
            }
            if (hipHostGetDevicePointer(reinterpret_cast<void**>(&failDev_), h, 0) != hipSuccess) {
                (void)hipHostFree(h);
                *dev = nullptr;
                return nullptr;
            }
            *h = 0;
            failHost_ = h;
        }
        *dev = failDev_;
        return failHost_;
    }

    HcclResult Exchange(uint32_t rank, const void* mine, size_t bytes, void* all)
    {
        std::unique_lock<std::mutex> lk(mu_);
        const uint64_t gen = generation_;
        slots_[rank].assign(static_cast<const char*>(mine), static_cast<const char*>(mine) + bytes);
        if (++arrived_ == n_) {
            // The last arrival completes the generation whatever happens, so no rank of this exchange is left
            // counted in the next one; a size mismatch fails every rank of the generation alike.
            result_.clear();
            bool sameSize = true;
            for (auto& s : slots_) {
                sameSize = sameSize && s.size() == bytes;
                result_.insert(result_.end(), s.begin(), s.end());
            }
            resultOk_ = sameSize;
            arrived_ = 0;
            generation_++;
            cv_.notify_all();
        } else if (!cv_.wait_for(lk, std::chrono::seconds(600), [&] { return generation_ != gen; })) {
            --arrived_;  // withdraw: a later exchange must not count this rank as arrived
            return HCCL_E_TIMEOUT;
        }
        if (!resultOk_ || result_.size() != bytes * n_) return HCCL_E_INTERNAL;
        std::memcpy(all, result_.data(), bytes * n_);
        return HCCL_SUCCESS;
    }
};

namespace {

constexpr auto kRendezvousTimeout = std::chrono::seconds(600);

class LoopbackTransport : public Transport {
public:
    LoopbackTransport(std::shared_ptr<LoopbackWorld> w, uint32_t rank) : w_(std::move(w)), me_(rank) {}
    const char* Name() const override { return "loopback"; }
    bool SharedDevice() const override { return true; }
    HcclResult AllGatherHost(const void* mine, size_t bytes, void* all) override
    {
        return w_->Exchange(me_, mine, bytes, all);
    }
    uint32_t* SharedFailWord(uint32_t** dev) override { return w_->FailWord(dev); }

    HcclResult Group(const std::vector<P2pOp>& ops, hipStream_t stream) override
    {
        LoopbackWorld& w = *w_;
        std::vector<std::shared_ptr<LoopbackWorld::Entry>> posted;
        for (const P2pOp& o : ops) {
            if (!o.isSend) continue;
            auto e = std::make_shared<LoopbackWorld::Entry>();
            e->src = o.ptr;
            e->bytes = o.bytes;
            HIP_CHK(hipEventCreateWithFlags(&e->ready, hipEventDisableTiming));
            HIP_CHK(hipEventRecord(e->ready, stream));
            {
                std::lock_guard<std::mutex> lk(w.mu_);
                w.boxes_[size_t(me_) * w.n_ + o.peer].push_back(e);
            }
            w.cv_.notify_all();
            posted.push_back(std::move(e));
        }
        HcclResult result = HCCL_SUCCESS;
        for (const P2pOp& o : ops) {
            if (o.isSend) continue;
            std::shared_ptr<LoopbackWorld::Entry> e;
            {
                std::unique_lock<std::mutex> lk(w.mu_);
                auto& box = w.boxes_[size_t(o.peer) * w.n_ + me_];
                if (!w.cv_.wait_for(lk, kRendezvousTimeout, [&] { return !box.empty(); })) {
                    HCCL_AMD_ERR("loopback rank %u: no send from rank %u", me_, o.peer);
                    return HCCL_E_TIMEOUT;
                }
                e = box.front();
                box.pop_front();
            }
            hipEvent_t done = nullptr;
            bool ok = e->bytes == o.bytes;
            if (!ok) {
                HCCL_AMD_ERR("loopback rank %u: recv of %llu B matched a send of %llu B from rank %u", me_,
                             (unsigned long long)o.bytes, (unsigned long long)e->bytes, o.peer);
                result = HCCL_E_INTERNAL;
            } else {
                ok = hipStreamWaitEvent(stream, e->ready, 0) == hipSuccess &&
                     LaunchCopyBytes(o.ptr, e->src, o.bytes, stream) == HCCL_SUCCESS &&
                     hipEventCreateWithFlags(&done, hipEventDisableTiming) == hipSuccess &&
                     hipEventRecord(done, stream) == hipSuccess;
                if (!ok) result = HCCL_E_RUNTIME;
            }
            {
                std::lock_guard<std::mutex> lk(w.mu_);
                e->done = done;
                e->failed = !ok;
                e->consumed = true;
            }
            w.cv_.notify_all();
        }
        for (auto& e : posted) {
            {
                std::unique_lock<std::mutex> lk(w.mu_);
                if (!w.cv_.wait_for(lk, kRendezvousTimeout, [&] { return e->consumed; })) {
                    HCCL_AMD_ERR("loopback rank %u: send never received", me_);
                    return HCCL_E_TIMEOUT;
                }
            }
            if (e->failed) result = HCCL_E_INTERNAL;
            if (e->done != nullptr && hipStreamWaitEvent(stream, e->done, 0) != hipSuccess) result = HCCL_E_RUNTIME;
            w.Retire(e->done);
            w.Retire(e->ready);
        }
        return result;
    }

private:
    std::shared_ptr<LoopbackWorld> w_;
    uint32_t me_;
};

}  // namespace

std::shared_ptr<LoopbackWorld> MakeLoopbackWorld(uint32_t nRanks) { return std::make_shared<LoopbackWorld>(nRanks); }

std::unique_ptr<Transport> MakeLoopbackTransport(std::shared_ptr<LoopbackWorld> world, uint32_t rank)
{
    return std::make_unique<LoopbackTransport>(std::move(world), rank);
}

namespace {

// Bootstrap-only transport of HcclAmdCommInitHostExchange: the host exchange is the caller's all-gather; there is
// no send/recv data path (the IPC AllReduce moves the data itself).
class HostExchangeTransport : public Transport {
public:
    HostExchangeTransport(HcclAmdHostAllGatherFn fn, void* ctx) : fn_(fn), ctx_(ctx) {}
    const char* Name() const override { return "host-exchange"; }
    bool HasSendRecv() const override { return false; }
    HcclResult Group(const std::vector<P2pOp>&, hipStream_t) override
    {
        HCCL_AMD_ERR("host-exchange communicator has no send/recv path (only the IPC AllReduce)");
        return HCCL_E_NOT_SUPPORT;
    }
    HcclResult AllGatherHost(const void* mine, size_t bytes, void* all) override
    {
        return fn_(ctx_, mine, bytes, all) == 0 ? HCCL_SUCCESS : HCCL_E_INTERNAL;
    }

private:
    HcclAmdHostAllGatherFn fn_;
    void* ctx_;
};

}  // namespace

std::unique_ptr<Transport> MakeHostExchangeTransport(HcclAmdHostAllGatherFn fn, void* ctx)
{
    return std::make_unique<HostExchangeTransport>(fn, ctx);
}

}  // namespace hccl_amd
