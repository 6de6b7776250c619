// comm.h — communicator, transports and executor of libhccl_amd.so.
//
// HcclComm (opaque in include/hccl_types.h) is a Comm*. One Comm per rank and device, like the reference's
// communicator (SURVEY.md §8b "Threading"). Its resources mirror what the reference's op layer allocates per
// communicator (op_common.cc:1203 HcclGetAlgRes): a staging "CCL buffer" (aiv_defines.h:44, 200 MiB there),
// helper streams (the reference's slave "threads") and events (its notifies).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "config.h"
#include "internal.h"
#include "ipc.h"
#include "schedule.h"

namespace hccl_amd {

struct P2pOp {
    bool isSend;
    uint32_t peer;
    void* ptr;
    uint64_t bytes;
};

// Posts one group of sends and receives on `stream`. The group is complete (in stream order) when every send's
// source may be overwritten and every receive's destination holds the data.
class Transport {
public:
    virtual ~Transport() = default;
    virtual HcclResult Group(const std::vector<P2pOp>& ops, hipStream_t stream) = 0;
    virtual const char* Name() const = 0;
    // Blocking all-gather of `bytes` host bytes per rank into all[nRanks * bytes] (setup and rendezvous only).
    virtual HcclResult AllGatherHost(const void* mine, size_t bytes, void* all) = 0;
    // True when every rank lives in this process on this device (loopback world).
    virtual bool SharedDevice() const { return false; }
    // False for a bootstrap-only transport: the communicator's only data path is the one-sided IPC kernel.
    virtual bool HasSendRecv() const { return true; }
    // An asynchronous failure of the transport (RCCL: ncclCommGetAsyncError), HCCL_SUCCESS if none. Non-blocking and
    // callable from any thread.
    virtual HcclResult AsyncError() { return HCCL_SUCCESS; }
    // True when a lost peer can leave this transport's device work waiting forever (RCCL): such a communicator keeps a
    // watchdog (Watchdog) that aborts it past HCCL_EXEC_TIMEOUT.
    virtual bool Abortable() const { return false; }
    // ncclCommAbort: in-flight device work returns, later groups fail. Callable from any thread.
    virtual void Abort() {}
    // on: the teardown will run later, on one rank alone (a destroy deferred behind live graphs), and must not wait on
    // peers (RCCL: abort instead of finalize); off: it runs now, with its peers (the deferral fell through).
    virtual void SetLocalTeardown(bool on) {}
    // Loopback world: the pinned failure word all its ranks share (the world's single IPC launch writes it), owned by
    // the world so that it outlives every rank's communicator; *dev receives its device address. nullptr elsewhere.
    virtual uint32_t* SharedFailWord(uint32_t** dev)
    {
        *dev = nullptr;
        return nullptr;
    }
};

std::unique_ptr<Transport> MakeRcclTransport(void* uniqueId, uint32_t nRanks, uint32_t rank, HcclResult* err);
// A one-rank RCCL communicator standing in for every peer of a larger world (HcclAmdCommInitSelfLoop): each group's
// sends are posted beside receives of the same size.
std::unique_ptr<Transport> MakeRcclSelfLoopTransport(HcclResult* err);
// One RCCL communicator per listed device, all in this process (ncclCommInitAll); (*out)[r] is rank r.
HcclResult MakeRcclTransportsAll(uint32_t ndev, const int32_t* devices, std::vector<std::unique_ptr<Transport>>* out);
HcclResult RcclGetUniqueId(void* id128);
// RCCL's per-peer p2p channels, set in the environment when the library is loaded (comm.cc).
void RcclP2pChannels(uint32_t* perPeer, uint32_t* minP2p);

class LoopbackWorld;
std::unique_ptr<Transport> MakeLoopbackTransport(std::shared_ptr<LoopbackWorld> world, uint32_t rank);
std::shared_ptr<LoopbackWorld> MakeLoopbackWorld(uint32_t nRanks);
std::unique_ptr<Transport> MakeHostExchangeTransport(HcclAmdHostAllGatherFn fn, void* ctx);

// The executor's units for one rank's IR (Execute issues exactly these): a transport group (link stream 0) or a
// batch of folds / a copy (reduce stream 1), each with the unit of the other stream it must wait for (the latest whose
// byte ranges conflict with it, RAW / WAR / WAW on absolute addresses), or -1.
struct UnitPlan {
    int stream = 0;
    bool isComm = false;
    size_t first = 0;  // IR records [first, first + count)
    size_t count = 0;
    int64_t waitUnit = -1;
    bool waitedOn = false;  // a later unit waits for this one: Execute records an event after it (no one else's)
};

// One rank's compiled collective: the schedule for a set of ScheduleParams and the executor's plan for it. The plan
// depends on the buffers only through how they overlap (conflicts compare absolute addresses, and a translation of
// one buffer changes nothing while it stays clear of the others), so it is kept with the overlap relation it was
// made for and rebuilt only when a call's relation differs (an in-place call after out-of-place ones).
struct CompiledSchedule {
    ScheduleParams params;
    Schedule sched;
    uint64_t extent[3] = {0, 0, 0};  // bytes of {sendBuf, recvBuf, scratch} the IR addresses
    uint32_t groups = 0;             // transport groups of the program
    int64_t relation[3] = {0, 0, 0};  // pairs (0,1), (0,2), (1,2): kDisjoint or the base difference
    bool hasPlan = false;
    std::vector<UnitPlan> plan;
    uint64_t lastUse = 0;
};

// One rank's executor program captured into a HIP graph for exact buffers, stream, dtype and op (RunCompiled).
struct GraphEntry {
    ScheduleParams params;
    void* bufs[3] = {nullptr, nullptr, nullptr};
    hipStream_t stream = nullptr;
    HcclDataType dt = HCCL_DATA_TYPE_RESERVED;
    HcclReduceOp op = HCCL_REDUCE_RESERVED;
    bool single = false;            // a single-stream program (Execute's singleStream)
    bool tried = false;             // the capture was attempted (the key's second call)
    hipGraphExec_t exec = nullptr;  // nullptr: not captured (first call) or the capture failed: run eagerly
    uint64_t lastUse = 0;
};

// An evicted executor graph, destroyed once `done` (recorded after its last possible launch) has completed.
struct RetiredGraph {
    hipGraphExec_t exec;
    hipEvent_t done;
};

struct Comm;

// HCCL_EXEC_TIMEOUT for the RCCL path in ms (0 = never; default 1836 s), and the bound of communicator set-up
// (HCCL_CONNECT_TIMEOUT + 20 s); watchdog.cc.
uint64_t RcclExecTimeoutMs();
uint64_t ConnectTimeoutMs();

// The execution bound of a communicator whose transport is Abortable (watchdog.cc has the contract). Begin enqueues
// a start stamp on the caller's stream before the collective's work (or, for a small single-stream program, lets the
// start be inferred), Commit a completion stamp after it: device stores of the call's sequence number into a pinned
// host ring (k_stamp), which the watchdog thread reads with plain loads (it makes no HIP call, so it can never
// disturb another thread's stream capture). Past the bound between the two, it aborts.
class Watchdog {
public:
    struct Ticket {
        uint64_t seq = 0;
        hipStream_t stream = nullptr;
        bool stamped = false;
    };
    static constexpr uint64_t kSlots = 4096;  // collectives in flight per communicator that the watchdog follows
    Watchdog(Comm* c, uint64_t boundMs);
    ~Watchdog();
    Watchdog(const Watchdog&) = delete;
    Watchdog& operator=(const Watchdog&) = delete;
    HcclResult Init();
    // stampStart = false: no start stamp; the collective counts as started once every earlier watched collective of
    // the communicator has completed (at once if none is outstanding).
    HcclResult Begin(hipStream_t s, Ticket* t, bool stampStart = true);
    void Commit(Ticket* t);

private:
    struct Slot {
        uint64_t start;
        uint64_t done;
    };
    struct Entry {
        uint64_t seq;
        bool stamped;  // a start stamp was enqueued
        bool started;
        std::chrono::steady_clock::time_point t0;
    };
    void Run();
    void Fire(HcclResult why);
    Comm* c_;
    uint64_t boundMs_;
    volatile Slot* host_ = nullptr;  // pinned, coherent: written by the device, read by the watchdog
    Slot* dev_ = nullptr;
    uint64_t nextSeq_ = 0;  // under Comm::mu (Begin is called inside a collective entry)
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Entry> pending_;
    bool stop_ = false;
    bool fired_ = false;
    std::thread th_;
};

// Brackets one collective's work with the watchdog's events (nothing when wd is null or the stream is capturing).
class WatchScope {
public:
    WatchScope(Watchdog* wd, hipStream_t s, bool stampStart = true) : wd_(wd)
    {
        if (wd_ != nullptr && wd_->Begin(s, &t_, stampStart) != HCCL_SUCCESS) wd_ = nullptr;
    }
    ~WatchScope()
    {
        if (wd_ != nullptr) wd_->Commit(&t_);
    }
    WatchScope(const WatchScope&) = delete;
    WatchScope& operator=(const WatchScope&) = delete;

private:
    Watchdog* wd_;
    Watchdog::Ticket t_;
};

struct Comm {
    uint32_t magic = 0x48434C41;  // "HCLA"
    uint32_t rank = 0;
    uint32_t nRanks = 1;
    int device = 0;
    CommConfig cfg;  // the environment at creation (config.h); HcclAmdCommSetConfig changes it under mu
    std::unique_ptr<Transport> transport;
    hipStream_t commStream = nullptr;
    hipStream_t reduceStream = nullptr;
    void* scratch = nullptr;    // executor staging, nullptr until EnsureScratch
    uint64_t cclBytes = 0;      // HCCL_BUFFSIZE: sizes the executor loops (ScheduleParams::cclBytes)
    uint64_t scratchBytes = 0;  // 2 x cclBytes (the staging's size once allocated)
    int32_t algoOverride = HCCL_AMD_ALGO_AUTO;
    uint64_t pieceBytes = 0;
    int32_t lastAlgo = -1;
    std::mutex mu;  // one collective at a time per communicator

    // event pool, recycled per collective
    std::vector<hipEvent_t> events;
    size_t nextEvent = 0;

    IpcState ipc;  // one-sided AllReduce path, set up on first use (collectively)
    uint32_t ipcBlocks = 0;  // workgroups per IPC launch, 0 = DefaultIpcBlocks(bytes) (HcclAmdCommSetIpcBlocks)

    // Failure state. Work is stream-ordered and asynchronous, so a failure (an IPC barrier timeout, an RCCL async
    // error) surfaces after the call that enqueued it has returned: the first collective entry that sees it returns
    // the error itself (HCCL_E_TIMEOUT for a barrier timeout) and marks the communicator failed; every later entry
    // returns HCCL_E_SUSPENDING, the reference's status gate (Selector, src/ops/op_common/op_common.cc:89-97: a
    // communicator whose status is not READY). HcclGetCommAsyncError reports the error without changing state.
    // failCode and failWord are read without the lock (HcclGetCommAsyncError is polled by watchdog threads while
    // another thread may sit in a collective).
    bool failed = false;
    std::atomic<int32_t> failCode{HCCL_SUCCESS};
    std::atomic<const volatile uint32_t*> failWord{nullptr};  // the pinned word the IPC launches set on a timeout
    std::unique_ptr<Watchdog> watchdog;  // RCCL transports: the execution bound (watchdog.cc)

    // Graphs captured on this communicator that are still alive (NoteCapture); HcclCommDestroy defers the teardown
    // until they are gone (DeferDestroy).
    std::atomic<int32_t> graphRefs{0};
    bool ipcQuiesced = false;  // the IPC teardown rendezvous already ran (at HcclCommDestroy of a deferred destroy)
    unsigned long long lastCaptureId = 0;

    // Fault injection for the timeout tests (HCCL_AMD_INJECT_STALL_GROUP=k): before the k-th transport group the link
    // stream runs a kernel that waits on this pinned word, as an RCCL kernel waits for a lost peer's message. The
    // watchdog's abort sets the word; the kernel also gives up by itself after a minute.
    uint64_t stallAtGroup = 0;
    uint64_t groupsPosted = 0;
    uint32_t* stallHost = nullptr;
    uint32_t* stallDev = nullptr;

    // Compiled collectives, least recently used evicted (a training loop repeats the same few bucket calls: they skip
    // BuildSchedule and PlanUnits after the first). HCCL_AMD_PLAN_CACHE=0 compiles every call.
    std::vector<std::unique_ptr<CompiledSchedule>> compiled;
    uint64_t compileTick = 0;
    uint64_t compileHits = 0;
    uint64_t compileMisses = 0;

    // Executor graphs (RunCompiled): the two-stream programs of the RCCL path, captured once on a private stream and
    // replayed with one hipGraphLaunch per call. graphLaunches / graphCaptures count them (HcclAmdCommGraphStats).
    std::vector<GraphEntry> graphs;
    std::vector<RetiredGraph> retiredGraphs;
    hipStream_t captureStream = nullptr;
    uint64_t graphLaunches = 0;
    uint64_t graphCaptures = 0;

    // Fold timing (CommConfig::foldTiming, HCCL_AMD_FOLD_TIMING; diagnostics of the fold's operating point inside a
    // program, bench.py's fold_piece row): the last eager Execute's fold launches, each bracketed by timing events on
    // its stream, with their algorithmic bytes, and the program's span on the caller's stream (HcclAmdCommFoldTiming).
    struct FoldTiming {
        std::vector<hipEvent_t> pool;  // timing-enabled, reused call after call
        size_t next = 0;
        std::vector<std::pair<hipEvent_t, hipEvent_t>> folds;
        std::vector<uint64_t> bytes;
        hipEvent_t spanStart = nullptr;
        hipEvent_t spanEnd = nullptr;
        HcclResult Next(hipEvent_t* e);
    } foldTiming;

    // The end of the last collective on its user stream: a call on another stream waits for it first, since every
    // call of a communicator shares its staging (OrderAfterTail / MarkTail).
    hipEvent_t tail = nullptr;
    hipStream_t tailStream = nullptr;

    HcclResult Init(int dev);
    // The executor's staging (2 x HCCL_BUFFSIZE), allocated by the first schedule program that runs: a communicator
    // whose calls all go to the one-sided kernel never holds it.
    HcclResult EnsureScratch();
    // Device bytes the library holds for this communicator now (executor staging + the IPC path's allocations; RCCL's
    // own buffers are not counted). HcclAmdCommDeviceBytes.
    uint64_t DeviceBytes() const;
    // After the transport is set: the watchdog for an Abortable transport and the fault-injection hook.
    HcclResult StartWatchdog();
    HcclResult NextEvent(hipEvent_t* e);
    // Non-blocking, lock-free: the first asynchronous error seen on this communicator, HCCL_SUCCESS if none.
    HcclResult PollAsyncError();
    // Entry gate of every collective (call with mu held).
    HcclResult Gate();
    ~Comm();
};

// One-sided AllReduce / ReduceScatter / Reduce over peer-mapped staging, any buffer alignment. `family` is the schedule
// family whose order the folds follow: AllReduce one-shot (O1) / two-shot (O2) / MeshChunk (O6), ReduceScatter mesh
// (O1) / MeshChunk (O6), Reduce one-shot (O1, root first) / two-shot (O1, owner first). Returns HCCL_E_NOT_SUPPORT,
// on every rank alike, when the peer mappings cannot be set up (the caller then runs the RCCL schedule of the same
// family).
HcclResult RunIpcCollective(Comm& c, int32_t opType, int32_t family, const void* sendBuf, void* recvBuf,
                            uint64_t count, HcclDataType dt, HcclReduceOp op, uint32_t root, hipStream_t stream);
// The same for an explicit plan (the AIV engine's variants, SelectAivPlan).
// vCounts / vDispls (kIpcGeomV, ReduceScatterV): every rank's block, as the caller passed them (equal on all ranks).
HcclResult RunIpcPlan(Comm& c, int32_t opType, const IpcPlan& plan, const void* sendBuf, void* recvBuf, uint64_t count,
                      HcclDataType dt, HcclReduceOp op, uint32_t root, hipStream_t stream,
                      const uint64_t* vCounts = nullptr, const uint64_t* vDispls = nullptr);
HcclResult IpcPlanRhd(uint32_t n, IpcPlan* pl);
HcclResult IpcPlanForFamily(int32_t opType, int32_t family, uint32_t n, uint64_t es, uint64_t cclBytes, IpcPlan* pl);

// The reference's AIV engine (HCCL_OP_EXPANSION_MODE=AIV): SelectAivAlgo's rules and the variant its kernel takes
// for the vector-core count `coreLimit` (aivCoreLimit / the device's vector cores). Returns the variant
// (HcclAmdAivVariant, include/hccl_amd.h), HCCL_AMD_AIV_NOT_MATCHED when the selector would fall back to the AICPU
// engine; *plan receives the one-sided kernel's plan for a matched variant.
int32_t SelectAivPlan(int32_t opType, uint32_t n, uint64_t count, HcclDataType dt, HcclReduceOp op, bool strict,
                      bool aivOnly, uint64_t cclBytes, uint32_t coreLimit, IpcPlan* plan, uint32_t* group);
// Collective: every rank's IPC kernels have finished before any rank unmaps or frees (called by ~Comm).
void IpcQuiesce(Comm& c);
void IpcRelease(Comm& c);
// The area sizes of staging tier t (kIpcTierSmall / kIpcTierLarge) for c: a function of the rank count and the (=)
// configuration, so equal on every rank. IpcDeviceBytes: the device bytes c's IPC path holds now.
IpcTier IpcTierSizes(const Comm& c, int t);
uint64_t IpcDeviceBytes(const Comm& c);
// The process's idle uncached blocks of the IPC path (kept for reuse by later communicators), in bytes
// (HcclAmdIpcIdleStaging).
uint64_t IpcIdleBytes();

Comm* AsComm(HcclComm c);

// Called at every collective entry with the caller's stream: under capture, counts the capturing graph against the
// communicator until the graph is destroyed (once per capture).
HcclResult NoteCapture(Comm& c, hipStream_t s);
// HcclCommDestroy while graphs hold the communicator: queue it for the reaper thread and return true.
bool DeferDestroy(Comm* c);
uint32_t PendingDestroys();
// HCCL_AMD_TEARDOWN_TRACE=1: time-stamped steps of ~Comm on stderr.
void TeardownTrace(uint32_t rank, const char* step, bool begin);
// The watchdog's stamp and the injected stall (watch_kernels.hip).
HcclResult LaunchStamp(uint64_t* slot, uint64_t seq, hipStream_t stream);
HcclResult LaunchStall(const uint32_t* word, uint64_t maxMs, hipStream_t stream);

// HCCL_BUFFSIZE (MB, default 200) in bytes; staging per communicator is twice that. Must be equal on every rank: the
// executor loops and the pipelining granule are derived from it.
uint64_t CclBytesDefault();
uint64_t ScratchBytesDefault();

// Runs one rank's schedule. bufs = {sendBuf, recvBuf, scratch}. Stream-ordered after `user`; `user` waits for the
// whole schedule before anything enqueued later on it runs. singleStream puts every unit on `user` in program order.
// plan = PlanUnits(ops, bufs, es) if the caller has it (CompileCollective), else nullptr.
HcclResult Execute(Comm& c, const std::vector<HcclAmdIrOp>& ops, void* const bufs[3], HcclDataType dt,
                   HcclReduceOp op, hipStream_t user, bool singleStream = false,
                   const std::vector<UnitPlan>* plan = nullptr);

std::vector<UnitPlan> PlanUnits(const std::vector<HcclAmdIrOp>& ops, void* const bufs[3], uint64_t es);

// Runs a compiled collective (the two-stream program, or with `single` the single-stream one): from the communicator's
// graph cache when the transport allows capture (RCCL) and HCCL_AMD_GRAPH_CACHE is not 0 (the first run of a compiled
// collective is eager, later ones with the same buffers, stream, dtype, op and mode replay one captured graph), else
// through Execute.
HcclResult RunCompiled(Comm& c, const CompiledSchedule& cs, void* const bufs[3], HcclDataType dt, HcclReduceOp op,
                       hipStream_t user, bool single = false);
void ReleaseGraphs(Comm& c);

// Entry/exit of every collective: under the caller's capture, NoteCapture; otherwise wait for the previous call's end
// when it ran on another stream, and record this call's end.
class EntryScope {
public:
    EntryScope(Comm& c, hipStream_t s);
    ~EntryScope();
    HcclResult status() const { return status_; }
    bool captured() const { return captured_; }
    EntryScope(const EntryScope&) = delete;
    EntryScope& operator=(const EntryScope&) = delete;

private:
    Comm& c_;
    hipStream_t s_;
    bool captured_ = false;
    HcclResult status_ = HCCL_SUCCESS;
};

// The compiled form of p for the buffers bufs (cached on c; call with c.mu held): BuildSchedule's result and, when
// withPlan, the plan for the buffers' overlap relation. The pointer stays valid until the next call on c.
HcclResult CompileCollective(Comm& c, const ScheduleParams& p, void* const bufs[3], bool withPlan,
                             const CompiledSchedule** out);
// The same for an IR program handed in whole (HcclAmdCommExecute), keyed by its records; always with its plan.
constexpr int32_t kProgramOpType = -1;
HcclResult CompileProgram(Comm& c, const HcclAmdIrOp* ops, uint64_t numOps, uint32_t elemSize, void* const bufs[3],
                          const CompiledSchedule** out);

}  // namespace hccl_amd
