// watchdog.cc — the execution bound of the RCCL path, graph references of a communicator, deferred destroy.
//
// The reference bounds every handshake wait of its write/read-reduce steps by HCCL_EXEC_TIMEOUT
// (HcommChannelNotifyWaitOnThread(..., execTimeout), alg_data_trans_wrapper.cc:258-268, 284-286; the bound from
// ExecTimeoutManager, exec_timeout_manager.cc:30-44, default CUSTOM_TIMEOUT = 1836 s, alg_param.h:79), and a failed
// communicator takes no more work (Selector, op_common.cc:89-97). On this path the waits are inside RCCL's send/recv
// kernels, which poll until the peer's matching message arrives. A communicator therefore keeps a watchdog thread:
//   * every collective it runs outside stream capture is bracketed by two device-written stamps on the caller's
//     stream (k_stamp stores into a pinned host ring), which the thread reads with plain loads: it makes no HIP
//     call, so it cannot invalidate a stream capture running on another thread (an earlier version polled events with
//     hipEventQuery, and HIP failed a concurrent torch.cuda.graph capture on it even in the relaxed capture mode);
//   * once the start stamp has landed (the collective's work has started on the GPU), the completion stamp must land
//     within the bound; the thread also polls ncclCommGetAsyncError. A small single-stream program (<= 1 MiB) has no
//     start stamp (each stamp costs about 1.8 us of GPU time): it counts as started once every earlier watched
//     collective of the communicator has completed, so user work queued between two collectives on a stream counts
//     against the later one's bound;
//   * past the bound, or on an asynchronous RCCL error, it records the error (HcclGetCommAsyncError reports it at
//     once), calls ncclCommAbort (RCCL's kernels poll the abort flag and return), and the communicator is failed:
//     the next collective entry returns the error (HCCL_E_TIMEOUT), every later one HCCL_E_SUSPENDING (Comm::Gate).
// This is the contract the one-sided IPC kernel already has with its in-kernel bound (ipc.cc IpcTimeoutTicks).
//
// Graph references. A HIP graph captured on a communicator's collective holds the communicator's staging, streams
// and RCCL plans. RCCL's ncclCommDestroy waits until every graph holding one of its plans is destroyed, so destroying
// a communicator while such a graph is alive did not return. Each capture now
// retains a HIP user object on the capturing graph that counts the graph against the communicator, and
// HcclCommDestroy of a communicator with live graphs returns at once: the teardown runs on a reaper thread when the
// last such graph is destroyed (and never, if the process exits first).
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

#include "comm.h"

namespace hccl_amd {

namespace {

using Clock = std::chrono::steady_clock;

// Non-negative integer from the environment, or dflt when unset / malformed.
bool EnvMs(const char* name, uint64_t lo, uint64_t hi, uint64_t* out)
{
    const char* e = std::getenv(name);
    if (e == nullptr || *e == '\0') return false;
    char* end = nullptr;
    const unsigned long long v = std::strtoull(e, &end, 10);
    if (end == e || *end != '\0' || v < lo || v > hi) return false;
    *out = v;
    return true;
}

bool EnvFlag(const char* name, bool dflt)
{
    const char* e = std::getenv(name);
    if (e == nullptr || *e == '\0') return dflt;
    return std::strcmp(e, "0") != 0;
}

}  // namespace

uint64_t RcclExecTimeoutMs()
{
    // HCCL_EXEC_TIMEOUT in the reference's AI_CPU-mode rule (docs/zh/user_guide/hccl_env/HCCL_EXEC_TIMEOUT.md:
    // seconds, [0, 2147483647], default 1836, 0 = never), parsed with ParseExecTimeout's format check
    // (alg_env_config.cc:43-110). HCCL_AMD_EXEC_TIMEOUT_MS (0 .. 2^40) overrides it for tests.
    uint64_t ms = 0;
    if (EnvMs("HCCL_AMD_EXEC_TIMEOUT_MS", 0, 1ull << 40, &ms)) return ms;
    double sec = 0;
    if (ParseExecTimeoutSeconds(std::getenv("HCCL_EXEC_TIMEOUT"), &sec) && sec <= 2147483647.0) {
        return sec == 0 ? 0 : std::max<uint64_t>(1, static_cast<uint64_t>(sec * 1000.0 + 0.5));
    }
    return 1836ull * 1000;
}

uint64_t ConnectTimeoutMs()
{
    // HCCL_CONNECT_TIMEOUT (docs/zh/user_guide/hccl_env/HCCL_CONNECT_TIMEOUT.md: seconds, [120, 7200], default 120)
    // plus 20 s of slack for the slowest rank's start; HCCL_AMD_CONNECT_TIMEOUT_MS overrides it for tests.
    uint64_t ms = 0;
    if (EnvMs("HCCL_AMD_CONNECT_TIMEOUT_MS", 1, 1ull << 40, &ms)) return ms;
    uint64_t s = 120;
    (void)EnvMs("HCCL_CONNECT_TIMEOUT", 120, 7200, &s);  // out of range or malformed: the default
    return (s + 20) * 1000;
}

// ------------------------------------------------------------------------------------------------ teardown trace

bool TeardownTraceEnabled()
{
    static const bool on = EnvFlag("HCCL_AMD_TEARDOWN_TRACE", false);
    return on;
}

void TeardownTrace(uint32_t rank, const char* step, bool begin)
{
    if (!TeardownTraceEnabled()) return;
    static const Clock::time_point t0 = Clock::now();
    const double ms = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    std::fprintf(stderr, "[hccl_amd] teardown rank %u: %-26s %-5s +%.3f ms\n", rank, step, begin ? "begin" : "end",
                 ms);
    std::fflush(stderr);
}

// ------------------------------------------------------------------------------------------------ watchdog

Watchdog::Watchdog(Comm* c, uint64_t boundMs) : c_(c), boundMs_(boundMs) {}

HcclResult Watchdog::Init()
{
    void* h = nullptr;
    HIP_CHK(hipHostMalloc(&h, kSlots * sizeof(Slot), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(h, 0, kSlots * sizeof(Slot));
    host_ = static_cast<volatile Slot*>(h);
    HIP_CHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev_), h, 0));
    th_ = std::thread([this] { Run(); });
    return HCCL_SUCCESS;
}

Watchdog::~Watchdog()
{
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
    if (host_ != nullptr) (void)hipHostFree(const_cast<Slot*>(host_));
}

HcclResult Watchdog::Begin(hipStream_t s, Ticket* t, bool stampStart)
{
    const uint64_t seq = ++nextSeq_;
    volatile Slot& slot = host_[seq % kSlots];
    {
        // a slot still in flight kSlots calls later: this call goes unwatched rather than overwrite it
        std::lock_guard<std::mutex> lk(mu_);
        if (!pending_.empty() && seq - pending_.front().seq >= kSlots) return HCCL_E_AGAIN;
    }
    slot.start = 0;
    slot.done = 0;
    if (stampStart) HCCL_CHK(LaunchStamp(&dev_[seq % kSlots].start, seq, s));
    t->seq = seq;
    t->stream = s;
    t->stamped = stampStart;
    return HCCL_SUCCESS;
}

void Watchdog::Commit(Ticket* t)
{
    if (t->stream == nullptr) return;
    if (LaunchStamp(&dev_[t->seq % kSlots].done, t->seq, t->stream) != HCCL_SUCCESS) {
        HCCL_AMD_ERR("rank %u: watchdog could not enqueue a completion stamp", c_->rank);
        t->stream = nullptr;
        return;
    }
    std::lock_guard<std::mutex> lk(mu_);
    pending_.push_back({t->seq, t->stamped, false, {}});
    t->stream = nullptr;
}

// A helper thread's HIP calls (event queries, teardown) must not invalidate a stream capture another thread runs in
// the global capture mode (torch's default): this thread is put in the relaxed mode.
void RelaxCaptureMode()
{
    hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&m);
}

void Watchdog::Run()
{
    RelaxCaptureMode();  // Fire's abort makes HIP calls from this thread
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
        // a 10 ms poll: no wake-up is paid per collective, and the bound is seconds
        cv_.wait_for(lk, std::chrono::milliseconds(10), [&] { return stop_; });
        if (stop_) break;
        const Clock::time_point now = Clock::now();
        bool overdue = false;
        for (size_t i = 0; i < pending_.size();) {
            Entry& e = pending_[i];
            volatile Slot& slot = host_[e.seq % kSlots];
            if (slot.done == e.seq) {
                pending_.erase(pending_.begin() + static_cast<std::ptrdiff_t>(i));
                continue;
            }
            // started: its start stamp landed, or (no start stamp) every earlier watched collective has completed
            if (!e.started && (e.stamped ? slot.start == e.seq : i == 0)) {
                e.started = true;
                e.t0 = now;
            }
            if (e.started && !fired_ && boundMs_ != 0 &&
                std::chrono::duration_cast<std::chrono::milliseconds>(now - e.t0).count() >
                    static_cast<int64_t>(boundMs_)) {
                overdue = true;
            }
            ++i;
        }
        if (fired_) continue;  // keep draining the entries as the aborted work ends
        HcclResult why = HCCL_SUCCESS;
        if (overdue) {
            why = HCCL_E_TIMEOUT;
        } else if (!pending_.empty()) {
            why = c_->transport != nullptr ? c_->transport->AsyncError() : HCCL_SUCCESS;
        }
        if (why == HCCL_SUCCESS) continue;
        fired_ = true;
        lk.unlock();
        Fire(why);
        lk.lock();
    }
}

void Watchdog::Fire(HcclResult why)
{
    int32_t expected = HCCL_SUCCESS;
    c_->failCode.compare_exchange_strong(expected, why, std::memory_order_acq_rel);
    if (why == HCCL_E_TIMEOUT) {
        HCCL_AMD_ERR("rank %u: a collective ran past HCCL_EXEC_TIMEOUT (%llu ms): aborting the RCCL communicator; "
                     "the next collective returns HCCL_E_TIMEOUT, later ones HCCL_E_SUSPENDING",
                     c_->rank, (unsigned long long)boundMs_);
    } else {
        HCCL_AMD_ERR("rank %u: RCCL reported an asynchronous error (%s): aborting the communicator", c_->rank,
                     HcclAmdGetErrorString(why));
    }
    // The injected stall (HCCL_AMD_INJECT_STALL_GROUP) stands for an RCCL kernel waiting on a lost peer: it returns
    // on the abort as RCCL's kernels do on their abort flag. It is released first, so that the RCCL kernels queued
    // behind it have run before RCCL reclaims the communicator.
    if (c_->stallHost != nullptr) __atomic_store_n(c_->stallHost, 1u, __ATOMIC_RELEASE);
    if (c_->transport != nullptr) c_->transport->Abort();
}

// ------------------------------------------------------------------------------------------------ graph references

namespace {

// Communicators whose HcclCommDestroy came while graphs captured on them were alive: torn down by the reaper thread
// once their last graph is destroyed. Allocated once and never freed (a graph may outlive main()).
struct Reaper {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Comm*> pending;
    uint32_t active = 0;  // teardowns in progress on the reaper thread
    bool started = false;
};

Reaper& TheReaper()
{
    static Reaper* r = new Reaper();
    return *r;
}

struct GraphRef {
    Comm* comm;
};

// The user object's destructor: runs on a HIP-internal thread when the graph (and every executable instantiated from
// it) is destroyed. No HIP call may be made here; it only counts down and wakes the reaper.
void ReleaseGraphRef(void* p)
{
    GraphRef* ref = static_cast<GraphRef*>(p);
    Reaper& r = TheReaper();
    {
        std::lock_guard<std::mutex> lk(r.mu);
        ref->comm->graphRefs.fetch_sub(1, std::memory_order_acq_rel);
    }
    r.cv.notify_all();
    delete ref;
}

void ReaperLoop()
{
    RelaxCaptureMode();
    Reaper& r = TheReaper();
    std::unique_lock<std::mutex> lk(r.mu);
    for (;;) {
        r.cv.wait(lk, [&] {
            for (Comm* c : r.pending) {
                if (c->graphRefs.load(std::memory_order_acquire) == 0) return true;
            }
            return false;
        });
        for (size_t i = 0; i < r.pending.size();) {
            Comm* c = r.pending[i];
            if (c->graphRefs.load(std::memory_order_acquire) != 0) {
                ++i;
                continue;
            }
            r.pending.erase(r.pending.begin() + static_cast<std::ptrdiff_t>(i));
            ++r.active;
            lk.unlock();
            TeardownTrace(c->rank, "deferred destroy (reaper)", true);
            delete c;
            lk.lock();
            --r.active;
            r.cv.notify_all();
        }
    }
}

}  // namespace

HcclResult NoteCapture(Comm& c, hipStream_t s)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    HIP_CHK(hipStreamGetCaptureInfo_v2(s, &st, &id, &g, nullptr, nullptr));
    if (st != hipStreamCaptureStatusActive || g == nullptr || id == c.lastCaptureId) return HCCL_SUCCESS;
    GraphRef* ref = new GraphRef{&c};
    hipUserObject_t obj = nullptr;
    if (hipUserObjectCreate(&obj, ref, ReleaseGraphRef, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
        delete ref;
        HCCL_AMD_ERR("rank %u: hipUserObjectCreate failed", c.rank);
        return HCCL_E_RUNTIME;
    }
    c.graphRefs.fetch_add(1, std::memory_order_acq_rel);
    if (hipGraphRetainUserObject(g, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
        (void)hipUserObjectRelease(obj, 1);  // runs ReleaseGraphRef: the count goes back
        HCCL_AMD_ERR("rank %u: hipGraphRetainUserObject failed", c.rank);
        return HCCL_E_RUNTIME;
    }
    c.lastCaptureId = id;
    return HCCL_SUCCESS;
}

// At process exit, a teardown the reaper has begun is let finish (bounded): exiting under it races RCCL's own
// teardown. Communicators still held by live graphs are left as they are.
void WaitForReaperAtExit()
{
    Reaper& r = TheReaper();
    std::unique_lock<std::mutex> lk(r.mu);
    r.cv.wait_for(lk, std::chrono::seconds(10), [&] { return r.active == 0; });
}

bool DeferDestroy(Comm* c)
{
    if (c->graphRefs.load(std::memory_order_acquire) == 0) return false;
    // The collective steps of the teardown run now, on this rank's destroy, as on every peer's: the IPC
    // rendezvous (after it no peer stores into this rank's staging, nor this rank into theirs), and the transport is
    // told that its own teardown, later and alone, must not wait on peers. Only the local frees the live graphs
    // depend on are deferred. (A graph replayed after its communicator's destroy is the caller's error.)
    TeardownTrace(c->rank, "IPC quiesce (destroy time)", true);
    IpcQuiesce(*c);
    if (c->transport != nullptr) c->transport->SetLocalTeardown(true);
    Reaper& r = TheReaper();
    std::lock_guard<std::mutex> lk(r.mu);
    if (c->graphRefs.load(std::memory_order_acquire) == 0) {
        // the last graph went meanwhile: the teardown runs now, on the caller's thread, and may still flush this
        // rank's outstanding work with its peers (bounded finalize), so the local-only flag is withdrawn
        if (c->transport != nullptr) c->transport->SetLocalTeardown(false);
        return false;
    }
    TeardownTrace(c->rank, "destroy deferred (graphs)", true);
    r.pending.push_back(c);
    if (!r.started) {
        r.started = true;
        std::thread(ReaperLoop).detach();
        std::atexit(WaitForReaperAtExit);
    }
    r.cv.notify_all();
    return true;
}

uint32_t PendingDestroys()
{
    Reaper& r = TheReaper();
    std::lock_guard<std::mutex> lk(r.mu);
    return static_cast<uint32_t>(r.pending.size()) + r.active;
}

}  // namespace hccl_amd

extern "C" uint32_t HcclAmdCommPendingDestroys(void) { return hccl_amd::PendingDestroys(); }
