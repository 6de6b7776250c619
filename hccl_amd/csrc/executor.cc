// executor.cc — runs one rank's schedule IR on two HIP streams.
//
// Replaces the reference's per-step orchestration (executors' OrchestrateLoop + templates' KernelRun, which post
// hcomm tasks on a main "thread" and slave threads joined by notifies: alg_data_trans_wrapper.cc:1005-1073,
// SURVEY.md §8a rows R5, R8). Here:
//   * SEND/RECV records with one group id become one transport group on the link stream (RCCL over xGMI);
//   * REDUCE and COPY records go to the reduce stream (the fold kernels and the copy kernel of reduce_kernels.hip);
//   * dependencies are not written by hand: every record's byte ranges (absolute device addresses, so in-place
//     buffers alias correctly) are checked against the earlier units of the OTHER stream, and the latest
//     conflicting unit (RAW, WAR or WAW) becomes a hipStreamWaitEvent. Same-stream order is program order.
// This is the reference ST's memory-conflict rule (test/st/algorithm/.../mem_conflict_check) turned into the
// synchronisation itself. The host never blocks (except loopback rendezvous); the user stream is joined at the end.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstring>

#include "comm.h"

namespace hccl_amd {

// ------------------------------------------------------------------------------------------------ host profile

// HCCL_AMD_HOST_PROFILE=1: host time by category (HcclAmdHostProfile): the executor's parts, and whole collective
// entries and one-sided launches (ops.cc, ipc.cc), for the breakdown of the enqueue cost. Off by default: one cached
// flag test per site.
namespace {

struct HostProfile {
    std::atomic<uint64_t> ns[HCCL_AMD_HP_COUNT];
    std::atomic<uint64_t> calls[HCCL_AMD_HP_COUNT];
};

HostProfile& Hp()
{
    static HostProfile p{};
    return p;
}

using HpScope = HostProfileScope;

}  // namespace

bool HostProfileOn()
{
    static const bool on = [] {
        const char* e = std::getenv("HCCL_AMD_HOST_PROFILE");
        return e != nullptr && std::strcmp(e, "1") == 0;
    }();
    return on;
}

void HostProfileAdd(int cat, uint64_t ns)
{
    Hp().ns[cat].fetch_add(ns, std::memory_order_relaxed);
    Hp().calls[cat].fetch_add(1, std::memory_order_relaxed);
}

namespace {

struct Range {
    uintptr_t lo;
    uintptr_t hi;
    bool write;
};

bool Conflicts(const std::vector<Range>& a, const std::vector<Range>& b)
{
    for (const Range& x : a) {
        for (const Range& y : b) {
            if ((x.write || y.write) && x.lo < y.hi && y.lo < x.hi) return true;
        }
    }
    return false;
}

// Length of the run of REDUCE records starting at ops[i] that can share one batched launch: same operand count
// (>= 2), at most kMaxBatchSegs, and no record's output overlapping another record's output or inputs (the batch
// runs them concurrently). The records of one schedule step qualify: a MeshChunk piece's O6 sub-slices, the folds of
// the R rings or of the RHD instances.
size_t BatchRun(const std::vector<HcclAmdIrOp>& ops, size_t i, uint64_t es, void* const bufs[3])
{
    const HcclAmdIrOp& o = ops[i];
    if (o.kind != HCCL_AMD_IR_REDUCE || o.nsrc < 2) return 1;
    auto addr = [&](int32_t buf, uint64_t off) { return reinterpret_cast<uintptr_t>(bufs[buf]) + off * es; };
    std::vector<Range> outs, ins;
    size_t k = i;
    for (; k < ops.size() && k - i < kMaxBatchSegs; ++k) {
        const HcclAmdIrOp& q = ops[k];
        if (q.kind != HCCL_AMD_IR_REDUCE || q.nsrc != o.nsrc) break;
        const uintptr_t d = addr(q.dstBuf, q.dstOff);
        const Range dr{d, d + q.count * es, true};
        std::vector<Range> qin;
        for (int j = 0; j < q.nsrc; ++j) {
            const uintptr_t a = addr(q.srcBuf[j], q.srcOff[j]);
            qin.push_back({a, a + q.count * es, false});
        }
        bool clash = false;
        for (const Range& r : outs) clash = clash || (dr.lo < r.hi && r.lo < dr.hi);
        for (const Range& r : ins) clash = clash || (dr.lo < r.hi && r.lo < dr.hi);
        for (const Range& r : qin) {
            for (const Range& w : outs) clash = clash || (r.lo < w.hi && w.lo < r.hi);
        }
        if (clash) break;
        outs.push_back(dr);
        ins.insert(ins.end(), qin.begin(), qin.end());
    }
    return std::max<size_t>(1, k - i);
}

// Launches REDUCE records ops[i, i+m) (one batch, or a single fold when m == 1).
HcclResult LaunchFoldsRaw(const std::vector<HcclAmdIrOp>& ops, size_t i, size_t m, uint64_t es, void* const bufs[3],
                       HcclDataType dt, HcclReduceOp op, hipStream_t stream)
{
    auto addr = [&](int32_t buf, uint64_t off) { return reinterpret_cast<uintptr_t>(bufs[buf]) + off * es; };
    if (m == 1) {
        const HcclAmdIrOp& o = ops[i];
        const void* srcs[HCCL_AMD_IR_MAX_SRC];
        for (int j = 0; j < o.nsrc; ++j) srcs[j] = reinterpret_cast<const void*>(addr(o.srcBuf[j], o.srcOff[j]));
        return LaunchReduceN(reinterpret_cast<void*>(addr(o.dstBuf, o.dstOff)), srcs, static_cast<uint32_t>(o.nsrc),
                             o.count, dt, op, stream);
    }
    FoldSeg segs[kMaxBatchSegs];
    for (size_t g = 0; g < m; ++g) {
        const HcclAmdIrOp& o = ops[i + g];
        segs[g].out = reinterpret_cast<void*>(addr(o.dstBuf, o.dstOff));
        for (int j = 0; j < o.nsrc; ++j) segs[g].srcs[j] = reinterpret_cast<const void*>(addr(o.srcBuf[j], o.srcOff[j]));
        segs[g].count = o.count;
    }
    return LaunchReduceNBatch(segs, static_cast<uint32_t>(m), static_cast<uint32_t>(ops[i].nsrc), dt, op, stream);
}

// LaunchFoldsRaw, bracketed by timing events when the communicator times its folds (Comm::FoldTiming).
HcclResult LaunchFolds(Comm& c, bool timed, const std::vector<HcclAmdIrOp>& ops, size_t i, size_t m, uint64_t es,
                       void* const bufs[3], HcclDataType dt, HcclReduceOp op, hipStream_t stream)
{
    if (!timed) return LaunchFoldsRaw(ops, i, m, es, bufs, dt, op, stream);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HCCL_CHK(c.foldTiming.Next(&e0));
    HCCL_CHK(c.foldTiming.Next(&e1));
    HIP_CHK(hipEventRecord(e0, stream));
    HCCL_CHK(LaunchFoldsRaw(ops, i, m, es, bufs, dt, op, stream));
    HIP_CHK(hipEventRecord(e1, stream));
    uint64_t bytes = 0;
    for (size_t g = i; g < i + m; ++g) bytes += uint64_t(ops[g].nsrc + 1) * ops[g].count * es;
    c.foldTiming.folds.emplace_back(e0, e1);
    c.foldTiming.bytes.push_back(bytes);
    return HCCL_SUCCESS;
}

// HCCL_AMD_INJECT_STALL_GROUP=k (timeout tests): before the communicator's k-th transport group, outside capture, the
// group's stream waits on the injected stall kernel, as if the peer never posted its half of the group.
HcclResult MaybeInjectStall(Comm& c, hipStream_t s)
{
    if (c.stallAtGroup == 0 || ++c.groupsPosted != c.stallAtGroup) return HCCL_SUCCESS;
    HCCL_AMD_ERR("rank %u: injected stall before transport group %llu (HCCL_AMD_INJECT_STALL_GROUP)", c.rank,
                 (unsigned long long)c.groupsPosted);
    return LaunchStall(c.stallDev, 60000, s);
}

}  // namespace

// Small collectives have one pipeline piece, so the two-stream split cannot overlap anything: every unit goes on
// the caller's stream in program order and no event is recorded or waited on (the latency floor of C5).
static HcclResult ExecuteSingleStream(Comm& c, const std::vector<HcclAmdIrOp>& ops, void* const bufs[3],
                                      HcclDataType dt, HcclReduceOp op, hipStream_t user, bool captured, bool timed)
{
    const uint64_t es = DataTypeSize(dt);
    auto addr = [&](int32_t buf, uint64_t off) -> uintptr_t {
        return reinterpret_cast<uintptr_t>(bufs[buf]) + off * es;
    };
    std::vector<P2pOp> p2p;
    size_t i = 0;
    while (i < ops.size()) {
        const HcclAmdIrOp& o = ops[i];
        if (o.kind == HCCL_AMD_IR_SEND || o.kind == HCCL_AMD_IR_RECV) {
            p2p.clear();
            const int32_t g = o.group;
            while (i < ops.size() && (ops[i].kind == HCCL_AMD_IR_SEND || ops[i].kind == HCCL_AMD_IR_RECV) &&
                   ops[i].group == g) {
                const HcclAmdIrOp& q = ops[i];
                const bool send = q.kind == HCCL_AMD_IR_SEND;
                uintptr_t a = send ? addr(q.srcBuf[0], q.srcOff[0]) : addr(q.dstBuf, q.dstOff);
                p2p.push_back({send, static_cast<uint32_t>(q.peer), reinterpret_cast<void*>(a), q.count * es});
                ++i;
            }
            if (!captured) HCCL_CHK(MaybeInjectStall(c, user));
            HpScope hp(HCCL_AMD_HP_GROUP);
            HCCL_CHK(c.transport->Group(p2p, user));
            continue;
        }
        void* dst = reinterpret_cast<void*>(addr(o.dstBuf, o.dstOff));
        if (o.kind == HCCL_AMD_IR_COPY) {
            HpScope hp(HCCL_AMD_HP_COPY);
            const void* src = reinterpret_cast<const void*>(addr(o.srcBuf[0], o.srcOff[0]));
            HCCL_CHK(LaunchCopyBytes(dst, src, o.count * es, user));
        } else if (o.kind == HCCL_AMD_IR_REDUCE) {
            HpScope hp(HCCL_AMD_HP_FOLD);
            const size_t m = BatchRun(ops, i, es, bufs);
            HCCL_CHK(LaunchFolds(c, timed, ops, i, m, es, bufs, dt, op, user));
            i += m;
            continue;
        } else {
            return HCCL_E_INTERNAL;
        }
        ++i;
    }
    return HCCL_SUCCESS;
}

std::vector<UnitPlan> PlanUnits(const std::vector<HcclAmdIrOp>& ops, void* const bufs[3], uint64_t es)
{
    auto addr = [&](int32_t buf, uint64_t off) -> uintptr_t {
        return reinterpret_cast<uintptr_t>(bufs[buf]) + off * es;
    };
    std::vector<UnitPlan> plan;
    std::vector<std::vector<Range>> ranges;
    std::vector<size_t> onStream[2];
    // synced[x][y]: index into onStream[y] of the last unit stream x has already waited for (+1)
    size_t synced[2][2] = {{0, 0}, {0, 0}};
    size_t i = 0;
    while (i < ops.size()) {
        UnitPlan u;
        std::vector<Range> rg;
        u.first = i;
        const HcclAmdIrOp& first = ops[i];
        u.isComm = first.kind == HCCL_AMD_IR_SEND || first.kind == HCCL_AMD_IR_RECV;
        u.stream = u.isComm ? 0 : 1;
        if (u.isComm) {
            const int32_t g = first.group;
            while (i < ops.size() && (ops[i].kind == HCCL_AMD_IR_SEND || ops[i].kind == HCCL_AMD_IR_RECV) &&
                   ops[i].group == g) {
                const HcclAmdIrOp& o = ops[i];
                const uint64_t bytes = o.count * es;
                const uintptr_t a = o.kind == HCCL_AMD_IR_SEND ? addr(o.srcBuf[0], o.srcOff[0]) : addr(o.dstBuf, o.dstOff);
                rg.push_back({a, a + bytes, o.kind == HCCL_AMD_IR_RECV});
                ++i;
            }
        } else {
            const size_t batch = BatchRun(ops, i, es, bufs);
            for (size_t g = 0; g < batch; ++g) {
                const HcclAmdIrOp& o = ops[i + g];
                const uint64_t bytes = o.count * es;
                const uintptr_t d = addr(o.dstBuf, o.dstOff);
                rg.push_back({d, d + bytes, true});
                for (int j = 0; j < o.nsrc; ++j) {
                    const uintptr_t sa = addr(o.srcBuf[j], o.srcOff[j]);
                    rg.push_back({sa, sa + bytes, false});
                }
            }
            i += batch;
        }
        u.count = i - u.first;
        // cross-stream hazards: wait for the latest conflicting unit on the other stream
        const int x = u.stream;
        const int y = 1 - x;
        for (size_t k = onStream[y].size(); k > synced[x][y]; --k) {
            const size_t prior = onStream[y][k - 1];
            if (Conflicts(ranges[prior], rg)) {
                u.waitUnit = static_cast<int64_t>(prior);
                synced[x][y] = k;
                break;
            }
        }
        onStream[x].push_back(plan.size());
        if (u.waitUnit >= 0) plan[size_t(u.waitUnit)].waitedOn = true;
        plan.push_back(u);
        ranges.push_back(std::move(rg));
    }
    return plan;
}

namespace {

constexpr int64_t kDisjoint = INT64_MIN;
constexpr size_t kCompiledMax = 32;

bool SameParams(const ScheduleParams& a, const ScheduleParams& b)
{
    return a.opType == b.opType && a.algo == b.algo && a.nRanks == b.nRanks && a.rank == b.rank && a.count == b.count &&
           a.elemSize == b.elemSize && a.root == b.root && a.pieceBytes == b.pieceBytes &&
           a.scratchCapBytes == b.scratchCapBytes && a.cclBytes == b.cclBytes && a.special == b.special &&
           a.counts == b.counts && a.displs == b.displs;
}

// How the buffers of pair (x, y) lie against each other over the bytes the IR addresses: kDisjoint, or base(y) -
// base(x) when the addressed ranges overlap (every conflict test between them is then fixed by that difference).
void Relation(const uint64_t ext[3], void* const bufs[3], int64_t rel[3])
{
    static const int kPair[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    for (int k = 0; k < 3; ++k) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(bufs[kPair[k][0]]);
        const uintptr_t b = reinterpret_cast<uintptr_t>(bufs[kPair[k][1]]);
        const uint64_t ea = ext[kPair[k][0]];
        const uint64_t eb = ext[kPair[k][1]];
        const bool overlap = ea != 0 && eb != 0 && a < b + eb && b < a + ea;
        rel[k] = overlap ? static_cast<int64_t>(b - a) : kDisjoint;
    }
}

}  // namespace

namespace {

// The compiled-collective cache of c: the entry for p (a hit moves it to the front of the LRU order), else a new one
// from make(), evicting the least recently used at kCompiledMax entries.
template <class Make>
HcclResult FindOrCompile(Comm& c, const ScheduleParams& p, void* const bufs[3], bool withPlan, Make make,
                         const CompiledSchedule** out)
{
    if (!c.cfg.planCache) c.compiled.clear();  // HCCL_AMD_PLAN_CACHE=0: compile every call
    CompiledSchedule* hit = nullptr;
    for (auto& e : c.compiled) {
        if (SameParams(e->params, p)) {
            hit = e.get();
            break;
        }
    }
    if (hit == nullptr) {
        ++c.compileMisses;
        auto e = std::make_unique<CompiledSchedule>();
        e->params = p;
        HCCL_CHK(make(&e->sched));
        int32_t lastGroup = -1;
        bool inGroup = false;
        for (const HcclAmdIrOp& o : e->sched.ops) {
            const bool p2p = o.kind == HCCL_AMD_IR_SEND || o.kind == HCCL_AMD_IR_RECV;
            if (p2p && (!inGroup || o.group != lastGroup)) ++e->groups;
            inGroup = p2p;
            lastGroup = o.group;
            const uint64_t bytes = o.count * p.elemSize;
            if (o.dstBuf >= 0 && o.dstBuf < 3) {
                e->extent[o.dstBuf] = std::max(e->extent[o.dstBuf], (o.dstOff + o.count) * p.elemSize);
            }
            const int nsrc = o.kind == HCCL_AMD_IR_RECV ? 0 : std::max(0, std::min(o.nsrc, HCCL_AMD_IR_MAX_SRC));
            for (int j = 0; j < nsrc; ++j) {
                const int32_t sb = o.srcBuf[j];
                if (sb >= 0 && sb < 3) e->extent[sb] = std::max(e->extent[sb], o.srcOff[j] * p.elemSize + bytes);
            }
        }
        if (c.compiled.size() >= kCompiledMax) {
            auto lru = std::min_element(c.compiled.begin(), c.compiled.end(),
                                        [](const auto& x, const auto& y) { return x->lastUse < y->lastUse; });
            c.compiled.erase(lru);
        }
        hit = e.get();
        c.compiled.push_back(std::move(e));
    } else {
        ++c.compileHits;
    }
    hit->lastUse = ++c.compileTick;
    if (withPlan) {
        int64_t rel[3];
        Relation(hit->extent, bufs, rel);
        if (!hit->hasPlan || std::memcmp(rel, hit->relation, sizeof rel) != 0) {
            hit->plan = PlanUnits(hit->sched.ops, bufs, p.elemSize);
            std::memcpy(hit->relation, rel, sizeof rel);
            hit->hasPlan = true;
        }
    }
    *out = hit;
    return HCCL_SUCCESS;
}

}  // namespace

HcclResult CompileCollective(Comm& c, const ScheduleParams& p, void* const bufs[3], bool withPlan,
                             const CompiledSchedule** out)
{
    return FindOrCompile(
        c, p, bufs, withPlan, [&](Schedule* s) { return static_cast<HcclResult>(BuildSchedule(p, s)); }, out);
}

HcclResult CompileProgram(Comm& c, const HcclAmdIrOp* ops, uint64_t numOps, uint32_t elemSize, void* const bufs[3],
                          const CompiledSchedule** out)
{
    // A program has no schedule parameters: it is keyed by its bytes (FNV-1a 64) and length, and a hit is confirmed
    // record by record.
    uint64_t h = 1469598103934665603ull;
    const unsigned char* b = reinterpret_cast<const unsigned char*>(ops);
    for (size_t i = 0; i < numOps * sizeof(HcclAmdIrOp); ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    ScheduleParams p;
    p.opType = kProgramOpType;
    p.count = h;
    p.nRanks = static_cast<uint32_t>(numOps);
    p.elemSize = elemSize;
    p.scratchCapBytes = c.scratchBytes;
    HCCL_CHK(FindOrCompile(
        c, p, bufs, true,
        [&](Schedule* s) {
            s->ops.assign(ops, ops + numOps);
            return HCCL_SUCCESS;
        },
        out));
    if ((*out)->sched.ops.size() != numOps ||
        std::memcmp((*out)->sched.ops.data(), ops, numOps * sizeof(HcclAmdIrOp)) != 0) {
        c.compiled.clear();  // a hash collision: compile afresh
        return CompileProgram(c, ops, numOps, elemSize, bufs, out);
    }
    return HCCL_SUCCESS;
}

HcclResult Execute(Comm& c, const std::vector<HcclAmdIrOp>& ops, void* const bufs[3], HcclDataType dt,
                   HcclReduceOp op, hipStream_t user, bool singleStream, const std::vector<UnitPlan>* cached)
{
    hipStreamCaptureStatus capture = hipStreamCaptureStatusNone;
    HIP_CHK(hipStreamIsCapturing(user, &capture));
    const bool captured = capture != hipStreamCaptureStatusNone;
    // A loopback world meets its peers through host rendezvous and events exchanged between threads on every group,
    // which a graph cannot replay: refused under capture, before anything is enqueued (every rank alike).
    if (captured && c.transport->SharedDevice()) return HCCL_E_NOT_SUPPORT;
    // The execution bound (watchdog.cc): this call's work on `user`, bracketed by the watchdog's events. A captured
    // call runs later, from a graph, outside any entry: not tracked.
    HpScope hpTotal(HCCL_AMD_HP_EXECUTE);
    WatchScope watch(captured ? nullptr : c.watchdog.get(), user, !singleStream);
    const bool timed = c.cfg.foldTiming && !captured;
    if (timed) {
        c.foldTiming.next = 0;
        c.foldTiming.folds.clear();
        c.foldTiming.bytes.clear();
        c.foldTiming.spanEnd = nullptr;
        HCCL_CHK(c.foldTiming.Next(&c.foldTiming.spanStart));
        HIP_CHK(hipEventRecord(c.foldTiming.spanStart, user));
    }
    if (singleStream) {
        HCCL_CHK(ExecuteSingleStream(c, ops, bufs, dt, op, user, captured, timed));
        if (timed) {
            HCCL_CHK(c.foldTiming.Next(&c.foldTiming.spanEnd));
            HIP_CHK(hipEventRecord(c.foldTiming.spanEnd, user));
        }
        return HCCL_SUCCESS;
    }
    const uint64_t es = DataTypeSize(dt);
    // Under stream capture the transport groups go on the capturing stream itself and only the folds on a forked
    // stream: an RCCL group captured on a stream joined to the capture (rather than its origin) brought down graph
    // instantiation (hipStreamEndCapture segfaulted; tools/rccl_capture_probe.py), while the same group on the origin
    // stream captures and replays. The plan and its waits are the same; only the link stream's identity changes.
    hipStream_t streams[2] = {captured ? user : c.commStream, c.reduceStream};
    c.nextEvent = 0;
    hipEvent_t start;
    HCCL_CHK(c.NextEvent(&start));
    HIP_CHK(hipEventRecord(start, user));
    if (!captured) HIP_CHK(hipStreamWaitEvent(c.commStream, start, 0));
    HIP_CHK(hipStreamWaitEvent(c.reduceStream, start, 0));

    auto addr = [&](int32_t buf, uint64_t off) -> uintptr_t {
        return reinterpret_cast<uintptr_t>(bufs[buf]) + off * es;
    };

    std::vector<UnitPlan> fresh;
    if (cached == nullptr) {
        HpScope hp(HCCL_AMD_HP_PLAN);
        fresh = PlanUnits(ops, bufs, es);
    }
    const std::vector<UnitPlan>& plan = cached != nullptr ? *cached : fresh;
    std::vector<hipEvent_t> evs(plan.size(), nullptr);
    bool used[2] = {false, false};
    std::vector<P2pOp> p2p;
    for (size_t ui = 0; ui < plan.size(); ++ui) {
        const UnitPlan& u = plan[ui];
        const int x = u.stream;
        if (u.waitUnit >= 0) {
            HpScope hp(HCCL_AMD_HP_WAIT);
            HIP_CHK(hipStreamWaitEvent(streams[x], evs[size_t(u.waitUnit)], 0));
        }
        if (u.isComm) {
            p2p.clear();
            for (size_t k = u.first; k < u.first + u.count; ++k) {
                const HcclAmdIrOp& o = ops[k];
                const bool send = o.kind == HCCL_AMD_IR_SEND;
                const uintptr_t a = send ? addr(o.srcBuf[0], o.srcOff[0]) : addr(o.dstBuf, o.dstOff);
                p2p.push_back({send, static_cast<uint32_t>(o.peer), reinterpret_cast<void*>(a), o.count * es});
            }
            if (!captured) HCCL_CHK(MaybeInjectStall(c, streams[x]));
            HpScope hp(HCCL_AMD_HP_GROUP);
            HCCL_CHK(c.transport->Group(p2p, streams[x]));
        } else {
            const HcclAmdIrOp& o = ops[u.first];
            void* dst = reinterpret_cast<void*>(addr(o.dstBuf, o.dstOff));
            HpScope hp(o.kind == HCCL_AMD_IR_COPY ? HCCL_AMD_HP_COPY : HCCL_AMD_HP_FOLD);
            if (o.kind == HCCL_AMD_IR_COPY) {
                const void* src = reinterpret_cast<const void*>(addr(o.srcBuf[0], o.srcOff[0]));
                HCCL_CHK(LaunchCopyBytes(dst, src, o.count * es, streams[x]));
            } else if (o.kind == HCCL_AMD_IR_REDUCE) {
                HCCL_CHK(LaunchFolds(c, timed, ops, u.first, u.count, es, bufs, dt, op, streams[x]));
            } else {
                return HCCL_E_INTERNAL;
            }
        }
        if (u.waitedOn) {
            HpScope hp(HCCL_AMD_HP_RECORD);
            HCCL_CHK(c.NextEvent(&evs[ui]));
            HIP_CHK(hipEventRecord(evs[ui], streams[x]));
        }
        used[x] = true;
    }

    for (int s = 0; s < 2; ++s) {
        // an unused stream needs no join, except under capture, where every stream forked into it must rejoin
        if ((!used[s] && !captured) || streams[s] == user) continue;
        hipEvent_t end;
        HCCL_CHK(c.NextEvent(&end));
        HIP_CHK(hipEventRecord(end, streams[s]));
        HIP_CHK(hipStreamWaitEvent(user, end, 0));
    }
    if (timed) {
        HCCL_CHK(c.foldTiming.Next(&c.foldTiming.spanEnd));
        HIP_CHK(hipEventRecord(c.foldTiming.spanEnd, user));
    }
    return HCCL_SUCCESS;
}

HcclResult Comm::FoldTiming::Next(hipEvent_t* e)
{
    if (next == pool.size()) {
        hipEvent_t ev;
        HIP_CHK(hipEventCreate(&ev));  // timing enabled
        pool.push_back(ev);
    }
    *e = pool[next++];
    return HCCL_SUCCESS;
}

}  // namespace hccl_amd

extern "C" HcclResult HcclAmdHostProfile(uint64_t* ns, uint64_t* calls, uint32_t n, int32_t reset)
{
    using hccl_amd::Hp;
    for (uint32_t i = 0; i < n && i < HCCL_AMD_HP_COUNT; ++i) {
        if (ns != nullptr) ns[i] = Hp().ns[i].load();
        if (calls != nullptr) calls[i] = Hp().calls[i].load();
    }
    if (reset != 0) {
        for (uint32_t i = 0; i < HCCL_AMD_HP_COUNT; ++i) {
            Hp().ns[i] = 0;
            Hp().calls[i] = 0;
        }
    }
    return HCCL_SUCCESS;
}

namespace hccl_amd {

// ------------------------------------------------------------------------------------------------ entry ordering

EntryScope::EntryScope(Comm& c, hipStream_t s) : c_(c), s_(s)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) {
        status_ = HCCL_E_RUNTIME;
        return;
    }
    captured_ = st != hipStreamCaptureStatusNone;
    if (captured_) {
        status_ = NoteCapture(c, s);
        return;
    }
    // Every call of a communicator shares its staging. Calls on one stream are ordered by it, and eager two-stream
    // calls by the communicator's own streams; a call that follows one on another stream waits for its end.
    if (c.tailStream != nullptr && c.tailStream != s && hipStreamWaitEvent(s, c.tail, 0) != hipSuccess) {
        status_ = HCCL_E_RUNTIME;
    }
}

EntryScope::~EntryScope()
{
    if (captured_ || status_ != HCCL_SUCCESS) return;
    // The tail keeps the runtime's default system-scope fence although it costs 3.0 us of device time per call behind
    // a device-bound kernel against 1.0 us without (tools/probes/event_record_cost.py,
    // profiles/r05_event_record_cost.jsonl): it is the last command of every eager call on the caller's stream, the
    // one a caller's later synchronisation and host read follow, and HIP documents an event recorded without the fence
    // as not synchronising memory with the host.
    if (c_.tail == nullptr && hipEventCreateWithFlags(&c_.tail, hipEventDisableTiming) != hipSuccess) {
        c_.tail = nullptr;
        return;
    }
    if (hipEventRecord(c_.tail, s_) == hipSuccess) c_.tailStream = s_;
}

// ------------------------------------------------------------------------------------------------ executor graphs

namespace {

// Captures the program on the communicator's private stream (thread-local capture mode: other threads' HIP calls do
// not disturb it, and it disturbs no capture of theirs). Under capture Execute posts the transport groups on the
// capturing stream and forks only the folds (executor.cc Execute), the RCCL capture pattern that instantiates.
HcclResult CaptureProgram(Comm& c, const CompiledSchedule& cs, void* const bufs[3], HcclDataType dt, HcclReduceOp op,
                          bool single, hipGraphExec_t* exec)
{
    *exec = nullptr;
    if (c.captureStream == nullptr) HIP_CHK(hipStreamCreateWithFlags(&c.captureStream, hipStreamNonBlocking));
    HIP_CHK(hipStreamBeginCapture(c.captureStream, hipStreamCaptureModeThreadLocal));
    const HcclResult r = Execute(c, cs.sched.ops, bufs, dt, op, c.captureStream, single, single ? nullptr : &cs.plan);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(c.captureStream, &g);
    if (r != HCCL_SUCCESS || e != hipSuccess || g == nullptr) {
        if (g != nullptr) (void)hipGraphDestroy(g);
        HCCL_AMD_ERR("rank %u: executor graph capture failed (%s / %s); the collective runs eagerly", c.rank,
                     HcclAmdGetErrorString(r), hipGetErrorString(e));
        return r != HCCL_SUCCESS ? r : HCCL_E_RUNTIME;
    }
    const hipError_t ie = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);  // the executable keeps what it needs (RCCL's plans are held by it)
    if (ie != hipSuccess) {
        *exec = nullptr;
        HCCL_AMD_ERR("rank %u: hipGraphInstantiate: %s; the collective runs eagerly", c.rank, hipGetErrorString(ie));
        return HCCL_E_RUNTIME;
    }
    return HCCL_SUCCESS;
}

}  // namespace

// Destroys the retired executables whose last launch has completed (all of them, waiting, when wait is set).
void ReapRetiredGraphs(Comm& c, bool wait)
{
    for (size_t i = 0; i < c.retiredGraphs.size();) {
        RetiredGraph& g = c.retiredGraphs[i];
        if (wait) (void)hipEventSynchronize(g.done);
        if (hipEventQuery(g.done) == hipErrorNotReady) {
            ++i;
            continue;
        }
        (void)hipGraphExecDestroy(g.exec);
        (void)hipEventDestroy(g.done);
        c.retiredGraphs.erase(c.retiredGraphs.begin() + static_cast<std::ptrdiff_t>(i));
    }
}

HcclResult RunCompiled(Comm& c, const CompiledSchedule& cs, void* const bufs[3], HcclDataType dt, HcclReduceOp op,
                       hipStream_t user, bool single)
{
    const size_t cap = c.cfg.graphCache;
    const std::vector<UnitPlan>* plan = single ? nullptr : &cs.plan;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    HIP_CHK(hipStreamIsCapturing(user, &st));
    // A single-stream program with one transport group stays eager: its two launches enqueue faster than a graph
    // launch (the C5 1 KiB one-shot over the RCCL self loop: 31.6 us eager, 36.2 us through the cache; an 8-rank RHD of
    // 6 groups: 54.9 us eager, 43.9 us through the cache; profiles/r05_host_cost_selfloop.jsonl).
    if (cap == 0 || st != hipStreamCaptureStatusNone || !c.transport->Abortable() || c.cfg.foldTiming ||
        (single && cs.groups <= 1)) {
        return Execute(c, cs.sched.ops, bufs, dt, op, user, single, plan);
    }
    if (!c.retiredGraphs.empty()) ReapRetiredGraphs(c, false);
    GraphEntry* hit = nullptr;
    for (GraphEntry& g : c.graphs) {
        if (g.stream == user && g.dt == dt && g.op == op && g.single == single &&
            std::memcmp(g.bufs, bufs, sizeof g.bufs) == 0 && SameParams(g.params, cs.params)) {
            hit = &g;
            break;
        }
    }
    if (hit == nullptr) {
        // A key's first call runs eagerly (it makes RCCL connect to the program's peers, which a capture must not have
        // to do) and leaves a placeholder; its second call captures. A workload whose buffers change from call to call
        // therefore never pays a capture it cannot replay.
        if (c.graphs.size() >= cap) {
            // The evicted executable may still run: the host is ahead of the device. It is retired with an
            // event recorded on this call's stream before this call's work: EntryScope has already ordered this stream
            // after the previous call's end, which every earlier launch precedes, so once the event has completed no
            // launch of the executable is in flight. It is destroyed then (ReapRetiredGraphs at a later call or at
            // teardown); the host never waits here.
            auto lru = std::min_element(c.graphs.begin(), c.graphs.end(),
                                        [](const GraphEntry& x, const GraphEntry& y) { return x.lastUse < y.lastUse; });
            if (lru->exec != nullptr) {
                RetiredGraph r{lru->exec, nullptr};
                HIP_CHK(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
                HIP_CHK(hipEventRecord(r.done, user));
                c.retiredGraphs.push_back(r);
            }
            c.graphs.erase(lru);
        }
        GraphEntry e;
        e.params = cs.params;
        std::memcpy(e.bufs, bufs, sizeof e.bufs);
        e.stream = user;
        e.dt = dt;
        e.op = op;
        e.single = single;
        e.lastUse = ++c.compileTick;
        c.graphs.push_back(e);
        return Execute(c, cs.sched.ops, bufs, dt, op, user, single, plan);
    }
    if (!hit->tried) {
        hit->tried = true;
        (void)CaptureProgram(c, cs, bufs, dt, op, single, &hit->exec);
        if (hit->exec != nullptr) ++c.graphCaptures;
    }
    hit->lastUse = ++c.compileTick;
    if (hit->exec == nullptr) return Execute(c, cs.sched.ops, bufs, dt, op, user, single, plan);
    // a single-stream program is not start-stamped eagerly either (the watchdog infers its start, watchdog.cc)
    WatchScope watch(c.watchdog.get(), user, !single);
    HIP_CHK(hipGraphLaunch(hit->exec, user));
    ++c.graphLaunches;
    return HCCL_SUCCESS;
}

void ReleaseGraphs(Comm& c)
{
    for (GraphEntry& g : c.graphs) {
        if (g.exec != nullptr) (void)hipGraphExecDestroy(g.exec);
    }
    c.graphs.clear();
    ReapRetiredGraphs(c, true);
    if (c.captureStream != nullptr) (void)hipStreamDestroy(c.captureStream);
    c.captureStream = nullptr;
}

}  // namespace hccl_amd

extern "C" HcclResult HcclAmdCommFoldTiming(HcclComm comm, uint64_t* folds, uint64_t* foldBytes, double* foldUs,
                                            double* spanUs)
{
    hccl_amd::Comm* c = hccl_amd::AsComm(comm);
    if (c == nullptr || folds == nullptr || foldBytes == nullptr || foldUs == nullptr || spanUs == nullptr) {
        return HCCL_E_PTR;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    const auto& t = c->foldTiming;
    if (t.spanEnd == nullptr) return HCCL_E_NOT_SUPPORT;
    HIP_CHK(hipEventSynchronize(t.spanEnd));
    float ms = 0;
    double sum = 0;
    uint64_t bytes = 0;
    for (size_t k = 0; k < t.folds.size(); ++k) {
        HIP_CHK(hipEventElapsedTime(&ms, t.folds[k].first, t.folds[k].second));
        sum += ms;
        bytes += t.bytes[k];
    }
    HIP_CHK(hipEventElapsedTime(&ms, t.spanStart, t.spanEnd));
    *folds = t.folds.size();
    *foldBytes = bytes;
    *foldUs = sum * 1e3;
    *spanUs = double(ms) * 1e3;
    return HCCL_SUCCESS;
}

extern "C" HcclResult HcclAmdCommGraphStats(HcclComm comm, uint64_t* launches, uint64_t* captures)
{
    hccl_amd::Comm* c = hccl_amd::AsComm(comm);
    if (c == nullptr || launches == nullptr || captures == nullptr) return HCCL_E_PTR;
    std::lock_guard<std::mutex> lk(c->mu);
    *launches = c->graphLaunches;
    *captures = c->graphCaptures;
    return HCCL_SUCCESS;
}
