// ipc.cc — host side of the one-sided collectives (ipc_kernel_body.h): peer-mapped staging set-up and launch.
//
// Set-up (collective, on the first IPC call of a communicator): every rank allocates uncached staging and a
// flag array, exports them with hipIpcGetMemHandle, all-gathers the handles over the communicator (ncclAllGather)
// and opens every peer's with hipIpcOpenMemHandle — the reference's channel set-up that hands each rank its peers'
// CCL buffers (ChannelInfo.remoteCclMem, alg_param.h:434-448; AIV GM_IN[r], aiv_communication_base_v2.h:121-150).
// In a loopback world the ranks share a device and the raw pointers are exchanged instead, and the whole world runs
// as one launch (all ranks' blocks must be resident together, which separate per-rank launches on 4 hardware queues
// would not guarantee).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>

#include "comm.h"

namespace hccl_amd {

namespace {

// The uncached allocations of the IPC path (the staging tiers; flags and LL area) are kept for the life of the process
// and handed to the next communicator's set-up that asks for the same size on the same device; they are never freed.
// Freeing hipDeviceMallocUncached memory corrupts later GPU work on this stack: the r03 test order's allocation history
// in a loop returned wrong results (ranks' operands missing) in 17 of 217 iterations with these blocks freed after
// every destroy and in 0 of 223 with them kept, and a loop that freed uncached blocks allocated outside the library
// faulted the GPU (memory aperture violation) where the same loop with cached blocks ran clean
// (profiles/r06_release_stress.txt).
struct UncachedPool {
    std::mutex mu;
    std::multimap<std::pair<int, size_t>, void*> idle;  // (device, bytes) -> allocation
};

UncachedPool& Pool()
{
    static UncachedPool* p = new UncachedPool;  // never destroyed: the runtime frees device memory at exit
    return *p;
}

bool UncachedAlloc(int device, void** ptr, size_t bytes)
{
    {
        UncachedPool& pool = Pool();
        std::lock_guard<std::mutex> lk(pool.mu);
        auto it = pool.idle.find({device, bytes});
        if (it != pool.idle.end()) {
            *ptr = it->second;
            pool.idle.erase(it);
            return true;
        }
    }
    return hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached) == hipSuccess;
}

void UncachedRelease(int device, void* ptr, size_t bytes)
{
    UncachedPool& pool = Pool();
    std::lock_guard<std::mutex> lk(pool.mu);
    pool.idle.insert({{device, bytes}, ptr});
}

}  // namespace

uint64_t IpcIdleBytes()
{
    UncachedPool& pool = Pool();
    std::lock_guard<std::mutex> lk(pool.mu);
    uint64_t b = 0;
    for (const auto& kv : pool.idle) b += kv.first.second;
    return b;
}

namespace {

size_t FlagAllocBytes() { return size_t(kIpcFlagBytes + 2 * kIpcLlParityBytes); }

// Maps one allocation of every rank (collective: every rank takes part whatever its local outcome, and the outcome
// is agreed: either every rank has every peer's allocation mapped, or none keeps a mapping and all report
// HCCL_E_NOT_SUPPORT; a failed host exchange returns the transport's error). peers[r] receives rank r's allocation
// as this rank addresses it (its own at [me]); opened[r] marks the ones opened with hipIpcOpenMemHandle. In a loopback
// world the ranks share the device and exchange raw pointers. ranksOnDevice (rank mode, optional) receives the most
// ranks any one device holds, from every rank's PCI bus id: the same number on every rank.
HcclResult MapPeers(Comm& c, void* mine, bool localOk, void* peers[kIpcMaxRanks], bool opened[kIpcMaxRanks],
                    uint32_t* ranksOnDevice)
{
    const uint32_t n = c.nRanks, me = c.rank;
    if (c.transport->SharedDevice()) {
        struct Raw {
            void* p;
            uint8_t ok;
        };
        const Raw m{mine, static_cast<uint8_t>(localOk ? 1 : 0)};
        std::vector<Raw> all(n);
        HCCL_CHK(c.transport->AllGatherHost(&m, sizeof m, all.data()));
        for (uint32_t r = 0; r < n; ++r) {
            if (all[r].ok == 0) return HCCL_E_NOT_SUPPORT;
        }
        for (uint32_t r = 0; r < n; ++r) peers[r] = all[r].p;
        return HCCL_SUCCESS;
    }
    struct Exported {
        hipIpcMemHandle_t h;
        char busId[32];  // the rank's device: ranks that share one count against its resident blocks together
        uint8_t ok;
    };
    Exported m{};
    bool ok = localOk && hipIpcGetMemHandle(&m.h, mine) == hipSuccess &&
              hipDeviceGetPCIBusId(m.busId, sizeof m.busId - 1, c.device) == hipSuccess;
    m.ok = ok ? 1 : 0;
    std::vector<Exported> all(n);
    HCCL_CHK(c.transport->AllGatherHost(&m, sizeof m, all.data()));
    for (uint32_t r = 0; r < n; ++r) ok = ok && all[r].ok != 0;  // nobody opens a handle some rank could not export
    if (ranksOnDevice != nullptr) {
        *ranksOnDevice = 1;
        for (uint32_t r = 0; r < n; ++r) {
            uint32_t k = 0;
            for (uint32_t q = 0; q < n; ++q) k += std::strncmp(all[r].busId, all[q].busId, sizeof m.busId) == 0;
            *ranksOnDevice = std::max(*ranksOnDevice, k);
        }
    }
    for (uint32_t r = 0; r < n && ok; ++r) {
        if (r == me) {
            peers[r] = mine;
            continue;
        }
        void* p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, all[r].h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            HCCL_AMD_ERR("rank %u: hipIpcOpenMemHandle of rank %u failed: %s", me, r, hipGetErrorString(e));
            ok = false;
            break;
        }
        peers[r] = p;
        opened[r] = true;
    }
    const uint8_t mineOk = ok ? 1 : 0;
    std::vector<uint8_t> allOk(n);
    const HcclResult xr = c.transport->AllGatherHost(&mineOk, 1, allOk.data());
    for (uint32_t r = 0; r < n && xr == HCCL_SUCCESS; ++r) ok = ok && allOk[r] != 0;
    if (xr == HCCL_SUCCESS && ok) return HCCL_SUCCESS;
    for (uint32_t r = 0; r < n; ++r) {
        if (opened[r]) (void)hipIpcCloseMemHandle(peers[r]);
        opened[r] = false;
        peers[r] = nullptr;
    }
    return xr != HCCL_SUCCESS ? xr : HCCL_E_NOT_SUPPORT;
}

// The four areas inside one staging allocation at base (every rank has the same layout).
void AreasOf(const IpcTier& t, void* base, void* areas[kIpcAreas])
{
    char* b = static_cast<char*>(base);
    areas[kIpcAreaIn] = b;
    areas[kIpcAreaRes] = b + t.inBytes;
    areas[kIpcAreaAlt0] = b + t.inBytes + t.resBytes;
    areas[kIpcAreaAlt1] = b + t.inBytes + t.resBytes + t.altBytes;
}

void ReleaseTier(Comm& c, IpcTier& t)
{
    for (uint32_t r = 0; r < kIpcMaxRanks; ++r) {
        if (t.opened[r]) (void)hipIpcCloseMemHandle(t.peerArea[kIpcAreaIn][r]);  // the peer's one allocation
    }
    if (t.area[0] != nullptr) UncachedRelease(c.device, t.area[0], t.allocBytes());
    const bool unavailable = t.unavailable;
    t = IpcTier{};
    t.unavailable = unavailable;
}

}  // namespace

IpcTier IpcTierSizes(const Comm& c, int t)
{
    constexpr uint64_t kGranule = 64ull << 10;
    const auto up = [](uint64_t b) { return (b + kGranule - 1) / kGranule * kGranule; };
    // the large tier: HCCL_BUFFSIZE / 2 per area (2 x HCCL_BUFFSIZE for the four), or HCCL_AMD_IPC_STAGING_MIB
    uint64_t large = c.cfg.ipcStagingBytes != 0 ? c.cfg.ipcStagingBytes : c.cclBytes / 2 / kGranule * kGranule;
    large = std::min<uint64_t>(std::max<uint64_t>(large, 1ull << 20), kIpcStagingAreaMaxBytes);
    uint64_t area = large;
    if (t == kIpcTierSmall) {
        area = std::min(large, up(uint64_t(std::max<uint32_t>(c.nRanks, 1)) *
                                  std::max<uint64_t>(c.cfg.smallIpcBytes, 64ull << 10)));
    }
    IpcTier s{};
    s.inBytes = area;
    s.resBytes = area;  // results of a whole round, in round coordinates
    // slots of the single-barrier kinds, two areas used alternately: as large as the others, within the one
    // allocation's bound (1000 MiB areas leave them 23.5 MiB)
    s.altBytes = std::min<uint64_t>(area, (kIpcStagingMaxBytes - 2 * area) / 2 / kGranule * kGranule);
    return s;
}

namespace {

// What every one-sided call needs (collective, at the communicator's first one-sided call): the flags and, behind
// them, the LL area (one uncached allocation mapped by every peer, zeroed), the status words, the host-visible failure
// word and the LL unpack area.
HcclResult IpcSetupBase(Comm& c)
{
    IpcState& s = c.ipc;
    if (s.ready) return HCCL_SUCCESS;
    if (s.unavailable) return HCCL_E_NOT_SUPPORT;
    s.blocks = kIpcBlocks;
    const size_t flagBytes = FlagAllocBytes();
    // The fresh uncached pages may carry lines of a freed cached buffer in some XCD's L2: scrub the L2s before the
    // flags are zeroed (ScrubL2), so that no stale line is ever read or written back over them.
    // HCCL_AMD_INJECT_IPC_ALLOC_FAIL (tests): this rank's allocations fail, as under memory pressure
    const bool inject = c.cfg.injectIpcAllocFail == static_cast<int32_t>(c.rank);
    bool ok = !inject && UncachedAlloc(c.device, reinterpret_cast<void**>(&s.flags), flagBytes) &&
              hipMalloc(reinterpret_cast<void**>(&s.status), kIpcStatusBytes) == hipSuccess &&
              hipMalloc(&s.llUnpack, kIpcLlUnpackBytes) == hipSuccess &&
              hipHostMalloc(reinterpret_cast<void**>(&s.failHost), 64, hipHostMallocCoherent | hipHostMallocMapped) ==
                  hipSuccess &&
              hipHostGetDevicePointer(reinterpret_cast<void**>(&s.failDev), s.failHost, 0) == hipSuccess &&
              hipDeviceSynchronize() == hipSuccess && (!c.cfg.ipcL2Scrub || ScrubL2(c.reduceStream) == HCCL_SUCCESS) &&
              hipMemset(s.flags, 0, flagBytes) == hipSuccess && hipMemset(s.status, 0, kIpcStatusBytes) == hipSuccess &&
              hipDeviceSynchronize() == hipSuccess;
    if (ok && c.cfg.ipcTrace) {
        // phase stamps (diagnostics, HCCL_AMD_IPC_TRACE; HcclAmdCommIpcTrace reads them back): every rank's and
        // block's row, so a loopback world's one launch fits too
        const size_t tb = size_t(kIpcMaxRanks) * kIpcMaxBlocks * kIpcTraceSlots * sizeof(uint64_t);
        ok = hipMalloc(reinterpret_cast<void**>(&s.trace), tb) == hipSuccess && hipMemset(s.trace, 0, tb) == hipSuccess &&
             hipDeviceSynchronize() == hipSuccess;
    }
    if (ok) {
        *s.failHost = 0;
    } else {
        HCCL_AMD_ERR("rank %u: IPC flag or status allocation failed", c.rank);
    }
    const volatile uint32_t* watch = s.failHost;
    uint32_t* wdev = nullptr;
    if (c.transport->SharedDevice()) {
        // The world runs one launch for all ranks (issued by rank 0): its timeouts go to the world's word, which every
        // rank watches and which outlives each rank's communicator.
        uint32_t* word = ok ? c.transport->SharedFailWord(&wdev) : nullptr;
        ok = ok && word != nullptr;
        watch = word;
    }
    void* peers[kIpcMaxRanks] = {};
    const HcclResult r = MapPeers(c, s.flags, ok, peers, s.flagsOpened, &s.ranksOnDevice);
    if (r != HCCL_SUCCESS) {
        IpcRelease(c);
        s.unavailable = true;
        return r;
    }
    for (uint32_t q = 0; q < c.nRanks; ++q) s.peerFlags[q] = static_cast<uint32_t*>(peers[q]);
    if (c.transport->SharedDevice()) s.failDev = wdev;
    c.failWord.store(watch, std::memory_order_release);
    s.ready = true;
    return HCCL_SUCCESS;
}

// Staging tier t (collective, at the first call that needs it): one uncached allocation below 2 GiB holding
// [in][results][alternate 0][alternate 1], mapped by every peer. hipIpcOpenMemHandle never returned for a 2 GiB
// allocation on this stack (r03: the 512 MiB areas in one 2 GiB block hung the rank-mode set-up;
// profiles/r03_probe_ipc_open*.jsonl: up to 2047 MiB opens in < 1 ms, 2048 MiB does not return).
HcclResult IpcSetupTier(Comm& c, int t)
{
    IpcTier& tr = c.ipc.tier[t];
    if (tr.ready) return HCCL_SUCCESS;
    if (tr.unavailable) return HCCL_E_NOT_SUPPORT;
    tr = IpcTierSizes(c, t);
    void* base = nullptr;
    bool ok = c.cfg.injectIpcAllocFail != static_cast<int32_t>(c.rank) && UncachedAlloc(c.device, &base, tr.allocBytes());
    if (!ok) {
        base = nullptr;
        HCCL_AMD_ERR("rank %u: IPC staging allocation of %llu B failed", c.rank, (unsigned long long)tr.allocBytes());
    }
    // no stale line of a freed cached buffer may be written back over the new staging (as for the flags)
    ok = ok && hipDeviceSynchronize() == hipSuccess && (!c.cfg.ipcL2Scrub || ScrubL2(c.reduceStream) == HCCL_SUCCESS);
    void* peers[kIpcMaxRanks] = {};
    const HcclResult r = MapPeers(c, base, ok, peers, tr.opened, nullptr);
    if (r != HCCL_SUCCESS) {
        if (base != nullptr) UncachedRelease(c.device, base, tr.allocBytes());
        tr = IpcTier{};
        tr.unavailable = true;
        return r;
    }
    AreasOf(tr, base, tr.area);
    for (uint32_t q = 0; q < c.nRanks; ++q) {
        void* areas[kIpcAreas];
        AreasOf(tr, peers[q], areas);
        for (int k = 0; k < kIpcAreas; ++k) tr.peerArea[k][q] = areas[k];
    }
    tr.ready = true;
    return HCCL_SUCCESS;
}

bool Aligned16(const void* p, const void* q)
{
    return ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(q)) & 15u) == 0;
}

// Barrier fences (IpcArgs::fence). Every byte a barrier hands over lives in uncached staging, which no L2 holds: the
// storing waves' vmcnt drains order the data before the flag (a store completes at memory), and an agent-scope acquire
// (the CU's L1) suffices for the reader, whose loads go to memory. The user buffers are never handed over inside the
// kernel (each element is read and written by the lane that owns it); across kernels they are ordered by the ordinary
// kernel boundaries, which make plain and non-temporal stores visible to the next kernel on every XCD
// (tools/probes/coherence_probe.hip, profiles/r04_coherence_probe.jsonl). The light fences skip the system-scope
// release and acquire, which write back and invalidate the whole XCD L2 for every block: 3-13 % per call in loopback
// worlds (profiles/r03_ipc_variant_ab_fence.jsonl). Default (CommConfig::ipcLightFence = -1): light in a loopback
// world, where every store goes through the owner's own uncached pointer; system scope in rank mode, whose stores reach
// the peers' staging through hipIpcOpenMemHandle mappings, and an imported mapping need not keep the exporter's uncached
// memory type (imported mappings). HCCL_AMD_IPC_LIGHT_FENCE=1 or 0 forces either. Equal on every rank.
bool IpcLightFence(const Comm& c)
{
    return c.cfg.ipcLightFence < 0 ? c.transport->SharedDevice() : c.cfg.ipcLightFence != 0;
}

}  // namespace

void IpcQuiesce(Comm& c)
{
    if (!c.ipc.ready || c.ipcQuiesced) return;
    c.ipcQuiesced = true;
    // Peers store into this rank's staging and flags: unmapping or freeing them while any peer's kernel may still
    // run would fault that peer. Wait for this device, then for every rank to get here (each has waited for its own).
    (void)hipDeviceSynchronize();
    // A loopback world has no rendezvous here: its ranks are destroyed one after another from any thread (a host
    // exchange would wait for ranks that are destroyed later on the same thread), and every one-sided launch of the
    // world is a single launch on this device, which the device synchronisation above has drained; a world whose ranks
    // are destroyed while others still issue collectives is outside the contract.
    if (c.transport->SharedDevice()) return;
    uint8_t mine = 1;
    std::vector<uint8_t> all(c.nRanks);
    if (c.transport->AllGatherHost(&mine, 1, all.data()) != HCCL_SUCCESS) {
        HCCL_AMD_ERR("rank %u: IPC teardown rendezvous failed; peer mappings are left in place", c.rank);
        c.ipc = IpcState{};  // leak rather than free memory a peer may still write
    }
}

void IpcRelease(Comm& c)
{
    IpcState& s = c.ipc;
    for (IpcTier& t : s.tier) ReleaseTier(c, t);
    for (uint32_t r = 0; r < kIpcMaxRanks; ++r) {
        if (s.flagsOpened[r]) (void)hipIpcCloseMemHandle(s.peerFlags[r]);
    }
    if (s.flags != nullptr) UncachedRelease(c.device, s.flags, FlagAllocBytes());
    if (s.status != nullptr) (void)hipFree(s.status);
    if (s.trace != nullptr) (void)hipFree(s.trace);
    if (s.llUnpack != nullptr) (void)hipFree(s.llUnpack);
    // the word is no longer watched before it is freed (a failure already seen stays in Comm::failCode)
    c.failWord.store(nullptr, std::memory_order_release);
    if (s.failHost != nullptr) (void)hipHostFree(s.failHost);
    const bool unavailable = s.unavailable;
    s = IpcState{};
    s.unavailable = unavailable;
}

uint64_t IpcDeviceBytes(const Comm& c)
{
    const IpcState& s = c.ipc;
    uint64_t b = 0;
    if (s.flags != nullptr) b += FlagAllocBytes();
    if (s.status != nullptr) b += kIpcStatusBytes;
    if (s.llUnpack != nullptr) b += kIpcLlUnpackBytes;
    if (s.trace != nullptr) b += uint64_t(kIpcMaxRanks) * kIpcMaxBlocks * kIpcTraceSlots * sizeof(uint64_t);
    for (const IpcTier& t : s.tier) {
        if (t.area[0] != nullptr) b += t.allocBytes();
    }
    return b;
}

// Default workgroups per launch by the bytes of one rank's input. Every block runs its own cross-rank barrier (a
// system-scope release, one flag store per peer, a poll), so small calls pay per block: 16 blocks run a 1 KiB
// AllReduce in 11 us where 128 take 25 us and 256 take 42 us; large calls want the whole chip (1 GiB: 256 blocks
// 10 % ahead of 128). Rank-mode sweep on one GPU, n = 2 and 4 (tools/probes/sweep_ipc_blocks.py,
// profiles/r01_sweep_ipc_blocks.jsonl); the best count agreed between n = 2 and 4 at every size. Below 16 blocks (r05,
// profiles/r05_sweep_small_blocks.jsonl): up to 64 KiB, 4 blocks are 0.2-0.5 us faster than 16 at n = 2 (1 KiB
// 10.26 vs 10.71 us) and no slower at n = 4; from 256 KiB on, fewer than 16 lose bandwidth.
// Workgroups of an LL launch: about two polled words per thread, (n - 1) x bytes / 4 words over 256-thread blocks. A
// block's pull, unpack and fold are serial latencies, so the LL form wants many small blocks where the staged kernel
// wants few: rank mode, n = 2 and 4 on one GPU (tools/probes/sweep_ipc_blocks.py with HCCL_AMD_IPC_LL_BYTES,
// profiles/r05_ll_sweep_blocks.jsonl): 1 KiB best at 1-2 blocks (7.4 us), 64 KiB at 32 (9.4 us; 55.5 us with 1).
// RHD's order folds a tree per part and chunk, so its blocks want about one word per thread, and never fewer than two
// blocks (n = 2, eager: 1 KiB 14.5 us on one block, 13.4 on two; 4 KiB 13.2 on four; profiles/r05_ll_rhd_blocks.jsonl).
uint32_t LlIpcBlocks(uint32_t n, uint64_t bytes, bool rhd)
{
    const uint64_t items = uint64_t(n > 1 ? n - 1 : 1) * ((bytes + 3) / 4);
    const uint64_t per = rhd ? 256 : 512;
    return static_cast<uint32_t>(std::min<uint64_t>(128, std::max<uint64_t>(2, (items + per - 1) / per)));
}

uint32_t DefaultIpcBlocks(uint64_t bytes)
{
    if (bytes <= (64ull << 10)) return 4;
    if (bytes <= (512ull << 10)) return 16;
    if (bytes <= (2ull << 20)) return 32;
    if (bytes <= (32ull << 20)) return 64;
    if (bytes <= (64ull << 20)) return 128;
    return 256;
}

// ------------------------------------------------------------------------------------------------ plans

namespace {

uint64_t LoopElems(uint64_t loopBytes, uint64_t es) { return std::max<uint64_t>(1, loopBytes / es); }

uint64_t RoundDown128(uint64_t b) { return b / 128 * 128; }

constexpr uint64_t kUbMaxDataSize = 256ull << 20;  // UB_MAX_DATA_SIZE, alg_param.h:37

}  // namespace

// The AICPU template whose order the kernel follows, by schedule family (the auto selector's families).
HcclResult IpcPlanForFamily(int32_t opType, int32_t family, uint32_t n, uint64_t es, uint64_t cclBytes, IpcPlan* pl)
{
    IpcPlan p{};
    switch (opType) {
        case HCCL_AMD_OP_ALLREDUCE:
            if (family == HCCL_AMD_ALGO_MESH_ONESHOT) {
                p.kind = kIpcAllReduceOneShot;
                p.order = kIpcO1;
                p.geom = kIpcGeomWhole;
            } else if (family == HCCL_AMD_ALGO_MESH_CHUNK) {
                // MeshChunk CalcSliceInfoVec (…mesh_chunk.cc:79-97), loops of min(ccl, ccl / 2) rounded down to
                // 128 B (scratch multiple 2)
                p.kind = kIpcAllReduce;
                p.order = kIpcO6;
                p.geom = kIpcGeomCeil;
                p.loopElems = LoopElems(std::min<uint64_t>(cclBytes, RoundDown128(cclBytes / 2)), es);
            } else {
                p.kind = kIpcAllReduce;  // two-shot: O2 does not depend on the slicing or the loops
                p.order = kIpcO2;
                p.geom = kIpcGeomAlignedCeil;
            }
            break;
        case HCCL_AMD_OP_REDUCE_SCATTER:
            p.kind = kIpcReduceScatter;
            p.geom = kIpcGeomBlock;
            if (family == HCCL_AMD_ALGO_MESH_CHUNK) {
                // ReduceScatter MeshChunk: loops of min(ccl - 1 MiB, (ccl - 1 MiB) / (n-1)) rounded down to 128 B
                const uint64_t tmp = cclBytes > (1ull << 20) ? cclBytes - (1ull << 20) : cclBytes;
                p.order = kIpcO6;
                p.subMode = kIpcSubRs4K;
                p.loopElems = LoopElems(std::min<uint64_t>(tmp, RoundDown128(tmp / (n - 1))), es);
            } else {
                p.order = kIpcO1;
            }
            break;
        case HCCL_AMD_OP_REDUCE:
            p.order = kIpcO1;
            if (family == HCCL_AMD_ALGO_MESH_ONESHOT) {
                p.kind = kIpcReduceOneShot;
                p.geom = kIpcGeomWhole;
            } else {
                // ReduceSoleExecutor loops (reduce_sole_executor.cc:120-170): min(UB_MAX_DATA_SIZE, ccl / n) rounded
                // down to 128 B, each sliced by ReduceMesh1DTwoShot::CalcSlice on its own
                p.kind = kIpcReduce;
                p.geom = kIpcGeomBalanced;
                p.group = 1;
                p.loopElems = LoopElems(std::min<uint64_t>(kUbMaxDataSize, RoundDown128(cclBytes / n)), es);
            }
            break;
        case HCCL_AMD_OP_ALLGATHER:
            p.kind = kIpcAllGather;  // data movement only: no order
            p.order = kIpcO1;
            p.geom = kIpcGeomWhole;
            break;
        default: return HCCL_E_NOT_SUPPORT;
    }
    *pl = p;
    return HCCL_SUCCESS;
}

// RHD's bits on the one-sided kernel (HCCL_AMD_ALGO_IPC_RHD): the one-shot kind in order kIpcRhd over the whole
// range. AllReduceRhd has no executor loops (it is not a reference template), so neither does this: its slicing is
// a function of the count alone.
HcclResult IpcPlanRhd(uint32_t n, IpcPlan* pl)
{
    if (RhdTable(n).empty() || n < 2) return HCCL_E_NOT_SUPPORT;
    IpcPlan p{};
    p.kind = kIpcAllReduceOneShot;
    p.order = kIpcRhd;
    p.geom = kIpcGeomWhole;
    *pl = p;
    return HCCL_SUCCESS;
}

int32_t SelectAivPlan(int32_t opType, uint32_t n, uint64_t count, HcclDataType dt, HcclReduceOp op, bool strict,
                      bool aivOnly, uint64_t cclBytes, uint32_t coreLimit, IpcPlan* plan, uint32_t* group)
{
    // Common rejections of AllReduceAutoSelector / ReduceScatterAutoSelector::SelectAivAlgo
    // (all_reduce_auto_selector.cc:591-683, reduce_scatter_auto_selector.cc:537-600): the order-preserved (STRICT)
    // mode, PROD, UINT64 / FP64 and more than MAX_RANK_SIZE ranks fall back to the AICPU engine; so does data of
    // AIV_MAX_PER_RANK_DATA_SIZE (8 MiB, auto_selector_base.h:24) x rankSize or more, or above 16 CCL buffers
    // (AIV_MAX_CCL_LOOP_NUM, hccl_aiv_utils.h:33). ReduceAutoSelector has no AIV selection: Reduce stays AICPU.
    // AIV_ONLY (OpExecuteConfig::AIV_ONLY) lifts the 8 MiB x rankSize bound, not the CCL one
    // (all_reduce_auto_selector.cc:650-661, reduce_scatter_auto_selector.cc:597-610).
    const uint64_t es = DataTypeSize(dt);
    if (es == 0 || n < 2 || n > 512) return HCCL_AMD_AIV_NOT_MATCHED;
    if (opType != HCCL_AMD_OP_ALLREDUCE && opType != HCCL_AMD_OP_REDUCE_SCATTER) return HCCL_AMD_AIV_NOT_MATCHED;
    if (strict || op == HCCL_REDUCE_PROD || dt == HCCL_DATA_TYPE_UINT64 || dt == HCCL_DATA_TYPE_FP64) {
        return HCCL_AMD_AIV_NOT_MATCHED;
    }
    const uint64_t maxPerRank = 8ull << 20;
    IpcPlan p{};
    uint32_t g = 1;
    int32_t variant;
    if (opType == HCCL_AMD_OP_ALLREDUCE) {
        const uint64_t dataSize = count * es;
        if ((!aivOnly && dataSize >= maxPerRank * n) || dataSize > cclBytes * 16) return HCCL_AMD_AIV_NOT_MATCHED;
        // n <= AR_AIV_BOARD_SIZE (8): one-shot below AR_AIV_SMALL_DATA_SIZE_IN_BOARD (128 KiB); above 8 ranks
        // IsSmallData (< 512 KiB, auto_selector_base.cc:94)
        const bool oneShot = n <= 8 ? dataSize < (128ull << 10) : dataSize < (512ull << 10);
        if (oneShot) {
            // aiv_all_reduce_mesh_1d_oneshot.h:33-48: out = slot 0, then out (op)= slot r, r = 1 .. n-1 (O2);
            // executor loops of min(UB_MAX_DATA_SIZE, ccl / n) (scratch multiple n), which do not change O2
            variant = HCCL_AMD_AIV_AR_ONESHOT;
            p.kind = kIpcAllReduceOneShot;
            p.order = kIpcO2;
            p.geom = kIpcGeomWhole;
            p.loopElems = LoopElems(std::min<uint64_t>(kUbMaxDataSize, RoundDown128(cclBytes / n)), es);
        } else {
            // AivTempAllReduceMesh1DTwoShot::CalNumBlocks (aiv_temp_all_reduce_mesh_1D_twoshot.cc:88-100) and the
            // kernel's split (aiv_all_reduce_mesh_1d_twoshot.h:330-346): 2n blocks or more take Prepare/Process,
            // fewer the small-core path. Executor loops of min(UB_MAX_DATA_SIZE, ccl / 4) (scratch multiple 4).
            const uint32_t blocks = coreLimit >= n + 1 ? coreLimit / (n + 1) * (n + 1) : coreLimit;
            p.loopElems = LoopElems(std::min<uint64_t>(kUbMaxDataSize, RoundDown128(cclBytes / 4)), es);
            p.kind = kIpcAllReduce;
            if (blocks >= 2 * n) {
                // ReduceScatterLocalReduce (:145-181): groupSize = (blocks - n) / n consumer slices per rank, the
                // loop split into groupSize * n balanced slices, rank r owning slices [r * g, (r + 1) * g); each
                // is folded own copy first, then the other ranks ascending (O1)
                g = (blocks - n) / n;
                variant = HCCL_AMD_AIV_AR_TWOSHOT_LARGE;
                p.order = kIpcO1;
                p.geom = kIpcGeomBalanced;
                p.group = g;
            } else {
                // SmallCoreReduceScatter (:224-271): chunks of ceil(count / n); slot 0 (op)= slot i, i = 1 .. n-1 (O2)
                variant = HCCL_AMD_AIV_AR_TWOSHOT_SMALL;
                p.order = kIpcO2;
                p.geom = kIpcGeomCeil;
            }
        }
    } else {
        const uint64_t totalSize = count * es * n;
        if ((!aivOnly && totalSize >= maxPerRank * n) || totalSize > cclBytes * 16) return HCCL_AMD_AIV_NOT_MATCHED;
        // AivTempReduceScatterMesh1D::CalNumBlocks (aiv_temp_reduce_scatter_mesh_1D.cc:87-97): the core limit, at most
        // 2n below 512 KiB of output; aiv_reduce_scatter_op.h:23-37 takes the big-data kernel above 2n blocks (out =
        // rank 0's copy, then (op)= rank 1 .. n-1: O2, aiv_reduce_scatter_mesh_1d_bigdata.h:85-101), the local tree
        // (O4, aiv_reduce_scatter_local_tree.h:138-172, and its core-control twin) otherwise. Executor loops of
        // min(UB_MAX_DATA_SIZE, ccl / 2n) per block (scratch multiple 2n); neither order depends on them.
        uint32_t blocks = coreLimit;
        if (count * es < (512ull << 10)) blocks = std::min(blocks, 2 * n);
        p.kind = kIpcReduceScatter;
        p.geom = kIpcGeomBlock;
        p.loopElems = LoopElems(std::min<uint64_t>(kUbMaxDataSize, RoundDown128(cclBytes / (2ull * n))), es);
        if (blocks > 2 * n) {
            variant = HCCL_AMD_AIV_RS_BIGDATA;
            p.order = kIpcO2;
        } else {
            variant = HCCL_AMD_AIV_RS_LOCAL_TREE;
            p.order = kIpcO4;
        }
    }
    if (plan != nullptr) *plan = p;
    if (group != nullptr) *group = g;
    return variant;
}

HcclResult RunIpcCollective(Comm& c, int32_t opType, int32_t family, const void* sendBuf, void* recvBuf,
                            uint64_t count, HcclDataType dt, HcclReduceOp op, uint32_t root, hipStream_t stream)
{
    const uint64_t es = DataTypeSize(dt);
    if (es == 0) return HCCL_E_NOT_SUPPORT;
    IpcPlan plan{};
    HCCL_CHK(IpcPlanForFamily(opType, family, c.nRanks, es, c.cclBytes, &plan));
    return RunIpcPlan(c, opType, plan, sendBuf, recvBuf, count, dt, op, root, stream);
}

HcclResult RunIpcPlan(Comm& c, int32_t opType, const IpcPlan& plan, const void* sendBuf, void* recvBuf,
                      uint64_t count, HcclDataType dt, HcclReduceOp op, uint32_t root, hipStream_t stream,
                      const uint64_t* vCounts, const uint64_t* vDispls)
{
    const HostProfileScope hp(HCCL_AMD_HP_IPC);
    if (plan.geom == kIpcGeomV && (vCounts == nullptr || vDispls == nullptr || plan.loopElems != 0)) {
        return HCCL_E_INTERNAL;
    }
    uint64_t es = DataTypeSize(dt);
    if (es == 0 || c.nRanks > kIpcMaxRanks) return HCCL_E_NOT_SUPPORT;
    uint64_t loopElems = plan.loopElems;
    if (opType == HCCL_AMD_OP_ALLGATHER) {
        // pure data movement: any dtype runs as the integer type of its size (16-B types as pairs of 8-B words)
        op = HCCL_REDUCE_SUM;
        switch (es) {
            case 1: dt = HCCL_DATA_TYPE_INT8; break;
            case 2: dt = HCCL_DATA_TYPE_INT16; break;
            case 4: dt = HCCL_DATA_TYPE_INT32; break;
            case 8: dt = HCCL_DATA_TYPE_INT64; break;
            case 16: dt = HCCL_DATA_TYPE_INT64; count *= 2; es = 8; break;
            default: return HCCL_E_NOT_SUPPORT;
        }
    }
    const IpcKind kind = static_cast<IpcKind>(plan.kind);
    // Stream capture: the barrier epochs live on the device (status word kIpcEpochWord, advanced once per launch by
    // the block that completes its arrival count), so a captured launch replays correctly: each replay takes the
    // next epochs, as a new call would. Two things cannot be captured: the collective set-up of the first call
    // (allocation, host exchange, device synchronisation) and the loopback world, which exchanges events between
    // host threads per call. Those report NOT_SUPPORT under capture; a communicator with RCCL then takes the RCCL
    // schedule of the same family. Every rank of a collective is captured alike, so they all decide the same way.
    hipStreamCaptureStatus capture = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &capture) != hipSuccess) return HCCL_E_NOT_SUPPORT;
    if (capture != hipStreamCaptureStatusNone && (!c.ipc.ready || c.transport->SharedDevice())) {
        return HCCL_E_NOT_SUPPORT;
    }
    const bool capturing = capture != hipStreamCaptureStatusNone;
    HCCL_CHK(IpcSetupBase(c));
    IpcState& s = c.ipc;
    const uint32_t n = c.nRanks;
    // workgroups per rank (equal on every rank: block b pairs with block b of each peer, and the default is a function
    // of the call's arguments alone). A loopback world runs every rank's blocks in one launch on one GPU, so it keeps
    // at most kIpcBlocks per rank to stay co-resident.
    const bool blockLayout = opType == HCCL_AMD_OP_REDUCE_SCATTER || opType == HCCL_AMD_OP_ALLGATHER;
    uint64_t callBytes = (blockLayout ? uint64_t(c.nRanks) : 1u) * count * es;  // RS input / AG output
    if (plan.geom == kIpcGeomV) {
        callBytes = 0;
        for (uint32_t q = 0; q < c.nRanks; ++q) callBytes += vCounts[q] * es;
    }
    // The LL form (HCCL_AMD_IPC_LL_BYTES; LlOneShot): a one-shot AllReduce of at most that many bytes per rank (and
    // kIpcLlMaxBytes), one launch of one round. The decision depends only on the call's arguments and the
    // configuration, which every rank shares, so every rank takes the same form.
    // The ReduceScatter takes it too (equal blocks of `count`, each at most that many bytes): like the one-shot, every
    // rank receives from every peer in every launch.
    IpcArgs a{};
    const bool llKind = (kind == kIpcAllReduceOneShot && opType == HCCL_AMD_OP_ALLREDUCE && plan.geom == kIpcGeomWhole) ||
                        (kind == kIpcReduceScatter && opType == HCCL_AMD_OP_REDUCE_SCATTER && plan.geom == kIpcGeomBlock);
    a.ll = (llKind && (loopElems == 0 || count <= loopElems) &&
            count * es <= std::min<uint64_t>(c.cfg.ipcLlBytes, kIpcLlMaxBytes))
               ? 1u
               : 0u;
    s.blocks = c.ipcBlocks != 0               ? c.ipcBlocks
               : a.ll != 0                    ? LlIpcBlocks(n, count * es, plan.order == kIpcRhd)
                                              : DefaultIpcBlocks(callBytes);
    if (c.transport->SharedDevice() && c.ipcBlocks == 0) s.blocks = std::min(s.blocks, kIpcBlocks);
    // Co-residency: every block waits at barriers for its peers' blocks, so all blocks on this device must be resident
    // at once (a loopback world puts every rank's blocks on it; in rank mode, the ranks whose processes share this
    // device, counted at set-up by PCI bus id). The count depends only on the kernel, the device and the placement,
    // so ranks of a node agree on it.
    {
        const uint32_t here = c.transport->SharedDevice() ? n : std::max<uint32_t>(1, s.ranksOnDevice);
        const uint32_t resident = IpcResidentBlocks(dt, op, plan.order == kIpcRhd, a.ll != 0, c.cfg.ipcThreads);
        if (resident != 0) s.blocks = std::max<uint32_t>(1, std::min(s.blocks, resident / here));
    }
    const uint64_t V = 16 / es;

    for (uint32_t r = 0; r < n; ++r) a.flags[r] = s.peerFlags[r];
    a.n = n;
    a.kind = kind;
    a.order = plan.order;
    a.subMode = plan.subMode;
    a.root = root;
    a.timeoutTicks = c.cfg.ipcTimeoutMs * 100000;  // a lost peer ends the kernel with status bit 0, never a hang
    a.status = s.status;
    a.failHost = s.failDev;
    a.callSeq = ++s.callSeq;  // equal on every rank of a loopback world (each runs this once per call)
    a.outStride = count;
    a.trace = s.trace;
    if (plan.order == kIpcRhd) {
        // the RHD schedule's parts and relabelling (AllReduceRhd): R instances over Chunk(count, R, j) parts
        const std::vector<std::vector<uint32_t>> table = RhdTable(n);
        const uint32_t parts = std::min<uint32_t>(static_cast<uint32_t>(table.size()), RhdInstances(n, count * es));
        if (parts == 0 || loopElems != 0) return HCCL_E_INTERNAL;
        a.rhdParts = parts;
        a.alignElems = static_cast<uint32_t>(std::max<uint64_t>(1, 128 / es));
        const uint64_t stride = (count + parts - 1) / parts;
        a.rhdPartStride = std::max<uint64_t>(1, (stride + a.alignElems - 1) / a.alignElems * a.alignElems);
        for (uint32_t j = 0; j < parts; ++j) {
            for (uint32_t v = 0; v < n; ++v) a.rhdReal[j][v] = static_cast<uint8_t>(table[j][v]);
        }
    }
    const bool single = SingleBarrierKind(kind);
    // slot capacity of a tier in elements (a round's piece of every chunk must fit n slots)
    const auto capOf = [&](const IpcTier& t) { return ((single ? t.altBytes : t.inBytes) / es / n) / V * V; };
    uint64_t slotCap = capOf(IpcTierSizes(c, kIpcTierSmall));

    // One launch per executor loop [off, off + cnt) of the reference template whose order the fold follows: its
    // slicing is per loop (schedule.cc RefLoopElems and the MeshChunk loops). A ReduceScatter loop takes elements
    // [off, off + cnt) of every block.
    struct Launch {
        uint64_t off, cnt;
    };
    std::vector<Launch> launches;
    if (plan.geom == kIpcGeomV) {
        // one launch on every rank, whatever this rank's own block: the launch is collective (every block meets its
        // peers at the barriers), and a rank whose block is empty still pushes its share of the others' blocks
        launches.push_back({0, 0});
    } else {
        if (loopElems == 0) loopElems = count;
        for (uint64_t off = 0; off < count; off += loopElems) {
            launches.push_back({off, std::min(loopElems, count - off)});
        }
    }
    auto geometry = [&](IpcArgs& g, uint64_t cnt) {
        g.balanced = false;
        g.vgeom = false;
        g.group = 1;
        g.rem = 0;
        g.total = cnt;
        switch (plan.geom) {
            case kIpcGeomV:
                // ReduceScatterV: rank c's block is counts[c] elements at displs[c] of every input (one launch: the
                // mesh order O1 does not depend on executor loops)
                g.vgeom = true;
                g.chunkStride = 0;
                g.chunkLen = 0;
                for (uint32_t q = 0; q < n; ++q) {
                    g.vStart[q] = vDispls[q];
                    g.vLen[q] = vCounts[q];
                    g.chunkLen = std::max(g.chunkLen, vCounts[q]);
                }
                break;
            case kIpcGeomBlock:
                // block c of the input (recvCount elements, stride recvCount) is chunk c (reduce_scatter_op.cc:158-159)
                g.chunkStride = count;
                g.chunkLen = cnt;
                g.total = uint64_t(n - 1) * count + cnt;
                break;
            case kIpcGeomBalanced: {
                const uint64_t slices = uint64_t(plan.group) * n;
                g.balanced = true;
                g.group = plan.group;
                g.chunkLen = cnt / slices;  // slice length; the first cnt % slices slices hold one more
                g.rem = cnt % slices;
                g.chunkStride = 0;
                break;
            }
            case kIpcGeomWhole:
                // every rank holds (and, for the AllReduce, folds) the whole range; AllGather: its whole input
                g.chunkStride = 0;
                g.chunkLen = cnt;
                break;
            case kIpcGeomCeil:
                g.chunkStride = g.chunkLen = (cnt + n - 1) / n;
                break;
            default: {
                const uint64_t align = 128 / es;  // HCCL_MIN_SLICE_ALIGN
                g.chunkStride = g.chunkLen = ((cnt + n - 1) / n + align - 1) / align * align;
                break;
            }
        }
        const uint64_t widest = g.balanced ? g.group * g.chunkLen + std::min<uint64_t>(g.group, g.rem) : g.chunkLen;
        g.piece = std::max<uint64_t>(V, std::min(slotCap, (widest + V - 1) / V * V));
        g.blockElems = ((g.piece + s.blocks - 1) / s.blocks + V - 1) / V * V;
        g.tileElems = c.cfg.ipcTileBytes / es / V * V;  // 0: contiguous windows (HCCL_AMD_IPC_TILE_KIB)
        g.nt = c.cfg.ipcNt ? 1u : 0u;                     // non-temporal loads and stores (HCCL_AMD_IPC_NT)
        g.fence = IpcLightFence(c) ? 1u : 0u;
        g.threads = c.cfg.ipcThreads;                    // HCCL_AMD_IPC_THREADS
        g.rounds = static_cast<uint32_t>((widest + g.piece - 1) / g.piece);
        g.epochSpan = (single ? 1 : 2) * g.rounds;
        if (g.ll != 0 && g.rounds == 1) {  // one window per block, no barrier epochs (the LL sequence advances)
            g.tileElems = 0;
            g.epochSpan = 0;
        } else {
            g.ll = 0;
        }
    };
    auto at = [es](const void* p, uint64_t off) { return static_cast<char*>(const_cast<void*>(p)) + off * es; };

    // The staging tier (IpcTier): the small one when every launch of the call fits one round there, else the large
    // one (also when the small tier's set-up failed). The choice depends on the call's arguments and the configuration
    // at the set-up, equal on every rank, and each tier's availability is agreed, so every rank takes the same tier.
    // The LL form uses no staging area (its words travel through the flags allocation's LL area).
    bool fitsSmall = true;
    for (const Launch& l : launches) {
        IpcArgs g = a;
        geometry(g, l.cnt);
        fitsSmall = fitsSmall && g.rounds == 1;
    }
    if (a.ll == 0) {
        int t = fitsSmall && !s.tier[kIpcTierSmall].unavailable ? kIpcTierSmall : kIpcTierLarge;
        if (capturing && !s.tier[t].ready) return HCCL_E_NOT_SUPPORT;  // no collective set-up under capture
        HcclResult r = IpcSetupTier(c, t);
        if (r == HCCL_E_NOT_SUPPORT && t == kIpcTierSmall) {
            t = kIpcTierLarge;
            if (capturing && !s.tier[t].ready) return HCCL_E_NOT_SUPPORT;
            r = IpcSetupTier(c, t);
        }
        HCCL_CHK(r);
        const IpcTier& tr = s.tier[t];
        slotCap = capOf(tr);
        for (uint32_t q = 0; q < n; ++q) {
            a.stgIn[q] = tr.peerArea[kIpcAreaIn][q];
            a.stgRes[q] = tr.peerArea[kIpcAreaRes][q];
            a.stgAlt[0][q] = tr.peerArea[kIpcAreaAlt0][q];
            a.stgAlt[1][q] = tr.peerArea[kIpcAreaAlt1][q];
        }
    }

    if (!c.transport->SharedDevice()) {
        a.me = static_cast<int32_t>(c.rank);
        a.aligned = Aligned16(sendBuf, recvBuf);
        a.llUnpack[c.rank] = s.llUnpack;
        for (const Launch& l : launches) {
            a.in[c.rank] = at(sendBuf, l.off);
            a.out[c.rank] = at(recvBuf, l.off);
            geometry(a, l.cnt);
            HCCL_CHK(LaunchIpcCollective(a, s.blocks, 0, dt, op, stream));
        }
        return HCCL_SUCCESS;
    }

    // loopback world: one launch for every rank, issued by rank 0 behind every rank's stream. Every rank takes part in
    // both exchanges whatever its local outcome (one that returned early would leave the others in the rendezvous),
    // and a failure anywhere is every rank's result.
    struct Part {
        const void* in;
        void* out;
        void* unpack;
        hipEvent_t ready;
        int32_t code;
    };
    Part mine{sendBuf, recvBuf, s.llUnpack, nullptr, HCCL_SUCCESS};
    c.nextEvent = 0;
    mine.code = c.NextEvent(&mine.ready);
    if (mine.code == HCCL_SUCCESS && hipEventRecord(mine.ready, stream) != hipSuccess) mine.code = HCCL_E_RUNTIME;
    std::vector<Part> all(n);
    HCCL_CHK(c.transport->AllGatherHost(&mine, sizeof mine, all.data()));
    HcclResult code = HCCL_SUCCESS;
    for (uint32_t r = 0; r < n && code == HCCL_SUCCESS; ++r) code = static_cast<HcclResult>(all[r].code);
    struct Done {
        hipEvent_t ev;
        int32_t code;
    };
    Done done{nullptr, code};
    if (c.rank == 0 && code == HCCL_SUCCESS) {
        a.me = -1;
        a.aligned = true;
        for (uint32_t r = 0; r < n && done.code == HCCL_SUCCESS; ++r) {
            a.aligned = a.aligned && Aligned16(all[r].in, all[r].out);
            if (hipStreamWaitEvent(stream, all[r].ready, 0) != hipSuccess) done.code = HCCL_E_RUNTIME;
        }
        for (size_t k = 0; k < launches.size() && done.code == HCCL_SUCCESS; ++k) {
            for (uint32_t r = 0; r < n; ++r) {
                a.in[r] = at(all[r].in, launches[k].off);
                a.out[r] = at(all[r].out, launches[k].off);
                a.llUnpack[r] = all[r].unpack;
            }
            geometry(a, launches[k].cnt);
            done.code = LaunchIpcCollective(a, s.blocks, n, dt, op, stream);
        }
        if (done.code == HCCL_SUCCESS) done.code = c.NextEvent(&done.ev);
        if (done.code == HCCL_SUCCESS && hipEventRecord(done.ev, stream) != hipSuccess) done.code = HCCL_E_RUNTIME;
    }
    std::vector<Done> dones(n);
    HCCL_CHK(c.transport->AllGatherHost(&done, sizeof done, dones.data()));
    if (dones[0].code != HCCL_SUCCESS) return static_cast<HcclResult>(dones[0].code);
    if (c.rank != 0) HIP_CHK(hipStreamWaitEvent(stream, dones[0].ev, 0));
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
    uint32_t w[4] = {0, 0, 0, 0};
    HIP_CHK(hipMemcpy(w, c->ipc.status, sizeof w, hipMemcpyDeviceToHost));
    const uint32_t wait = w[3] == c->ipc.callSeq ? w[2] : 0;  // an older tag: no block of the last call waited
    uint32_t lg = 0;
    while (lg < 32 && (uint64_t(1) << lg) <= wait) ++lg;  // bit length of the longest wait
    *status = (w[0] & 0xFFu) | (lg << 8);
    return HCCL_SUCCESS;
}

extern "C" HcclResult HcclAmdCommIpcLlLaunches(HcclComm comm, uint32_t* launches)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || launches == nullptr) return HCCL_E_PTR;
    *launches = 0;
    if (!c->ipc.ready) return HCCL_SUCCESS;
    HIP_CHK(hipSetDevice(c->device));
    HIP_CHK(hipMemcpy(launches, c->ipc.status + kIpcLlSeqWord, sizeof *launches, hipMemcpyDeviceToHost));
    return HCCL_SUCCESS;
}

extern "C" HcclResult HcclAmdCommIpcTrace(HcclComm comm, uint64_t* stamps, uint64_t cap, uint32_t* blocks)
{
    Comm* c = AsComm(comm);
    if (c == nullptr || stamps == nullptr || blocks == nullptr) return HCCL_E_PTR;
    *blocks = 0;
    if (!c->ipc.ready || c->ipc.trace == nullptr) return HCCL_E_NOT_SUPPORT;
    const uint64_t want = uint64_t(kIpcMaxRanks) * kIpcMaxBlocks * kIpcTraceSlots;
    if (cap < want) return HCCL_E_PARA;
    HIP_CHK(hipSetDevice(c->device));
    HIP_CHK(hipDeviceSynchronize());
    HIP_CHK(hipMemcpy(stamps, c->ipc.trace, want * sizeof(uint64_t), hipMemcpyDeviceToHost));
    *blocks = c->ipc.blocks;
    return HCCL_SUCCESS;
}
