// ipc_kernel_body.h — device code of the one-sided AllReduce / ReduceScatter / Reduce / AllGather over peer-mapped
// staging buffers. The two-shot AllReduce is described first; the other kinds are variations of it (IpcKind).
//
// The reference's AIV engine runs AllReduce as ONE kernel whose blocks write into every peer's CCL buffer
// (GM_IN[r]) and synchronise with per-block flags (aiv_all_reduce_mesh_1d_twoshot.h:20-217,
// aiv_communication_base_v2.h:296-357). This is the MI355X form of that model, two-shot with the reference's
// deterministic order O2 (acc = x_0, then x_1 .. x_{n-1}; ins_temp_all_reduce_mesh_1D_two_shot.cc:327-335).
// PUSH only: every access to a peer's memory is a store; every load reads this rank's own uncached staging or its own
// user buffers. (A load through an imported mapping may be served by this XCD's L2, which no in-kernel acquire
// evicts, so a pull design re-reading a peer's staging in a later round can see stale lines.)
//   per round of `roundElems` elements (bounded staging), chunk c of the round is owned by rank c:
//     phase 0  rank r stores its values of chunk c into owner c's staging slot r (c != r; the owner reads its own
//              slot straight from its input)
//     barrier  block b tells block b of every rank "my stores are out", waits for theirs
//     phase 1  owner c folds slots 0..n-1 in rank order (O2), writes recvBuf and stores the result into every
//              peer's result area
//     barrier
//     phase 2  every rank copies the other chunks from its own result area
// Two barriers per round suffice: a peer's next-round phase-0 stores into my staging come after it passed barrier 2
// (so after my phase-1 reads), and its next phase-1 stores into my result area come after barrier 1 of the next
// round (so after my phase-2 reads); the same holds across calls (kernels of a stream run in order). The kinds with
// no result push and no phase 2 (ReduceScatter, one-shot) keep only the first barrier and alternate their slots
// between two areas of their own instead (k_ipc_collective; model-checked by tests/test_ipc_protocol.py).
// Every round of one launch has the same geometry (the host launches a shorter last round separately), so block b
// of every rank touches the same slot and result addresses in every round and only waits for block b of its peers;
// nothing in a GPU waits for another block of the same GPU. Every storing wave drains (s_waitcnt vmcnt(0)) before the
// workgroup barrier; since every handed-over byte is in uncached staging that drain is the release (IpcArgs::fence 1,
// the loopback world's default; fence 0, rank mode's default, adds the system-scope L2 write-back), and one wave stores
// the flags with system-scope stores;
// flags are polled with system-scope relaxed loads and followed by an acquire (agent scope: the CU's L1; fence 0:
// system scope; IpcLightFence in ipc.cc). Every wait is bounded
// in wall time (s_memrealtime, HCCL_AMD_IPC_TIMEOUT_MS): on timeout the kernel sets status bit 0 and finishes (wrong
// data, never a hang); the bit is sticky for the communicator, so later launches return at once. World mode (me < 0) runs all
// n ranks of a loopback world as blockIdx.y of one launch on one GPU, which is how the protocol is tested without a
// second GPU; the rank-mode path (one launch per process, peers opened from IPC handles) is tested with n processes
// sharing the GPU.
#pragma once
// Included by the per-dtype translation units ipc_k_*.hip (compiled in parallel); ipc_kernels.hip holds the
// dispatch over them. Every TU instantiates its dtypes' kernels from this one definition.
#include <hip/hip_runtime.h>

#include <atomic>
#include <type_traits>

#include "internal.h"
#include "ipc.h"
#include "reduce_elem.h"

namespace hccl_amd {

namespace {

// Returns false when this block's wait was cut short: its own timeout, or a timeout another block of this rank already
// set (status bit 0). The caller then stops at once, so a rank never stores into a peer it has lost track of. The
// longest wait (in polls) stays in the lane's `waitMax` and is published once per launch (PublishWait), off the
// barrier's critical path.
// The flag words lane t (< n) of block b uses in every barrier: the one it stores into on peer t, and the one peer t
// stores into here (the pointer table is in kernel-argument memory, indexed per lane).
struct FlagLane {
    uint32_t* remote;
    uint32_t* mine;
};

__device__ __forceinline__ FlagLane LaneFlags(const IpcArgs& a, uint32_t me)
{
    const uint32_t t = threadIdx.x;
    if (t >= a.n) return {nullptr, nullptr};
    return {a.flags[t] + blockIdx.x * a.n + me, a.flags[me] + blockIdx.x * a.n + t};
}

__device__ __forceinline__ bool Barrier(const IpcArgs& a, FlagLane fl, uint32_t epoch, uint32_t& waitMax)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its stores have left the CU
    __syncthreads();
    __shared__ uint32_t failed;
    const uint32_t t = threadIdx.x;
    if (t < a.n) {
        if (t == 0) failed = 0;  // every thread read the previous barrier's value before the __syncthreads above
        // System-scope release: the L2 write-back (buffer_wbl2 sc0 sc1). Every wave of the block has drained its
        // stores (vmcnt(0)) before the workgroup barrier, so the write-back covers the whole block's data. The flag
        // store must wait for the write-back, and ROCm 7.2 drops that s_waitcnt vmcnt(0) where it can prove the
        // wave's counter empty (MI355X_MICROARCH.md, "Compiler hazard"): the release store form lost it in 8 of the
        // 73 instantiations (the epoch load before it is a waited load), so a peer could read the data before it
        // left this XCD's L2. The explicit wait, invisible to that pass, keeps the flag behind the write-back.
        // IpcArgs::fence = 1 (light): the handed-off bytes are all in uncached staging, whose stores no L2 holds, so
        // the waves' vmcnt(0) drains above are the release; no XCD-wide write-back.
        if (a.fence == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(fl.remote, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        uint32_t* mine = fl.mine;
        uint32_t polls = 0;
        bool cut = false;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
        // wrap-safe: the 32-bit epochs never reset (2 per round and call); a peer's flag is behind while the signed
        // difference is negative, which stays true across the wrap at 2^32
        while (static_cast<int32_t>(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) <
               0) {
            ++polls;
            if ((polls & 63u) == 0) {
                // a timeout anywhere (this or another block of this rank) ends the wait at once
                if ((__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 1u) != 0) {
                    cut = true;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeoutTicks) {
                    __hip_atomic_fetch_or(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    // the host sees the failure without a device synchronisation: the next collective on this
                    // communicator returns HCCL_E_TIMEOUT (Comm::Gate), every later one HCCL_E_SUSPENDING
                    __hip_atomic_store(a.failHost, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    cut = true;
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(2);
        }
        waitMax = max(waitMax, polls);
        if (cut) failed = 1;
        // light: the CU's L1 only (agent scope); the system-scope acquire also invalidates the XCD's whole L2
        if (a.fence == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        } else {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate has completed before the barrier opens
    }
    __syncthreads();
    return failed == 0;
}

// Longest barrier wait of this call: one 64-bit max per lane and launch into status words 2..3, tagged with the
// call's sequence number in the high half, so a new call needs no reset (HcclAmdCommIpcStatus keeps only its own tag).
__device__ __forceinline__ void PublishWait(const IpcArgs& a, uint32_t waitMax)
{
    if (threadIdx.x < a.n && waitMax != 0) {
        __hip_atomic_fetch_max(reinterpret_cast<unsigned long long*>(a.status + 2),
                               (static_cast<unsigned long long>(a.callSeq) << 32) | waitMax, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Epoch counter protocol. Every block reads the counter at its start, then counts itself in the arrival word
// (kIpcDoneWord), in that order: the count is issued only once the read has returned. The block whose arrival
// completes the grid advances the counter by the launch's barriers per block and resets the count (EndLaunch).
// Every block read before it arrived, so no block of this launch can see the advanced value. The next launch in
// stream order starts only after this one has ended, so it sees it. The arrival is a returning atomic issued at the
// start, and its value is consumed only at the end, so its round trip overlaps the launch's work. A launch that
// returns at once on a failed communicator (sticky bit) never arrives; no later launch waits on it.
__device__ __forceinline__ uint32_t Arrive(const IpcArgs& a, uint32_t epoch)
{
    if (threadIdx.x != 0) return 0;
    asm volatile("" ::"v"(epoch) : "memory");  // the counter read has returned before the arrival is issued
    // The offset is zero, but the compiler cannot see it: an address it takes for uniform across the wave gets the
    // wave-combined atomic, whose per-lane result is computed (and waited for) right here instead of at EndLaunch.
    uint32_t zero = 0;
    asm volatile("" : "+v"(zero));
    return __hip_atomic_fetch_add(a.status + kIpcDoneWord + zero, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void EndLaunch(const IpcArgs& a, uint32_t arrivedBefore)
{
    // opaque until here: otherwise the compiler folds the comparison's + 1 into Arrive's branch and waits for the
    // arrival's round trip at the launch's start, before the first store
    asm volatile("" : "+v"(arrivedBefore));
    if (threadIdx.x == 0 && arrivedBefore + 1 == gridDim.x * gridDim.y) {
        __hip_atomic_store(a.status + kIpcDoneWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // an LL launch has no barrier epochs; it advances the LL sequence instead (LlOneShot)
        __hip_atomic_fetch_add(a.status + (a.ll != 0 ? kIpcLlSeqWord : kIpcEpochWord), a.ll != 0 ? 1u : a.epochSpan,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Phase stamp (HCCL_AMD_IPC_TRACE): lane 0 of the block, one 8-B vector store per stamp; nothing when tracing is off.
__device__ __forceinline__ void Stamp(const IpcArgs& a, uint32_t me, uint32_t slot)
{
    if (a.trace == nullptr || threadIdx.x != 0) return;
    a.trace[(uint64_t(me) * kIpcMaxBlocks + blockIdx.x) * kIpcTraceSlots + slot] = __builtin_amdgcn_s_memrealtime();
}

struct Range {
    uint64_t lo, hi;  // piece coordinates
};

__device__ __forceinline__ uint64_t ChunkStart(const IpcArgs& a, uint32_t c)
{
    if (a.vgeom) return a.vStart[c];
    const uint64_t s = uint64_t(c) * a.group;  // first slice of chunk c (balanced)
    return a.balanced ? s * a.chunkLen + min(s, a.rem) : uint64_t(c) * a.chunkStride;
}

__device__ __forceinline__ uint64_t ChunkElems(const IpcArgs& a, uint32_t c)
{
    if (a.vgeom) return a.vLen[c];
    if (a.balanced) {
        const uint64_t s = uint64_t(c) * a.group;
        return a.group * a.chunkLen + (a.rem > s ? min(a.group, a.rem - s) : 0);
    }
    const uint64_t start = uint64_t(c) * a.chunkStride;
    return start >= a.total ? 0 : min(a.chunkLen, a.total - start);
}

// 16-B vectors for chunk c: the user buffers are aligned and so is the chunk's first element
template <typename S>
__device__ __forceinline__ bool ChunkVec(const IpcArgs& a, uint32_t c)
{
    return a.aligned && ChunkStart(a, c) % (16 / sizeof(S)) == 0;
}

// Elements of chunk c in round k (piece coordinates [0, len)), and the block's fixed window clipped to it.
__device__ __forceinline__ uint64_t PieceLen(const IpcArgs& a, uint32_t c, uint64_t kP)
{
    const uint64_t clen = ChunkElems(a, c);
    return kP >= clen ? 0 : min(a.piece, clen - kP);
}

__device__ __forceinline__ Range BlockWindow(const IpcArgs& a, uint64_t len)
{
    const uint64_t lo = min(len, uint64_t(blockIdx.x) * a.blockElems);
    return {lo, min(len, lo + a.blockElems)};
}

// The block's share of piece coordinates [0, len): f(range) for one window of blockElems (tileElems == 0), or for
// each tile of tileElems at b, b + B, b + 2B, ... (B = blocks of the launch). Both depend on the block and the piece
// only, so block b touches the same coordinates in every round, which its per-block barrier relies on.
template <class F>
__device__ __forceinline__ void ForBlockShare(const IpcArgs& a, uint64_t len, F&& f)
{
    if (a.tileElems == 0) {
        f(BlockWindow(a, len));
        return;
    }
    const uint64_t step = uint64_t(gridDim.x) * a.tileElems;
    for (uint64_t lo = uint64_t(blockIdx.x) * a.tileElems; lo < len; lo += step) f(Range{lo, min(len, lo + a.tileElems)});
}

constexpr int kIpcU = 4;  // vectors per lane in flight (r03 A/B of 2, 4, 8: profiles/r03_ipc_variant_ab_unroll.jsonl)

template <int NT>
__device__ __forceinline__ void CopyVecs(u32x4* d, const u32x4* s, uint64_t& v, uint64_t vhi, uint32_t bt)
{
    for (; v + (kIpcU - 1) * bt < vhi; v += kIpcU * bt) {
        u32x4 x[kIpcU];
#pragma unroll
        for (int u = 0; u < kIpcU; ++u) x[u] = ld<NT>(s + v + u * bt);
#pragma unroll
        for (int u = 0; u < kIpcU; ++u) st<NT>(d + v + u * bt, x[u]);
    }
    for (; v < vhi; v += bt) st<NT>(d + v, ld<NT>(s + v));
}

// dst[e] = src[e] for e in r. vec = both pointers are 16-B aligned; otherwise every element goes through the scalar
// loop. nt: non-temporal loads and stores (IpcArgs::nt).
template <typename S>
__device__ __forceinline__ void CopyRange(S* dst, const S* src, Range r, bool vec, bool nt, uint32_t bt)
{
    constexpr uint64_t V = 16 / sizeof(S);
    // r.lo is vector aligned unless the window is empty at the end of a piece (lo = hi = len); r.hi may be anything
    const uint64_t vlo = r.lo / V, vhi = vec ? max(vlo, r.hi / V) : vlo;
    const u32x4* s = reinterpret_cast<const u32x4*>(src);
    u32x4* d = reinterpret_cast<u32x4*>(dst);
    uint64_t v = vlo + threadIdx.x;
    if (nt) {
        CopyVecs<3>(d, s, v, vhi, bt);
    } else {
        CopyVecs<0>(d, s, v, vhi, bt);
    }
    for (uint64_t e = max(vhi * V, r.lo) + threadIdx.x; e < r.hi; e += bt) dst[e] = src[e];
}

// Rank of operand i (0 .. n-1) of a fold of chunk t in the given order; j = the sub-slice (kIpcO6 only).
__device__ __forceinline__ uint32_t OperandRank(uint32_t order, uint32_t n, uint32_t t, uint32_t j, uint32_t i)
{
    if (order == kIpcO2) return i;
    if (i == 0) return t;
    if (order == kIpcO1) return i <= t ? i - 1 : i;
    uint32_t x = i + j;  // kIpcO6: step s = i - 1 brings nextNum = s + j + 1, plus one once it reaches n
    if (x >= n) x += 1;
    return (t + x) % n;
}

// First element (chunk coordinates) of sub-slice j of a chunk of L elements; SubStart(n-1) = L.
template <typename S>
__device__ __forceinline__ uint64_t SubStart(const IpcArgs& a, uint64_t L, uint32_t j)
{
    const uint32_t parts = a.n - 1;
    if (j >= parts) return L;
    if (a.subMode == kIpcSubRs4K && parts >= 2) {
        const uint64_t al = L * sizeof(S) / parts / 4096 * 4096 / sizeof(S);
        if (al != 0) return uint64_t(j) * al;
    }
    const uint64_t base = L / parts, big = L % parts;
    return uint64_t(j) * base + min(uint64_t(j), big);
}

template <class E, int OP>
__device__ __forceinline__ u32x4 Comb(u32x4 s, u32x4 d)
{
    return combine<E, OP>(s, d);
}

template <class E, int OP>
__device__ __forceinline__ typename E::S Comb(typename E::S s, typename E::S d)
{
    return E::template ap<OP>(s, d);
}

// Bit reversal of t over log2(M) bits (M a power of two), and the number of trailing one bits of t.
template <int M>
constexpr uint32_t BitRev(uint32_t t)
{
    uint32_t r = 0;
    for (int m = M >> 1, b = 1; m > 0; m >>= 1, b <<= 1) {
        if (t & uint32_t(b)) r |= uint32_t(m);
    }
    return r;
}

constexpr int TrailingOnes(int t)
{
    int c = 0;
    while (t & 1) {
        ++c;
        t >>= 1;
    }
    return c;
}

constexpr int Log2(int m) { return m <= 1 ? 0 : 1 + Log2(m >> 1); }

// Step T of TreeFold: first-round value number BitRev(T), then the merges its position completes.
template <class E, int OP, int M, int T, int D, class Leaf, class V>
__device__ __forceinline__ V TreeStep(uint32_t n, const Leaf& leaf, V (&st)[D])
{
    constexpr uint32_t jj = BitRev<M>(uint32_t(T));
    V x = leaf(jj);
    if (jj + M < n) x = Comb<E, OP>(leaf(jj + M), x);
    constexpr int lvl = TrailingOnes(T);
#pragma unroll
    for (int b = 0; b < lvl; ++b) x = Comb<E, OP>(x, st[b]);  // the later partial is src, the earlier one dst
    if constexpr (T + 1 < M) {
        st[lvl] = x;
        return TreeStep<E, OP, M, T + 1>(n, leaf, st);
    } else {
        return x;
    }
}

// Order O4 over the n sources (leaf(q) = operand of rank q), M = the largest power of two below n
// (GetLargestPowerOf2, aiv_reduce_scatter_local_tree.h:95-105). Round one folds x_{j+M} into x_j for j + M < n; the
// rounds after it halve a power-of-two set: L'(j) = L(j + h) (op) L(j). Visiting the first-round values in bit-reversed
// index order makes every later pair adjacent, so the rounds become a binary counter over a register stack: each
// value merges as src into the partial below it (dst), exactly the (src, dst) roles of the template's
// CpGM2GM(front, back, reduceOp) = front (op)= back. Every stack index is a compile-time constant.
template <class E, int OP, int M, class Leaf>
__device__ __forceinline__ auto TreeFold(uint32_t n, const Leaf& leaf)
{
    using V = decltype(leaf(0u));
    V st[Log2(M) > 0 ? Log2(M) : 1];
    return TreeStep<E, OP, M, 0>(n, leaf, st);
}

// Dispatch of TreeFold on M (n <= 16: M <= 8).
template <class E, int OP, class Leaf>
__device__ __forceinline__ auto TreeFoldN(uint32_t n, const Leaf& leaf)
{
    if (n > 8) return TreeFold<E, OP, 8>(n, leaf);
    if (n > 4) return TreeFold<E, OP, 4>(n, leaf);
    if (n > 2) return TreeFold<E, OP, 2>(n, leaf);
    return TreeFold<E, OP, 1>(n, leaf);
}

// Order O4 over the piece range r: operand q of the tree is rank rankOf(q)'s (rankSrc gives a rank's operand in piece
// coordinates). One vector (or element) per lane and step keeps the register stack small.
template <class E, int OP, class Dst, class RankSrc, class RankOf>
__device__ __forceinline__ void TreeSeg(uint32_t n, const RankSrc& rankSrc, const RankOf& rankOf, Dst dsts,
                                        uint32_t ndst, Range r, bool vec, uint32_t bt)
{
    using S = typename E::S;
    constexpr uint64_t V = 16 / sizeof(S);
    const uint64_t vb = (r.lo + V - 1) / V, ve = r.hi / V;
    auto scalarTree = [&](uint64_t lo, uint64_t hi) {
        for (uint64_t e = lo + threadIdx.x; e < hi; e += bt) {
            const S acc = TreeFoldN<E, OP>(n, [&](uint32_t q) { return rankSrc(rankOf(q))[e]; });
            for (uint32_t d = 0; d < ndst; ++d) dsts(d)[e] = acc;
        }
    };
    if (!vec || vb >= ve) {
        scalarTree(r.lo, r.hi);
        return;
    }
    scalarTree(r.lo, vb * V);
    for (uint64_t v = vb + threadIdx.x; v < ve; v += bt) {
        const u32x4 acc = TreeFoldN<E, OP>(
            n, [&](uint32_t q) { return reinterpret_cast<const u32x4*>(rankSrc(rankOf(q)))[v]; });
        for (uint32_t d = 0; d < ndst; ++d) reinterpret_cast<u32x4*>(dsts(d))[v] = acc;
    }
    scalarTree(ve * V, r.hi);
}

// Fold of the piece range r (piece coordinates) of chunk `me` over the n operands, operand i being rank
// OperandRank(order, n, me, j, i) (order O4: the tree over the ranks), written to ndst destinations. own = this rank's
// operand, slots = its staging (slot q at q * piece). vec: the chunk's operands are 16-B aligned at piece coordinate
// 0; r may start and end anywhere (scalar head and tail around the vector body).
template <class E, int OP, class Dst>
__device__ __forceinline__ void FoldSeg(const IpcArgs& a, uint32_t me, uint32_t j, const typename E::S* own,
                                        const typename E::S* slots, Dst dsts, uint32_t ndst, Range r, bool vec)
{
    using S = typename E::S;
    constexpr uint64_t V = 16 / sizeof(S);
    const uint32_t n = a.n;
    auto rankSrc = [&](uint32_t q) { return q == me ? own : slots + uint64_t(q) * a.piece; };
    if (a.order == kIpcO4) {
        // rank-independent tree
        TreeSeg<E, OP>(n, rankSrc, [](uint32_t q) { return q; }, dsts, ndst, r, vec, a.threads);
        return;
    }
    auto src = [&](uint32_t i) { return rankSrc(OperandRank(a.order, n, me, j, i)); };
    auto scalar = [&](uint64_t lo, uint64_t hi) {
        for (uint64_t e = lo + threadIdx.x; e < hi; e += a.threads) {
            S acc = src(0)[e];
            for (uint32_t i = 1; i < n; ++i) acc = E::template ap<OP>(src(i)[e], acc);
            for (uint32_t d = 0; d < ndst; ++d) dsts(d)[e] = acc;
        }
    };
    const uint64_t vb = (r.lo + V - 1) / V, ve = r.hi / V;
    if (!vec || vb >= ve) {
        scalar(r.lo, r.hi);
        return;
    }
    scalar(r.lo, vb * V);
    uint64_t v = vb + threadIdx.x;
    auto body = [&](auto ntTag) {
        constexpr int NT = decltype(ntTag)::value;
        constexpr int U = kIpcU;
        for (; v + (U - 1) * a.threads < ve; v += U * a.threads) {
            u32x4 acc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] = ld<NT>(reinterpret_cast<const u32x4*>(src(0)) + v + u * a.threads);
            for (uint32_t i = 1; i < n; ++i) {
                u32x4 x[U];
#pragma unroll
                for (int u = 0; u < U; ++u) x[u] = ld<NT>(reinterpret_cast<const u32x4*>(src(i)) + v + u * a.threads);
#pragma unroll
                for (int u = 0; u < U; ++u) acc[u] = combine<E, OP>(x[u], acc[u]);
            }
            for (uint32_t d = 0; d < ndst; ++d) {
#pragma unroll
                for (int u = 0; u < U; ++u) st<NT>(reinterpret_cast<u32x4*>(dsts(d)) + v + u * a.threads, acc[u]);
            }
        }
    };
    if (a.nt != 0) {
        body(std::integral_constant<int, 3>{});
    } else {
        body(std::integral_constant<int, 0>{});
    }
    for (; v < ve; v += a.threads) {
        u32x4 acc = reinterpret_cast<const u32x4*>(src(0))[v];
        for (uint32_t i = 1; i < n; ++i) acc = combine<E, OP>(reinterpret_cast<const u32x4*>(src(i))[v], acc);
        for (uint32_t d = 0; d < ndst; ++d) reinterpret_cast<u32x4*>(dsts(d))[v] = acc;
    }
    scalar(ve * V, r.hi);
}

// Order kIpcRhd (one-shot kind, whole range: piece coordinate e is element kP + e of the launch). The RHD AllReduce
// (schedule.cc AllReduceRhd) splits the buffer into R parts, instance j running the classic recursive halving on
// virtual ranks (virtual v = real rhdReal[j][v]) over n chunks of its part, each fold dst = partner (op) mine. The
// element's value is then the O4 tree over the operands of virtual ranks v ^ q, q = 0 .. n-1, v its chunk's owner:
// round M of O4 folds leaf q + M into leaf q, which is exactly the step at distance M folding partner v ^ q ^ M into
// v ^ q (tests/test_ipc_rhd_order.py checks the identity against the schedule's closed form). Split the window at
// part and chunk boundaries (Chunk() of schedule.cc: ceil splits rounded up to HCCL_MIN_SLICE_ALIGN).
template <class E, int OP, class Dst>
__device__ __forceinline__ void RhdFold(const IpcArgs& a, uint32_t me, uint64_t kP, const typename E::S* own,
                                        const typename E::S* slots, Dst dsts, uint32_t ndst, Range r, bool vec)
{
    const uint32_t n = a.n;
    auto rankSrc = [&](uint32_t q) { return q == me ? own : slots + uint64_t(q) * a.piece; };
    uint64_t g = kP + r.lo;
    const uint64_t g1 = kP + r.hi;
    while (g < g1) {
        const uint32_t j = static_cast<uint32_t>(g / a.rhdPartStride);
        const uint64_t pb = uint64_t(j) * a.rhdPartStride;
        const uint64_t plen = min(a.total, pb + a.rhdPartStride) - pb;
        const uint64_t sc = ((plen + n - 1) / n + a.alignElems - 1) / a.alignElems * a.alignElems;
        const uint32_t v = static_cast<uint32_t>((g - pb) / sc);
        const uint64_t end = min(g1, pb + min(plen, uint64_t(v + 1) * sc));
        // operand q of the tree is real rank rhdReal[j][v ^ q], packed 4 bits per operand (n <= 16) so the tree's
        // compile-time operand numbers select it with a shift
        uint64_t packed = 0;
        for (uint32_t q = 0; q < n; ++q) packed |= uint64_t(a.rhdReal[j][v ^ q]) << (4 * q);
        TreeSeg<E, OP>(n, rankSrc, [packed](uint32_t q) { return uint32_t(packed >> (4 * q)) & 15u; }, dsts, ndst,
                       Range{g - kP, end - kP}, vec, a.threads);
        g = end;
    }
}

// The block's window r of round k (piece coordinates, chunk offset kP) of chunk `me`: one FoldSeg, or, in order O6,
// one per sub-slice the window meets (kIpcRhd: one tree per RHD chunk the window meets).
template <class E, int OP, bool kRhd, class Dst>
__device__ __forceinline__ void FoldRange(const IpcArgs& a, uint32_t me, uint64_t kP, const typename E::S* own,
                                          const typename E::S* slots, Dst dsts, uint32_t ndst, Range r, bool vec)
{
    using S = typename E::S;
    if constexpr (kRhd) {
        RhdFold<E, OP>(a, me, kP, own, slots, dsts, ndst, r, vec);
        return;
    }
    if (a.order != kIpcO6) {
        FoldSeg<E, OP>(a, me, 0, own, slots, dsts, ndst, r, vec);
        return;
    }
    const uint64_t L = ChunkElems(a, me);
    for (uint32_t j = 0; j + 1 < a.n; ++j) {
        const uint64_t sb = SubStart<S>(a, L, j), se = SubStart<S>(a, L, j + 1);
        const uint64_t lo = max(r.lo, sb > kP ? sb - kP : 0), hi = min(r.hi, se > kP ? se - kP : 0);
        if (lo < hi) FoldSeg<E, OP>(a, me, j, own, slots, dsts, ndst, Range{lo, hi}, vec);
    }
}

// A generic pointer into device memory as a global-address-space one (global, not flat, loads and stores).
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* AsGlobal(T* p)
{
    return (__attribute__((address_space(1))) T*)p;
}

// The LL word w of source rank q in rank c's LL area for parity p: 8 bytes {data bytes 4w .. 4w+3, flag}.
__device__ __forceinline__ uint64_t* LlWord(const IpcArgs& a, uint32_t c, uint32_t p, uint32_t q, uint64_t w)
{
    char* area = reinterpret_cast<char*>(a.flags[c]) + kIpcFlagBytes;
    return reinterpret_cast<uint64_t*>(area + p * kIpcLlParityBytes + q * kIpcLlSlotBytes) + w;
}

// Bytes 4w .. 4w+3 of a buffer of `bytes` bytes, little-endian in a word (zeros past the end; a base that is not
// 4-byte aligned reads bytewise).
__device__ __forceinline__ uint32_t LoadWord(const uint8_t* b, uint64_t bytes, uint64_t w)
{
    const uint64_t o = 4 * w;
    if ((reinterpret_cast<uintptr_t>(b) & 3u) == 0 && o + 4 <= bytes) return *reinterpret_cast<const uint32_t*>(b + o);
    uint32_t v = 0;
    for (uint32_t i = 0; i < 4 && o + i < bytes; ++i) v |= uint32_t(b[o + i]) << (8 * i);
    return v;
}

// The one-shot AllReduce (kIpcAllReduceOneShot, its own order or kIpcRhd) and the ReduceScatter (kIpcReduceScatter over
// equal blocks) in the LL form (IpcArgs::ll; pieces of at most kIpcLlMaxBytes, one round, windows of BlockWindow).
// Both receive from every peer in every launch, which the reuse argument below needs (a one-shot Reduce's non-roots
// receive nothing, so it stays staged). Each block pushes its window of this rank's input to every peer's
// LL slot `me` as 8-byte words {4 data bytes, flag}, one atomic store each, so a word's data is visible exactly when its
// flag is: no drain, release or separate flag store, and no barrier. It then polls its window of every peer's slot
// in its own LL area until the flags equal this launch's, unpacks the data into its own cached unpack area (the fold's
// slot layout) and folds exactly as the staged one-shot does (FoldRange), so the bits are the same.
// Flags and reuse: launch s (the device's LL sequence word, identical on every rank: every rank makes the same LL
// calls) writes parity s & 1 with flag s + 1. Rank i writes launch s + 2 into peer p's area only after its launch s + 1
// has received p's words of s + 1, which p pushed from a launch that its stream started after its launch s had ended,
// so p has finished reading parity s & 1 by then. A stale word in the polled range carries an older flag of the same
// parity: equal to the current one only after 2^32 LL launches.
template <class E, int OP, bool kRhd>
__device__ __forceinline__ void LlOneShot(const IpcArgs& a, uint32_t me)
{
    using S = typename E::S;
    const uint32_t n = a.n;
    Stamp(a, me, kTrEntry);
    // The sticky word, the LL sequence word and the first batch of input words are all loaded before any of them is
    // waited for: one memory latency before the first store instead of three.
    uint32_t sticky = __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t seq = __hip_atomic_load(a.status + kIpcLlSeqWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // Every destination's piece has the same length: the whole input (one-shot AllReduce) or one block of the
    // ReduceScatter's equal blocks (peer c receives block c, this rank folds block me).
    const bool perDest = a.kind == kIpcReduceScatter;
    const uint64_t len = PieceLen(a, me, 0);
    const Range r = BlockWindow(a, len);
    const uint64_t bytes = len * sizeof(S);
    // words [wlo, whi) of the window; an empty window (a block past the end) has none, so the partial last word is
    // the last non-empty window's alone
    const uint64_t wlo = r.lo * sizeof(S) / 4, whi = r.hi > r.lo ? (r.hi * sizeof(S) + 3) / 4 : wlo, nw = whi - wlo;
    const uint8_t* in = static_cast<const uint8_t*>(a.in[me]);
    // ChunkStart for the LL geometries (Whole and Block: neither vgeom nor balanced), without ChunkStart's vStart
    // table, which a per-lane peer index would read from the argument memory with a round trip per word
    auto src = [&](uint32_t c) { return in + uint64_t(c) * a.chunkStride * sizeof(S); };
    // kLlBatch words per thread in flight at once: the first look at a batch costs one memory latency, not one per word
    constexpr uint32_t kLlBatch = 8;
    // Push items: a one-shot's words (each loaded once, stored to every peer), a ReduceScatter's (peer, word) pairs,
    // the word fastest (peer c's word w comes from c's block). Every batch is loaded before any of it is stored, and
    // the stores wait for nothing but their data: a store loop holding a load makes the compiler wait for each store
    // to complete before the next.
    const uint32_t T = a.threads;
    const uint32_t pushItems = static_cast<uint32_t>(perDest ? uint64_t(n - 1) * nw : nw);
    auto itemAt = [&](uint32_t i, uint32_t& c, uint64_t& w) {
        c = perDest ? (me + 1 + i / static_cast<uint32_t>(nw)) % n : me;
        w = wlo + (perDest ? i % static_cast<uint32_t>(nw) : i);
    };
    uint32_t d[kLlBatch];
    auto loadBatch = [&](uint32_t base) {
#pragma unroll
        for (uint32_t k = 0; k < kLlBatch; ++k) {
            const uint32_t i = base + k * T;
            if (i < pushItems) {
                uint32_t c;
                uint64_t w;
                itemAt(i, c, w);
                d[k] = LoadWord(src(c), bytes, w);
            }
        }
    };
    // a ReduceScatter's lanes store to different peers: their LL areas from LDS, not by a per-lane index into the
    // arguments (a memory round trip per store)
    __shared__ char* llArea[kIpcMaxRanks];
    if (perDest && threadIdx.x < n) llArea[threadIdx.x] = reinterpret_cast<char*>(a.flags[threadIdx.x]) + kIpcFlagBytes;
    loadBatch(threadIdx.x);
    // the status words are used only from here, so the loads above are all issued before the first wait
    asm volatile("" : "+v"(sticky), "+v"(seq)::"memory");
    // a communicator whose IPC wait ever timed out stays failed (sticky bit): never wait on its peers again
    if ((sticky & 1u) != 0) return;
    if (perDest) __syncthreads();
    // issued before the stores (its result is consumed only at EndLaunch), so it waits for none of them
    const uint32_t arrivedBefore = Arrive(a, seq);
    const uint32_t par = seq & 1u, flag = seq + 1u;
    for (uint32_t base = threadIdx.x; base < pushItems; base += kLlBatch * T) {
        if (base != threadIdx.x) loadBatch(base);  // the first batch is loaded above
        if (perDest) {
#pragma unroll
            for (uint32_t k = 0; k < kLlBatch; ++k) {
                const uint32_t i = base + k * T;
                if (i >= pushItems) continue;
                uint32_t c;
                uint64_t w;
                itemAt(i, c, w);
                // LlWord(a, c, par, me, w), as a global pointer: a generic one makes a flat store, which the compiler
                // waits for before the next LDS read
                char* slot = llArea[c] + par * kIpcLlParityBytes + me * kIpcLlSlotBytes;
                __hip_atomic_store(AsGlobal(reinterpret_cast<uint64_t*>(slot) + w),
                                   uint64_t(d[k]) | (uint64_t(flag) << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {
            // peer-major: the loop over peers holds stores only, so the batch's loads are waited for once, before it
            for (uint32_t j = 1; j < n; ++j) {
                const auto slot = AsGlobal(LlWord(a, (me + j) % n, par, me, wlo));
#pragma unroll
                for (uint32_t k = 0; k < kLlBatch; ++k) {
                    const uint32_t i = base + k * T;
                    if (i >= pushItems) continue;
                    __hip_atomic_store(slot + i, uint64_t(d[k]) | (uint64_t(flag) << 32), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
    Stamp(a, me, kTrPhase0);
    // pull: every peer's words of this window, once their flag is this launch's, into the unpack slots
    uint32_t* unpack = static_cast<uint32_t*>(a.llUnpack[me]);
    const uint64_t slotWords = a.piece * sizeof(S) / 4;  // piece is a multiple of 16 B
    uint32_t polls = 0;
    bool cut = false;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t items = uint64_t(n - 1) * nw;
    for (uint64_t base = threadIdx.x; base < items && !cut; base += uint64_t(kLlBatch) * a.threads) {
        uint64_t v[kLlBatch];
        const uint64_t* src[kLlBatch];
        uint32_t dst[kLlBatch];
        uint32_t pending = 0;
#pragma unroll
        for (uint32_t k = 0; k < kLlBatch; ++k) {
            const uint64_t i = base + uint64_t(k) * a.threads;
            src[k] = nullptr;
            if (i < items) {
                const uint32_t q = (me + 1 + static_cast<uint32_t>(i / nw)) % n;
                const uint64_t w = wlo + i % nw;
                src[k] = LlWord(a, me, par, q, w);
                dst[k] = static_cast<uint32_t>(q * slotWords + w);
                pending |= 1u << k;
            }
        }
        // every pending word of the batch is (re)loaded in one round, so a round costs one memory latency however
        // many of the batch's words are still on their way
        for (;;) {
#pragma unroll
            for (uint32_t k = 0; k < kLlBatch; ++k) {
                if (pending & (1u << k)) v[k] = __hip_atomic_load(src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
#pragma unroll
            for (uint32_t k = 0; k < kLlBatch; ++k) {
                if ((pending & (1u << k)) && static_cast<uint32_t>(v[k] >> 32) == flag) {
                    unpack[dst[k]] = static_cast<uint32_t>(v[k]);
                    pending &= ~(1u << k);
                }
            }
            if (pending == 0) break;
            ++polls;
            if ((polls & 63u) == 0) {
                if ((__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 1u) != 0) {
                    cut = true;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeoutTicks) {
                    __hip_atomic_fetch_or(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(a.failHost, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    cut = true;
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __shared__ uint32_t failed;
    if (threadIdx.x == 0) failed = 0;
    __syncthreads();
    if (cut) failed = 1;
    __syncthreads();  // the unpacked words are the block's own stores: visible to its waves after the barrier
    Stamp(a, me, kTrBarrier1);
    if (failed == 0) {
        const S* own = static_cast<const S*>(a.in[me]) + ChunkStart(a, me);
        S* out = static_cast<S*>(a.out[me]) + (perDest ? 0 : ChunkStart(a, me));
        FoldRange<E, OP, kRhd>(a, me, 0, own, reinterpret_cast<const S*>(unpack), [out](uint32_t) { return out; },
                               1u, r, ChunkVec<S>(a, me));
    }
    Stamp(a, me, kTrPhase1);
    if (a.trace != nullptr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        Stamp(a, me, kTrExit);
    }
    PublishWait(a, polls);
    EndLaunch(a, arrivedBefore);
}

// The LL form as a kernel of its own (IpcArgs::ll): its batched polling needs more registers than the staged kernel,
// whose occupancy it must not lower.
template <class E, int OP, bool kRhd>
__global__ __launch_bounds__(kIpcMaxThreads) void k_ipc_ll(IpcArgs a)
{
    const uint32_t me = a.me >= 0 ? static_cast<uint32_t>(a.me) : blockIdx.y;
    LlOneShot<E, OP, kRhd>(a, me);  // checks the sticky bit itself
}

// kRhd: the kIpcRhd instantiation (one-shot AllReduce only, kind and order fixed at compile time). It is a kernel of
// its own so that the RHD tree's register use never lowers the occupancy of the others: a loopback world needs every
// rank's blocks resident at once.
template <class E, int OP, bool kRhd>
__global__ __launch_bounds__(kIpcMaxThreads) void k_ipc_collective(IpcArgs a)
{
    const uint32_t kind = kRhd ? uint32_t(kIpcAllReduceOneShot) : a.kind;
    using S = typename E::S;
    const uint32_t n = a.n;
    const uint32_t me = a.me >= 0 ? static_cast<uint32_t>(a.me) : blockIdx.y;
    const S* in = static_cast<const S*>(a.in[me]);
    S* out = static_cast<S*>(a.out[me]);
    const bool oneShot = kind == kIpcAllReduceOneShot || kind == kIpcReduceOneShot;
    const bool reduceKind = kind == kIpcReduce || kind == kIpcReduceOneShot;
    // a communicator whose IPC barrier ever timed out stays failed (sticky bit): never wait on its peers again. The
    // epoch counter (below) is loaded together with it: one memory latency for both.
    const uint32_t sticky = __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t epoch = __hip_atomic_load(a.status + kIpcEpochWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((sticky & 1u) != 0) return;
    // Slots: the two-barrier kinds use stgIn. The single-barrier kinds alternate between two areas by the parity of
    // the round's barrier epoch e, and fold after the barrier with no second one, so rank i may store round k+2
    // (parity of k) while a peer still folds round k. That is safe because block b of rank i passed barrier k+1
    // first, and:
    //   * rounds k, k+1, k+2 in one launch: every peer's block b signalled k+1 after its fold of round k, and block b
    //     of every rank touches only its own window of the area in every round of a launch;
    //   * k+1 in the launch of k, k+2 in a later one: rank i's launch of k ended only after all its blocks passed
    //     k+1 (the block count is the same on every rank), so every block of every peer had folded round k;
    //   * k+1 in a later launch than k: the peer's block b signalled k+1 from that later launch, which its stream
    //     started only after the launch with round k had ended.
    // No two-barrier kind touches these areas, so a peer still in phase 2 of an earlier call is never disturbed, and a
    // later two-shot call never stores over a fold that runs after the last barrier.
    const bool single = SingleBarrierKind(kind);
    auto slotArea = [&](uint32_t c, uint32_t e) -> char* {
        return static_cast<char*>(single ? a.stgAlt[e & 1u][c] : a.stgIn[c]);
    };
    // Epochs come from the device counter (Arrive / EndLaunch), so the next launch in stream order, a call or a graph
    // replay alike, starts where this one ended. Every rank runs the same launch sequence, so the counters agree.
    Stamp(a, me, kTrEntry);
    const uint32_t arrivedBefore = Arrive(a, epoch);
    uint32_t waitMax = 0;
    for (uint32_t k = 0; k < a.rounds; ++k) {
        const uint64_t kP = uint64_t(k) * a.piece;
        Stamp(a, me, kTrRound);
        // phase 0: my piece of chunk c -> owner c's slot `me` (one-shot: my whole piece to every peer; to the root
        // only for a one-shot Reduce). Each block starts at a different peer (offset rotated by blockIdx.x), so at any
        // moment the blocks of a rank spread their stores over all n-1 xGMI links instead of all feeding one peer.
        for (uint32_t i = 0; i + 1 < n; ++i) {
            const uint32_t c = (me + 1 + (i + blockIdx.x) % (n - 1)) % n;
            if (kind == kIpcReduceOneShot && c != a.root) continue;
            S* slot = reinterpret_cast<S*>(slotArea(c, epoch + 1)) + uint64_t(me) * a.piece;
            ForBlockShare(a, PieceLen(a, c, kP), [&](Range r) {
                CopyRange<S>(slot, in + ChunkStart(a, c) + kP, r, ChunkVec<S>(a, c), a.nt != 0, a.threads);
            });
        }
        Stamp(a, me, kTrPhase0);
        // this lane's flag words, loaded behind the phase's stores: the barrier's drain waits for both at once
        // (computed before the push, the per-lane pointer load held up the first store by a memory round trip)
        const FlagLane fl = LaneFlags(a, me);
        if (!Barrier(a, fl, ++epoch, waitMax)) break;
        Stamp(a, me, kTrBarrier1);
        if (kind == kIpcAllGather) {
            // phase 1 of an AllGather: rank q's piece, from my slot q (mine from my input), to output block q
            const S* slots = reinterpret_cast<const S*>(slotArea(me, epoch));
            constexpr uint64_t V = 16 / sizeof(S);
            ForBlockShare(a, PieceLen(a, me, kP), [&](Range r) {
                for (uint32_t q = 0; q < n; ++q) {
                    const S* src = q == me ? in + kP : slots + uint64_t(q) * a.piece;
                    S* dst = out + uint64_t(q) * a.outStride + kP;
                    if (src != dst) {
                        CopyRange<S>(dst, src, r, a.aligned && (uint64_t(q) * a.outStride) % V == 0, a.nt != 0,
                                     a.threads);
                    }
                }
            });
        } else if (!(kind == kIpcReduceOneShot && me != a.root)) {
            // phase 1: fold my chunk's piece over the slots (my own operand straight from my input)
            const S* own = in + ChunkStart(a, me) + kP;
            const S* slots = reinterpret_cast<const S*>(slotArea(me, epoch));
            // destination 0: my output (or, for a non-root two-shot Reduce rank, the root's result area); the
            // two-shot AllReduce also pushes to every peer's result area (destinations 1 .. n-1 = the peers in
            // ascending order)
            S* first = kind == kIpcReduceScatter ? out + kP
                     : (kind == kIpcReduce && me != a.root)
                         ? static_cast<S*>(a.stgRes[a.root]) + uint64_t(me) * a.piece
                         : out + ChunkStart(a, me) + kP;
            auto dst = [&](uint32_t d) {
                if (d == 0) return first;
                const uint32_t p = d - 1 < me ? d - 1 : d;
                return static_cast<S*>(a.stgRes[p]) + uint64_t(me) * a.piece;
            };
            ForBlockShare(a, PieceLen(a, me, kP), [&](Range r) {
                FoldRange<E, OP, kRhd>(a, me, kP, own, slots, dst, kind == kIpcAllReduce ? n : 1u, r,
                                       ChunkVec<S>(a, me));
            });
        }
        Stamp(a, me, kTrPhase1);
        if (!single && !Barrier(a, fl, ++epoch, waitMax)) break;
        Stamp(a, me, kTrBarrier2);
        // phase 2: the other chunks' results from my own result area (two-shot AllReduce: every rank; two-shot
        // Reduce: the root)
        if (!oneShot && (kind == kIpcAllReduce || (reduceKind && me == a.root))) {
            for (uint32_t c = 0; c < n; ++c) {
                if (c == me) continue;
                ForBlockShare(a, PieceLen(a, c, kP), [&](Range r) {
                    CopyRange<S>(out + ChunkStart(a, c) + kP,
                                 static_cast<const S*>(a.stgRes[me]) + uint64_t(c) * a.piece, r, ChunkVec<S>(a, c),
                                 a.nt != 0, a.threads);
                });
            }
        }
        Stamp(a, me, kTrPhase2);
    }
    if (a.trace != nullptr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        Stamp(a, me, kTrExit);
    }
    PublishWait(a, waitMax);
    EndLaunch(a, arrivedBefore);
}

template <class E, bool kRhd>
hipError_t LaunchIpcLl(int op, const IpcArgs& a, dim3 grid, hipStream_t s)
{
    switch (op) {
        case R_SUM: hipLaunchKernelGGL((k_ipc_ll<E, R_SUM, kRhd>), grid, dim3(a.threads), 0, s, a); break;
        case R_PROD: hipLaunchKernelGGL((k_ipc_ll<E, R_PROD, kRhd>), grid, dim3(a.threads), 0, s, a); break;
        case R_MAX: hipLaunchKernelGGL((k_ipc_ll<E, R_MAX, kRhd>), grid, dim3(a.threads), 0, s, a); break;
        default: hipLaunchKernelGGL((k_ipc_ll<E, R_MIN, kRhd>), grid, dim3(a.threads), 0, s, a); break;
    }
    return hipGetLastError();
}

template <class E>
hipError_t LaunchIpcT(int op, const IpcArgs& a, dim3 grid, hipStream_t s)
{
    if (a.ll != 0) return a.order == kIpcRhd ? LaunchIpcLl<E, true>(op, a, grid, s) : LaunchIpcLl<E, false>(op, a, grid, s);
    if (a.order == kIpcRhd) {
        switch (op) {
            case R_SUM: hipLaunchKernelGGL((k_ipc_collective<E, R_SUM, true>), grid, dim3(a.threads), 0, s, a); break;
            case R_PROD: hipLaunchKernelGGL((k_ipc_collective<E, R_PROD, true>), grid, dim3(a.threads), 0, s, a); break;
            case R_MAX: hipLaunchKernelGGL((k_ipc_collective<E, R_MAX, true>), grid, dim3(a.threads), 0, s, a); break;
            default: hipLaunchKernelGGL((k_ipc_collective<E, R_MIN, true>), grid, dim3(a.threads), 0, s, a); break;
        }
        return hipGetLastError();
    }
    switch (op) {
        case R_SUM: hipLaunchKernelGGL((k_ipc_collective<E, R_SUM, false>), grid, dim3(a.threads), 0, s, a); break;
        case R_PROD: hipLaunchKernelGGL((k_ipc_collective<E, R_PROD, false>), grid, dim3(a.threads), 0, s, a); break;
        case R_MAX: hipLaunchKernelGGL((k_ipc_collective<E, R_MAX, false>), grid, dim3(a.threads), 0, s, a); break;
        default: hipLaunchKernelGGL((k_ipc_collective<E, R_MIN, false>), grid, dim3(a.threads), 0, s, a); break;
    }
    return hipGetLastError();
}

template <class E, bool kRhd>
const void* IpcLlKernelT(int op)
{
    switch (op) {
        case R_SUM: return reinterpret_cast<const void*>(&k_ipc_ll<E, R_SUM, kRhd>);
        case R_PROD: return reinterpret_cast<const void*>(&k_ipc_ll<E, R_PROD, kRhd>);
        case R_MAX: return reinterpret_cast<const void*>(&k_ipc_ll<E, R_MAX, kRhd>);
        default: return reinterpret_cast<const void*>(&k_ipc_ll<E, R_MIN, kRhd>);
    }
}

template <class E>
const void* IpcKernelT(int op, bool rhd, bool ll)
{
    if (ll) return rhd ? IpcLlKernelT<E, true>(op) : IpcLlKernelT<E, false>(op);
    if (rhd) {
        switch (op) {
            case R_SUM: return reinterpret_cast<const void*>(&k_ipc_collective<E, R_SUM, true>);
            case R_PROD: return reinterpret_cast<const void*>(&k_ipc_collective<E, R_PROD, true>);
            case R_MAX: return reinterpret_cast<const void*>(&k_ipc_collective<E, R_MAX, true>);
            default: return reinterpret_cast<const void*>(&k_ipc_collective<E, R_MIN, true>);
        }
    }
    switch (op) {
        case R_SUM: return reinterpret_cast<const void*>(&k_ipc_collective<E, R_SUM, false>);
        case R_PROD: return reinterpret_cast<const void*>(&k_ipc_collective<E, R_PROD, false>);
        case R_MAX: return reinterpret_cast<const void*>(&k_ipc_collective<E, R_MAX, false>);
        default: return reinterpret_cast<const void*>(&k_ipc_collective<E, R_MIN, false>);
    }
}

}  // namespace

// One dtype's entry points (ipc.h declares them): the kernel launch by op and the kernel's address (occupancy).
#define HCCL_AMD_IPC_DTYPE(NAME, ...)                                                                           \
    hipError_t LaunchIpc_##NAME(int op, const IpcArgs& a, dim3 grid, hipStream_t s)                              \
    {                                                                                                            \
        return LaunchIpcT<__VA_ARGS__>(op, a, grid, s);                                                              \
    }                                                                                                            \
    const void* IpcKernel_##NAME(int op, bool rhd, bool ll) { return IpcKernelT<__VA_ARGS__>(op, rhd, ll); }

}  // namespace hccl_amd
