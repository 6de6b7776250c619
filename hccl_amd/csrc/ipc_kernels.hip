// ipc_kernels.hip — one-sided AllReduce over peer-mapped staging buffers.
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
// round (so after my phase-2 reads); the same holds across calls (kernels of a stream run in order).
// Every round of one launch has the same geometry (the host launches a shorter last round separately), so block b
// of every rank touches the same slot and result addresses in every round and only waits for block b of its peers;
// nothing in a GPU waits for another block of the same GPU. Every storing wave drains (s_waitcnt vmcnt(0)) before the
// workgroup barrier, one wave then releases at system scope (L2 write-back) and stores the flags with system-scope
// release stores; flags are polled with system-scope relaxed loads and followed by an acquire. Every wait is bounded
// in wall time (s_memrealtime, HCCL_AMD_IPC_TIMEOUT_MS): on timeout the kernel sets status bit 0 and finishes (wrong
// data, never a hang); the bit is sticky for the communicator, so later launches return at once. World mode (me < 0) runs all
// n ranks of a loopback world as blockIdx.y of one launch on one GPU, which is how the protocol is tested without a
// second GPU; the rank-mode path (one launch per process, peers opened from IPC handles) is tested with n processes
// sharing the GPU.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "ipc.h"
#include "reduce_elem.h"

namespace hccl_amd {

namespace {

constexpr int kIpcBlock = 256;
constexpr int kIpcU = 4;

// Returns false when a barrier of this launch timed out (status bit 0): the caller then stops at once, so a rank
// never stores into a peer it has lost track of.
__device__ __forceinline__ bool Barrier(const IpcArgs& a, uint32_t me, uint32_t epoch)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its stores have left the CU
    __syncthreads();
    const uint32_t t = threadIdx.x;
    if (t < a.n) {
        __threadfence_system();
        uint32_t* remote = a.flags[t] + blockIdx.x * a.n + me;
        __hip_atomic_store(remote, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        uint32_t* mine = a.flags[me] + blockIdx.x * a.n + t;
        uint32_t polls = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
        while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
            ++polls;
            if ((polls & 63u) == 0) {
                // a timeout anywhere (this or another block of this rank) ends the wait at once
                if ((__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 1u) != 0) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeoutTicks) {
                    __hip_atomic_fetch_or(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (polls != 0) __hip_atomic_fetch_max(a.status + 1, polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate has completed before the barrier opens
    }
    __shared__ uint32_t failed;
    if (t == 0) failed = __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 1u;
    __syncthreads();
    return failed == 0;
}

struct Range {
    uint64_t lo, hi;  // piece coordinates
};

__device__ __forceinline__ uint64_t ChunkStart(const IpcArgs& a, uint32_t c)
{
    return a.balanced ? uint64_t(c) * a.chunkLen + min(uint64_t(c), a.rem) : uint64_t(c) * a.chunkStride;
}

__device__ __forceinline__ uint64_t ChunkElems(const IpcArgs& a, uint32_t c)
{
    if (a.balanced) return a.chunkLen + (c < a.rem ? 1 : 0);
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

// dst[e] = src[e] for e in r. vec = both pointers are 16-B aligned; otherwise every element goes through the scalar
// loop.
template <typename S>
__device__ __forceinline__ void CopyRange(S* dst, const S* src, Range r, bool vec)
{
    constexpr uint64_t V = 16 / sizeof(S);
    // r.lo is vector aligned unless the window is empty at the end of a piece (lo = hi = len); r.hi may be anything
    const uint64_t vlo = r.lo / V, vhi = vec ? max(vlo, r.hi / V) : vlo;
    const u32x4* s = reinterpret_cast<const u32x4*>(src);
    u32x4* d = reinterpret_cast<u32x4*>(dst);
    uint64_t v = vlo + threadIdx.x;
    for (; v + (kIpcU - 1) * kIpcBlock < vhi; v += kIpcU * kIpcBlock) {
        u32x4 x[kIpcU];
#pragma unroll
        for (int u = 0; u < kIpcU; ++u) x[u] = s[v + u * kIpcBlock];
#pragma unroll
        for (int u = 0; u < kIpcU; ++u) d[v + u * kIpcBlock] = x[u];
    }
    for (; v < vhi; v += kIpcBlock) d[v] = s[v];
    for (uint64_t e = max(vhi * V, r.lo) + threadIdx.x; e < r.hi; e += kIpcBlock) dst[e] = src[e];
}

// Fold of chunk `me` over the n operands in the kind's order, written to up to kIpcMaxRanks destinations.
//   all-reduce (O2):            operand i = rank i
//   reduce-scatter / reduce (O1): operand 0 = rank me (the owner), then the others ascending
template <class E, int OP, class Dst>
__device__ __forceinline__ void FoldRange(const IpcArgs& a, uint32_t me, const typename E::S* own,
                                          const typename E::S* slots, Dst dsts, uint32_t ndst, Range r, bool vec)
{
    using S = typename E::S;
    constexpr uint64_t V = 16 / sizeof(S);
    const uint32_t n = a.n;
    const bool o2 = a.kind == kIpcAllReduce;
    auto src = [&](uint32_t i) {
        const uint32_t q = o2 ? i : (i == 0 ? me : (i <= me ? i - 1 : i));
        return q == me ? own : slots + uint64_t(q) * a.piece;
    };
    const uint64_t vlo = r.lo / V, vhi = vec ? max(vlo, r.hi / V) : vlo;
    uint64_t v = vlo + threadIdx.x;
    for (; v + (kIpcU - 1) * kIpcBlock < vhi; v += kIpcU * kIpcBlock) {
        u32x4 acc[kIpcU];
#pragma unroll
        for (int u = 0; u < kIpcU; ++u) acc[u] = reinterpret_cast<const u32x4*>(src(0))[v + u * kIpcBlock];
        for (uint32_t i = 1; i < n; ++i) {
            u32x4 x[kIpcU];
#pragma unroll
            for (int u = 0; u < kIpcU; ++u) x[u] = reinterpret_cast<const u32x4*>(src(i))[v + u * kIpcBlock];
#pragma unroll
            for (int u = 0; u < kIpcU; ++u) acc[u] = combine<E, OP>(x[u], acc[u]);
        }
        for (uint32_t d = 0; d < ndst; ++d) {
#pragma unroll
            for (int u = 0; u < kIpcU; ++u) reinterpret_cast<u32x4*>(dsts(d))[v + u * kIpcBlock] = acc[u];
        }
    }
    for (; v < vhi; v += kIpcBlock) {
        u32x4 acc = reinterpret_cast<const u32x4*>(src(0))[v];
        for (uint32_t i = 1; i < n; ++i) acc = combine<E, OP>(reinterpret_cast<const u32x4*>(src(i))[v], acc);
        for (uint32_t d = 0; d < ndst; ++d) reinterpret_cast<u32x4*>(dsts(d))[v] = acc;
    }
    for (uint64_t e = max(vhi * V, r.lo) + threadIdx.x; e < r.hi; e += kIpcBlock) {
        S acc = src(0)[e];
        for (uint32_t i = 1; i < n; ++i) acc = E::template ap<OP>(src(i)[e], acc);
        for (uint32_t d = 0; d < ndst; ++d) dsts(d)[e] = acc;
    }
}

template <class E, int OP>
__global__ __launch_bounds__(kIpcBlock) void k_ipc_collective(IpcArgs a)
{
    using S = typename E::S;
    const uint32_t n = a.n;
    const uint32_t me = a.me >= 0 ? static_cast<uint32_t>(a.me) : blockIdx.y;
    const S* in = static_cast<const S*>(a.in[me]);
    S* out = static_cast<S*>(a.out[me]);
    // a communicator whose IPC barrier ever timed out stays failed (sticky bit): never wait on its peers again
    if ((__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 1u) != 0) return;
    uint32_t epoch = a.epochBase;
    for (uint32_t k = 0; k < a.rounds; ++k) {
        const uint64_t kP = uint64_t(k) * a.piece;
        // phase 0: my piece of chunk c -> owner c's slot `me`
        for (uint32_t c = 0; c < n; ++c) {
            if (c == me) continue;
            const Range r = BlockWindow(a, PieceLen(a, c, kP));
            S* slot = static_cast<S*>(a.stgIn[c]) + uint64_t(me) * a.piece;
            CopyRange<S>(slot, in + ChunkStart(a, c) + kP, r, ChunkVec<S>(a, c));
        }
        if (!Barrier(a, me, ++epoch)) return;
        // phase 1: fold my chunk's piece over the slots (my own operand straight from my input)
        {
            const Range r = BlockWindow(a, PieceLen(a, me, kP));
            const S* own = in + ChunkStart(a, me) + kP;
            const S* slots = static_cast<const S*>(a.stgIn[me]);
            // destination 0: my output (or, for a non-root Reduce rank, the root's result area); all-reduce also
            // pushes to every peer's result area (destinations 1 .. n-1 = the peers in ascending order)
            S* first = a.kind == kIpcReduceScatter ? out + kP
                     : (a.kind == kIpcReduce && me != a.root)
                         ? static_cast<S*>(a.stgRes[a.root]) + uint64_t(me) * a.piece
                         : out + ChunkStart(a, me) + kP;
            auto dst = [&](uint32_t d) {
                if (d == 0) return first;
                const uint32_t p = d - 1 < me ? d - 1 : d;
                return static_cast<S*>(a.stgRes[p]) + uint64_t(me) * a.piece;
            };
            FoldRange<E, OP>(a, me, own, slots, dst, a.kind == kIpcAllReduce ? n : 1u, r, ChunkVec<S>(a, me));
        }
        if (!Barrier(a, me, ++epoch)) return;
        // phase 2: the other chunks' results from my own result area (all-reduce: every rank; reduce: the root)
        if (a.kind == kIpcAllReduce || (a.kind == kIpcReduce && me == a.root)) {
            for (uint32_t c = 0; c < n; ++c) {
                if (c == me) continue;
                const Range r = BlockWindow(a, PieceLen(a, c, kP));
                CopyRange<S>(out + ChunkStart(a, c) + kP,
                             static_cast<const S*>(a.stgRes[me]) + uint64_t(c) * a.piece, r, ChunkVec<S>(a, c));
            }
        }
    }
}

template <class E>
hipError_t LaunchIpcT(int op, const IpcArgs& a, dim3 grid, hipStream_t s)
{
    switch (op) {
        case R_SUM: hipLaunchKernelGGL((k_ipc_collective<E, R_SUM>), grid, dim3(kIpcBlock), 0, s, a); break;
        case R_PROD: hipLaunchKernelGGL((k_ipc_collective<E, R_PROD>), grid, dim3(kIpcBlock), 0, s, a); break;
        case R_MAX: hipLaunchKernelGGL((k_ipc_collective<E, R_MAX>), grid, dim3(kIpcBlock), 0, s, a); break;
        default: hipLaunchKernelGGL((k_ipc_collective<E, R_MIN>), grid, dim3(kIpcBlock), 0, s, a); break;
    }
    return hipGetLastError();
}

}  // namespace

HcclResult LaunchIpcCollective(const IpcArgs& a, uint32_t blocks, uint32_t worldRanks, HcclDataType dt,
                              HcclReduceOp op, hipStream_t stream)
{
    dim3 grid(blocks, worldRanks == 0 ? 1 : worldRanks);
    hipError_t e;
    switch (dt) {
        case HCCL_DATA_TYPE_INT8: e = LaunchIpcT<EInt<int8_t, uint32_t>>(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_INT16: e = LaunchIpcT<EInt<int16_t, uint32_t>>(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_INT32: e = LaunchIpcT<EInt<int32_t, uint32_t>>(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_INT64: e = LaunchIpcT<EInt<int64_t, uint64_t>>(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_UINT64: e = LaunchIpcT<EInt<uint64_t, uint64_t>>(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_FP16: e = LaunchIpcT<EF16>(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_BFP16: e = LaunchIpcT<EBF16>(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_FP32: e = LaunchIpcT<EFp<float>>(op, a, grid, stream); break;
        case HCCL_DATA_TYPE_FP64: e = LaunchIpcT<EFp<double>>(op, a, grid, stream); break;
        default: return HCCL_E_NOT_SUPPORT;
    }
    if (e != hipSuccess) {
        HCCL_AMD_ERR("ipc collective launch failed: %s", hipGetErrorString(e));
        return HCCL_E_RUNTIME;
    }
    return HCCL_SUCCESS;
}

}  // namespace hccl_amd
