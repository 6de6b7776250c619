// ipc_kernels.hip — one-sided AllReduce over peer-mapped staging buffers.
//
// The reference's AIV engine runs AllReduce as ONE kernel whose blocks write into every peer's CCL buffer
// (GM_IN[r]) and synchronise with per-block flags (aiv_all_reduce_mesh_1d_twoshot.h:20-217,
// aiv_communication_base_v2.h:296-357). This is the MI355X form of that model, two-shot with the reference's
// deterministic order O2 (acc = x_0, then x_1 .. x_{n-1}; ins_temp_all_reduce_mesh_1D_two_shot.cc:327-335):
//   per round of `roundElems` elements (bounded staging):
//     phase 0  every rank copies its input slice into its own staging (local HBM)
//     barrier  block b tells block b of every rank "my staging is written", waits for theirs
//     phase 1  rank c folds chunk c reading all n stagings (n-1 of them over xGMI), writes recvBuf and a result area
//     barrier
//     phase 2  every rank copies the other chunks' results from their owners' result areas (xGMI reads)
//     barrier  (the staging may be overwritten by the next round / call)
// Block b of every rank always handles the same element ranges, so a block only waits for block b of its peers;
// nothing in a GPU waits for another block of the same GPU. Staging and flags are uncached device memory (fine
// grained), stores are drained and released at system scope before a flag store, flags are polled with system-scope
// relaxed loads followed by an acquire. Every poll loop is bounded: on timeout the kernel sets status bit 0 and
// finishes (wrong data, never a hang). World mode (me < 0) runs all n ranks of a loopback world as blockIdx.y of one
// launch on one GPU, which is how the protocol is tested without a second GPU.
#include <hip/hip_runtime.h>

#include "internal.h"
#include "ipc.h"
#include "reduce_elem.h"

namespace hccl_amd {

namespace {

constexpr int kIpcBlock = 256;
constexpr int kIpcU = 4;

__device__ __forceinline__ void Barrier(const IpcArgs& a, uint32_t me, uint32_t epoch)
{
    __syncthreads();
    const uint32_t t = threadIdx.x;
    if (t < a.n) {
        __threadfence_system();
        uint32_t* remote = a.flags[t] + blockIdx.x * a.n + me;
        __hip_atomic_store(remote, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        uint32_t* mine = a.flags[me] + blockIdx.x * a.n + t;
        uint32_t polls = 0;
        while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
            ++polls;
            // a timeout anywhere is sticky: later barriers of this launch stop waiting at once
            if (polls > a.maxPolls ||
                ((polls & 1023u) == 0 &&
                 (__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 1u) != 0)) {
                __hip_atomic_fetch_or(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
}

struct Range {
    uint64_t lo, hi;  // elements, relative to the round base
};

// Chunk c of a round of `len` elements, rounded to whole 16-B vectors; the block's share of it likewise.
__device__ __forceinline__ Range BlockRange(uint64_t len, uint32_t n, uint32_t c, uint64_t vecElems)
{
    uint64_t cs = (len + n - 1) / n;
    cs = (cs + vecElems - 1) / vecElems * vecElems;
    uint64_t clo = min(len, uint64_t(c) * cs), chi = min(len, clo + cs);
    uint64_t bs = (chi - clo + gridDim.x - 1) / gridDim.x;
    bs = (bs + vecElems - 1) / vecElems * vecElems;
    uint64_t lo = min(chi, clo + uint64_t(blockIdx.x) * bs);
    return {lo, min(chi, lo + bs)};
}

__device__ __forceinline__ uint64_t ChunkLo(uint64_t len, uint32_t n, uint32_t c, uint64_t vecElems)
{
    uint64_t cs = (len + n - 1) / n;
    cs = (cs + vecElems - 1) / vecElems * vecElems;
    return min(len, uint64_t(c) * cs);
}

template <typename S>
__device__ __forceinline__ void CopyRange(S* dst, const S* src, Range r)
{
    constexpr uint64_t V = 16 / sizeof(S);
    const uint64_t vlo = r.lo / V, vhi = r.hi / V;  // r.lo is vector aligned; r.hi may not be (last chunk)
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
    for (uint64_t e = vhi * V + threadIdx.x; e < r.hi; e += kIpcBlock) dst[e] = src[e];
}

template <class E, int OP>
__global__ __launch_bounds__(kIpcBlock) void k_allreduce_ipc(IpcArgs a)
{
    using S = typename E::S;
    constexpr uint64_t V = 16 / sizeof(S);
    const uint32_t n = a.n;
    const uint32_t me = a.me >= 0 ? static_cast<uint32_t>(a.me) : blockIdx.y;
    const S* in = static_cast<const S*>(a.in[me]);
    S* out = static_cast<S*>(a.out[me]);
    uint32_t epoch = a.epochBase;
    for (uint64_t base = 0; base < a.count; base += a.roundElems) {
        const uint64_t len = min(a.roundElems, a.count - base);
        // phase 0: own input -> own staging, every chunk's block-b range
        S* stg = static_cast<S*>(a.stgIn[me]);
        for (uint32_t c = 0; c < n; ++c) {
            Range r = BlockRange(len, n, c, V);
            CopyRange<S>(stg, in + base, r);
        }
        Barrier(a, me, ++epoch);
        // phase 1: fold chunk `me` over all stagings in rank order (O2)
        {
            Range r = BlockRange(len, n, me, V);
            const uint64_t clo = ChunkLo(len, n, me, V);
            S* res = static_cast<S*>(a.stgRes[me]);
            const uint64_t vlo = r.lo / V, vhi = r.hi / V;
            uint64_t v = vlo + threadIdx.x;
            for (; v + (kIpcU - 1) * kIpcBlock < vhi; v += kIpcU * kIpcBlock) {
                u32x4 acc[kIpcU];
                const u32x4* s0 = reinterpret_cast<const u32x4*>(a.stgIn[0]);
#pragma unroll
                for (int u = 0; u < kIpcU; ++u) acc[u] = s0[v + u * kIpcBlock];
                for (uint32_t q = 1; q < n; ++q) {
                    const u32x4* sq = reinterpret_cast<const u32x4*>(a.stgIn[q]);
                    u32x4 x[kIpcU];
#pragma unroll
                    for (int u = 0; u < kIpcU; ++u) x[u] = sq[v + u * kIpcBlock];
#pragma unroll
                    for (int u = 0; u < kIpcU; ++u) acc[u] = combine<E, OP>(x[u], acc[u]);
                }
#pragma unroll
                for (int u = 0; u < kIpcU; ++u) {
                    reinterpret_cast<u32x4*>(out + base)[v + u * kIpcBlock] = acc[u];
                    reinterpret_cast<u32x4*>(res - clo)[v + u * kIpcBlock] = acc[u];
                }
            }
            for (; v < vhi; v += kIpcBlock) {
                u32x4 acc = reinterpret_cast<const u32x4*>(a.stgIn[0])[v];
                for (uint32_t q = 1; q < n; ++q) {
                    acc = combine<E, OP>(reinterpret_cast<const u32x4*>(a.stgIn[q])[v], acc);
                }
                reinterpret_cast<u32x4*>(out + base)[v] = acc;
                reinterpret_cast<u32x4*>(res - clo)[v] = acc;
            }
            for (uint64_t e = vhi * V + threadIdx.x; e < r.hi; e += kIpcBlock) {
                S acc = static_cast<const S*>(a.stgIn[0])[e];
                for (uint32_t q = 1; q < n; ++q) acc = E::template ap<OP>(static_cast<const S*>(a.stgIn[q])[e], acc);
                out[base + e] = acc;
                res[e - clo] = acc;
            }
        }
        Barrier(a, me, ++epoch);
        // phase 2: the other chunks from their owners' result areas
        for (uint32_t c = 0; c < n; ++c) {
            if (c == me) continue;
            Range r = BlockRange(len, n, c, V);
            const uint64_t clo = ChunkLo(len, n, c, V);
            CopyRange<S>(out + base, static_cast<const S*>(a.stgRes[c]) - clo, r);
        }
        Barrier(a, me, ++epoch);
    }
}

template <class E>
hipError_t LaunchIpcT(int op, const IpcArgs& a, dim3 grid, hipStream_t s)
{
    switch (op) {
        case R_SUM: hipLaunchKernelGGL((k_allreduce_ipc<E, R_SUM>), grid, dim3(kIpcBlock), 0, s, a); break;
        case R_PROD: hipLaunchKernelGGL((k_allreduce_ipc<E, R_PROD>), grid, dim3(kIpcBlock), 0, s, a); break;
        case R_MAX: hipLaunchKernelGGL((k_allreduce_ipc<E, R_MAX>), grid, dim3(kIpcBlock), 0, s, a); break;
        default: hipLaunchKernelGGL((k_allreduce_ipc<E, R_MIN>), grid, dim3(kIpcBlock), 0, s, a); break;
    }
    return hipGetLastError();
}

}  // namespace

HcclResult LaunchIpcAllReduce(const IpcArgs& a, uint32_t blocks, uint32_t worldRanks, HcclDataType dt,
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
        HCCL_AMD_ERR("ipc allreduce launch failed: %s", hipGetErrorString(e));
        return HCCL_E_RUNTIME;
    }
    return HCCL_SUCCESS;
}

}  // namespace hccl_amd
