// reduce_kernels.hip — the element-wise reduce at the bottom of every HCCL reducing schedule, for CDNA4 (gfx950).
//
// Replaces:
//   AicpuReduceTemplate<T> / AicpuReduceFp16 / AicpuReduce  alg_data_trans_wrapper.cc:1232-1353 (CPU scalar loop)
//   LocalReduce -> HcommLocalReduceOnThread                  alg_data_trans_wrapper.cc:901-928 (external SDMA task)
//   AivCommBase::CpGM2GM(atomic) / Reduce64                  aiv_communication_base_v2.h:527-616 (AIV vector core)
//
// This is a pure HBM stream (1 flop per 12 B for fp32), so the design is about bytes in flight, not math:
//   * every lane moves 16-B vectors (global_load_dwordx4 / global_store_dwordx4), a wave 1 KiB per instruction;
//   * each lane issues all U loads of both operands of a tile before the first combine (2*U*16 B in flight per lane);
//   * a persistent grid of blocksPerCu x CUs workgroups of 256 threads walks the tiles (grid-stride), so the launch
//     is a fixed ~1-2k workgroups whatever the size;
//   * optional non-temporal loads/stores (nt bit) for once-touched streams;
//   * no LDS: staging a pure stream through LDS adds a round trip and buys no reuse (measured in DESIGN.md).
// Element rules are AicpuReduceTemplate's: dst = src (op) dst with std::max/std::min operand semantics (ties and NaN
// yield src), integer SUM/PROD wrap, fp16/bf16 computed as fp32 then rounded to nearest even. No fast-math: fp32
// denormals are preserved (checked in the code object: .amdhsa_float_denorm_mode_32 = 3).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>

#include "internal.h"
#include "reduce_elem.h"

namespace hccl_amd {


// Scalar elements outside the 16-B aligned body (head < 16 B before it, tail < 16 B after it): done by block 0.
struct Edges {
    uint32_t head;  // elements before the vector body
    uint32_t tail;  // elements after it
    uint64_t tailStart;
};

constexpr int kBlock = 256;

// ------------------------------------------------------------------------------------------------ out = src (op) dst

// ORD 0: tiles dealt round-robin to the persistent grid (the chip-wide access front stays a few MiB wide);
// ORD 1: each workgroup walks one contiguous run of tiles.
template <int ORD>
struct TileRange {
    uint64_t begin, end, step;
    __device__ TileRange(uint64_t fullTiles)
    {
        if constexpr (ORD == 0) {
            begin = blockIdx.x;
            end = fullTiles;
            step = gridDim.x;
        } else {
            uint64_t per = (fullTiles + gridDim.x - 1) / gridDim.x;
            begin = uint64_t(blockIdx.x) * per;
            end = begin + per < fullTiles ? begin + per : fullTiles;
            step = 1;
        }
    }
};

template <class E, int OP, int U, int NT, int ORD>
__global__ __launch_bounds__(kBlock) void k_reduce2(typename E::S* out, const typename E::S* src,
                                                      const typename E::S* dst, uint64_t nvec, Edges edges)
{
    constexpr uint64_t kTile = uint64_t(kBlock) * U;
    // vector body starts after the head elements
    u32x4* vout = reinterpret_cast<u32x4*>(out + edges.head);
    const u32x4* vsrc = reinterpret_cast<const u32x4*>(src + edges.head);
    const u32x4* vdst = reinterpret_cast<const u32x4*>(dst + edges.head);
    const uint64_t fullTiles = nvec / kTile;
    const TileRange<ORD> tr(fullTiles);
    for (uint64_t t = tr.begin; t < tr.end; t += tr.step) {
        const uint64_t base = t * kTile + threadIdx.x;
        u32x4 a[U];
        u32x4 b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = ld<NT>(vsrc + base + u * kBlock);
            b[u] = ld<NT>(vdst + base + u * kBlock);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            st<NT>(vout + base + u * kBlock, combine<E, OP>(a[u], b[u]));
        }
    }
    for (uint64_t i = fullTiles * kTile + uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < nvec;
         i += uint64_t(gridDim.x) * kBlock) {
        st<NT>(vout + i, combine<E, OP>(ld<NT>(vsrc + i), ld<NT>(vdst + i)));
    }
    if (blockIdx.x == 0) {
        uint32_t tid = threadIdx.x;
        if (tid < edges.head) {
            out[tid] = E::template ap<OP>(src[tid], dst[tid]);
        } else if (tid >= 64 && tid - 64 < edges.tail) {
            uint64_t i = edges.tailStart + (tid - 64);
            out[i] = E::template ap<OP>(src[i], dst[i]);
        }
    }
}

// Fallback when the three pointers are not congruent modulo 16 B: one element per lane, grid-stride.
template <class E, int OP>
__global__ __launch_bounds__(kBlock) void k_reduce2_scalar(typename E::S* out, const typename E::S* src,
                                                             const typename E::S* dst, uint64_t count)
{
    for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < count; i += uint64_t(gridDim.x) * kBlock) {
        out[i] = E::template ap<OP>(src[i], dst[i]);
    }
}

// ------------------------------------------------------------------------------------------------ ordered n-ary fold

struct SrcPack {
    const void* p[HCCL_AMD_IR_MAX_SRC];
};

// Vector body of operand j (16-B vectors from the first aligned element).
template <class E>
__device__ __forceinline__ const u32x4* VecSrc(const SrcPack& srcs, int j, const Edges& edges)
{
    return reinterpret_cast<const u32x4*>(static_cast<const typename E::S*>(srcs.p[j]) + edges.head);
}

// Fold of one tile (U vectors per lane at base, base + kBlock, ...) over the operands, in operand order.
// MODE 0 (serial): operand j+1 is loaded once operand j is folded, so a wave has U vectors of loads in flight.
// MODE 1 (prefetch): operand j+1's loads are issued before operand j is folded (a register double buffer), so a wave
// keeps 2U vectors in flight across the whole operand loop. The fold order (acc = x_j (op) acc) is the same.
// NS > 0: the operand count is a compile-time constant and every operand's loads of the tile are issued before the
// first combine (NS * U vectors in flight).
template <class E, int OP, int U, int NT, int MODE, int NS>
__device__ __forceinline__ void FoldTile(u32x4 (&acc)[U], const SrcPack& srcs, int nsrc, const Edges& edges,
                                         uint64_t base)
{
    if constexpr (NS > 0) {
        u32x4 v[NS][U];
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const u32x4* pj = VecSrc<E>(srcs, j, edges);
#pragma unroll
            for (int u = 0; u < U; ++u) v[j][u] = ld<NT>(pj + base + u * kBlock);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = v[0][u];
#pragma unroll
        for (int j = 1; j < NS; ++j) {
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] = combine<E, OP>(v[j][u], acc[u]);
        }
    } else if constexpr (MODE == 1) {
        u32x4 nxt[U];
        const u32x4* p0 = VecSrc<E>(srcs, 0, edges);
        const u32x4* p1 = VecSrc<E>(srcs, 1, edges);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = ld<NT>(p0 + base + u * kBlock);
#pragma unroll
        for (int u = 0; u < U; ++u) nxt[u] = ld<NT>(p1 + base + u * kBlock);
        for (int j = 1; j < nsrc; ++j) {
            u32x4 cur[U];
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
            if (j + 1 < nsrc) {
                const u32x4* pn = VecSrc<E>(srcs, j + 1, edges);
#pragma unroll
                for (int u = 0; u < U; ++u) nxt[u] = ld<NT>(pn + base + u * kBlock);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] = combine<E, OP>(cur[u], acc[u]);
        }
    } else {
        const u32x4* p0 = VecSrc<E>(srcs, 0, edges);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = ld<NT>(p0 + base + u * kBlock);
        for (int j = 1; j < nsrc; ++j) {
            const u32x4* pj = VecSrc<E>(srcs, j, edges);
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ld<NT>(pj + base + u * kBlock);
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] = combine<E, OP>(v[u], acc[u]);
        }
    }
}

// One ordered fold over `nvec` 16-B vectors (plus scalar edges), worked by `nblocks` workgroups, this one `bid`.
// ORD 0: tiles dealt round-robin over the grid; ORD 1: each workgroup folds one contiguous run of tiles.
template <class E, int OP, int U, int NT, int MODE = 0, int NS = 0, int ORD = 0>
__device__ __forceinline__ void ReduceNBody(typename E::S* out, const SrcPack& srcs, int nsrc, uint64_t nvec,
                                            Edges edges, uint32_t bid, uint32_t nblocks)
{
    using S = typename E::S;
    constexpr uint64_t kTile = uint64_t(kBlock) * U;
    u32x4* vout = reinterpret_cast<u32x4*>(out + edges.head);
    const uint64_t fullTiles = nvec / kTile;
    const uint64_t per = ORD == 0 ? 0 : (fullTiles + nblocks - 1) / nblocks;
    const uint64_t tBegin = ORD == 0 ? bid : uint64_t(bid) * per;
    const uint64_t tEnd = ORD == 0 ? fullTiles : (tBegin + per < fullTiles ? tBegin + per : fullTiles);
    const uint64_t tStep = ORD == 0 ? nblocks : 1;
    for (uint64_t t = tBegin; t < tEnd; t += tStep) {
        const uint64_t base = t * kTile + threadIdx.x;
        u32x4 acc[U];
        FoldTile<E, OP, U, NT, MODE, NS>(acc, srcs, nsrc, edges, base);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            st<NT>(vout + base + u * kBlock, acc[u]);
        }
    }
    for (uint64_t i = fullTiles * kTile + uint64_t(bid) * kBlock + threadIdx.x; i < nvec;
         i += uint64_t(nblocks) * kBlock) {
        u32x4 acc = ld<NT>(reinterpret_cast<const u32x4*>(static_cast<const S*>(srcs.p[0]) + edges.head) + i);
        for (int j = 1; j < nsrc; ++j) {
            acc = combine<E, OP>(ld<NT>(reinterpret_cast<const u32x4*>(static_cast<const S*>(srcs.p[j]) + edges.head) + i),
                                 acc);
        }
        st<NT>(vout + i, acc);
    }
    if (bid == 0) {
        uint32_t tid = threadIdx.x;
        uint64_t i;
        bool act = false;
        if (tid < edges.head) {
            i = tid;
            act = true;
        } else if (tid >= 64 && tid - 64 < edges.tail) {
            i = edges.tailStart + (tid - 64);
            act = true;
        }
        if (act) {
            S acc = static_cast<const S*>(srcs.p[0])[i];
            for (int j = 1; j < nsrc; ++j) {
                acc = E::template ap<OP>(static_cast<const S*>(srcs.p[j])[i], acc);
            }
            out[i] = acc;
        }
    }
}

template <class E, int OP, int U, int NT, int MODE = 0, int NS = 0, int ORD = 0>
__global__ __launch_bounds__(kBlock) void k_reduceN(typename E::S* out, SrcPack srcs, int nsrc, uint64_t nvec,
                                                      Edges edges)
{
    ReduceNBody<E, OP, U, NT, MODE, NS, ORD>(out, srcs, nsrc, nvec, edges, blockIdx.x, gridDim.x);
}

// A batch of independent folds (one schedule step's), in one of two layouts chosen by segment size (RunBatch):
// * flat (k_reduceN_batch): the segments' full tiles are one concatenated tile space that the whole grid strides over,
//   as a single fold would; at any moment the workgroups sit in a window of consecutive tiles, one or two segments
//   wide, so the DRAM sees a few operand streams instead of every segment's at once; each segment's leftover vectors
//   and scalar edges follow, spread over the grid;
// * rows (k_reduceN_batch_rows): a grid row per segment.
// Measured (tools/batch_fold_bench.py, 7 segments; profiles/r02_batch_fold_layout_ab.txt): at 4 and 16 MiB segments
// flat runs 6.1-6.5 TB/s against rows' 5.5-6.1 (2 and 8 operands); at 1-2 MiB rows is as fast or faster, and beside the
// RCCL kernels of a self-loop MeshChunk program (1.8 MiB sub-slices) rows' folds took 0.95-1.0 ms against flat's 1.4.
constexpr uint64_t kBatchFlatSegBytes = 4ull << 20;  // segments this large (on average) take the flat layout

struct BatchPack {
    void* out[kMaxBatchSegs];
    SrcPack srcs[kMaxBatchSegs];
    uint64_t nvec[kMaxBatchSegs];
    Edges edges[kMaxBatchSegs];
    uint64_t tileStart[kMaxBatchSegs + 1];  // prefix sums of the segments' full tiles
    int nseg;
    int nsrc;
};

// The other layout: one grid row (blockIdx.y) per segment, each row striding over its own segment.
template <class E, int OP, int U, int NT>
__global__ __launch_bounds__(kBlock) void k_reduceN_batch_rows(BatchPack pk)
{
    const uint32_t g = blockIdx.y;
    ReduceNBody<E, OP, U, NT>(static_cast<typename E::S*>(pk.out[g]), pk.srcs[g], pk.nsrc, pk.nvec[g], pk.edges[g],
                              blockIdx.x, gridDim.x);
}

template <class E, int OP, int U, int NT>
__global__ __launch_bounds__(kBlock) void k_reduceN_batch(BatchPack pk)
{
    using S = typename E::S;
    constexpr uint64_t kTile = uint64_t(kBlock) * U;
    const uint32_t bid = blockIdx.x, nblocks = gridDim.x;
    int g = 0;
    for (uint64_t t = bid; t < pk.tileStart[pk.nseg]; t += nblocks) {
        while (t >= pk.tileStart[g + 1]) ++g;  // t only grows: the segment index only moves forward
        const uint64_t base = (t - pk.tileStart[g]) * kTile + threadIdx.x;
        u32x4 acc[U];
        FoldTile<E, OP, U, NT, 0, 0>(acc, pk.srcs[g], pk.nsrc, pk.edges[g], base);
        u32x4* vout = reinterpret_cast<u32x4*>(static_cast<S*>(pk.out[g]) + pk.edges[g].head);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(vout + base + u * kBlock, acc[u]);
    }
    for (int h = 0; h < pk.nseg; ++h) {
        S* out = static_cast<S*>(pk.out[h]);
        const SrcPack& srcs = pk.srcs[h];
        const Edges& edges = pk.edges[h];
        u32x4* vout = reinterpret_cast<u32x4*>(out + edges.head);
        const uint64_t nvec = pk.nvec[h];
        for (uint64_t i = (pk.tileStart[h + 1] - pk.tileStart[h]) * kTile + uint64_t(bid) * kBlock + threadIdx.x;
             i < nvec; i += uint64_t(nblocks) * kBlock) {
            u32x4 acc = ld<NT>(reinterpret_cast<const u32x4*>(static_cast<const S*>(srcs.p[0]) + edges.head) + i);
            for (int j = 1; j < pk.nsrc; ++j) {
                acc = combine<E, OP>(
                    ld<NT>(reinterpret_cast<const u32x4*>(static_cast<const S*>(srcs.p[j]) + edges.head) + i), acc);
            }
            st<NT>(vout + i, acc);
        }
        if (bid == uint32_t(h) % nblocks) {  // the scalar head and tail of segment h
            const uint32_t tid = threadIdx.x;
            uint64_t i = 0;
            bool act = false;
            if (tid < edges.head) {
                i = tid;
                act = true;
            } else if (tid >= 64 && tid - 64 < edges.tail) {
                i = edges.tailStart + (tid - 64);
                act = true;
            }
            if (act) {
                S acc = static_cast<const S*>(srcs.p[0])[i];
                for (int j = 1; j < pk.nsrc; ++j) acc = E::template ap<OP>(static_cast<const S*>(srcs.p[j])[i], acc);
                out[i] = acc;
            }
        }
    }
}

template <class E, int OP>
__global__ __launch_bounds__(kBlock) void k_reduceN_scalar(typename E::S* out, SrcPack srcs, int nsrc, uint64_t count)
{
    using S = typename E::S;
    for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < count; i += uint64_t(gridDim.x) * kBlock) {
        S acc = static_cast<const S*>(srcs.p[0])[i];
        for (int j = 1; j < nsrc; ++j) {
            acc = E::template ap<OP>(static_cast<const S*>(srcs.p[j])[i], acc);
        }
        out[i] = acc;
    }
}

// ------------------------------------------------------------------------------------------------ host launch

namespace {

// Launch shape of one kernel family: workgroups per CU in the persistent grid, 16-B vectors per lane per
// operand per iteration (U), cache policy bits (NT) and tile order (ORD).
struct LaunchCfg {
    uint32_t blocksPerCu;
    uint32_t unroll;
    uint32_t nt;
    uint32_t order;
};

// 0 = "use the default" for every field.
std::atomic<uint32_t> g_blocksPerCu{0};
std::atomic<uint32_t> g_unroll{0};
std::atomic<uint32_t> g_policy{0};
std::atomic<uint32_t> g_order{0};
std::atomic<uint32_t> g_foldMode{0};  // n-ary fold operand pipelining: 0 default, 1 serial, 2 prefetch, 3 fixed n

// Defaults from the interleaved launch sweep on MI355X (tools/sweep_local.py): the HBM stream
// peaks with ~16 KiB of loads in flight per CU (2 workgroups x 256 lanes x 2 operands x 16 B) and nt loads+stores;
// more bytes in flight lowers throughput.
constexpr LaunchCfg kDefault2{2, 1, 3, 0};
// The n-ary fold's input loop is serial per wave (input j+1 is loaded after input j is folded), so its loads in flight
// per CU are blocksPerCu x waves x U vectors, whatever n is. Two inputs behave like the 2-input kernel (U = 1 best);
// from three inputs up, U = 4 keeps enough bytes in flight (tools/sweep_fold_launch.py, interleaved rounds, fp32 SUM,
// 1 GiB per input: n = 2 498 vs 554 us at U = 2; n = 3 714 vs 745; n = 4 913 vs 927; n = 8 1709 vs 1787).
constexpr LaunchCfg kDefaultN2{2, 1, 3, 0};
constexpr LaunchCfg kDefaultN{2, 4, 3, 0};

constexpr const LaunchCfg& DefaultFor(uint32_t nsrc) { return nsrc <= 2 ? kDefaultN2 : kDefaultN; }

LaunchCfg CurrentCfg(const LaunchCfg& dflt)
{
    LaunchCfg c;
    c.blocksPerCu = g_blocksPerCu.load(std::memory_order_relaxed);
    c.unroll = g_unroll.load(std::memory_order_relaxed);
    uint32_t pol = g_policy.load(std::memory_order_relaxed);
    uint32_t ord = g_order.load(std::memory_order_relaxed);
    if (c.blocksPerCu == 0) c.blocksPerCu = dflt.blocksPerCu;
    if (c.unroll == 0) c.unroll = dflt.unroll;
    c.nt = pol == 0 ? dflt.nt : pol - 1;
    c.order = ord == 0 ? dflt.order : ord - 1;
    return c;
}

int CuCount()
{
    static std::mutex mu;
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        return 256;
    }
    std::lock_guard<std::mutex> lk(mu);
    if (cached[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) {
            n = 256;
        }
        cached[dev] = n;
    }
    return cached[dev];
}

uint32_t GridFor(uint64_t work, uint32_t perBlock, const LaunchCfg& cfg)
{
    uint64_t need = (work + perBlock - 1) / perBlock;
    uint64_t cap = uint64_t(CuCount()) * cfg.blocksPerCu;
    if (need > cap) need = cap;
    if (need == 0) need = 1;
    return static_cast<uint32_t>(need);
}

// Split [0, count) into head / 16-B vector body / tail for pointers that share one alignment phase.
template <typename S>
bool SplitAligned(const void* const* ptrs, int n, uint64_t count, Edges* e, uint64_t* nvec)
{
    constexpr uint64_t kVec = 16 / sizeof(S);
    uintptr_t phase = reinterpret_cast<uintptr_t>(ptrs[0]) & 15u;
    for (int i = 1; i < n; ++i) {
        if ((reinterpret_cast<uintptr_t>(ptrs[i]) & 15u) != phase) return false;
    }
    if (phase % sizeof(S) != 0) return false;
    uint64_t head = phase == 0 ? 0 : (16 - phase) / sizeof(S);
    if (head > count) head = count;
    uint64_t rest = count - head;
    *nvec = rest / kVec;
    e->head = static_cast<uint32_t>(head);
    e->tailStart = head + *nvec * kVec;
    e->tail = static_cast<uint32_t>(count - e->tailStart);
    return true;
}

template <class E, int OP, int U, int NT, int ORD = 0>
hipError_t Run2Variant(void* out, const void* src, const void* dst, uint64_t nvec, Edges edges, uint32_t grid,
                       hipStream_t stream)
{
    using S = typename E::S;
    hipLaunchKernelGGL((k_reduce2<E, OP, U, NT, ORD>), dim3(grid), dim3(kBlock), 0, stream, static_cast<S*>(out),
                       static_cast<const S*>(src), static_cast<const S*>(dst), nvec, edges);
    return hipGetLastError();
}

template <class E, int OP, int U, int NT, int MODE = 0, int NS = 0, int ORD = 0>
hipError_t RunNVariant(void* out, const SrcPack& pk, int n, uint64_t nvec, Edges edges, uint32_t grid,
                       hipStream_t stream)
{
    using S = typename E::S;
    hipLaunchKernelGGL((k_reduceN<E, OP, U, NT, MODE, NS, ORD>), dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<S*>(out), pk, n, nvec, edges);
    return hipGetLastError();
}

// Operand pipelining variants of the fold (FoldTile): FM 1 serial, 2 prefetch, 3 compile-time operand count (n = 3..8;
// larger n takes the prefetch form).
template <class E, int OP, int U, int FM>
hipError_t RunNMode(void* out, const SrcPack& pk, int n, uint64_t nvec, Edges edges, uint32_t grid, hipStream_t stream)
{
    if constexpr (FM == 3) {
        switch (n) {
            case 3: return RunNVariant<E, OP, U, 3, 0, 3>(out, pk, n, nvec, edges, grid, stream);
            case 4: return RunNVariant<E, OP, U, 3, 0, 4>(out, pk, n, nvec, edges, grid, stream);
            case 5: return RunNVariant<E, OP, U, 3, 0, 5>(out, pk, n, nvec, edges, grid, stream);
            case 6: return RunNVariant<E, OP, U, 3, 0, 6>(out, pk, n, nvec, edges, grid, stream);
            case 7: return RunNVariant<E, OP, U, 3, 0, 7>(out, pk, n, nvec, edges, grid, stream);
            case 8: return RunNVariant<E, OP, U, 3, 0, 8>(out, pk, n, nvec, edges, grid, stream);
            default: return RunNVariant<E, OP, U, 3, 1, 0>(out, pk, n, nvec, edges, grid, stream);
        }
    } else {
        return RunNVariant<E, OP, U, 3, FM == 2 ? 1 : 0, 0>(out, pk, n, nvec, edges, grid, stream);
    }
}

// fp32 SUM (the headline path) carries every tuning variant; other (dtype, op) pairs are built at the default.
template <class E, int OP>
constexpr bool kTunable = std::is_same<E, EFp<float>>::value && OP == R_SUM;

template <class E, int OP, int U>
hipError_t Run2U(const LaunchCfg& c, void* out, const void* src, const void* dst, uint64_t nvec, Edges edges,
                 uint32_t grid, hipStream_t stream)
{
    switch (c.nt + 4 * c.order) {
        case 0: return Run2Variant<E, OP, U, 0, 0>(out, src, dst, nvec, edges, grid, stream);
        case 1: return Run2Variant<E, OP, U, 1, 0>(out, src, dst, nvec, edges, grid, stream);
        case 2: return Run2Variant<E, OP, U, 2, 0>(out, src, dst, nvec, edges, grid, stream);
        case 3: return Run2Variant<E, OP, U, 3, 0>(out, src, dst, nvec, edges, grid, stream);
        case 7: return Run2Variant<E, OP, U, 3, 1>(out, src, dst, nvec, edges, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

template <class E, int OP>
hipError_t Run2(void* out, const void* src, const void* dst, uint64_t count, hipStream_t stream)
{
    using S = typename E::S;
    LaunchCfg cfg = CurrentCfg(kDefault2);
    const void* ptrs[3] = {out, src, dst};
    Edges edges{};
    uint64_t nvec = 0;
    if (!SplitAligned<S>(ptrs, 3, count, &edges, &nvec)) {
        uint32_t grid = GridFor(count, kBlock * 4, cfg);
        hipLaunchKernelGGL((k_reduce2_scalar<E, OP>), dim3(grid), dim3(kBlock), 0, stream, static_cast<S*>(out),
                           static_cast<const S*>(src), static_cast<const S*>(dst), count);
        return hipGetLastError();
    }
    if constexpr (kTunable<E, OP>) {
        uint32_t grid = GridFor(nvec, kBlock * cfg.unroll, cfg);
        switch (cfg.unroll) {
            case 1: return Run2U<E, OP, 1>(cfg, out, src, dst, nvec, edges, grid, stream);
            case 2: return Run2U<E, OP, 2>(cfg, out, src, dst, nvec, edges, grid, stream);
            case 4: return Run2U<E, OP, 4>(cfg, out, src, dst, nvec, edges, grid, stream);
            case 8: return Run2U<E, OP, 8>(cfg, out, src, dst, nvec, edges, grid, stream);
            default: return hipErrorInvalidValue;
        }
    } else {
        uint32_t grid = GridFor(nvec, kBlock * kDefault2.unroll, cfg);
        return Run2Variant<E, OP, kDefault2.unroll, kDefault2.nt>(out, src, dst, nvec, edges, grid, stream);
    }
}

template <class E, int OP>
hipError_t RunN(void* out, const void* const* srcs, uint32_t n, uint64_t count, hipStream_t stream)
{
    using S = typename E::S;
    LaunchCfg cfg = CurrentCfg(DefaultFor(n));
    SrcPack pk{};
    const void* ptrs[HCCL_AMD_IR_MAX_SRC + 1];
    ptrs[0] = out;
    for (uint32_t j = 0; j < n; ++j) {
        pk.p[j] = srcs[j];
        ptrs[j + 1] = srcs[j];
    }
    Edges edges{};
    uint64_t nvec = 0;
    if (!SplitAligned<S>(ptrs, int(n) + 1, count, &edges, &nvec)) {
        uint32_t grid = GridFor(count, kBlock * 4, cfg);
        hipLaunchKernelGGL((k_reduceN_scalar<E, OP>), dim3(grid), dim3(kBlock), 0, stream, static_cast<S*>(out), pk,
                           int(n), count);
        return hipGetLastError();
    }
    if constexpr (kTunable<E, OP>) {
        uint32_t grid = GridFor(nvec, kBlock * cfg.unroll, cfg);
        const uint32_t fm = g_foldMode.load(std::memory_order_relaxed);
        if (fm >= 2 && cfg.nt == 3) {
            switch (cfg.unroll * 4 + fm) {
                case 4 + 2: return RunNMode<E, OP, 1, 2>(out, pk, int(n), nvec, edges, grid, stream);
                case 4 + 3: return RunNMode<E, OP, 1, 3>(out, pk, int(n), nvec, edges, grid, stream);
                case 8 + 2: return RunNMode<E, OP, 2, 2>(out, pk, int(n), nvec, edges, grid, stream);
                case 8 + 3: return RunNMode<E, OP, 2, 3>(out, pk, int(n), nvec, edges, grid, stream);
                case 16 + 2: return RunNMode<E, OP, 4, 2>(out, pk, int(n), nvec, edges, grid, stream);
                case 16 + 3: return RunNMode<E, OP, 4, 3>(out, pk, int(n), nvec, edges, grid, stream);
                default: return hipErrorInvalidValue;
            }
        }
        if (cfg.order == 1 && cfg.nt == 3) {  // SetReduceLaunch cache policy 5: contiguous tile runs (A/B)
            switch (cfg.unroll) {
                case 1: return RunNVariant<E, OP, 1, 3, 0, 0, 1>(out, pk, int(n), nvec, edges, grid, stream);
                case 2: return RunNVariant<E, OP, 2, 3, 0, 0, 1>(out, pk, int(n), nvec, edges, grid, stream);
                case 4: return RunNVariant<E, OP, 4, 3, 0, 0, 1>(out, pk, int(n), nvec, edges, grid, stream);
                default: return hipErrorInvalidValue;
            }
        }
        switch (cfg.unroll * 4 + cfg.nt) {
            case 4 + 0: return RunNVariant<E, OP, 1, 0>(out, pk, int(n), nvec, edges, grid, stream);
            case 4 + 1: return RunNVariant<E, OP, 1, 1>(out, pk, int(n), nvec, edges, grid, stream);
            case 4 + 2: return RunNVariant<E, OP, 1, 2>(out, pk, int(n), nvec, edges, grid, stream);
            case 4 + 3: return RunNVariant<E, OP, 1, 3>(out, pk, int(n), nvec, edges, grid, stream);
            case 8 + 0: return RunNVariant<E, OP, 2, 0>(out, pk, int(n), nvec, edges, grid, stream);
            case 8 + 1: return RunNVariant<E, OP, 2, 1>(out, pk, int(n), nvec, edges, grid, stream);
            case 8 + 2: return RunNVariant<E, OP, 2, 2>(out, pk, int(n), nvec, edges, grid, stream);
            case 8 + 3: return RunNVariant<E, OP, 2, 3>(out, pk, int(n), nvec, edges, grid, stream);
            case 16 + 0: return RunNVariant<E, OP, 4, 0>(out, pk, int(n), nvec, edges, grid, stream);
            case 16 + 1: return RunNVariant<E, OP, 4, 1>(out, pk, int(n), nvec, edges, grid, stream);
            case 16 + 2: return RunNVariant<E, OP, 4, 2>(out, pk, int(n), nvec, edges, grid, stream);
            case 16 + 3: return RunNVariant<E, OP, 4, 3>(out, pk, int(n), nvec, edges, grid, stream);
            default: return hipErrorInvalidValue;
        }
    } else {
        if (n <= 2) {
            uint32_t grid = GridFor(nvec, kBlock * kDefaultN2.unroll, cfg);
            return RunNVariant<E, OP, kDefaultN2.unroll, kDefaultN2.nt>(out, pk, int(n), nvec, edges, grid, stream);
        }
        uint32_t grid = GridFor(nvec, kBlock * kDefaultN.unroll, cfg);
        return RunNVariant<E, OP, kDefaultN.unroll, kDefaultN.nt>(out, pk, int(n), nvec, edges, grid, stream);
    }
}

template <class E>
hipError_t Dispatch2(int op, void* out, const void* src, const void* dst, uint64_t count, hipStream_t s)
{
    switch (op) {
        case R_SUM: return Run2<E, R_SUM>(out, src, dst, count, s);
        case R_PROD: return Run2<E, R_PROD>(out, src, dst, count, s);
        case R_MAX: return Run2<E, R_MAX>(out, src, dst, count, s);
        default: return Run2<E, R_MIN>(out, src, dst, count, s);
    }
}

template <class E>
hipError_t DispatchN(int op, void* out, const void* const* srcs, uint32_t n, uint64_t count, hipStream_t s)
{
    switch (op) {
        case R_SUM: return RunN<E, R_SUM>(out, srcs, n, count, s);
        case R_PROD: return RunN<E, R_PROD>(out, srcs, n, count, s);
        case R_MAX: return RunN<E, R_MAX>(out, srcs, n, count, s);
        default: return RunN<E, R_MIN>(out, srcs, n, count, s);
    }
}

using EI8 = EInt<int8_t, uint32_t>;
using EI16 = EInt<int16_t, uint32_t>;
using EI32 = EInt<int32_t, uint32_t>;
using EI64 = EInt<int64_t, uint64_t>;
using EU64 = EInt<uint64_t, uint64_t>;
using EF32 = EFp<float>;
using EF64 = EFp<double>;

bool ValidOp(HcclReduceOp op) { return op >= HCCL_REDUCE_SUM && op <= HCCL_REDUCE_MIN; }

}  // namespace

HcclResult SetReduceLaunch(uint32_t blocksPerCu, uint32_t unroll, uint32_t cachePolicy)
{
    // cachePolicy: 0 = default, 1 = plain, 2 = nt loads, 3 = nt stores, 4 = nt loads + stores,
    //              5 = nt loads + stores with contiguous per-workgroup tile runs (ORD 1)
    if (blocksPerCu > 32 || (unroll != 0 && unroll != 1 && unroll != 2 && unroll != 4 && unroll != 8) ||
        cachePolicy > 5) {
        return HCCL_E_PARA;
    }
    g_blocksPerCu.store(blocksPerCu);
    g_unroll.store(unroll);
    if (cachePolicy == 5) {
        g_policy.store(4);
        g_order.store(2);
    } else {
        g_policy.store(cachePolicy);
        g_order.store(cachePolicy == 0 ? 0 : 1);
    }
    return HCCL_SUCCESS;
}

HcclResult SetFoldMode(uint32_t mode)
{
    if (mode > 3) return HCCL_E_PARA;
    g_foldMode.store(mode);
    return HCCL_SUCCESS;
}

HcclResult LaunchReduce2(void* out, const void* src, const void* dst, uint64_t count, HcclDataType dt,
                         HcclReduceOp op, hipStream_t stream)
{
    if (count == 0) return HCCL_SUCCESS;
    if (!ValidOp(op)) return HCCL_E_PARA;
    hipError_t e;
    switch (dt) {
        case HCCL_DATA_TYPE_INT8: e = Dispatch2<EI8>(op, out, src, dst, count, stream); break;
        case HCCL_DATA_TYPE_INT16: e = Dispatch2<EI16>(op, out, src, dst, count, stream); break;
        case HCCL_DATA_TYPE_INT32: e = Dispatch2<EI32>(op, out, src, dst, count, stream); break;
        case HCCL_DATA_TYPE_INT64: e = Dispatch2<EI64>(op, out, src, dst, count, stream); break;
        case HCCL_DATA_TYPE_UINT64: e = Dispatch2<EU64>(op, out, src, dst, count, stream); break;
        case HCCL_DATA_TYPE_FP16: e = Dispatch2<EF16>(op, out, src, dst, count, stream); break;
        case HCCL_DATA_TYPE_BFP16: e = Dispatch2<EBF16>(op, out, src, dst, count, stream); break;
        case HCCL_DATA_TYPE_FP32: e = Dispatch2<EF32>(op, out, src, dst, count, stream); break;
        case HCCL_DATA_TYPE_FP64: e = Dispatch2<EF64>(op, out, src, dst, count, stream); break;
        default: return HCCL_E_NOT_SUPPORT;
    }
    if (e != hipSuccess) {
        HCCL_AMD_ERR("reduce launch failed: %s", hipGetErrorString(e));
        return HCCL_E_RUNTIME;
    }
    return HCCL_SUCCESS;
}

HcclResult LaunchReduceN(void* out, const void* const* srcs, uint32_t n, uint64_t count, HcclDataType dt,
                         HcclReduceOp op, hipStream_t stream)
{
    if (count == 0) return HCCL_SUCCESS;
    if (!ValidOp(op) || n == 0 || n > HCCL_AMD_IR_MAX_SRC) return HCCL_E_PARA;
    if (n == 1) {
        if (out == srcs[0]) return HCCL_SUCCESS;
        uint32_t es = DataTypeSize(dt);
        if (es == 0) return HCCL_E_NOT_SUPPORT;
        return LaunchCopyBytes(out, srcs[0], count * es, stream);
    }
    if (n == 2) {
        // acc = srcs[1] (op) srcs[0]
        return LaunchReduce2(out, srcs[1], srcs[0], count, dt, op, stream);
    }
    hipError_t e;
    switch (dt) {
        case HCCL_DATA_TYPE_INT8: e = DispatchN<EI8>(op, out, srcs, n, count, stream); break;
        case HCCL_DATA_TYPE_INT16: e = DispatchN<EI16>(op, out, srcs, n, count, stream); break;
        case HCCL_DATA_TYPE_INT32: e = DispatchN<EI32>(op, out, srcs, n, count, stream); break;
        case HCCL_DATA_TYPE_INT64: e = DispatchN<EI64>(op, out, srcs, n, count, stream); break;
        case HCCL_DATA_TYPE_UINT64: e = DispatchN<EU64>(op, out, srcs, n, count, stream); break;
        case HCCL_DATA_TYPE_FP16: e = DispatchN<EF16>(op, out, srcs, n, count, stream); break;
        case HCCL_DATA_TYPE_BFP16: e = DispatchN<EBF16>(op, out, srcs, n, count, stream); break;
        case HCCL_DATA_TYPE_FP32: e = DispatchN<EF32>(op, out, srcs, n, count, stream); break;
        case HCCL_DATA_TYPE_FP64: e = DispatchN<EF64>(op, out, srcs, n, count, stream); break;
        default: return HCCL_E_NOT_SUPPORT;
    }
    if (e != hipSuccess) {
        HCCL_AMD_ERR("reduceN launch failed: %s", hipGetErrorString(e));
        return HCCL_E_RUNTIME;
    }
    return HCCL_SUCCESS;
}

namespace {

template <class E, int OP>
hipError_t RunBatch(const BatchPack& pk, uint32_t nseg, uint64_t maxVec, hipStream_t stream)
{
    BatchPack p = pk;
    p.nseg = int(nseg);
    uint64_t totalVec = 0;
    for (uint32_t g = 0; g < nseg; ++g) totalVec += pk.nvec[g];
    if (totalVec * 16 / nseg < kBatchFlatSegBytes) {  // 16-B vectors: the average segment's bytes
        // rows: the per-CU budget of the n-ary default split over the segments, each row sized for the longest
        const LaunchCfg& c0 = DefaultFor(static_cast<uint32_t>(pk.nsrc));
        const uint64_t cap = std::max<uint64_t>(1, uint64_t(CuCount()) * c0.blocksPerCu / nseg);
        const uint64_t need = std::max<uint64_t>(1, (maxVec + kBlock * c0.unroll - 1) / (kBlock * c0.unroll));
        const uint32_t gr = static_cast<uint32_t>(std::min(cap, need));
        if (pk.nsrc <= 2) {
            hipLaunchKernelGGL((k_reduceN_batch_rows<E, OP, kDefaultN2.unroll, kDefaultN2.nt>), dim3(gr, nseg),
                               dim3(kBlock), 0, stream, p);
        } else {
            hipLaunchKernelGGL((k_reduceN_batch_rows<E, OP, kDefaultN.unroll, kDefaultN.nt>), dim3(gr, nseg),
                               dim3(kBlock), 0, stream, p);
        }
        return hipGetLastError();
    }
    // flat: one persistent grid over the concatenated tiles, sized like a single fold of the batch's bytes. U = 4 for
    // every operand count: with two operands too the tile walk wants the larger tile (5.0 / 5.6 / 6.1 TB/s at U = 1 /
    // 2 / 4 for 4 MiB segments, 5.7 / 6.3 / 6.4 at 16 MiB).
    const LaunchCfg& cfg = kDefaultN;
    const uint64_t tileVec = uint64_t(kBlock) * cfg.unroll;
    p.tileStart[0] = 0;
    for (uint32_t g = 0; g < nseg; ++g) p.tileStart[g + 1] = p.tileStart[g] + pk.nvec[g] / tileVec;
    const uint32_t gx = GridFor(totalVec, static_cast<uint32_t>(tileVec), cfg);
    hipLaunchKernelGGL((k_reduceN_batch<E, OP, kDefaultN.unroll, kDefaultN.nt>), dim3(gx), dim3(kBlock), 0, stream, p);
    return hipGetLastError();
}

template <class E>
hipError_t DispatchBatch(int op, const BatchPack& pk, uint32_t nseg, uint64_t maxVec, hipStream_t s)
{
    switch (op) {
        case R_SUM: return RunBatch<E, R_SUM>(pk, nseg, maxVec, s);
        case R_PROD: return RunBatch<E, R_PROD>(pk, nseg, maxVec, s);
        case R_MAX: return RunBatch<E, R_MAX>(pk, nseg, maxVec, s);
        default: return RunBatch<E, R_MIN>(pk, nseg, maxVec, s);
    }
}

}  // namespace

HcclResult LaunchReduceNBatch(const FoldSeg* segs, uint32_t nseg, uint32_t nsrc, HcclDataType dt, HcclReduceOp op,
                              hipStream_t stream)
{
    if (!ValidOp(op) || nsrc < 2 || nsrc > HCCL_AMD_IR_MAX_SRC || nseg > kMaxBatchSegs) return HCCL_E_PARA;
    const uint32_t es = DataTypeSize(dt);
    if (es == 0) return HCCL_E_NOT_SUPPORT;
    BatchPack pk{};
    pk.nsrc = int(nsrc);
    uint32_t nb = 0;
    uint64_t maxVec = 0;
    for (uint32_t g = 0; g < nseg; ++g) {
        const FoldSeg& f = segs[g];
        if (f.count == 0) continue;
        const void* ptrs[HCCL_AMD_IR_MAX_SRC + 1];
        ptrs[0] = f.out;
        for (uint32_t j = 0; j < nsrc; ++j) ptrs[j + 1] = f.srcs[j];
        Edges edges{};
        uint64_t nvec = 0;
        bool ok = false;
        switch (es) {
            case 1: ok = SplitAligned<uint8_t>(ptrs, int(nsrc) + 1, f.count, &edges, &nvec); break;
            case 2: ok = SplitAligned<uint16_t>(ptrs, int(nsrc) + 1, f.count, &edges, &nvec); break;
            case 4: ok = SplitAligned<uint32_t>(ptrs, int(nsrc) + 1, f.count, &edges, &nvec); break;
            default: ok = SplitAligned<uint64_t>(ptrs, int(nsrc) + 1, f.count, &edges, &nvec); break;
        }
        // a segment whose pointers do not share a 16-B phase runs on its own (scalar kernel)
        if (!ok) {
            HCCL_CHK(LaunchReduceN(f.out, f.srcs, nsrc, f.count, dt, op, stream));
            continue;
        }
        pk.out[nb] = f.out;
        for (uint32_t j = 0; j < nsrc; ++j) pk.srcs[nb].p[j] = f.srcs[j];
        pk.nvec[nb] = nvec;
        pk.edges[nb] = edges;
        maxVec = std::max(maxVec, nvec);
        ++nb;
    }
    if (nb == 0) return HCCL_SUCCESS;
    hipError_t e;
    switch (dt) {
        case HCCL_DATA_TYPE_INT8: e = DispatchBatch<EI8>(op, pk, nb, maxVec, stream); break;
        case HCCL_DATA_TYPE_INT16: e = DispatchBatch<EI16>(op, pk, nb, maxVec, stream); break;
        case HCCL_DATA_TYPE_INT32: e = DispatchBatch<EI32>(op, pk, nb, maxVec, stream); break;
        case HCCL_DATA_TYPE_INT64: e = DispatchBatch<EI64>(op, pk, nb, maxVec, stream); break;
        case HCCL_DATA_TYPE_UINT64: e = DispatchBatch<EU64>(op, pk, nb, maxVec, stream); break;
        case HCCL_DATA_TYPE_FP16: e = DispatchBatch<EF16>(op, pk, nb, maxVec, stream); break;
        case HCCL_DATA_TYPE_BFP16: e = DispatchBatch<EBF16>(op, pk, nb, maxVec, stream); break;
        case HCCL_DATA_TYPE_FP32: e = DispatchBatch<EF32>(op, pk, nb, maxVec, stream); break;
        case HCCL_DATA_TYPE_FP64: e = DispatchBatch<EF64>(op, pk, nb, maxVec, stream); break;
        default: return HCCL_E_NOT_SUPPORT;
    }
    if (e != hipSuccess) {
        HCCL_AMD_ERR("batched reduce launch failed: %s", hipGetErrorString(e));
        return HCCL_E_RUNTIME;
    }
    return HCCL_SUCCESS;
}


// ------------------------------------------------------------------------------------------------ device copies

namespace {

// dst[0, bytes) = src[0, bytes) in units of W bytes (W = the widest of 16, 8, 4, 2, 1 in which dst and src share their
// alignment phase: every schedule's copy is at least element-aligned, and 16 B whenever its offsets are): kCopyU units
// per lane in flight (loads first, then stores; non-temporal both ways, like the reduce kernels) over a grid of tiles
// dealt round-robin; the ragged head (before dst reaches a W boundary) and tail bytes one by one. A kernel of this
// library, so the copy's stores are ordered before the next kernel of the stream by the ordinary end-of-kernel release
// like every other kernel here (root cause of the stale operands).
constexpr int kCopyU = 4;

template <int W>
struct CopyUnit;
template <>
struct CopyUnit<16> {
    using T = u32x4;
};
template <>
struct CopyUnit<8> {
    using T = uint64_t;
};
template <>
struct CopyUnit<4> {
    using T = uint32_t;
};
template <>
struct CopyUnit<2> {
    using T = uint16_t;
};
template <>
struct CopyUnit<1> {
    using T = unsigned char;
};

template <int W>
__device__ __forceinline__ typename CopyUnit<W>::T CopyLd(const typename CopyUnit<W>::T* p)
{
    if constexpr (W == 16) {
        return ld<3>(p);
    } else {
        return __builtin_nontemporal_load(p);
    }
}

template <int W>
__device__ __forceinline__ void CopySt(typename CopyUnit<W>::T* p, typename CopyUnit<W>::T v)
{
    if constexpr (W == 16) {
        st<3>(p, v);
    } else {
        __builtin_nontemporal_store(v, p);
    }
}

template <int W>
__global__ __launch_bounds__(256) void k_copy_units(unsigned char* dst, const unsigned char* src, uint64_t head,
                                                    uint64_t nunits, uint64_t bytes)
{
    using T = typename CopyUnit<W>::T;
    const T* s = reinterpret_cast<const T*>(src + head);
    T* d = reinterpret_cast<T*>(dst + head);
    constexpr uint64_t kTile = uint64_t(256) * kCopyU;
    const uint64_t fullTiles = nunits / kTile;
    for (uint64_t t = blockIdx.x; t < fullTiles; t += gridDim.x) {
        const uint64_t base = t * kTile + threadIdx.x;
        T x[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) x[u] = CopyLd<W>(s + base + u * 256);
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) CopySt<W>(d + base + u * 256, x[u]);
    }
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = fullTiles * kTile + tid; i < nunits; i += stride) d[i] = s[i];
    for (uint64_t i = tid; i < head; i += stride) dst[i] = src[i];
    for (uint64_t i = head + nunits * W + tid; i < bytes; i += stride) dst[i] = src[i];
}

template <int W>
hipError_t RunCopy(unsigned char* dst, const unsigned char* src, uint64_t bytes, hipStream_t stream)
{
    const uint64_t mis = (W - (reinterpret_cast<uintptr_t>(dst) & (W - 1))) & (W - 1);
    const uint64_t head = std::min<uint64_t>(bytes, mis);
    const uint64_t nunits = (bytes - head) / W;
    // One tile per workgroup up to 16 tiles per CU (latency-bound sizes: 16 MiB ran 8.96 us on a 2-per-CU persistent
    // grid against hipMemcpyAsync's 7.88, profiles/r04_copy_kernel.jsonl); beyond that a persistent grid of two
    // workgroups per CU, the reduce kernels' measured best (1 GiB: 356-410 us against hipMemcpyAsync's 417-455).
    const uint64_t tiles = std::max<uint64_t>(1, (std::max<uint64_t>(nunits, 1) + 256 * kCopyU - 1) / (256 * kCopyU));
    const uint64_t cus = uint64_t(CuCount());
    const uint64_t blocks = tiles <= cus * 16 ? tiles : cus * 2;
    hipLaunchKernelGGL((k_copy_units<W>), dim3(uint32_t(blocks)), dim3(256), 0, stream, dst, src, head, nunits, bytes);
    return hipGetLastError();
}

}  // namespace

HcclResult LaunchCopyBytes(void* dst, const void* src, uint64_t bytes, hipStream_t stream)
{
    if (bytes == 0 || dst == src) return HCCL_SUCCESS;
    auto* d = static_cast<unsigned char*>(dst);
    const auto* sp = static_cast<const unsigned char*>(src);
    const uintptr_t x = reinterpret_cast<uintptr_t>(dst) ^ reinterpret_cast<uintptr_t>(src);  // phase difference
    hipError_t e;
    if ((x & 15u) == 0) {
        e = RunCopy<16>(d, sp, bytes, stream);
    } else if ((x & 7u) == 0) {
        e = RunCopy<8>(d, sp, bytes, stream);
    } else if ((x & 3u) == 0) {
        e = RunCopy<4>(d, sp, bytes, stream);
    } else if ((x & 1u) == 0) {
        e = RunCopy<2>(d, sp, bytes, stream);
    } else {
        e = RunCopy<1>(d, sp, bytes, stream);
    }
    if (e != hipSuccess) {
        HCCL_AMD_ERR("copy launch failed: %s", hipGetErrorString(e));
        return HCCL_E_RUNTIME;
    }
    return HCCL_SUCCESS;
}

}  // namespace hccl_amd
