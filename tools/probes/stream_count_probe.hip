// stream_count_probe.hip — does the number of concurrent HBM streams lower the ceiling? (measurement tool, not
// product code). Pure reads of NS streams (XOR kept in registers, one store per lane at the end) and the fold's shape
// (NS reads + 1 write, XOR combine, so no arithmetic cost), both persistent-grid / grid-stride over 16-B vectors with
// the product's launch (256-thread workgroups, nt loads and stores), every stream's U vectors issued before use.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/stream_count_probe.hip -o tools/libstream_count_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kB = 256;

struct Ptrs {
    const u32x4* p[16];
};

template <int NS, int U, bool WRITE>
__global__ __launch_bounds__(kB) void k_streams(Ptrs in, u32x4* out, u32x4* sink, uint64_t nvec)
{
    const uint64_t tile = uint64_t(kB) * U;
    u32x4 keep = {0, 0, 0, 0};
    for (uint64_t t = blockIdx.x; t < nvec / tile; t += gridDim.x) {
        const uint64_t base = t * tile + threadIdx.x;
        u32x4 v[NS][U];
#pragma unroll
        for (int j = 0; j < NS; ++j) {
#pragma unroll
            for (int u = 0; u < U; ++u) v[j][u] = __builtin_nontemporal_load(in.p[j] + base + u * kB);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 acc = v[0][u];
#pragma unroll
            for (int j = 1; j < NS; ++j) acc ^= v[j][u];
            if constexpr (WRITE) {
                __builtin_nontemporal_store(acc, out + base + u * kB);
            } else {
                keep ^= acc;
            }
        }
    }
    if constexpr (!WRITE) sink[uint64_t(blockIdx.x) * kB + threadIdx.x] = keep;
}

template <int NS, bool W>
hipError_t Go(int u, uint32_t grid, const Ptrs& p, u32x4* o, u32x4* sink, uint64_t nvec, hipStream_t s)
{
    switch (u) {
        case 1: hipLaunchKernelGGL((k_streams<NS, 1, W>), dim3(grid), dim3(kB), 0, s, p, o, sink, nvec); break;
        case 2: hipLaunchKernelGGL((k_streams<NS, 2, W>), dim3(grid), dim3(kB), 0, s, p, o, sink, nvec); break;
        default: hipLaunchKernelGGL((k_streams<NS, 4, W>), dim3(grid), dim3(kB), 0, s, p, o, sink, nvec); break;
    }
    return hipGetLastError();
}

template <bool W>
hipError_t GoN(int ns, int u, uint32_t grid, const Ptrs& p, u32x4* o, u32x4* sink, uint64_t nvec, hipStream_t s)
{
    switch (ns) {
        case 1: return Go<1, W>(u, grid, p, o, sink, nvec, s);
        case 2: return Go<2, W>(u, grid, p, o, sink, nvec, s);
        case 3: return Go<3, W>(u, grid, p, o, sink, nvec, s);
        case 4: return Go<4, W>(u, grid, p, o, sink, nvec, s);
        case 8: return Go<8, W>(u, grid, p, o, sink, nvec, s);
        default: return hipErrorInvalidValue;
    }
}

// write = 0: NS pure read streams; write = 1: NS reads + 1 write. grid = blocksPerCu x 256 CUs.
extern "C" int probe_streams(int ns, int write, int u, int blocksPerCu, void* const* ins, void* out, void* sink,
                             uint64_t nvec, void* stream)
{
    Ptrs p{};
    for (int j = 0; j < ns; ++j) p.p[j] = static_cast<const u32x4*>(ins[j]);
    const uint32_t grid = 256u * uint32_t(blocksPerCu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = write ? GoN<true>(ns, u, grid, p, static_cast<u32x4*>(out), static_cast<u32x4*>(sink), nvec, s)
                         : GoN<false>(ns, u, grid, p, static_cast<u32x4*>(out), static_cast<u32x4*>(sink), nvec, s);
    return e == hipSuccess ? 0 : 1;
}
