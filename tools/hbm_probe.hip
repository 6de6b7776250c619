// hbm_probe.hip — HBM stream ceilings on MI355X for the reduce kernel's access pattern (measurement tool, not
// product code). Variants, all persistent-grid / grid-stride over 16-B vectors, 256-thread workgroups:
//   read2   : 2 read streams (sum kept in registers; one 16-B store per lane at the end)
//   write1  : 1 write stream
//   copy    : 1 read + 1 write
//   r2w1    : the reduce shape (2 reads + 1 write), global_load/store with cache-policy bits LDP/STP
//   r2w1buf : same through buffer_load/store (SRD) with aux policy bits
//   r2w1lds : loads by LDS-DMA (global_load_lds_dwordx4) into a per-wave LDS window, then ds_read, add, store
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/hbm_probe.hip -o tools/libhbm_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kB = 256;

template <int NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__device__ __forceinline__ u32x4 addf(u32x4 a, u32x4 b)
{
    f32x4 x = __builtin_bit_cast(f32x4, a) + __builtin_bit_cast(f32x4, b);
    return __builtin_bit_cast(u32x4, x);
}

template <int U, int NT>
__global__ __launch_bounds__(kB) void k_read2(const u32x4* a, const u32x4* b, u32x4* sink, uint64_t nvec)
{
    u32x4 acc = {0, 0, 0, 0};
    const uint64_t tile = uint64_t(kB) * U;
    for (uint64_t t = blockIdx.x; t < nvec / tile; t += gridDim.x) {
        uint64_t base = t * tile + threadIdx.x;
        u32x4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x[u] = ld<NT>(a + base + u * kB);
            y[u] = ld<NT>(b + base + u * kB);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= x[u] ^ y[u];
    }
    sink[uint64_t(blockIdx.x) * kB + threadIdx.x] = acc;
}

template <int U, int NT>
__global__ __launch_bounds__(kB) void k_write1(u32x4* o, uint64_t nvec)
{
    const uint64_t tile = uint64_t(kB) * U;
    u32x4 v = {threadIdx.x, blockIdx.x, 1, 2};
    for (uint64_t t = blockIdx.x; t < nvec / tile; t += gridDim.x) {
        uint64_t base = t * tile + threadIdx.x;
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(o + base + u * kB, v);
    }
}

template <int U, int NT>
__global__ __launch_bounds__(kB) void k_copy(const u32x4* a, u32x4* o, uint64_t nvec)
{
    const uint64_t tile = uint64_t(kB) * U;
    for (uint64_t t = blockIdx.x; t < nvec / tile; t += gridDim.x) {
        uint64_t base = t * tile + threadIdx.x;
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<NT>(a + base + u * kB);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(o + base + u * kB, x[u]);
    }
}

template <int U, int NT>
__global__ __launch_bounds__(kB) void k_r2w1(const u32x4* a, const u32x4* b, u32x4* o, uint64_t nvec)
{
    const uint64_t tile = uint64_t(kB) * U;
    for (uint64_t t = blockIdx.x; t < nvec / tile; t += gridDim.x) {
        uint64_t base = t * tile + threadIdx.x;
        u32x4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x[u] = ld<NT>(a + base + u * kB);
            y[u] = ld<NT>(b + base + u * kB);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(o + base + u * kB, addf(x[u], y[u]));
    }
}

// buffer_load / buffer_store with explicit cache-policy aux bits (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16).
// Each workgroup tile is addressed through a descriptor rebased at the tile so the 32-bit offsets never overflow.
template <int U, int LDA, int STA>
__global__ __launch_bounds__(kB) void k_r2w1buf(const u32x4* a, const u32x4* b, u32x4* o, uint64_t nvec)
{
    const uint64_t tile = uint64_t(kB) * U;
    for (uint64_t t = blockIdx.x; t < nvec / tile; t += gridDim.x) {
        const uint64_t base = t * tile;
        auto ra = __builtin_amdgcn_make_buffer_rsrc((void*)(a + base), 0, int(tile * 16), 0x00020000);
        auto rb = __builtin_amdgcn_make_buffer_rsrc((void*)(b + base), 0, int(tile * 16), 0x00020000);
        auto ro = __builtin_amdgcn_make_buffer_rsrc((void*)(o + base), 0, int(tile * 16), 0x00020000);
        u32x4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int off = int((threadIdx.x + u * kB) * 16);
            x[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, LDA));
            y[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, LDA));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int off = int((threadIdx.x + u * kB) * 16);
            __builtin_amdgcn_raw_buffer_store_b128(addf(x[u], y[u]), ro, off, 0, STA);
        }
    }
}

// LDS-DMA loads: each wave owns a (2 x U x 1 KiB) LDS window; lanes read back their own 16 B, so only the wave's
// own vmcnt wait orders the DMA before the ds_read (no workgroup barrier).
template <int U, int AUX, int NT>
__global__ __launch_bounds__(kB) void k_r2w1lds(const u32x4* a, const u32x4* b, u32x4* o, uint64_t nvec)
{
    __shared__ u32x4 lds[2 * U * kB];
    const int wave = threadIdx.x / 64;
    const int lane = threadIdx.x % 64;
    const uint64_t tile = uint64_t(kB) * U;
    u32x4* wa = lds + wave * 64 * 2 * U;
    for (uint64_t t = blockIdx.x; t < nvec / tile; t += gridDim.x) {
        uint64_t base = t * tile + threadIdx.x;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            __builtin_amdgcn_global_load_lds((const void*)(a + base + u * kB), (__attribute__((address_space(3))) void*)(wa + (2 * u) * 64), 16, 0, AUX);
            __builtin_amdgcn_global_load_lds((const void*)(b + base + u * kB), (__attribute__((address_space(3))) void*)(wa + (2 * u + 1) * 64), 16, 0, AUX);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15) (gfx9 encoding)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 x = wa[(2 * u) * 64 + lane];
            u32x4 y = wa[(2 * u + 1) * 64 + lane];
            st<NT>(o + base + u * kB, addf(x, y));
        }
    }
}

extern "C" {

// kind: 0 read2, 1 write1, 2 copy, 3 r2w1, 4 r2w1buf, 5 r2w1lds. param: variant code (see switch).
int probe_launch(int kind, int variant, int blocksPerCu, const void* a, const void* b, void* o, uint64_t nvec,
                 void* sink, hipStream_t s)
{
    int cus = 256;
    int grid = cus * blocksPerCu;
    const u32x4* A = (const u32x4*)a;
    const u32x4* B = (const u32x4*)b;
    u32x4* O = (u32x4*)o;
#define L(K, ...) hipLaunchKernelGGL((K), dim3(grid), dim3(kB), 0, s, __VA_ARGS__)
    switch (kind * 100 + variant) {
        case 0: L((k_read2<1, 1>), A, B, (u32x4*)sink, nvec); break;
        case 1: L((k_read2<2, 1>), A, B, (u32x4*)sink, nvec); break;
        case 2: L((k_read2<4, 1>), A, B, (u32x4*)sink, nvec); break;
        case 3: L((k_read2<2, 0>), A, B, (u32x4*)sink, nvec); break;
        case 100: L((k_write1<1, 1>), O, nvec); break;
        case 101: L((k_write1<2, 1>), O, nvec); break;
        case 102: L((k_write1<4, 1>), O, nvec); break;
        case 103: L((k_write1<2, 0>), O, nvec); break;
        case 200: L((k_copy<1, 1>), A, O, nvec); break;
        case 201: L((k_copy<2, 1>), A, O, nvec); break;
        case 202: L((k_copy<4, 1>), A, O, nvec); break;
        case 203: L((k_copy<2, 0>), A, O, nvec); break;
        case 300: L((k_r2w1<1, 1>), A, B, O, nvec); break;
        case 301: L((k_r2w1<2, 1>), A, B, O, nvec); break;
        case 302: L((k_r2w1<4, 1>), A, B, O, nvec); break;
        case 400: L((k_r2w1buf<1, 2, 2>), A, B, O, nvec); break;    // nt / nt
        case 401: L((k_r2w1buf<1, 0, 2>), A, B, O, nvec); break;    // plain / nt
        case 402: L((k_r2w1buf<1, 2, 18>), A, B, O, nvec); break;   // nt / sc1 nt
        case 403: L((k_r2w1buf<1, 2, 17>), A, B, O, nvec); break;   // nt / sc0 sc1
        case 404: L((k_r2w1buf<1, 18, 2>), A, B, O, nvec); break;   // sc1 nt / nt
        case 405: L((k_r2w1buf<1, 3, 3>), A, B, O, nvec); break;    // sc0 nt / sc0 nt
        case 406: L((k_r2w1buf<2, 2, 2>), A, B, O, nvec); break;
        case 407: L((k_r2w1buf<1, 2, 16>), A, B, O, nvec); break;   // nt / sc1
        case 408: L((k_r2w1buf<1, 19, 19>), A, B, O, nvec); break;  // sc0 sc1 nt both
        case 500: L((k_r2w1lds<1, 2, 1>), A, B, O, nvec); break;
        case 501: L((k_r2w1lds<2, 2, 1>), A, B, O, nvec); break;
        case 502: L((k_r2w1lds<4, 2, 1>), A, B, O, nvec); break;
        case 503: L((k_r2w1lds<2, 0, 1>), A, B, O, nvec); break;
        default: return -1;
    }
#undef L
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
}

// Uncached (MTYPE UC) allocations, the IPC staging's memory type, to compare streams that read or write it.
extern "C" void* probe_alloc_uncached(uint64_t bytes)
{
    void* p = nullptr;
    return hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess ? p : nullptr;
}

extern "C" int probe_free(void* p) { return hipFree(p) == hipSuccess ? 0 : 1; }
