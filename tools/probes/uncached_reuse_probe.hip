// uncached_reuse_probe.hip — VERDICT r05 next #2: does a cached allocation placed on memory that was just mapped
// uncached (hipExtMallocWithFlags(hipDeviceMallocUncached), then hipFree) read and write correctly on every XCD?
//
// Per iteration, the IPC path's flags + LL block life, then an executor staging life, in one process on one device:
//   1. uncached allocation of the flags + LL block's size (4 MiB + 32 KiB); L2 scrub (one system-scope fence per CU);
//      hipMemset 0; 8-byte system-scope atomic stores of pattern P over it from 256 workgroups (the LL push); sync;
//      hipFree;
//   2. hipMalloc of the executor staging's size (2 MiB at HCCL_BUFFSIZE=1) — recorded whether it lands in the freed
//      block; a copy kernel (16-B non-temporal loads/stores, 256 workgroups, as k_copy_units) fills it from a source
//      holding pattern Q; then 256 workgroups (every XCD) read all of it with plain and non-temporal loads and count
//      words != Q; then a host copy counts words != Q and classifies them (0, P, the sentinel, other); hipFree.
// Output: one JSON line per configuration with totals. `uncached_reuse_probe fresh [iters]`: the fresh-allocation mode
// below. Build: hipcc --offload-arch=gfx950 -O2 -o uncached_reuse_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                   \
        }                                                                                   \
    } while (0)

__global__ __launch_bounds__(64) void k_scrub()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ __launch_bounds__(256) void k_ll_push(unsigned long long* p, uint64_t words, uint32_t pat)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < words; i += gridDim.x * 256ull) {
        const unsigned long long v = (static_cast<unsigned long long>(pat) << 32) | static_cast<uint32_t>(i);
        __hip_atomic_store(p + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(256) void k_fill(uint32_t* p, uint64_t words, uint32_t pat)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < words; i += gridDim.x * 256ull) p[i] = pat ^ uint32_t(i);
}

__global__ __launch_bounds__(256) void k_copy_nt(uint4* dst, const uint4* src, uint64_t vecs)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < vecs; i += gridDim.x * 256ull) {
        uint4 v;
        v.x = __builtin_nontemporal_load(&src[i].x);
        v.y = __builtin_nontemporal_load(&src[i].y);
        v.z = __builtin_nontemporal_load(&src[i].z);
        v.w = __builtin_nontemporal_load(&src[i].w);
        __builtin_nontemporal_store(v.x, &dst[i].x);
        __builtin_nontemporal_store(v.y, &dst[i].y);
        __builtin_nontemporal_store(v.z, &dst[i].z);
        __builtin_nontemporal_store(v.w, &dst[i].w);
    }
}

// every workgroup reads the whole range (plain, then non-temporal loads) and counts words != pat ^ i
__global__ __launch_bounds__(256) void k_read_all(const uint32_t* p, uint64_t words, uint32_t pat, uint32_t* out)
{
    uint32_t bad = 0, badNt = 0;
    for (uint64_t i = threadIdx.x; i < words; i += 256) {
        bad += p[i] != (pat ^ uint32_t(i));
        badNt += __builtin_nontemporal_load(p + i) != (pat ^ uint32_t(i));
    }
    __shared__ uint32_t sb, sn;
    if (threadIdx.x == 0) sb = sn = 0;
    __syncthreads();
    atomicAdd(&sb, bad);
    atomicAdd(&sn, badNt);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        out[3 * blockIdx.x + 0] = sb;
        out[3 * blockIdx.x + 1] = sn;
        out[3 * blockIdx.x + 2] = xcc & 15u;
    }
}

// "fresh" mode (r06): does the first kernel that writes a freshly allocated buffer have its bytes kept? Per iteration:
// optionally allocate and free a 1 GiB uncached block first (work for the driver's wipe of released VRAM), then
// allocate S bytes (cached or uncached), launch at once a 256-workgroup kernel writing a pattern over all of it, then a
// kernel that counts mismatching words from 256 workgroups on every XCD; then a host copy of the first and last 4 MiB.
// A zero word where the pattern should be means the write was lost or overwritten after the fact.
__global__ __launch_bounds__(256) void k_count(const uint32_t* p, uint64_t words, uint32_t pat, unsigned long long* bad,
                                               unsigned long long* zero)
{
    unsigned long long b = 0, z = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < words; i += gridDim.x * 256ull) {
        const uint32_t x = p[i];
        b += x != (pat ^ uint32_t(i));
        z += x == 0;
    }
    atomicAdd(bad, b);
    atomicAdd(zero, z);
}

int fresh(int iters)
{
    unsigned long long* cnt = nullptr;
    CHK(hipMalloc(&cnt, 16));
    const size_t sizes[] = {2ull << 20, 64ull << 20, 512ull << 20};
    for (int unc = 0; unc < 2; ++unc) {
        for (size_t S : sizes) {
            for (int churn = 0; churn < 2; ++churn) {
                long runsBad = 0, gpuBad = 0, gpuZero = 0, hostBad = 0;
                for (int it = 0; it < iters; ++it) {
                    if (churn) {
                        void* big = nullptr;
                        CHK(hipExtMallocWithFlags(&big, 1ull << 30, hipDeviceMallocUncached));
                        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, nullptr, static_cast<uint32_t*>(big),
                                           uint64_t((1ull << 30) / 4), 0x77u);
                        CHK(hipDeviceSynchronize());
                        CHK(hipFree(big));
                    }
                    void* b = nullptr;
                    if (unc) {
                        CHK(hipExtMallocWithFlags(&b, S, hipDeviceMallocUncached));
                    } else {
                        CHK(hipMalloc(&b, S));
                    }
                    const uint32_t pat = 0x1C000000u | uint32_t(it * 131 + int(S >> 20));
                    hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, nullptr, static_cast<uint32_t*>(b),
                                       uint64_t(S / 4), pat);
                    CHK(hipMemsetAsync(cnt, 0, 16, nullptr));
                    hipLaunchKernelGGL(k_count, dim3(256), dim3(256), 0, nullptr, static_cast<const uint32_t*>(b),
                                       uint64_t(S / 4), pat, cnt, cnt + 1);
                    unsigned long long hc[2];
                    CHK(hipMemcpy(hc, cnt, 16, hipMemcpyDeviceToHost));
                    const size_t part = std::min<size_t>(S, 4ull << 20);
                    std::vector<uint32_t> h(part / 4);
                    long hb = 0;
                    for (int end = 0; end < 2; ++end) {
                        const size_t off = end ? S - part : 0;
                        CHK(hipMemcpy(h.data(), static_cast<char*>(b) + off, part, hipMemcpyDeviceToHost));
                        for (size_t i = 0; i < h.size(); ++i) hb += h[i] != (pat ^ uint32_t(off / 4 + i));
                    }
                    gpuBad += long(hc[0]);
                    gpuZero += long(hc[1]);
                    hostBad += hb;
                    runsBad += (hc[0] != 0 || hb != 0);
                    CHK(hipFree(b));
                }
                std::printf("{\"probe\": \"fresh_write\", \"uncached\": %d, \"bytes\": %zu, \"churn_1GiB_free\": %d, "
                            "\"iters\": %d, \"iters_with_wrong_words\": %ld, \"gpu_wrong\": %ld, \"gpu_zero\": %ld, "
                            "\"host_wrong_first_last_4MiB\": %ld}\n", unc, S, churn, iters, runsBad, gpuBad, gpuZero, hostBad);
                std::fflush(stdout);
            }
        }
    }
    CHK(hipFree(cnt));
    return 0;
}

int main(int argc, char** argv)
{
    if (argc > 1 && std::strcmp(argv[1], "fresh") == 0) return fresh(argc > 2 ? std::atoi(argv[2]) : 50);
    const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
    const size_t flagBytes = (32ull << 10) + (4ull << 20);
    const size_t stgBytes = 2ull << 20;
    int cus = 256;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* src = nullptr;
    uint32_t* counts = nullptr;
    CHK(hipMalloc(&src, stgBytes));
    CHK(hipMalloc(&counts, 3 * 256 * sizeof(uint32_t)));
    std::vector<uint32_t> host(stgBytes / 4), hc(3 * 256);
    // configurations: whether the uncached block is freed (else kept, so staging cannot land there), and whether the
    // L2s are scrubbed between the free and the cached allocation
    const char* names[3] = {"free", "free_scrub_before_free", "keep"};
    for (int cfg = 0; cfg < 3; ++cfg) {
        long landed = 0, gpuBad = 0, gpuBadNt = 0, hostBad = 0, hostZero = 0, hostP = 0, hostOther = 0, runsBad = 0;
        std::vector<void*> kept;
        for (int it = 0; it < iters; ++it) {
            const uint32_t P = 0x5A000000u | uint32_t(it);
            const uint32_t Q = 0x3C000000u | uint32_t(it * 7 + cfg);
            void* u = nullptr;
            CHK(hipExtMallocWithFlags(&u, flagBytes, hipDeviceMallocUncached));
            hipLaunchKernelGGL(k_scrub, dim3(cus), dim3(64), 0, nullptr);
            CHK(hipDeviceSynchronize());
            CHK(hipMemset(u, 0, flagBytes));
            hipLaunchKernelGGL(k_ll_push, dim3(256), dim3(256), 0, nullptr, static_cast<unsigned long long*>(u),
                               uint64_t(flagBytes / 8), P);
            CHK(hipDeviceSynchronize());
            if (cfg == 1) {
                hipLaunchKernelGGL(k_scrub, dim3(cus), dim3(64), 0, nullptr);
                CHK(hipDeviceSynchronize());
            }
            if (cfg == 2) {
                kept.push_back(u);
            } else {
                CHK(hipFree(u));
            }
            hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, nullptr, src, uint64_t(stgBytes / 4), Q);
            void* c = nullptr;
            CHK(hipMalloc(&c, stgBytes));
            const bool in = static_cast<char*>(c) >= static_cast<char*>(u) &&
                            static_cast<char*>(c) < static_cast<char*>(u) + flagBytes;
            landed += in;
            hipLaunchKernelGGL(k_copy_nt, dim3(256), dim3(256), 0, nullptr, static_cast<uint4*>(c),
                               reinterpret_cast<const uint4*>(src), uint64_t(stgBytes / 16));
            hipLaunchKernelGGL(k_read_all, dim3(256), dim3(256), 0, nullptr, static_cast<const uint32_t*>(c),
                               uint64_t(stgBytes / 4), Q, counts);
            CHK(hipDeviceSynchronize());
            CHK(hipMemcpy(hc.data(), counts, hc.size() * 4, hipMemcpyDeviceToHost));
            CHK(hipMemcpy(host.data(), c, stgBytes, hipMemcpyDeviceToHost));
            long b = 0;
            for (int k = 0; k < 256; ++k) {
                gpuBad += hc[3 * k];
                gpuBadNt += hc[3 * k + 1];
                b += hc[3 * k] + hc[3 * k + 1];
            }
            for (size_t i = 0; i < host.size(); ++i) {
                const uint32_t want = Q ^ uint32_t(i);
                if (host[i] == want) continue;
                ++hostBad;
                ++b;
                if (host[i] == 0) {
                    ++hostZero;
                } else if ((host[i] & 0xFF000000u) == 0x5A000000u) {
                    ++hostP;
                } else {
                    ++hostOther;
                }
            }
            runsBad += b != 0;
            CHK(hipFree(c));
        }
        for (void* u : kept) CHK(hipFree(u));
        std::printf("{\"probe\": \"uncached_reuse\", \"config\": \"%s\", \"iters\": %d, \"staging_in_freed_block\": %ld, "
                    "\"iters_with_wrong_words\": %ld, \"gpu_wrong_plain\": %ld, \"gpu_wrong_nt\": %ld, "
                    "\"host_wrong\": %ld, \"host_wrong_zero\": %ld, \"host_wrong_P\": %ld, \"host_wrong_other\": %ld}\n",
                    names[cfg], iters, landed, runsBad, gpuBad, gpuBadNt, hostBad, hostZero, hostP, hostOther);
        std::fflush(stdout);
    }
    CHK(hipFree(src));
    CHK(hipFree(counts));
    return 0;
}
