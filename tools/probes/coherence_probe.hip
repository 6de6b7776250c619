// coherence_probe.hip — which writes leave another XCD's L2 holding an old copy of a line (r04 diagnosis of the
// stale-operand failures, VERDICT r03 "What's weak" #1).
//
// Every scenario: fill B (256 KiB) with P0 from all XCDs, PRIME every XCD's L2 with it (every block reads all of B),
// write P1 by one method, then CHECK from all XCDs (every block reads all of B, counts words != P1 and words == P0,
// per XCC id). A control runs a system-scope L2 write-back + invalidate on every CU before the check.
// The "ipc_like" scenarios replay the test's order without a prime: H2D zeros -> kernel stores -> D2H -> H2D -> read.
//   hipcc -O3 --offload-arch=gfx950 tools/coherence_probe.hip -o tools/coherence_probe && tools/coherence_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                              \
        }                                                                              \
    } while (0)

constexpr uint32_t kWords = 64 * 1024;  // 256 KiB
constexpr uint32_t kBlocks = 256;        // 32 per XCD
constexpr uint32_t kThreads = 256;

__device__ __forceinline__ uint32_t XccId()
{
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 15u;
}

__global__ void k_fill(uint32_t* b, uint32_t v, uint32_t n)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) b[i] = v;
}

__global__ void k_fill_nt(uint32_t* b, uint32_t v, uint32_t n)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        __builtin_nontemporal_store(v, b + i);
    }
}

// every block reads all of b (plain loads): each XCD's L2 ends up holding every line
__global__ void k_prime(const uint32_t* b, uint32_t n, uint32_t* sink)
{
    uint32_t s = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) s += b[i];
    if (s == 0x9e3779b9u) sink[blockIdx.x] = s;  // keeps the loads
}

// the same with non-temporal loads (the executor's folds and the one-sided kernel load this way)
__global__ void k_prime_nt(const uint32_t* b, uint32_t n, uint32_t* sink)
{
    uint32_t s = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) s += __builtin_nontemporal_load(b + i);
    if (s == 0x9e3779b9u) sink[blockIdx.x] = s;
}

template <bool NT>
__global__ void k_check_t(const uint32_t* b, uint32_t n, uint32_t expect, uint32_t old, uint32_t* out)
{
    uint32_t bad = 0, stale = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t x = NT ? __builtin_nontemporal_load(b + i) : b[i];
        bad += x != expect;
        stale += x == old;
    }
    __shared__ uint32_t sb, ss;
    if (threadIdx.x == 0) sb = ss = 0;
    __syncthreads();
    atomicAdd(&sb, bad);
    atomicAdd(&ss, stale);
    __syncthreads();
    if (threadIdx.x == 0) {
        out[blockIdx.x * 3 + 0] = sb;
        out[blockIdx.x * 3 + 1] = ss;
        out[blockIdx.x * 3 + 2] = XccId();
    }
}

// every block reads all of b: words != expect, words == old, per block; the block's XCC id
__global__ void k_check(const uint32_t* b, uint32_t n, uint32_t expect, uint32_t old, uint32_t* out)
{
    uint32_t bad = 0, stale = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t x = b[i];
        bad += x != expect;
        stale += x == old;
    }
    __shared__ uint32_t sb, ss;
    if (threadIdx.x == 0) sb = ss = 0;
    __syncthreads();
    atomicAdd(&sb, bad);
    atomicAdd(&ss, stale);
    __syncthreads();
    if (threadIdx.x == 0) {
        out[blockIdx.x * 3 + 0] = sb;
        out[blockIdx.x * 3 + 1] = ss;
        out[blockIdx.x * 3 + 2] = XccId();
    }
}

// system-scope write-back + invalidate of the L2 of every CU's XCD (the library's k_l2_maintain)
__global__ void k_l2_sys()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

struct Ctx {
    uint32_t* b;
    uint32_t* src;
    uint32_t* sink;
    uint32_t* out;
    uint32_t* hostPinned;
    uint32_t* hostPage;
    hipStream_t s1, s2;
};

void Report(const char* name, int rep, Ctx& c, hipStream_t s, uint32_t expect, uint32_t old, bool ntCheck = false,
            const uint32_t* buf = nullptr)
{
    if (buf == nullptr) buf = c.b;
    if (ntCheck) {
        hipLaunchKernelGGL((k_check_t<true>), dim3(kBlocks), dim3(kThreads), 0, s, buf, kWords, expect, old, c.out);
    } else {
        hipLaunchKernelGGL((k_check_t<false>), dim3(kBlocks), dim3(kThreads), 0, s, buf, kWords, expect, old, c.out);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> h(kBlocks * 3);
    CK(hipMemcpy(h.data(), c.out, h.size() * 4, hipMemcpyDeviceToHost));
    uint64_t bad = 0, stale = 0, blocksBad = 0;
    uint64_t byXcc[16] = {0};
    for (uint32_t k = 0; k < kBlocks; ++k) {
        bad += h[k * 3];
        stale += h[k * 3 + 1];
        blocksBad += h[k * 3] != 0;
        byXcc[h[k * 3 + 2] & 15] += h[k * 3];
    }
    std::printf("{\"scenario\": \"%s\", \"rep\": %d, \"bad_words\": %llu, \"old_words\": %llu, \"blocks_bad\": %llu, "
                "\"blocks\": %u, \"bad_by_xcc\": [",
                name, rep, (unsigned long long)bad, (unsigned long long)stale, (unsigned long long)blocksBad, kBlocks);
    for (int x = 0; x < 8; ++x) std::printf("%s%llu", x ? ", " : "", (unsigned long long)byXcc[x]);
    std::printf("]}\n");
    std::fflush(stdout);
}

void FillHost(uint32_t* h, uint32_t v)
{
    for (uint32_t i = 0; i < kWords; ++i) h[i] = v;
}

// fill P0 everywhere, prime every L2, then the writer
void Prime(Ctx& c, uint32_t p0, bool ntPrime = false)
{
    hipLaunchKernelGGL(k_fill, dim3(kBlocks), dim3(kThreads), 0, c.s1, c.b, p0, kWords);
    if (ntPrime) {
        hipLaunchKernelGGL(k_prime_nt, dim3(kBlocks), dim3(kThreads), 0, c.s1, c.b, kWords, c.sink);
    } else {
        hipLaunchKernelGGL(k_prime, dim3(kBlocks), dim3(kThreads), 0, c.s1, c.b, kWords, c.sink);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
}

int main(int argc, char** argv)
{
    CK(hipSetDevice(0));
    Ctx c{};
    CK(hipMalloc(&c.b, kWords * 4));
    CK(hipMalloc(&c.src, kWords * 4));
    CK(hipMalloc(&c.sink, kBlocks * 4));
    CK(hipMalloc(&c.out, kBlocks * 3 * 4));
    CK(hipHostMalloc(&c.hostPinned, kWords * 4, hipHostMallocDefault));
    c.hostPage = static_cast<uint32_t*>(std::malloc(kWords * 4));
    CK(hipStreamCreateWithFlags(&c.s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&c.s2, hipStreamNonBlocking));

    for (int rep = 0; rep < 3; ++rep) {
        const uint32_t p0 = 0x11110000u + rep, p1 = 0x22220000u + rep, p2 = 0x33330000u + rep;
        struct W {
            const char* name;
            int kind;
        };
        const W ws[] = {{"none_control", 0},       {"kernel_plain_1block", 1}, {"kernel_nt_1block", 2},
                        {"kernel_plain_all", 3},   {"kernel_nt_all", 4},       {"memset_s1", 5},
                        {"d2d_memcpy_s1", 6},      {"h2d_pinned_s1", 7},       {"h2d_pageable_s1", 8},
                        {"d2d_memcpy_s2_sync", 9}, {"h2d_pageable_null_sync", 10}, {"h2d_pageable_null_sync_l2sys", 11},
                        {"d2h_then_h2d_pageable_null", 12}};
        for (int pol = 0; pol < 3; ++pol)  // 0: plain prime, plain check; 1: nt prime, nt check; 2: plain prime, nt check
        for (const W& w : ws) {
            const bool ntPrime = pol == 1, ntCheck = pol >= 1;
            Prime(c, p0, ntPrime);
            uint32_t expect = p1;
            switch (w.kind) {
                case 0: expect = p0; break;
                case 1: hipLaunchKernelGGL(k_fill, dim3(1), dim3(kThreads), 0, c.s1, c.b, p1, kWords); break;
                case 2: hipLaunchKernelGGL(k_fill_nt, dim3(1), dim3(kThreads), 0, c.s1, c.b, p1, kWords); break;
                case 3: hipLaunchKernelGGL(k_fill, dim3(kBlocks), dim3(kThreads), 0, c.s1, c.b, p1, kWords); break;
                case 4: hipLaunchKernelGGL(k_fill_nt, dim3(kBlocks), dim3(kThreads), 0, c.s1, c.b, p1, kWords); break;
                case 5: CK(hipMemsetD32Async(c.b, p1, kWords, c.s1)); break;
                case 6:
                    hipLaunchKernelGGL(k_fill, dim3(kBlocks), dim3(kThreads), 0, c.s1, c.src, p1, kWords);
                    CK(hipMemcpyAsync(c.b, c.src, kWords * 4, hipMemcpyDeviceToDevice, c.s1));
                    break;
                case 7:
                    FillHost(c.hostPinned, p1);
                    CK(hipMemcpyAsync(c.b, c.hostPinned, kWords * 4, hipMemcpyHostToDevice, c.s1));
                    break;
                case 8:
                    FillHost(c.hostPage, p1);
                    CK(hipMemcpyAsync(c.b, c.hostPage, kWords * 4, hipMemcpyHostToDevice, c.s1));
                    break;
                case 9:
                    hipLaunchKernelGGL(k_fill, dim3(kBlocks), dim3(kThreads), 0, c.s2, c.src, p1, kWords);
                    CK(hipMemcpyAsync(c.b, c.src, kWords * 4, hipMemcpyDeviceToDevice, c.s2));
                    CK(hipDeviceSynchronize());
                    break;
                case 10:
                case 11:
                    FillHost(c.hostPage, p1);
                    CK(hipMemcpy(c.b, c.hostPage, kWords * 4, hipMemcpyHostToDevice));
                    CK(hipDeviceSynchronize());
                    if (w.kind == 11) {
                        hipLaunchKernelGGL(k_l2_sys, dim3(256), dim3(64), 0, c.s1);
                    }
                    break;
                case 12:
                    CK(hipMemcpy(c.hostPage, c.b, kWords * 4, hipMemcpyDeviceToHost));
                    FillHost(c.hostPage, p1);
                    CK(hipMemcpy(c.b, c.hostPage, kWords * 4, hipMemcpyHostToDevice));
                    CK(hipDeviceSynchronize());
                    break;
            }
            CK(hipGetLastError());
            std::string name = std::string(w.name) + (pol == 0 ? "" : pol == 1 ? "/nt_prime_nt_check" : "/nt_check");
            Report(name.c_str(), rep, c, c.s1, expect, p0, ntCheck);
        }

        // Freed and reallocated: lines of a freed buffer primed in every L2, a new allocation (likely the same pages)
        // filled by a D2D copy, then read (plain and nt).
        for (int ntc = 0; ntc < 2; ++ntc) {
            uint32_t* a = nullptr;
            CK(hipMalloc(&a, kWords * 4));
            hipLaunchKernelGGL(k_fill, dim3(kBlocks), dim3(kThreads), 0, c.s1, a, p0, kWords);
            hipLaunchKernelGGL(k_prime_nt, dim3(kBlocks), dim3(kThreads), 0, c.s1, a, kWords, c.sink);
            hipLaunchKernelGGL(k_prime, dim3(kBlocks), dim3(kThreads), 0, c.s1, a, kWords, c.sink);
            CK(hipDeviceSynchronize());
            CK(hipFree(a));
            uint32_t* b2 = nullptr;
            CK(hipMalloc(&b2, kWords * 4));
            hipLaunchKernelGGL(k_fill, dim3(kBlocks), dim3(kThreads), 0, c.s1, c.src, p1, kWords);
            CK(hipMemcpyAsync(b2, c.src, kWords * 4, hipMemcpyDeviceToDevice, c.s2));
            CK(hipDeviceSynchronize());
            std::string name = std::string("realloc_d2d") + (ntc ? "/nt_check" : "") + (a == b2 ? "/same_va" : "/new_va");
            Report(name.c_str(), rep, c, c.s1, p1, p0, ntc != 0, b2);
            CK(hipFree(b2));
        }

        // The test's order without a prime: H2D zeros (null stream), the collective's stores from every XCD (plain or
        // nt) on s1, D2H of the result, H2D of new inputs (null stream), then a reader on s2.
        for (int nt = 0; nt < 2; ++nt) {
            std::memset(c.hostPage, 0, kWords * 4);
            CK(hipMemcpy(c.b, c.hostPage, kWords * 4, hipMemcpyHostToDevice));
            CK(hipDeviceSynchronize());
            if (nt) {
                hipLaunchKernelGGL(k_fill_nt, dim3(kBlocks), dim3(kThreads), 0, c.s1, c.b, p1, kWords);
            } else {
                hipLaunchKernelGGL(k_fill, dim3(kBlocks), dim3(kThreads), 0, c.s1, c.b, p1, kWords);
            }
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(c.hostPage, c.b, kWords * 4, hipMemcpyDeviceToHost));
            uint32_t wrong = 0;
            for (uint32_t i = 0; i < kWords; ++i) wrong += c.hostPage[i] != p1;
            FillHost(c.hostPage, p2);
            CK(hipMemcpy(c.b, c.hostPage, kWords * 4, hipMemcpyHostToDevice));
            CK(hipDeviceSynchronize());
            std::string name = std::string(nt ? "ipc_like_nt" : "ipc_like_plain") + "_d2h_wrong_" + std::to_string(wrong);
            Report(name.c_str(), rep, c, c.s2, p2, 0u, nt != 0);
        }
    }
    std::printf("{\"done\": true}\n");
    return 0;
}
