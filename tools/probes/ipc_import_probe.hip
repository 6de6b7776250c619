// ipc_import_probe.hip — is a store made through a hipIpcOpenMemHandle mapping of another process's UNCACHED allocation
// (same device) visible to the owner's loads without an L2 write-back? (imported mappings; VERDICT r04
// next #1.)
//
// The one-sided kernel's light barrier fences (IpcArgs::fence = 1) rely on every handed-over byte being in uncached
// staging: the storing waves' vmcnt(0) drain is then the release. In rank mode the stores reach the peer's staging
// through an imported mapping, whose memory type the importer's driver chooses. If that mapping is cached, a store
// sits dirty in the importer's XCD L2 after its drain, and only a system-scope release (buffer_wbl2) pushes it to
// memory: a light-fence barrier would then hand over stale bytes, a wrong result with no timeout.
//
// Two processes (forked before any HIP call). The owner allocates [flags 4 KiB][data] uncached and exports it. Per
// iteration e the importer's one workgroup stores the pattern f(e, i) into the data through its imported mapping (plain
// or non-temporal stores), drains (s_waitcnt vmcnt(0)), optionally runs a system-scope release, then stores e into
// flag 0 with a system-scope store, and stays resident polling flag 1 (so no end-of-kernel write-back happens). The
// owner's 256 workgroups (spread over every XCD) wait for flag 0 >= e, read the data with plain loads, count words
// that differ from f(e, i), and the last of them stores e into flag 1. Every wait is bounded (2 s).
//
// Output: one JSON line per (store kind, fence) with the stale words summed over the iterations.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/probes/ipc_import_probe tools/probes/ipc_import_probe.hip
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#define CHK(x)                                                                                   \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            _exit(2);                                                                            \
        }                                                                                        \
    } while (0)

constexpr uint64_t kFlagWords = 1024;       // 4 KiB of flags ahead of the data
constexpr uint64_t kTimeoutTicks = 200000000;  // 2 s of s_memrealtime (100 MHz)

__device__ __forceinline__ uint32_t Pattern(uint32_t e, uint64_t i) { return e * 2654435761u + uint32_t(i) * 40503u + 1u; }

__device__ __forceinline__ bool WaitFlag(uint32_t* f, uint32_t e)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) return false;
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}

// importer: one workgroup of 256 threads
__global__ void k_importer(uint32_t* base, uint64_t words, uint32_t e, int nt, int release, uint32_t* timeouts)
{
    uint32_t* data = base + kFlagWords;
    for (uint64_t i = threadIdx.x; i < words; i += blockDim.x) {
        if (nt) {
            __builtin_nontemporal_store(Pattern(e, i), data + i);
        } else {
            data[i] = Pattern(e, i);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: buffer_wbl2 sc0 sc1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(base + 0, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (!WaitFlag(base + 1, e)) atomicAdd(timeouts, 1u);  // resident until the owner has read
    }
}

// owner: every workgroup reads the whole data after flag 0
__global__ void k_owner(uint32_t* base, uint64_t words, uint32_t e, uint32_t* stale, uint32_t* arrived,
                        uint32_t* timeouts)
{
    __shared__ uint32_t ok;
    uint32_t* data = base + kFlagWords;
    if (threadIdx.x == 0) {
        ok = WaitFlag(base + 0, e) ? 1u : 0u;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    uint32_t bad = 0;
    if (ok) {
        for (uint64_t i = threadIdx.x; i < words; i += blockDim.x) bad += data[i] != Pattern(e, i);
    }
    atomicAdd(stale, bad);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!ok) atomicAdd(timeouts, 1u);
        if (atomicAdd(arrived, 1u) + 1 == gridDim.x) {
            *arrived = 0;
            __hip_atomic_store(base + 1, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

struct Sizes {
    uint64_t words;
    int iters;
};

int Owner(int wr, int rd, const Sizes* sz, int nsz)
{
    CHK(hipSetDevice(0));
    uint64_t maxWords = 0;
    for (int k = 0; k < nsz; ++k) maxWords = sz[k].words > maxWords ? sz[k].words : maxWords;
    uint32_t* buf = nullptr;
    CHK(hipExtMallocWithFlags(reinterpret_cast<void**>(&buf), (kFlagWords + maxWords) * 4, hipDeviceMallocUncached));
    CHK(hipMemset(buf, 0, (kFlagWords + maxWords) * 4));
    uint32_t* cnt = nullptr;  // stale, arrived, timeouts
    CHK(hipMalloc(reinterpret_cast<void**>(&cnt), 64));
    CHK(hipMemset(cnt, 0, 64));
    CHK(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    CHK(hipIpcGetMemHandle(&h, buf));
    if (write(wr, &h, sizeof h) != sizeof h) return 2;
    uint32_t e = 0;
    for (int k = 0; k < nsz; ++k) {
        for (int mode = 0; mode < 4; ++mode) {  // bit 0: nt stores, bit 1: system release
            uint64_t staleTotal = 0, staleIters = 0, timeouts = 0;
            for (int it = 0; it < sz[k].iters; ++it) {
                ++e;
                CHK(hipMemset(cnt, 0, 64));
                hipLaunchKernelGGL(k_owner, dim3(256), dim3(256), 0, nullptr, buf, sz[k].words, e, cnt, cnt + 1, cnt + 2);
                CHK(hipDeviceSynchronize());
                uint32_t h3[3];
                CHK(hipMemcpy(h3, cnt, sizeof h3, hipMemcpyDeviceToHost));
                staleTotal += h3[0];
                staleIters += h3[0] != 0;
                timeouts += h3[2];
            }
            char c = 0;
            if (read(rd, &c, 1) != 1) return 2;  // the importer's counts for this mode follow in its own line
            std::printf("{\"side\": \"owner\", \"words\": %llu, \"stores\": \"%s\", \"fence\": \"%s\", \"iters\": %d, "
                        "\"stale_words\": %llu, \"stale_iters\": %llu, \"owner_timeouts\": %llu}\n",
                        (unsigned long long)sz[k].words, (mode & 1) ? "nt" : "plain",
                        (mode & 2) ? "system_release" : "drain_only", sz[k].iters, (unsigned long long)staleTotal,
                        (unsigned long long)staleIters, (unsigned long long)timeouts);
            std::fflush(stdout);
        }
    }
    CHK(hipFree(buf));
    return 0;
}

int Importer(int rd, int wr, const Sizes* sz, int nsz)
{
    hipIpcMemHandle_t h;
    if (read(rd, &h, sizeof h) != sizeof h) return 2;
    CHK(hipSetDevice(0));
    uint32_t* p = nullptr;
    CHK(hipIpcOpenMemHandle(reinterpret_cast<void**>(&p), h, hipIpcMemLazyEnablePeerAccess));
    uint32_t* to = nullptr;
    CHK(hipMalloc(reinterpret_cast<void**>(&to), 4));
    uint32_t e = 0;
    for (int k = 0; k < nsz; ++k) {
        for (int mode = 0; mode < 4; ++mode) {
            CHK(hipMemset(to, 0, 4));
            for (int it = 0; it < sz[k].iters; ++it) {
                ++e;
                hipLaunchKernelGGL(k_importer, dim3(1), dim3(256), 0, nullptr, p, sz[k].words, e, mode & 1,
                                   (mode >> 1) & 1, to);
                CHK(hipDeviceSynchronize());
            }
            uint32_t t = 0;
            CHK(hipMemcpy(&t, to, 4, hipMemcpyDeviceToHost));
            if (t != 0) std::fprintf(stderr, "importer: %u timeouts in mode %d\n", t, mode);
            const char c = 1;
            if (write(wr, &c, 1) != 1) return 2;
        }
    }
    CHK(hipIpcCloseMemHandle(p));
    return 0;
}

int main()
{
    const Sizes sz[] = {{16384, 200}, {1 << 20, 50}};  // 64 KiB (fits one XCD's L2 easily) and 4 MiB
    const int nsz = 2;
    int a2b[2], b2a[2];
    if (pipe(a2b) != 0 || pipe(b2a) != 0) return 2;
    const pid_t pid = fork();  // before any HIP call in either process
    if (pid == 0) {
        close(a2b[1]);
        close(b2a[0]);
        _exit(Importer(a2b[0], b2a[1], sz, nsz));
    }
    close(a2b[0]);
    close(b2a[1]);
    const int rc = Owner(a2b[1], b2a[0], sz, nsz);
    int st = 0;
    waitpid(pid, &st, 0);
    return rc != 0 ? rc : (WIFEXITED(st) ? WEXITSTATUS(st) : 3);
}
