// memcpy_visibility_probe.hip — are the bytes of a device-to-device hipMemcpyAsync visible to the next kernel of the
// stream on every XCD, and in memory after hipDeviceSynchronize? (r04 root cause of the stale-operand failures,
// DESIGN.md §5b.) The loopback transport's link is exactly this sequence: the receiver's stream waits on the sender's
// event, copies the sender's bytes into fresh (never read) staging with hipMemcpyAsync, records an event the sender
// waits on, waits on the sender's event in turn, and launches the fold, whose workgroups are spread over all XCDs.
// Each rep copies into a region of a 512 MiB allocation nobody has touched yet (its bytes are zero), then a kernel of
// 256 workgroups reads the region from every XCD and counts wrong words, then a host copy counts wrong words in memory.
// The same with this library's kind of copy: a kernel with plain stores.
//   hipcc -O3 --offload-arch=gfx950 tools/memcpy_visibility_probe.hip -o tools/memcpy_visibility_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                          \
        }                                                                                          \
    } while (0)

__global__ void k_fill(uint32_t* b, uint32_t seed, uint64_t n)
{
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        b[i] = seed * 2654435761u + uint32_t(i) + 1u;  // never zero for these seeds
    }
}

__global__ void k_copy(uint32_t* d, const uint32_t* s, uint64_t n)
{
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        d[i] = s[i];
    }
}

// every workgroup reads the whole region: out[b] = words that differ from the source's pattern
__global__ void k_check(const uint32_t* b, uint32_t seed, uint64_t n, uint32_t* out)
{
    uint32_t bad = 0;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) bad += b[i] != seed * 2654435761u + uint32_t(i) + 1u;
    __shared__ uint32_t sb;
    if (threadIdx.x == 0) sb = 0;
    __syncthreads();
    atomicAdd(&sb, bad);
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = sb;
}

int main()
{
    CK(hipSetDevice(0));
    const uint64_t arena = 512ull << 20;
    uint32_t *scr = nullptr, *src = nullptr, *out = nullptr;
    CK(hipMalloc(&scr, arena));
    CK(hipMalloc(&src, 4u << 20));
    CK(hipMalloc(&out, 256 * 4));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    std::vector<uint32_t> host(1u << 20), hout(256);
    uint64_t off = 0;  // bytes of the arena used so far (every rep takes a fresh region)
    const int reps = 24;
    struct V {
        const char* name;
        uint64_t bytes;
        bool events;
        bool kernelCopy;
    };
    const V vs[] = {{"memcpy_16KiB_events", 16 << 10, true, false}, {"memcpy_16KiB_plain", 16 << 10, false, false},
                    {"memcpy_1MiB_events", 1 << 20, true, false},   {"memcpy_1MiB_plain", 1 << 20, false, false},
                    {"kernel_16KiB_events", 16 << 10, true, true},  {"kernel_1MiB_events", 1 << 20, true, true}};
    for (const V& v : vs) {
        int kernelBad = 0, memBad = 0;
        uint64_t kernelWords = 0, memWords = 0;
        for (int r = 0; r < reps; ++r) {
            const uint64_t n = v.bytes / 4;
            if (off + v.bytes + (64 << 10) > arena) off = 0;  // (not reached with these sizes)
            uint32_t* slot = scr + off / 4;
            off += (v.bytes + (64 << 10)) / (64 << 10) * (64 << 10);
            const uint32_t seed = 1000u + r;
            hipEvent_t ready, done, back;
            CK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&back, hipEventDisableTiming));
            hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, a, src, seed, n);
            CK(hipEventRecord(ready, a));
            CK(hipDeviceSynchronize());
            if (v.events) CK(hipStreamWaitEvent(b, ready, 0));
            if (v.kernelCopy) {
                hipLaunchKernelGGL(k_copy, dim3(64), dim3(256), 0, b, slot, src, n);
            } else {
                CK(hipMemcpyAsync(slot, src, v.bytes, hipMemcpyDeviceToDevice, b));
            }
            if (v.events) {
                CK(hipEventRecord(done, b));
                CK(hipStreamWaitEvent(a, done, 0));
                CK(hipEventRecord(back, a));
                CK(hipStreamWaitEvent(b, back, 0));
            }
            hipLaunchKernelGGL(k_check, dim3(256), dim3(256), 0, b, slot, seed, n, out);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hout.data(), out, 256 * 4, hipMemcpyDeviceToHost));
            uint64_t kb = 0;
            for (uint32_t x : hout) kb += x;
            CK(hipMemcpy(host.data(), slot, v.bytes, hipMemcpyDeviceToHost));
            uint64_t mb = 0;
            for (uint64_t i = 0; i < n; ++i) mb += host[i] != seed * 2654435761u + uint32_t(i) + 1u;
            kernelBad += kb != 0;
            memBad += mb != 0;
            kernelWords += kb;
            memWords += mb;
            CK(hipEventDestroy(ready));
            CK(hipEventDestroy(done));
            CK(hipEventDestroy(back));
        }
        std::printf("{\"variant\": \"%s\", \"reps\": %d, \"reps_kernel_saw_wrong\": %d, \"reps_memory_wrong\": %d, "
                    "\"kernel_wrong_words\": %llu, \"memory_wrong_words\": %llu}\n",
                    v.name, reps, kernelBad, memBad, (unsigned long long)kernelWords, (unsigned long long)memWords);
        std::fflush(stdout);
    }
    return 0;
}
