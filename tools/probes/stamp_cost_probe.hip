// stamp_cost_probe.hip — what a completion stamp costs per call on one stream (r03, watchdog design).
// A call is one small kernel (stand-in for a fold); per variant, N calls are enqueued back to back and the wall time
// per call (enqueue + GPU, one sync at the end) and the host enqueue time per call are printed as JSON lines:
//   none       the kernel alone
//   event      + hipEventRecord
//   write1     + hipStreamWriteValue64 into pinned host memory
//   write2     + two of them (start and done)
//   kernel1    + a one-wave kernel that stores the stamp (vector store)
//   fused      the kernel itself stores the stamp from its last block (atomic arrival count)
// Build: hipcc -O2 --offload-arch=gfx950 tools/stamp_cost_probe.hip -o tools/stamp_cost_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

__global__ void k_work(float* x, int n, uint64_t* stamp, unsigned* arrivals, uint64_t v, uint64_t spinTicks)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = x[i] * 0.5f + 1.0f;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spinTicks) __builtin_amdgcn_s_sleep(2);
    if (stamp == nullptr) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const unsigned a = __hip_atomic_fetch_add(arrivals, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (a == gridDim.x - 1) {
            __hip_atomic_store(arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(stamp, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ void k_stamp(uint64_t* stamp, uint64_t v)
{
    if (threadIdx.x == 0) __hip_atomic_store(stamp, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main()
{
    const int n = 256 * 16, iters = 2000;
    float* x = nullptr;
    CHK(hipMalloc(&x, n * sizeof(float)));
    CHK(hipMemset(x, 0, n * sizeof(float)));
    unsigned* arrivals = nullptr;
    CHK(hipMalloc(&arrivals, 64));
    CHK(hipMemset(arrivals, 0, 64));
    uint64_t* host = nullptr;
    CHK(hipHostMalloc(reinterpret_cast<void**>(&host), 64, hipHostMallocCoherent | hipHostMallocMapped));
    uint64_t* dev = nullptr;
    CHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), host, 0));
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const char* names[] = {"none", "event", "write1", "write2", "kernel1", "fused"};
    // rep 1: host-bound (tiny kernel); rep 2: GPU-bound (each kernel spins 20 us), where a stamp's GPU-side cost shows
    for (int rep = 0; rep < 3; ++rep) {
        const uint64_t spin = rep == 2 ? 2000 : 0;  // 100 MHz ticks
        for (int v = 0; v < 6; ++v) {
            CHK(hipStreamSynchronize(s));
            const auto t0 = std::chrono::steady_clock::now();
            for (int k = 0; k < iters; ++k) {
                if (v == 3) CHK(hipStreamWriteValue64(s, dev, k, 0));
                hipLaunchKernelGGL(k_work, dim3(n / 256), dim3(256), 0, s, x, n, v == 5 ? dev + 1 : nullptr, arrivals,
                                   uint64_t(k), spin);
                if (v == 1) CHK(hipEventRecord(ev, s));
                if (v == 2 || v == 3) CHK(hipStreamWriteValue64(s, dev + 1, k, 0));
                if (v == 4) hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, s, dev + 1, uint64_t(k));
            }
            const auto t1 = std::chrono::steady_clock::now();
            CHK(hipStreamSynchronize(s));
            const auto t2 = std::chrono::steady_clock::now();
            if (rep >= 1) {
                std::printf("{\"regime\": \"%s\", \"variant\": \"%s\", \"us_per_call\": %.2f, "
                            "\"enqueue_us_per_call\": %.2f, \"last_stamp\": %llu}\n",
                            rep == 1 ? "host-bound" : "gpu-bound (20 us kernel)", names[v], std::chrono::duration<double, std::micro>(t2 - t0).count() / iters,
                            std::chrono::duration<double, std::micro>(t1 - t0).count() / iters,
                            (unsigned long long)host[1]);
            }
        }
    }
    return 0;
}
