// Does the size of a kernel's arguments change the device time of back-to-back launches? (r05)
// The one-sided kernel takes its whole IpcArgs (about 1.7 KB: every rank's pointers, the RHD tables) by value. This
// probe launches a one-workgroup kernel that does one store (or first spins 10 us, so the device sets the pace),
// 20,000 times back to back on one stream, with 16 B, 1 KiB and 2 KiB of arguments, and prints the per-launch time
// (HIP events) as JSON lines.
//   hipcc --offload-arch=gfx950 -O2 -o tools/probes/kernarg_cost_probe tools/probes/kernarg_cost_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int B>
struct Args {
    unsigned long long w[B / 8];
};

template <int B>
__global__ void k_args(int* out, Args<B> a)
{
    // spin a.w[0] ticks of the 100 MHz clock (0: none), so that with a spin the device, not the host, sets the pace
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < a.w[0]) {
    }
    if (threadIdx.x == 0) out[0] = static_cast<int>(a.w[B / 8 - 1]);
}

template <int B>
static double PerLaunchUs(hipStream_t s, int* out, int iters, unsigned long long spin)
{
    Args<B> a{};
    a.w[0] = spin;
    a.w[B / 8 - 1] = 7;
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL((k_args<B>), dim3(1), dim3(64), 0, s, out, a);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipStreamSynchronize(s);
    (void)hipEventRecord(e0, s);
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((k_args<B>), dim3(1), dim3(64), 0, s, out, a);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return double(ms) * 1e3 / iters;
}

int main()
{
    hipStream_t s;
    int* out = nullptr;
    if (hipStreamCreate(&s) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    const int iters = 20000;
    for (unsigned long long spin : {0ull, 1000ull}) {  // no spin (the host's pace), 10 us (the device's)
        std::printf("{\"arg_bytes\": 16, \"spin_us\": %llu, \"us_per_launch\": %.3f}\n", spin / 100,
                    PerLaunchUs<16>(s, out, iters, spin));
        std::printf("{\"arg_bytes\": 1024, \"spin_us\": %llu, \"us_per_launch\": %.3f}\n", spin / 100,
                    PerLaunchUs<1024>(s, out, iters, spin));
        std::printf("{\"arg_bytes\": 2048, \"spin_us\": %llu, \"us_per_launch\": %.3f}\n", spin / 100,
                    PerLaunchUs<2048>(s, out, iters, spin));
    }
    (void)hipFree(out);
    (void)hipStreamDestroy(s);
    return 0;
}
