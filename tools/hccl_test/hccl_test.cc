// hccl_test.cc — the HCCL performance test tool's workflow (docs/en/build/build.md:184-204: `mpirun -n 8
// ./bin/all_reduce_test -b 8K -e 64M -f 2 -d fp32 -o sum -p 8`, printing data_size / aveg_time / alg_bandwidth /
// check_result per size) over libhccl_amd.so, as one native binary. The operator is the program name
// (all_reduce_test, reduce_scatter_test, reduce_test, all_gather_test) or --op. There is no MPI here: the tool starts
// its own ranks.
//   -t rccl      (default) -p processes, forked before any HIP call, one per device (rank r on device r); rank 0's
//                HcclGetRootInfo blob reaches the others through shared memory, every rank calls HcclCommInitRootInfo
//   -t ipc       -p processes over the IPC-only communicator (HcclAmdCommInitHostExchange, the all-gather through
//                shared memory); several may share one device
//   -t loopback  -p threads of one process over HcclAmdCommInitLoopback (one device)
// Sizes (-b, -e, -f) are the largest buffer of a rank: the AllReduce / Reduce buffer, the ReduceScatter input and the
// AllGather output. Inputs are small integers, exact in every order and dtype, so check_result compares every element
// with the exact result. aveg_time is the max over ranks of the mean per call (-n timed after -w warm-up calls);
// alg_bandwidth = data_size / aveg_time, and bus_bandwidth applies the nccl-tests factor of the operator.
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "hccl.h"
#include "hccl_amd.h"

#define HIP_TRY(x)                                                                   \
    do {                                                                             \
        const hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));     \
            return 1;                                                                \
        }                                                                            \
    } while (0)

namespace {

enum Op { kAllReduce, kReduceScatter, kReduce, kAllGather };

struct Options {
    Op op = kAllReduce;
    uint64_t minBytes = 8 << 10, maxBytes = 64 << 20;
    double factor = 2;
    HcclDataType dt = HCCL_DATA_TYPE_FP32;
    HcclReduceOp red = HCCL_REDUCE_SUM;
    int ranks = 1;
    uint32_t root = 0;
    int iters = 20, warmup = 5;
    bool check = true;
    std::string transport = "rccl";
    int algo = -1;  // HcclAmdCommSetAlgo, -1 = leave the default selection
};

constexpr int kMaxRanks = 16;
constexpr size_t kSlot = 64 << 10;  // host-exchange payload per rank

// Shared between the forked ranks (MAP_SHARED | MAP_ANONYMOUS, created before fork).
struct Shared {
    std::atomic<uint32_t> arrived;
    std::atomic<uint32_t> generation;
    HcclRootInfo root;
    int failed[kMaxRanks];
    char slot[kMaxRanks][kSlot];
};

// Cross-process barrier over the shared page. A rank that died never arrives: the others give up after a bound
// instead of spinning forever, and the parent reports the failure.
void Barrier(Shared* s, int n)
{
    const uint32_t gen = s->generation.load();
    if (s->arrived.fetch_add(1) + 1 == uint32_t(n)) {
        s->arrived.store(0);
        s->generation.fetch_add(1);
        return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    while (s->generation.load() == gen) {
        std::this_thread::yield();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600)) {
            std::fprintf(stderr, "hccl_test: a rank did not reach the barrier within 600 s\n");
            _exit(3);
        }
    }
}

uint64_t ParseBytes(const char* s)
{
    char* end = nullptr;
    double v = std::strtod(s, &end);
    switch (end && *end ? (*end | 0x20) : 0) {
        case 'k': v *= 1024; break;
        case 'm': v *= 1024 * 1024; break;
        case 'g': v *= 1024.0 * 1024 * 1024; break;
        default: break;
    }
    return static_cast<uint64_t>(v);
}

bool ParseDtype(const std::string& s, HcclDataType* dt)
{
    static const struct {
        const char* name;
        HcclDataType dt;
    } kTypes[] = {{"int8", HCCL_DATA_TYPE_INT8},   {"int16", HCCL_DATA_TYPE_INT16}, {"int32", HCCL_DATA_TYPE_INT32},
                  {"int64", HCCL_DATA_TYPE_INT64}, {"uint64", HCCL_DATA_TYPE_UINT64}, {"fp16", HCCL_DATA_TYPE_FP16},
                  {"bf16", HCCL_DATA_TYPE_BFP16},  {"fp32", HCCL_DATA_TYPE_FP32}, {"fp64", HCCL_DATA_TYPE_FP64}};
    for (const auto& t : kTypes) {
        if (s == t.name) {
            *dt = t.dt;
            return true;
        }
    }
    return false;
}

// ------------------------------------------------------------------------------------------------ data

// Rank r's input at element i: small integers whose sum / product / max / min is exact in every dtype and order.
double Input(HcclReduceOp red, int r, uint64_t i)
{
    if (red == HCCL_REDUCE_PROD) return ((i + uint64_t(r)) % 4 == 0) ? 2.0 : 1.0;  // at most ceil(n/4) twos
    return double((i * 7 + uint64_t(r) * 3) % 5);
}

double Combine(HcclReduceOp red, double a, double b)
{
    switch (red) {
        case HCCL_REDUCE_PROD: return a * b;
        case HCCL_REDUCE_MAX: return std::max(a, b);
        case HCCL_REDUCE_MIN: return std::min(a, b);
        default: return a + b;
    }
}

uint16_t HalfBits(double v)  // exact for the small integers used here
{
    if (v == 0) return 0;
    int e = 0;
    const double m = std::frexp(v, &e);  // v = m * 2^e, m in [0.5, 1)
    const uint32_t mant = static_cast<uint32_t>((m * 2 - 1) * 1024.0 + 0.5);
    return static_cast<uint16_t>(((e - 1 + 15) << 10) | mant);
}

uint16_t Bf16Bits(double v)
{
    const float f = static_cast<float>(v);
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return static_cast<uint16_t>(u >> 16);
}

void Store(HcclDataType dt, void* base, uint64_t i, double v)
{
    switch (dt) {
        case HCCL_DATA_TYPE_INT8: static_cast<int8_t*>(base)[i] = static_cast<int8_t>(v); break;
        case HCCL_DATA_TYPE_INT16: static_cast<int16_t*>(base)[i] = static_cast<int16_t>(v); break;
        case HCCL_DATA_TYPE_INT32: static_cast<int32_t*>(base)[i] = static_cast<int32_t>(v); break;
        case HCCL_DATA_TYPE_INT64: static_cast<int64_t*>(base)[i] = static_cast<int64_t>(v); break;
        case HCCL_DATA_TYPE_UINT64: static_cast<uint64_t*>(base)[i] = static_cast<uint64_t>(v); break;
        case HCCL_DATA_TYPE_FP16: static_cast<uint16_t*>(base)[i] = HalfBits(v); break;
        case HCCL_DATA_TYPE_BFP16: static_cast<uint16_t*>(base)[i] = Bf16Bits(v); break;
        case HCCL_DATA_TYPE_FP64: static_cast<double*>(base)[i] = v; break;
        default: static_cast<float*>(base)[i] = static_cast<float>(v); break;
    }
}

// ------------------------------------------------------------------------------------------------ one rank

struct RankCtx {
    const Options* o;
    int rank;
    HcclComm comm;
    std::vector<double>* usOut;  // per size
    std::vector<int>* badOut;    // per size: mismatching elements
    Shared* shared;              // forked modes: the barrier before each timed loop
};

bool Verbose() { return std::getenv("HCCL_TEST_VERBOSE") != nullptr; }

int RunRank(RankCtx& c, const std::vector<uint64_t>& sizes)
{
    const Options& o = *c.o;
    const int n = o.ranks;
    const uint64_t es = HcclAmdDataTypeSize(o.dt);
    hipStream_t stream;
    if (hipStreamCreate(&stream) != hipSuccess) return 1;
    if (o.algo >= 0 && HcclAmdCommSetAlgo(c.comm, o.algo) != HCCL_SUCCESS) return 1;
    const uint64_t maxBytes = sizes.back();
    void *send = nullptr, *recv = nullptr;
    if (hipMalloc(&send, maxBytes) != hipSuccess || hipMalloc(&recv, maxBytes) != hipSuccess) return 1;
    std::vector<char> host(maxBytes), want(maxBytes);
    for (size_t k = 0; k < sizes.size(); ++k) {
        const uint64_t bytes = sizes[k];
        const uint64_t elems = bytes / es;
        const uint64_t count = (o.op == kReduceScatter || o.op == kAllGather) ? elems / n : elems;
        const uint64_t inElems = o.op == kAllGather ? count : o.op == kReduceScatter ? count * n : elems;
        const uint64_t outElems = o.op == kReduceScatter ? count : o.op == kAllGather ? count * n : elems;
        for (uint64_t i = 0; i < inElems; ++i) Store(o.dt, host.data(), i, Input(o.red, c.rank, i));
        HIP_TRY(hipMemcpy(send, host.data(), inElems * es, hipMemcpyHostToDevice));
        HIP_TRY(hipMemset(recv, 0, outElems * es));
        auto call = [&]() -> HcclResult {
            switch (o.op) {
                case kReduceScatter: return HcclReduceScatter(send, recv, count, o.dt, o.red, c.comm, stream);
                case kReduce: return HcclReduce(send, recv, count, o.dt, o.red, o.root, c.comm, stream);
                case kAllGather: return HcclAllGather(send, recv, count, o.dt, c.comm, stream);
                default: return HcclAllReduce(send, recv, count, o.dt, o.red, c.comm, stream);
            }
        };
        if (count == 0) {
            (*c.usOut)[k] = 0;
            (*c.badOut)[k] = 0;
            continue;
        }
        // check first (one call), then warm-up and timing
        HcclResult rc = call();
        HIP_TRY(hipStreamSynchronize(stream));
        int bad = rc == HCCL_SUCCESS ? 0 : -1;
        if (rc == HCCL_SUCCESS && o.check && !(o.op == kReduce && uint32_t(c.rank) != o.root)) {
            HIP_TRY(hipMemcpy(host.data(), recv, outElems * es, hipMemcpyDeviceToHost));
            for (uint64_t i = 0; i < outElems; ++i) {
                double v;
                if (o.op == kAllGather) {
                    v = Input(o.red, int(i / count), i % count);
                } else {
                    const uint64_t g = o.op == kReduceScatter ? uint64_t(c.rank) * count + i : i;
                    v = Input(o.red, 0, g);
                    for (int r = 1; r < n; ++r) v = Combine(o.red, v, Input(o.red, r, g));
                }
                Store(o.dt, want.data(), 0, v);
                if (std::memcmp(want.data(), host.data() + i * es, es) != 0) ++bad;
            }
        }
        for (int w = 0; w < o.warmup && rc == HCCL_SUCCESS; ++w) rc = call();
        HIP_TRY(hipStreamSynchronize(stream));
        if (c.shared != nullptr) Barrier(c.shared, n);
        hipEvent_t e0, e1;
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        HIP_TRY(hipEventRecord(e0, stream));
        for (int it = 0; it < o.iters && rc == HCCL_SUCCESS; ++it) rc = call();
        HIP_TRY(hipEventRecord(e1, stream));
        HIP_TRY(hipEventSynchronize(e1));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        HIP_TRY(hipEventDestroy(e0));
        HIP_TRY(hipEventDestroy(e1));
        (*c.usOut)[k] = rc == HCCL_SUCCESS ? ms * 1e3 / std::max(1, o.iters) : -1;
        (*c.badOut)[k] = rc == HCCL_SUCCESS ? bad : -1;
    }
    HIP_TRY(hipFree(send));
    HIP_TRY(hipFree(recv));
    HIP_TRY(hipStreamDestroy(stream));
    return 0;
}

// ------------------------------------------------------------------------------------------------ report

double BusFactor(Op op, int n)
{
    if (op == kAllReduce) return 2.0 * (n - 1) / n;
    if (op == kReduce) return 1.0;
    return double(n - 1) / n;
}

int Report(const Options& o, const std::vector<uint64_t>& sizes, const std::vector<std::vector<double>>& us,
           const std::vector<std::vector<int>>& bad)
{
    std::printf("the minbytes is %llu, maxbytes is %llu, iters is %d, warmup_iters is %d, ranks is %d, transport is "
                "%s\n",
                (unsigned long long)o.minBytes, (unsigned long long)o.maxBytes, o.iters, o.warmup, o.ranks,
                o.transport.c_str());
    std::printf("%18s %16s %22s %22s %16s\n", "data_size(Bytes):", "aveg_time(us):", "alg_bandwidth(GB/s):",
                "bus_bandwidth(GB/s):", "check_result:");
    int rc = 0;
    for (size_t k = 0; k < sizes.size(); ++k) {
        double t = 0;
        int b = 0;
        bool failed = false;
        for (int r = 0; r < o.ranks; ++r) {
            if (us[r][k] < 0 || bad[r][k] < 0) failed = true;
            t = std::max(t, us[r][k]);
            b += std::max(0, bad[r][k]);
        }
        const double alg = t > 0 ? double(sizes[k]) / (t * 1e-6) / 1e9 : 0;
        const char* res = failed ? "error" : (!o.check ? "skipped" : (b == 0 ? "success" : "failed"));
        if (failed || (o.check && b != 0)) rc = 1;
        std::printf("%18llu %16.2f %22.4f %22.4f %16s\n", (unsigned long long)sizes[k], t, alg,
                    alg * BusFactor(o.op, o.ranks), res);
    }
    return rc;
}

void Usage(const char* prog)
{
    std::fprintf(stderr,
                 "usage: %s [-b minbytes] [-e maxbytes] [-f factor] [-d int8|int16|int32|int64|uint64|fp16|bf16|fp32|"
                 "fp64] [-o sum|prod|max|min] [-p ranks] [-r root] [-n iters] [-w warmup] [-c 0|1] "
                 "[-t rccl|ipc|loopback] [-a algo] [--op all_reduce|reduce_scatter|reduce|all_gather]\n",
                 prog);
}

}  // namespace

int main(int argc, char** argv)
{
    Options o;
    std::string base = argv[0];
    base = base.substr(base.find_last_of('/') + 1);
    if (base.rfind("reduce_scatter", 0) == 0) o.op = kReduceScatter;
    if (base.rfind("reduce_test", 0) == 0) o.op = kReduce;
    if (base.rfind("all_gather", 0) == 0) o.op = kAllGather;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        const char* v = i + 1 < argc ? argv[i + 1] : nullptr;
        if (v == nullptr) {
            Usage(argv[0]);
            return 2;
        }
        ++i;
        if (a == "-b") o.minBytes = ParseBytes(v);
        else if (a == "-e") o.maxBytes = ParseBytes(v);
        else if (a == "-f") o.factor = std::atof(v);
        else if (a == "-d") {
            if (!ParseDtype(v, &o.dt)) { Usage(argv[0]); return 2; }
        } else if (a == "-o") {
            const std::string s = v;
            o.red = s == "prod" ? HCCL_REDUCE_PROD : s == "max" ? HCCL_REDUCE_MAX : s == "min" ? HCCL_REDUCE_MIN
                                                                                                 : HCCL_REDUCE_SUM;
        } else if (a == "-p") o.ranks = std::atoi(v);
        else if (a == "-r") o.root = static_cast<uint32_t>(std::atoi(v));
        else if (a == "-n") o.iters = std::atoi(v);
        else if (a == "-w") o.warmup = std::atoi(v);
        else if (a == "-c") o.check = std::atoi(v) != 0;
        else if (a == "-t") o.transport = v;
        else if (a == "-a") o.algo = std::atoi(v);
        else if (a == "--op") {
            const std::string s = v;
            o.op = s == "reduce_scatter" ? kReduceScatter : s == "reduce" ? kReduce : s == "all_gather" ? kAllGather
                                                                                                      : kAllReduce;
        } else {
            Usage(argv[0]);
            return 2;
        }
    }
    if (o.ranks < 1 || o.ranks > kMaxRanks || o.minBytes == 0 || o.maxBytes < o.minBytes || o.factor <= 1 ||
        o.root >= uint32_t(o.ranks)) {
        Usage(argv[0]);
        return 2;
    }
    std::vector<uint64_t> sizes;
    for (double b = double(o.minBytes); b <= double(o.maxBytes) * 1.0000001; b *= o.factor) {
        sizes.push_back(static_cast<uint64_t>(b));
    }
    const int n = o.ranks;
    std::vector<std::vector<double>> us(n, std::vector<double>(sizes.size(), -1));
    std::vector<std::vector<int>> bad(n, std::vector<int>(sizes.size(), -1));

    if (o.transport == "loopback") {
        std::vector<HcclComm> comms(n);
        if (HcclAmdCommInitLoopback(uint32_t(n), comms.data()) != HCCL_SUCCESS) {
            std::fprintf(stderr, "HcclAmdCommInitLoopback failed\n");
            return 1;
        }
        std::vector<std::thread> th;
        std::vector<RankCtx> ctx(n);
        for (int r = 0; r < n; ++r) {
            ctx[r] = RankCtx{&o, r, comms[r], &us[r], &bad[r], nullptr};
            th.emplace_back([&, r] {
                (void)hipSetDevice(0);
                RunRank(ctx[r], sizes);
            });
        }
        for (auto& t : th) t.join();
        for (int r = 0; r < n; ++r) HcclCommDestroy(comms[r]);
        return Report(o, sizes, us, bad);
    }
    if (o.transport != "rccl" && o.transport != "ipc") {
        Usage(argv[0]);
        return 2;
    }
    // forked ranks: no HIP call in the parent before the fork
    void* mem = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (mem == MAP_FAILED) return 1;
    Shared* sh = new (mem) Shared();
    const size_t perRankDoubles = sizes.size();
    std::vector<double*> usShared(n);
    std::vector<int*> badShared(n);
    void* res = mmap(nullptr, size_t(n) * perRankDoubles * (sizeof(double) + sizeof(int)), PROT_READ | PROT_WRITE,
                     MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (res == MAP_FAILED) return 1;
    for (int r = 0; r < n; ++r) {
        usShared[r] = static_cast<double*>(res) + size_t(r) * perRankDoubles;
        badShared[r] = reinterpret_cast<int*>(static_cast<double*>(res) + size_t(n) * perRankDoubles) +
                       size_t(r) * perRankDoubles;
        std::fill(usShared[r], usShared[r] + perRankDoubles, -1.0);  // a rank that never reports shows as "error"
        std::fill(badShared[r], badShared[r] + perRankDoubles, -1);
    }
    std::vector<pid_t> pids;
    for (int r = 0; r < n; ++r) {
        const pid_t pid = fork();
        if (pid < 0) return 1;
        if (pid == 0) {
            int devices = 1;
            (void)hipGetDeviceCount(&devices);
            if (o.transport == "rccl" && devices < n) {
                // RCCL takes one rank per device; every rank sees the same count and stops before any RCCL call
                if (r == 0) std::fprintf(stderr, "-t rccl needs a device per rank (%d ranks, %d devices)\n", n, devices);
                _exit(2);
            }
            (void)hipSetDevice(o.transport == "rccl" ? r : 0);
            HcclComm comm = nullptr;
            HcclResult rc;
            // the IPC communicator calls the all-gather again at its first collective (the IPC set-up), so its
            // context lives as long as the rank
            struct Ctx {
                Shared* s;
                int rank, n;
            } agCtx{sh, r, n};
            if (o.transport == "rccl") {
                if (r == 0) {
                    sh->failed[0] = HcclGetRootInfo(&sh->root) != HCCL_SUCCESS;
                }
                Barrier(sh, n);
                rc = sh->failed[0] ? HCCL_E_INTERNAL : HcclCommInitRootInfo(uint32_t(n), &sh->root, uint32_t(r), &comm);
            } else {
                auto ag = [](void* p, const void* mine, uint64_t bytes, void* all) -> int32_t {
                    Ctx* x = static_cast<Ctx*>(p);
                    if (bytes > kSlot) return 1;
                    std::memcpy(x->s->slot[x->rank], mine, bytes);
                    Barrier(x->s, x->n);
                    for (int q = 0; q < x->n; ++q) std::memcpy(static_cast<char*>(all) + q * bytes, x->s->slot[q], bytes);
                    Barrier(x->s, x->n);
                    return 0;
                };
                rc = HcclAmdCommInitHostExchange(uint32_t(n), uint32_t(r), ag, &agCtx, &comm);
                if (rc == HCCL_SUCCESS && o.algo < 0) rc = HcclAmdCommSetAlgo(comm, HCCL_AMD_ALGO_IPC);
            }
            if (rc != HCCL_SUCCESS) {
                std::fprintf(stderr, "rank %d: communicator init failed: %s\n", r, HcclAmdGetErrorString(rc));
                _exit(1);
            }
            if (Verbose()) std::fprintf(stderr, "rank %d: communicator ready\n", r);
            std::vector<double> u(sizes.size(), -1);
            std::vector<int> b(sizes.size(), -1);
            RankCtx c{&o, r, comm, &u, &b, sh};
            const int ret = RunRank(c, sizes);
            if (Verbose()) std::fprintf(stderr, "rank %d: RunRank returned %d\n", r, ret);
            std::copy(u.begin(), u.end(), usShared[r]);
            std::copy(b.begin(), b.end(), badShared[r]);
            Barrier(sh, n);  // no rank unmaps its peers' memory while they may still use it
            HcclCommDestroy(comm);
            _exit(ret);
        }
        pids.push_back(pid);
    }
    int worst = 0;
    for (pid_t p : pids) {
        int st = 0;
        waitpid(p, &st, 0);
        if (WIFSIGNALED(st)) std::fprintf(stderr, "a rank died of signal %d\n", WTERMSIG(st));
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) worst = 1;
    }
    for (int r = 0; r < n; ++r) {
        us[r].assign(usShared[r], usShared[r] + perRankDoubles);
        bad[r].assign(badShared[r], badShared[r] + perRankDoubles);
    }
    const int rc = Report(o, sizes, us, bad);
    return worst != 0 ? 1 : rc;
}
