// Host-code sanitizer run (ASan + UBSan): the schedule builder (hccl_amd/csrc/schedule.cc) and the oracle's replay
// (oracle/hccl_oracle.c) over every collective x family x rank count x ragged counts, at the default and a 1 MiB
// HCCL_BUFFSIZE (many executor loops). Buffers are malloc'd at exactly their declared sizes (input, output, scratch),
// so an IR offset outside them is an ASan report. Values are checked too: int64 inputs i * 2^20 + 2^r make each SUM
// exact, so every output element must hold every rank once at its own offset (AllGather: rank q's block q).
// Built and run by tests/test_sanitize.py; test infrastructure only.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../hccl_amd/csrc/schedule.h"

extern "C" int orc_replay(uint32_t nRanks, int dtype, int op, const HcclAmdIrOp* const* progs, const uint64_t* nops,
                          void* const* bufs);

namespace {

constexpr int kInt64 = 5;
constexpr int kSum = 0;

int RunCase(int opType, int algo, uint32_t n, uint64_t count, uint64_t cclBytes, uint32_t root,
            uint64_t pieceBytes = 4096)
{
    std::vector<hccl_amd::Schedule> sch(n);
    for (uint32_t r = 0; r < n; ++r) {
        hccl_amd::ScheduleParams p;
        p.opType = opType;
        p.algo = algo;
        p.nRanks = n;
        p.rank = r;
        p.count = count;
        p.elemSize = 8;
        p.root = root;
        p.cclBytes = cclBytes;
        p.pieceBytes = pieceBytes;
        if (hccl_amd::BuildSchedule(p, &sch[r]) != 0) return -1;  // combination not offered (e.g. RHD at n = 3)
    }
    const uint64_t inCount = opType == HCCL_AMD_OP_REDUCE_SCATTER ? count * n : count;
    const uint64_t outCount = opType == HCCL_AMD_OP_ALLGATHER ? count * n : count;
    std::vector<int64_t*> mem;
    std::vector<void*> bufs(3 * n);
    std::vector<const HcclAmdIrOp*> progs(n);
    std::vector<uint64_t> nops(n);
    for (uint32_t r = 0; r < n; ++r) {
        int64_t* in = static_cast<int64_t*>(malloc(inCount * 8));
        int64_t* out = static_cast<int64_t*>(calloc(outCount, 8));
        int64_t* scr = static_cast<int64_t*>(calloc(sch[r].scratchElems ? sch[r].scratchElems : 1, 8));
        for (uint64_t i = 0; i < inCount; ++i) in[i] = static_cast<int64_t>(i) * (int64_t(1) << 20) + (int64_t(1) << r);
        bufs[3 * r] = in;
        bufs[3 * r + 1] = out;
        bufs[3 * r + 2] = scr;
        mem.push_back(in);
        mem.push_back(out);
        mem.push_back(scr);
        progs[r] = sch[r].ops.data();
        nops[r] = sch[r].ops.size();
    }
    int bad = orc_replay(n, kInt64, kSum, progs.data(), nops.data(), bufs.data()) != 0;
    const int64_t full = (int64_t(1) << n) - 1;
    for (uint32_t r = 0; r < n && !bad; ++r) {
        const int64_t* out = static_cast<const int64_t*>(bufs[3 * r + 1]);
        for (uint64_t i = 0; i < outCount && !bad; ++i) {
            int64_t want;
            if (opType == HCCL_AMD_OP_ALLGATHER) {
                const uint64_t q = i / count, j = i % count;
                want = static_cast<int64_t>(j) * (int64_t(1) << 20) + (int64_t(1) << q);
            } else if (opType == HCCL_AMD_OP_REDUCE && r != root) {
                want = 0;
            } else {
                const uint64_t g = opType == HCCL_AMD_OP_REDUCE_SCATTER ? r * count + i : i;
                want = int64_t(n) * static_cast<int64_t>(g) * (int64_t(1) << 20) + full;
            }
            bad = out[i] != want;
            if (bad) {
                std::printf("MISMATCH op %d algo %d n %u count %llu rank %u elem %llu: %lld vs %lld\n", opType,
                            algo, n, (unsigned long long)count, r, (unsigned long long)i, (long long)out[i],
                            (long long)want);
            }
        }
    }
    for (int64_t* m : mem) free(m);
    return bad;
}

}  // namespace

int main()
{
    const int ops[] = {HCCL_AMD_OP_ALLREDUCE, HCCL_AMD_OP_REDUCE_SCATTER, HCCL_AMD_OP_REDUCE, HCCL_AMD_OP_ALLGATHER};
    const uint32_t ns[] = {2, 3, 4, 5, 8};
    const uint64_t counts[] = {1, 7, 1000, 65537};
    const uint64_t ccls[] = {200ull << 20, 1ull << 20};
    int cases = 0, failures = 0;
    for (int op : ops) {
        for (int algo = 0; algo <= 9; ++algo) {
            for (uint32_t n : ns) {
                for (uint64_t count : counts) {
                    for (uint64_t ccl : ccls) {
                        const int rc = RunCase(op, algo, n, count, ccl, n / 2);
                        if (rc < 0) continue;
                        ++cases;
                        failures += rc;
                    }
                }
            }
        }
    }
    // The ring and RHD spread over more rings / instances as calls grow (RhdInstances, Rings): calls large enough for
    // two and for all of them, ragged, with 1 MiB pieces.
    struct Big {
        int op, algo;
        uint32_t n;
        uint64_t count;
    };
    const Big bigs[] = {
        {HCCL_AMD_OP_ALLREDUCE, HCCL_AMD_ALGO_RHD, 8, (2ull << 20) / 8 + 3},          // 2 instances
        {HCCL_AMD_OP_ALLREDUCE, HCCL_AMD_ALGO_RHD, 8, (49ull << 19) / 8 + 5},         // 7 instances (24.5 MiB)
        {HCCL_AMD_OP_ALLREDUCE, HCCL_AMD_ALGO_RHD, 4, (16ull << 20) / 8 + 1},         // 3 instances at n = 4
        {HCCL_AMD_OP_ALLREDUCE, HCCL_AMD_ALGO_RING, 8, (8ull << 20) / 8 + 7},         // 2 rings
        {HCCL_AMD_OP_ALLREDUCE, HCCL_AMD_ALGO_RING, 8, (58ull << 20) / 8 + 1},        // 7 rings
        {HCCL_AMD_OP_REDUCE_SCATTER, HCCL_AMD_ALGO_RING, 8, (58ull << 20) / 64 + 3},  // 7 rings (input bytes)
        {HCCL_AMD_OP_ALLGATHER, HCCL_AMD_ALGO_RING, 8, (58ull << 20) / 64 + 1},       // 7 rings (output bytes)
        {HCCL_AMD_OP_ALLREDUCE, HCCL_AMD_ALGO_RING, 5, (40ull << 20) / 8 + 3},        // 4 rings at n = 5
    };
    for (const Big& b : bigs) {
        const int rc = RunCase(b.op, b.algo, b.n, b.count, 200ull << 20, b.n / 2, 1ull << 20);
        if (rc < 0) {
            std::printf("NOT BUILT op %d algo %d n %u\n", b.op, b.algo, b.n);
            ++failures;
            continue;
        }
        ++cases;
        failures += rc;
    }
    std::printf("cases %d failures %d\n", cases, failures);
    return failures == 0 && cases > 0 ? 0 : 1;
}
