/*
 * A plain C caller of libhccl_amd.so on the GPU: the shape of the reference sample
 * (examples/02_collectives/01_allreduce/main.cc:51-136) with the device runtime calls swapped for HIP
 * (INTEGRATION.md §1). Run by tests/test_gpu_c_sample.py; built by __graft_entry__.build().
 *   1. HcclGetRootInfo + HcclCommInitRootInfo (one rank: RCCL), HcclAllReduce in place: the input comes back.
 *   2. HcclAmdCommInitLoopback(4) driven by 4 pthreads, one per rank: HcclAllReduce, HcclReduceScatter and
 *      HcclReduce of integer-valued fp32 (exact in any order), checked element by element.
 *   3. HcclAmdLocalReduce (the inner primitive): dst = src + dst.
 * Prints "C SAMPLE OK" and returns 0, or names the first failure and returns 1.
 */
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hccl.h"
#include "hccl_amd.h"

#define RANKS 4
#define COUNT 100003

#define CHECK(cond, ...)                      \
    do {                                      \
        if (!(cond)) {                        \
            fprintf(stderr, __VA_ARGS__);     \
            fprintf(stderr, "\n");            \
            exit(1);                          \
        }                                     \
    } while (0)

typedef struct {
    HcclComm comm;
    int rank;
    float* send;  /* COUNT * RANKS elements (ReduceScatter input) */
    float* recv;  /* COUNT * RANKS elements */
    HcclResult rc[3];
} RankArgs;

static void* rank_main(void* p)
{
    RankArgs* a = (RankArgs*)p;
    hipStream_t s;
    (void)hipSetDevice(0);
    (void)hipStreamCreate(&s);
    a->rc[0] = HcclAllReduce(a->send, a->recv, COUNT, HCCL_DATA_TYPE_FP32, HCCL_REDUCE_SUM, a->comm, (aclrtStream)s);
    (void)hipStreamSynchronize(s);
    a->rc[1] = HcclReduceScatter(a->send, a->recv + (size_t)COUNT * RANKS / 2, COUNT / 2, HCCL_DATA_TYPE_FP32,
                                 HCCL_REDUCE_SUM, a->comm, (aclrtStream)s);
    (void)hipStreamSynchronize(s);
    a->rc[2] = HcclReduce(a->send, a->recv + (size_t)COUNT * 3, COUNT, HCCL_DATA_TYPE_FP32, HCCL_REDUCE_MAX, 1,
                          a->comm, (aclrtStream)s);
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    return NULL;
}

int main(void)
{
    CHECK(hipSetDevice(0) == hipSuccess, "hipSetDevice failed");
    const size_t n = (size_t)COUNT * RANKS;
    float* host = (float*)malloc(n * sizeof(float));
    float* back = (float*)malloc(n * sizeof(float));
    CHECK(host != NULL && back != NULL, "host allocation failed");

    /* 1. one-rank communicator over RCCL, as the reference sample builds it */
    HcclRootInfo root;
    CHECK(HcclGetRootInfo(&root) == HCCL_SUCCESS, "HcclGetRootInfo failed");
    HcclComm comm;
    CHECK(HcclCommInitRootInfo(1, &root, 0, &comm) == HCCL_SUCCESS, "HcclCommInitRootInfo failed");
    uint32_t size = 0, id = 9;
    CHECK(HcclGetRankSize(comm, &size) == HCCL_SUCCESS && size == 1, "HcclGetRankSize");
    CHECK(HcclGetRankId(comm, &id) == HCCL_SUCCESS && id == 0, "HcclGetRankId");
    float* buf = NULL;
    CHECK(hipMalloc((void**)&buf, COUNT * sizeof(float)) == hipSuccess, "hipMalloc failed");
    for (size_t i = 0; i < COUNT; ++i) host[i] = (float)(i % 1000);
    CHECK(hipMemcpy(buf, host, COUNT * sizeof(float), hipMemcpyHostToDevice) == hipSuccess, "H2D failed");
    hipStream_t s;
    CHECK(hipStreamCreate(&s) == hipSuccess, "hipStreamCreate failed");
    CHECK(HcclAllReduce(buf, buf, COUNT, HCCL_DATA_TYPE_FP32, HCCL_REDUCE_SUM, comm, (aclrtStream)s) == HCCL_SUCCESS,
          "one-rank HcclAllReduce failed");
    CHECK(hipStreamSynchronize(s) == hipSuccess, "sync failed");
    CHECK(hipMemcpy(back, buf, COUNT * sizeof(float), hipMemcpyDeviceToHost) == hipSuccess, "D2H failed");
    CHECK(memcmp(back, host, COUNT * sizeof(float)) == 0, "one-rank AllReduce changed its input");
    /* reference error codes from C: a null stream is HCCL_E_PTR */
    CHECK(HcclAllReduce(buf, buf, COUNT, HCCL_DATA_TYPE_FP32, HCCL_REDUCE_SUM, comm, NULL) == HCCL_E_PTR,
          "null stream not refused");
    CHECK(HcclCommDestroy(comm) == HCCL_SUCCESS, "HcclCommDestroy failed");

    /* 2. four ranks in this process, one pthread each */
    HcclComm comms[RANKS];
    CHECK(HcclAmdCommInitLoopback(RANKS, comms) == HCCL_SUCCESS, "HcclAmdCommInitLoopback failed");
    RankArgs args[RANKS];
    pthread_t th[RANKS];
    for (int r = 0; r < RANKS; ++r) {
        args[r].comm = comms[r];
        args[r].rank = r;
        CHECK(hipMalloc((void**)&args[r].send, n * sizeof(float)) == hipSuccess, "hipMalloc send");
        CHECK(hipMalloc((void**)&args[r].recv, n * sizeof(float)) == hipSuccess, "hipMalloc recv");
        for (size_t i = 0; i < n; ++i) host[i] = (float)((i % 4096) + (size_t)r);
        CHECK(hipMemcpy(args[r].send, host, n * sizeof(float), hipMemcpyHostToDevice) == hipSuccess, "H2D");
        CHECK(hipMemset(args[r].recv, 0, n * sizeof(float)) == hipSuccess, "memset");
    }
    for (int r = 0; r < RANKS; ++r) CHECK(pthread_create(&th[r], NULL, rank_main, &args[r]) == 0, "pthread_create");
    for (int r = 0; r < RANKS; ++r) pthread_join(th[r], NULL);
    CHECK(hipDeviceSynchronize() == hipSuccess, "device sync failed");
    for (int r = 0; r < RANKS; ++r) {
        CHECK(args[r].rc[0] == HCCL_SUCCESS && args[r].rc[1] == HCCL_SUCCESS && args[r].rc[2] == HCCL_SUCCESS,
              "rank %d: codes %d %d %d", r, args[r].rc[0], args[r].rc[1], args[r].rc[2]);
        CHECK(hipMemcpy(back, args[r].recv, n * sizeof(float), hipMemcpyDeviceToHost) == hipSuccess, "D2H");
        for (size_t i = 0; i < COUNT; ++i) {  /* AllReduce: sum over ranks of (i % 4096) + q */
            const float want = (float)(RANKS * (i % 4096) + RANKS * (RANKS - 1) / 2);
            CHECK(back[i] == want, "rank %d AllReduce elem %zu: %f vs %f", r, i, back[i], want);
        }
        for (size_t i = 0; i < COUNT / 2; ++i) {  /* ReduceScatter: block r of every input */
            const size_t g = (size_t)r * (COUNT / 2) + i;
            const float want = (float)(RANKS * (g % 4096) + RANKS * (RANKS - 1) / 2);
            const float got = back[(size_t)COUNT * RANKS / 2 + i];
            CHECK(got == want, "rank %d ReduceScatter elem %zu: %f vs %f", r, i, got, want);
        }
        for (size_t i = 0; i < COUNT; ++i) {  /* Reduce MAX at root 1; other ranks' buffers untouched */
            const float want = r == 1 ? (float)((i % 4096) + RANKS - 1) : 0.0f;
            const float got = back[(size_t)COUNT * 3 + i];
            CHECK(got == want, "rank %d Reduce elem %zu: %f vs %f", r, i, got, want);
        }
    }
    for (int r = 0; r < RANKS; ++r) {
        CHECK(HcclCommDestroy(comms[r]) == HCCL_SUCCESS, "destroy");
        (void)hipFree(args[r].send);
        (void)hipFree(args[r].recv);
    }

    /* 3. the inner primitive */
    float* src = NULL;
    CHECK(hipMalloc((void**)&src, COUNT * sizeof(float)) == hipSuccess, "hipMalloc src");
    for (size_t i = 0; i < COUNT; ++i) host[i] = (float)(i % 77);
    CHECK(hipMemcpy(src, host, COUNT * sizeof(float), hipMemcpyHostToDevice) == hipSuccess, "H2D");
    CHECK(hipMemcpy(buf, host, COUNT * sizeof(float), hipMemcpyHostToDevice) == hipSuccess, "H2D");
    CHECK(HcclAmdLocalReduce(buf, src, COUNT, HCCL_DATA_TYPE_FP32, HCCL_REDUCE_SUM, (aclrtStream)s) == HCCL_SUCCESS,
          "HcclAmdLocalReduce failed");
    CHECK(hipStreamSynchronize(s) == hipSuccess, "sync");
    CHECK(hipMemcpy(back, buf, COUNT * sizeof(float), hipMemcpyDeviceToHost) == hipSuccess, "D2H");
    for (size_t i = 0; i < COUNT; ++i) CHECK(back[i] == 2.0f * (float)(i % 77), "local reduce elem %zu", i);
    (void)hipFree(src);
    (void)hipFree(buf);
    (void)hipStreamDestroy(s);
    free(host);
    free(back);
    printf("C SAMPLE OK\n");
    return 0;
}
