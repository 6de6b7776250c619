// schedule.h — per-rank schedule IR generators for the reducing collectives.
//
// A schedule is the list of HcclAmdIrOp records one rank executes (include/hccl_amd.h). It plays the role of the
// reference's algorithm templates (src/ops/*/template/aicpu/*.cc): which slices are sent to
// which peer, and which slices are folded in which order. Everything here is host-only integer logic; the same
// records are executed by the HIP/RCCL executor (executor.cc) and replayed by the CPU oracle.
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/hccl_amd.h"

namespace hccl_amd {

struct ScheduleParams {
    int32_t opType = HCCL_AMD_OP_ALLREDUCE;
    int32_t algo = HCCL_AMD_ALGO_AUTO;
    uint32_t nRanks = 1;
    uint32_t rank = 0;
    uint64_t count = 0;  // AllReduce/Reduce: elements per rank; ReduceScatter: recvCount
    uint32_t elemSize = 4;
    uint32_t root = 0;
    uint64_t pieceBytes = 0;        // 0 = default
    uint64_t scratchCapBytes = 0;   // 0 = unbounded
    uint64_t cclBytes = 200ull << 20;  // HCCL_BUFFSIZE: sizes the reference's executor loops (see RefLoopElems)
    bool special = false;  // INT64 / UINT64 / FP64 data or PROD: the selectors' isDataTypeOrReduceTypeSpecial
    // ReduceScatterV (HCCL_AMD_OP_REDUCE_SCATTER_V): rank q's block of every input is [displs[q], displs[q] +
    // counts[q]) (elements); nRanks entries each. count is then counts[rank].
    std::vector<uint64_t> counts;
    std::vector<uint64_t> displs;
};

struct Schedule {
    std::vector<HcclAmdIrOp> ops;
    int32_t algo = -1;
    uint64_t scratchElems = 0;
};

// Reference selector policy for a single-node full mesh (Level0Shape::MESH_1D, one net layer), bytes = count x size:
//   AllReduce   special: <= 8 MiB one-shot, else two-shot; otherwise <= 8 MiB one-shot,
//               bytes * 8/n^2 > 32 MiB MeshChunk, else two-shot            all_reduce_auto_selector.cc:517-550
//   ReduceScatter (bytes of recvCount)  special: mesh; bytes * (8/n)^2 > 16 MiB MeshChunk, else mesh
//                                                                            reduce_scatter_auto_selector.cc:473-512
//   Reduce      <  8 MiB one-shot mesh, else two-shot                      reduce_auto_selector.cc:312-324
int32_t SelectAlgo(int32_t opType, uint32_t nRanks, uint64_t bytes, bool special);

// The directed rings the ring schedules run for n ranks: arc-disjoint Hamiltonian cycles (rank lists).
std::vector<std::vector<uint32_t>> RingTable(uint32_t n);

// The RHD instances for a power-of-two n (empty otherwise): per instance, the real rank of every virtual rank.
std::vector<std::vector<uint32_t>> RhdTable(uint32_t n);

// How many RHD instances (parts of the buffer) an AllReduce of `bytes` per rank runs (AllReduceRhd).
uint32_t RhdInstances(uint32_t n, uint64_t bytes);

// Returns HCCL_E_PARA for an invalid combination, HCCL_SUCCESS otherwise.
int BuildSchedule(const ScheduleParams& p, Schedule* out);

}  // namespace hccl_amd
