// ipc.h — one-sided AllReduce / ReduceScatter / Reduce / AllGather over peer-mapped staging (host state + launch).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/hccl_types.h"

namespace hccl_amd {

constexpr int kIpcMaxRanks = 16;
// Staging areas of a rank, parts of one allocation (one IPC handle): slots, results, and the two alternate slot areas
// of the single-barrier kinds.
constexpr int kIpcAreas = 4;
constexpr int kIpcAreaIn = 0;
constexpr int kIpcAreaRes = 1;
constexpr int kIpcAreaAlt0 = 2;
constexpr int kIpcAreaAlt1 = 3;
constexpr int kIpcBlock = 256;        // threads per workgroup of the one-sided kernel (default)
constexpr int kIpcMaxThreads = 512;   // HCCL_AMD_IPC_THREADS may take 512 (r03 A/B)

enum IpcKind : uint32_t {
    kIpcAllReduce = 0,         // two-shot: owner c folds chunk c, every rank gets every chunk
    kIpcReduceScatter = 1,     // owner c folds block c into its recvBuf
    kIpcReduce = 2,            // two-shot Reduce: owner c folds chunk c, only the root gets the result
    kIpcAllReduceOneShot = 3,  // every rank receives every peer's whole piece and folds all of it (no phase 2)
    kIpcReduceOneShot = 4,     // the peers push their whole piece to the root, which folds it
    kIpcAllGather = 5,         // every rank pushes its whole piece to every peer; each copies the n pieces out
};

// Operand order of a fold of chunk t.
enum IpcOrder : uint32_t {
    kIpcO2 = 0,  // x_0, x_1, .., x_{n-1}                          two-shot AllReduce; AIV one-shot, small-core
                 //                                                 two-shot, big-data ReduceScatter
    kIpcO1 = 1,  // x_t, then ascending q != t                      one-shot, mesh ReduceScatter, Reduce; AIV
                 //                                                 large-core two-shot
    kIpcO6 = 2,  // sub-slice j: x_t, then x_{t+o}, o = j+1..n-1, 1..j   MeshChunk AllReduce / ReduceScatter
    kIpcO4 = 3,  // pow-2 tree over the source ranks (rank-independent): M = largest power of two below n,
                 // x_j = x_{j+M} (op) x_j for j + M < n, then pairwise halving  AIV local-tree ReduceScatter
                 // (aiv_reduce_scatter_local_tree.h:138-172) = the STRICT order-preserved tree
    kIpcRhd = 4,  // one-shot kind only: the RHD AllReduce's bits (schedule.cc AllReduceRhd), per element the O4 tree
                  // over virtual ranks v ^ q of its RHD instance, v = the owner of its chunk (RhdFold)
};

// Chunk layout of one launch (input coordinates, elements; rank c owns chunk c).
enum IpcGeom : uint32_t {
    kIpcGeomAlignedCeil = 0,  // ceil(cnt / n) rounded up to 128 B (two-shot AllReduce, CalcSliceInfo)
    kIpcGeomCeil = 1,         // ceil(cnt / n), no alignment (MeshChunk CalcSliceInfoVec; AIV small-core two-shot)
    kIpcGeomBalanced = 2,     // g * n balanced slices (the first cnt % (g*n) one longer), chunk c = slices
                              // [c*g, (c+1)*g): Reduce two-shot (g = 1, reduce_mesh_1D_two_shot.cc:108-131) and
                              // the AIV large-core two-shot (g = groupSize, aiv_all_reduce_mesh_1d_twoshot.h:21-58)
    kIpcGeomBlock = 3,        // ReduceScatter: chunk c = input block c (reduce_scatter_op.cc:158-159)
    kIpcGeomWhole = 4,        // one-shot kinds and AllGather: every chunk is the whole range
    kIpcGeomV = 5,            // ReduceScatterV: chunk c = counts[c] elements at displs[c] (per-rank, any alignment)
};

// Everything that decides a one-sided call's bits: the kind, the fold order, the chunk layout and the executor loop
// that the layout is applied to (the reference slices every loop on its own).
struct IpcPlan {
    uint32_t kind;       // IpcKind
    uint32_t order;      // IpcOrder
    uint32_t geom;       // IpcGeom
    uint32_t group = 1;  // kIpcGeomBalanced: slices per chunk
    uint32_t subMode = 0;  // IpcSubMode (kIpcO6)
    uint64_t loopElems = 0;  // elements per executor loop (per block for ReduceScatter); 0 = one loop
};

// Sub-slices of a chunk for kIpcO6 (chunk coordinates): the MeshChunk AllReduce's even split (the first L % (n-1)
// one longer) or the MeshChunk ReduceScatter's 4-KiB split (schedule.cc SubSlicesEven / SubSlicesRs).
enum IpcSubMode : uint32_t {
    kIpcSubEven = 0,
    kIpcSubRs4K = 1,
};

// Kinds whose fold reads only slots and writes only the rank's own output (no result push, no phase 2). They need
// one barrier per round: their slots alternate between two areas that no other kind touches, so the next round's
// stores never meet this round's fold (k_ipc_collective). The others keep two (results must be complete before phase 2).
__host__ __device__ constexpr bool SingleBarrierKind(uint32_t kind)
{
    return kind == kIpcReduceScatter || kind == kIpcAllReduceOneShot || kind == kIpcReduceOneShot ||
           kind == kIpcAllGather;
}

// Kernel arguments. In rank mode (me >= 0) only in[me] / out[me] are used; stgIn / stgRes / flags hold every rank's
// mapping (own allocation at [me], peers opened through hipIpcOpenMemHandle). In world mode (me < 0) every table is
// full and blockIdx.y is the rank.
//
// Geometry (elements): chunk c of the input starts at c * chunkStride and holds min(chunkLen, total - c*chunkStride)
// elements (clamped at 0), or, balanced (group * n slices of chunkLen, the first rem one longer; chunk c = slices
// [c*group, (c+1)*group)), as the fields below say; rank c owns chunk c. The one-shot kinds use chunkStride = 0, chunkLen = total: every "chunk"
// is the whole range and every rank owns it. Round k handles piece k of every chunk: chunk elements
// [k*piece, (k+1)*piece). Block b always handles piece coordinates [b*blockElems, (b+1)*blockElems), so every round
// of a launch touches the same slot and result addresses per block and the per-block barrier is sound.
// Staging: owner c's slot q = stgIn[c] + q*piece; results of chunk c at stgRes[p] + c*piece. The single-barrier kinds
// (SingleBarrierKind) put their slots in one of two alternate areas instead, stgAlt[e & 1][c] + q*piece for the round
// whose barrier has epoch e (see k_ipc_collective).
struct IpcArgs {
    const void* in[kIpcMaxRanks];
    void* out[kIpcMaxRanks];
    void* stgIn[kIpcMaxRanks];
    void* stgRes[kIpcMaxRanks];
    void* stgAlt[2][kIpcMaxRanks];
    uint32_t* flags[kIpcMaxRanks];  // [blocks][n] per rank
    uint32_t n;
    int32_t me;
    uint32_t kind;  // IpcKind
    uint32_t order;    // IpcOrder
    uint32_t subMode;  // IpcSubMode (kIpcO6 only)
    uint32_t root;  // kIpcReduce, kIpcReduceOneShot
    uint64_t total;
    uint64_t chunkStride;
    uint64_t chunkLen;
    uint64_t rem;   // balanced: chunkLen is the slice length, rem the number of one-longer slices
    uint64_t group;  // balanced: slices per chunk; chunk c starts at c*group*chunkLen + min(c*group, rem) and holds
                     // group*chunkLen + min(group, rem - c*group clamped at 0) elements
    bool balanced;
    uint64_t piece;
    uint64_t blockElems;
    uint64_t tileElems;  // 0: block b's share of a piece is one window of blockElems; else tiles of tileElems at
                         // b, b + B, b + 2B, ... (B = blocks): the same piece coordinates in every round either way
    uint32_t nt;         // non-temporal loads and stores in the copy and fold loops
    uint32_t threads;    // threads per workgroup (kIpcBlock, or 512 by HCCL_AMD_IPC_THREADS)
    uint32_t fence;      // barrier fences: 1 = light (default): the waves' drains release the uncached staging, an
                         // agent-scope acquire (L1); 0 = system-scope release (XCD-wide L2 write-back) and acquire
                         // (L2 invalidate): HCCL_AMD_IPC_LIGHT_FENCE=0, and always with cached staging
    uint32_t rounds;
    uint32_t epochSpan;  // barriers per block in this launch: the device epoch counter advances by this much
    uint64_t outStride;  // kIpcAllGather: elements between consecutive ranks' blocks of the output (sendCount)
    uint64_t timeoutTicks;  // per barrier wait, in s_memrealtime ticks (100 MHz)
    uint32_t* failHost;  // host-visible word (pinned, coherent): set to 1 by the block whose barrier times out, read by
                         // the host at every collective entry (Comm::Gate) and by HcclGetCommAsyncError
    uint32_t* status;  // [0] bit 0: a barrier timed out (sticky per communicator); [2..3]: (callSeq << 32) | longest
                       // wait of that call, in polls (64-bit max); [4]: epoch counter (barriers so far, per block);
                       // [5]: blocks of the running launch that have finished (kIpcEpochWord, kIpcDoneWord)
    uint32_t callSeq;  // this call's sequence number on the communicator
    bool aligned;      // every in[] / out[] is 16-B aligned (chunks whose start is not are still element-wise)
    bool vgeom;                          // kIpcGeomV: chunk c is vStart[c], vLen[c] (elements)
    uint64_t vStart[kIpcMaxRanks];
    uint64_t vLen[kIpcMaxRanks];
    uint32_t rhdParts;       // kIpcRhd: RHD instances R (parts of the launch's range)
    uint32_t alignElems;     // kIpcRhd: HCCL_MIN_SLICE_ALIGN (128 B) in elements
    uint64_t rhdPartStride;  // kIpcRhd: elements per part (the last part may be shorter)
    uint8_t rhdReal[kIpcMaxRanks - 1][kIpcMaxRanks];  // kIpcRhd: per instance j, virtual rank -> real rank
    uint64_t* trace;  // HCCL_AMD_IPC_TRACE=1: per rank and block, kIpcTraceSlots s_memrealtime stamps of the phases
                      // (IpcTraceSlot); nullptr = off
    uint32_t ll;      // 1: the one-shot AllReduce through the LL area (flags beside the data, no barrier; LlOneShot)
    void* llUnpack[kIpcMaxRanks];  // ll: each rank's own cached unpack area, slot q at q * piece elements
};

// Phase stamps of one block (HCCL_AMD_IPC_TRACE, HcclAmdCommIpcTrace): 100 MHz s_memrealtime ticks, lane 0 of the
// block. The round stamps are those of the launch's last round. "issued" = lane 0's wave has issued the phase's last
// access (a barrier's own drain counts toward the barrier).
enum IpcTraceSlot : uint32_t {
    kTrEntry = 0,       // kernel entry (after the failed-communicator check)
    kTrRound = 1,       // start of the round
    kTrPhase0 = 2,      // phase 0 issued
    kTrBarrier1 = 3,    // first barrier passed
    kTrPhase1 = 4,      // phase 1 issued
    kTrBarrier2 = 5,    // second barrier passed (two-barrier kinds)
    kTrPhase2 = 6,      // phase 2 issued
    kTrExit = 7,        // lane 0's stores drained, before the launch's end count
    kIpcTraceSlots = 8,
};

HcclResult LaunchIpcCollective(const IpcArgs& a, uint32_t blocks, uint32_t worldRanks, HcclDataType dt,
                              HcclReduceOp op, hipStream_t stream);

// Per-dtype entry points of the kernels (ipc_k_*.hip, one translation unit per dtype group): the launch by op, and the
// kernel's address for the occupancy query (rhd: the kIpcRhd instantiation; ll: the LL kernel).
#define HCCL_AMD_IPC_DTYPE_DECL(NAME)                                                          \
    hipError_t LaunchIpc_##NAME(int op, const IpcArgs& a, dim3 grid, hipStream_t s); \
    const void* IpcKernel_##NAME(int op, bool rhd, bool ll);
HCCL_AMD_IPC_DTYPE_DECL(Int8)
HCCL_AMD_IPC_DTYPE_DECL(Int16)
HCCL_AMD_IPC_DTYPE_DECL(Int32)
HCCL_AMD_IPC_DTYPE_DECL(Int64)
HCCL_AMD_IPC_DTYPE_DECL(Uint64)
HCCL_AMD_IPC_DTYPE_DECL(Fp16)
HCCL_AMD_IPC_DTYPE_DECL(Bf16)
HCCL_AMD_IPC_DTYPE_DECL(Fp32)
HCCL_AMD_IPC_DTYPE_DECL(Fp64)
#undef HCCL_AMD_IPC_DTYPE_DECL

// Workgroups of the IPC kernel for (dt, op) that the device holds at once (occupancy x CUs; 0 if unknown). Every
// block of a launch waits at barriers for its peers' blocks, so the blocks that share a device must all be resident.
uint32_t IpcResidentBlocks(HcclDataType dt, HcclReduceOp op, bool rhd, bool ll, uint32_t threads);

// Writes back and invalidates every XCD's L2 at system scope (one maintenance block per CU); synchronous on `stream`.
HcclResult ScrubL2(hipStream_t stream);

// Staging of the one-sided kernel comes in two tiers, each one uncached allocation per rank holding the four areas
// (kIpcAreaIn, kIpcAreaRes, kIpcAreaAlt0, kIpcAreaAlt1), mapped by every peer, and each set up collectively by the
// first call that needs it:
//   kIpcTierSmall — areas of n x HCCL_AMD_SMALL_IPC_BYTES (at least n x 64 KiB): every call whose staging fits one
//                   round there (the small-call rule's calls and any other small one-sided call);
//   kIpcTierLarge — areas of HCCL_BUFFSIZE / 2, so the four hold 2 x HCCL_BUFFSIZE, the reference's CCL buffer pair
//                   (HCCL_BUFFSIZE.md; aiv_defines.h:44), unless HCCL_AMD_IPC_STAGING_MIB sets the area size.
// A communicator that only makes small calls therefore holds MiBs, not the large tier.
constexpr int kIpcTierSmall = 0;
constexpr int kIpcTierLarge = 1;
constexpr int kIpcTiers = 2;

struct IpcTier {
    bool ready = false;
    bool unavailable = false;  // its set-up failed on some rank: calls that need it report NOT_SUPPORT
    void* area[kIpcAreas] = {};  // own areas, parts of one uncached allocation at area[0]
    void* peerArea[kIpcAreas][kIpcMaxRanks] = {};
    bool opened[kIpcMaxRanks] = {};  // rank mode: the peer's allocation was opened with hipIpcOpenMemHandle
    uint64_t inBytes = 0;
    uint64_t resBytes = 0;
    uint64_t altBytes = 0;  // each of the two alternate slot areas of the single-barrier kinds
    uint64_t allocBytes() const { return inBytes + resBytes + 2 * altBytes; }
};

// Per-communicator state of the IPC path. `ready` covers what every call needs: the flags and LL area (one uncached
// allocation mapped by every peer), the status words, the failure word and the LL unpack area.
struct IpcState {
    bool ready = false;
    bool unavailable = false;      // set-up failed on some rank: every later call reports NOT_SUPPORT
    uint32_t* flags = nullptr;     // own flags, uncached, zeroed
    uint32_t* status = nullptr;    // device words: [0] bit 0 = barrier timeout, [2..3] = tagged longest wait (IpcArgs)
    uint32_t callSeq = 0;          // IPC calls issued on the communicator (tags the wait diagnostic)
    uint32_t* failHost = nullptr;  // pinned host word the kernel sets on a barrier timeout (hipHostMalloc, coherent)
    uint32_t* failDev = nullptr;   // the device address the launches write (IpcArgs::failHost): of failHost, or in a
                                   // loopback world of the world's word (Transport::SharedFailWord)
    uint32_t* peerFlags[kIpcMaxRanks] = {};
    bool flagsOpened[kIpcMaxRanks] = {};
    IpcTier tier[kIpcTiers];
    uint32_t blocks = 0;
    uint32_t ranksOnDevice = 1;    // rank mode: the most ranks that share one device (by PCI bus id), same on all ranks
    uint64_t* trace = nullptr;     // HCCL_AMD_IPC_TRACE=1 at set-up: [kIpcMaxRanks][kIpcMaxBlocks][kIpcTraceSlots]
    void* llUnpack = nullptr;      // own unpack area of the LL path (cached, kIpcLlUnpackBytes)
};

constexpr uint32_t kIpcBlocks = 128;     // workgroups per rank and launch in a loopback world (cap)
constexpr uint32_t kIpcMaxBlocks = 512;  // flags are sized for this many (HcclAmdCommSetIpcBlocks)
uint32_t DefaultIpcBlocks(uint64_t bytes);  // workgroups per launch when the communicator sets none (ipc.cc)
uint32_t LlIpcBlocks(uint32_t n, uint64_t bytes, bool rhd);  // the same for a launch in the LL form (ipc.cc)
constexpr size_t kIpcStatusBytes = 32;  // status words (IpcArgs::status)
constexpr int kIpcEpochWord = 4;
constexpr int kIpcDoneWord = 5;
constexpr int kIpcLlSeqWord = 6;  // LL launches so far (each advances it by one; the flag of launch s is s + 1)
// Flag words of a rank: [kIpcMaxBlocks][kIpcMaxRanks], at the start of its flag allocation.
constexpr uint64_t kIpcFlagBytes = uint64_t(kIpcMaxBlocks) * kIpcMaxRanks * sizeof(uint32_t);
// LL area (HCCL_AMD_IPC_LL_BYTES): behind the flags in the same uncached allocation (one IPC handle), two parities of
// kIpcMaxRanks source slots; a slot holds a call's input as 8-byte words {4 data bytes, 32-bit flag}, so twice the
// bytes of the largest LL call. The unpack area (own, cached) holds the n operands in the fold's slot layout.
constexpr uint64_t kIpcLlMaxBytes = 64ull << 10;
constexpr uint64_t kIpcLlSlotBytes = 2 * kIpcLlMaxBytes;
constexpr uint64_t kIpcLlParityBytes = uint64_t(kIpcMaxRanks) * kIpcLlSlotBytes;
constexpr uint64_t kIpcLlUnpackBytes = uint64_t(kIpcMaxRanks) * (kIpcLlMaxBytes + 256);
// The staging allocation of a rank (slot, result and two alternate areas) stays below 2 GiB: hipIpcOpenMemHandle never
// returned for a 2 GiB allocation on this stack (IpcSetup). The area size is CommConfig::ipcStagingBytes.
constexpr uint64_t kIpcStagingMaxBytes = 2047ull << 20;
// One staging area (HCCL_AMD_IPC_STAGING_MIB's range, and the cap of HCCL_BUFFSIZE / 2): two such areas leave the
// alternate areas 23.5 MiB each within kIpcStagingMaxBytes.
constexpr uint64_t kIpcStagingAreaMaxBytes = 1000ull << 20;

}  // namespace hccl_amd
