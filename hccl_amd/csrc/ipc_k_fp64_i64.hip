// ipc_k_fp64_i64.hip — the one-sided kernels for Fp64, Int64, Uint64 (ipc_kernel_body.h; one translation unit per dtype group so the
// instantiations compile in parallel).
#include "ipc_kernel_body.h"

namespace hccl_amd {

HCCL_AMD_IPC_DTYPE(Fp64, EFp<double>)
HCCL_AMD_IPC_DTYPE(Int64, EInt<int64_t, uint64_t>)
HCCL_AMD_IPC_DTYPE(Uint64, EInt<uint64_t, uint64_t>)

}  // namespace hccl_amd
